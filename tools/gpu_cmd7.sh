#!/bin/bash
# full GPU suite (arena + graphs included), graph / arena benches, LPIPS layout experiment, BERTScore pairing check
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "step $name rc=$rc" >&2; if [ $rc -ne 0 ]; then exit $rc; fi; }
run new_tests 300 python -u -m pytest tests/test_graphs_gpu.py tests/unittests/bases/test_arena.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/new_tests.log 2>&1
tail -3 $OUT/new_tests.log
run graph_bench 300 python -u tools/graph_bench.py > $OUT/graph_bench.json 2> $OUT/graph_bench.err
cat $OUT/graph_bench.json
run arena_bench 300 python -u tools/arena_bench.py > $OUT/arena_bench.json 2> $OUT/arena_bench.err
cat $OUT/arena_bench.json
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -2 $OUT/pytest_gpu.log
run lpips_exp 300 python -u tools/lpips_trunk_exp.py > $OUT/lpips_trunk_exp.json 2> $OUT/lpips_trunk_exp.err
cat $OUT/lpips_trunk_exp.json
run refcfg 400 python -u tools/ref_config_bench.py --which bert --steps 1 > $OUT/ref_config_bert.json 2> $OUT/ref_config_bert.err
cat $OUT/ref_config_bert.json
