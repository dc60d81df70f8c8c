#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "step $name rc=$rc" >&2; if [ $rc -ne 0 ]; then exit $rc; fi; }
run refcfg 400 python -u tools/ref_config_bench.py --which bert --steps 1 > $OUT/ref_config_bert.json 2> $OUT/ref_config_bert.err
cat $OUT/ref_config_bert.json
run arena_bench 300 python -u tools/arena_bench.py > $OUT/arena_bench.json 2> $OUT/arena_bench.err
cat $OUT/arena_bench.json
run graph_bench 300 python -u tools/graph_bench.py > $OUT/graph_bench.json 2> $OUT/graph_bench.err
cat $OUT/graph_bench.json
