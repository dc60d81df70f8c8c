#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "step $name rc=$rc" >&2; if [ $rc -ne 0 ]; then exit $rc; fi; }
run new_tests 300 python -u -m pytest tests/unittests/text/test_lcs_native.py tests/test_graphs_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/new_tests2.log 2>&1
tail -2 $OUT/new_tests2.log
run lcs_bench 200 python -u tools/lcs_bench.py > $OUT/lcs_bench.json 2> $OUT/lcs_bench.err
cat $OUT/lcs_bench.json
