#!/bin/bash
# headline bench (20 / 50 steps), a kernel trace and the GPU test-suite
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "step $name rc=$rc" >&2; if [ $rc -ne 0 ]; then exit $rc; fi; }
run bench 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
run bench50 300 python bench.py --steps 50 --warmup 5 > $OUT/bench50.json 2> $OUT/bench50.err
cat $OUT/bench50.json
rm -rf $OUT/prof
run prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 > $OUT/prof.log 2>&1
run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -3 $OUT/pytest_gpu.log
