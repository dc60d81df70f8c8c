#!/bin/bash
# round-end rehearsal: GPU suite, smoke(), headline bench at 20 and 50 steps; one timeout per GPU step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "step $name rc=$rc" >&2; if [ $rc -ne 0 ]; then exit $rc; fi; }
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu_final.log 2>&1
tail -1 $OUT/pytest_gpu_final.log
run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
run bench20 300 python bench.py --steps 20 --warmup 3 > $OUT/bench20.json 2> $OUT/bench20.err
cat $OUT/bench20.json
run bench50 300 python bench.py --steps 50 --warmup 5 > $OUT/bench50.json 2> $OUT/bench50.err
cat $OUT/bench50.json
