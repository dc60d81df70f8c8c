#!/bin/bash
# Round-end rehearsal on one MI355X: GPU suite, smoke(), headline bench at 20 and 50 steps, and a rocprofv3 kernel-stats
# pass of the headline bench.  One timeout per GPU step; the script stops at the first failing step.
#   usage (from this container): gpurun --timeout 1100 -- bash tools/gpu_rehearsal.sh [suite|bench|prof ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
STEPS="${*:-suite bench prof}"
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "step $name rc=$rc" >&2; if [ $rc -ne 0 ]; then exit $rc; fi; }
for s in $STEPS; do
  case $s in
    suite)
      run pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
      tail -1 $OUT/pytest_gpu.log
      run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      tail -1 $OUT/smoke.log ;;
    bench)
      run bench20 300 python bench.py --steps 20 --warmup 5 > $OUT/bench20.json 2> $OUT/bench20.err
      cat $OUT/bench20.json
      run bench50 300 python bench.py --steps 50 --warmup 5 > $OUT/bench50.json 2> $OUT/bench50.err
      cat $OUT/bench50.json ;;
    prof)
      run prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o headline -- python3 bench.py --steps 20 --warmup 5 > $OUT/prof.log 2>&1
      find $OUT/prof -name "*kernel_stats.csv" | head -3 ;;
  esac
done
