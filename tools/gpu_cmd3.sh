#!/bin/bash
# GPU session: tests, headline bench, kernel trace, FETCH/WRITE counters (one counter group per pass)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "step $name rc=$rc" | tee -a $OUT/session.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
STEPS="${STEPS:-pytest,bench,prof,pmc}"
if [[ $STEPS == *pytest* ]]; then
  run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  tail -3 $OUT/pytest_gpu.log
fi
if [[ $STEPS == *bench* ]]; then
  run bench 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
  cat $OUT/bench.json
  run bench50 300 python bench.py --steps 50 --warmup 5 > $OUT/bench50.json 2> $OUT/bench50.err
  cat $OUT/bench50.json
fi
if [[ $STEPS == *prof* ]]; then
  rm -rf $OUT/prof
  run prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 > $OUT/prof.log 2>&1
fi
if [[ $STEPS == *pmc* ]]; then
  rm -rf $OUT/pmc_fetch $OUT/pmc_write
  run pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 > $OUT/pmc_fetch.log 2>&1
  run pmc_write 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 > $OUT/pmc_write.log 2>&1
fi
echo done
