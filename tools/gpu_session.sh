#!/bin/bash
# One GPU session: gpu tests, headline bench, rocprofv3 kernel stats, reference baseline.
# Every GPU step has its own timeout; a fault/abort/timeout stops the session (no further GPU work).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
stop_if_fatal() {  # $1 = exit code, $2 = step name
  local rc=$1
  # any failing GPU step ends the session: a fault, abort, timeout or error leaves nothing else to run
  if [ $rc -ne 0 ]; then
    echo "FATAL step '$2' rc=$rc - stopping GPU session" | tee -a $OUT/session.log; exit $rc
  fi
  echo "step '$2' rc=$rc" | tee -a $OUT/session.log
}
STEPS="${STEPS:-pytest,bench,prof}"
if [[ $STEPS == *pytest* ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; stop_if_fatal $? pytest; tail -5 $OUT/pytest_gpu.log
fi
if [[ $STEPS == *kexp* ]]; then
  timeout -k 10 120 ./build/curve_hist_exp > $OUT/kexp.json 2> $OUT/kexp.err; stop_if_fatal $? kexp; cat $OUT/kexp.json
fi
if [[ $STEPS == *kbench* ]]; then
  timeout -k 10 300 python tools/kbench.py > $OUT/kbench.json 2> $OUT/kbench.err; stop_if_fatal $? kbench; cat $OUT/kbench.json
fi
if [[ $STEPS == *,bench* ]] || [[ $STEPS == bench* ]]; then
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err; stop_if_fatal $? bench; cat $OUT/bench.json
fi
if [[ $STEPS == *prof* ]]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 > $OUT/prof.log 2>&1; stop_if_fatal $? prof
  find $OUT/prof -name "*kernel_stats.csv" | head -3
fi
if [[ $STEPS == *domain* ]]; then
  timeout -k 10 900 python tools/domain_bench.py ${DOMAIN_ARGS:-} > $OUT/domain_bench.json 2> $OUT/domain_bench.err; stop_if_fatal $? domain; cat $OUT/domain_bench.json
fi
if [[ $STEPS == *kkern* ]]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_kern -o kern --output-format csv -- python3 tools/kbench_kernels.py > $OUT/kbench_kernels.log 2>&1; stop_if_fatal $? kkern
  grep '^{' $OUT/kbench_kernels.log > $OUT/kbench_kernels.json || true
  cat $OUT/kbench_kernels.json
fi
if [[ $STEPS == *ref* ]]; then
  timeout -k 10 900 python tools/ref_bench.py --steps 10 --warmup 2 > $OUT/ref_bench.json 2> $OUT/ref_bench.err; stop_if_fatal $? ref; cat $OUT/ref_bench.json
fi
echo "session done"
