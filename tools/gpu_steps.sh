#!/bin/bash
# Generic GPU session: runs the named steps in order, each under its own timeout; the first failure ends the session.
#   STEPS="t:tests/test_ops_detection_gpu.py b:map p:map" bash tools/gpu_steps.sh
#   t:<pytest target>   GPU pytest on that target
#   b:<config>          bench.py --config <config>  (auroc = headline)
#   p:<config>          rocprofv3 kernel-trace stats of bench.py --config <config>
#   k:<script>          python <script> (kernel micro-benchmarks)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "step $name rc=$rc" | tee -a $OUT/session.log >&2; if [ $rc -ne 0 ]; then exit $rc; fi; }
for s in ${STEPS}; do
  kind=${s%%:*}; arg=${s#*:}; tag=$(echo "$arg" | tr '/.:' '___')
  case $kind in
    t) run "pytest $arg" 600 python -u -m pytest "$arg" -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$tag.log 2>&1; tail -3 $OUT/pytest_$tag.log ;;
    b) run "bench $arg" 600 python bench.py --config $arg ${BENCH_ARGS:-} > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err; cat $OUT/bench_$tag.json ;;
    p) run "prof $arg" 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$tag -o run --output-format csv -- python3 bench.py --config $arg ${BENCH_ARGS:-} > $OUT/prof_$tag.log 2>&1 ;;
    k) run "script $arg" 600 env PYTHONPATH=$PWD python $arg > $OUT/script_$tag.log 2>&1; tail -20 $OUT/script_$tag.log ;;
  esac
done
echo "session done"
