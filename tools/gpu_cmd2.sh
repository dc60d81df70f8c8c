#!/bin/bash
# round-2 GPU session: new kernel tests, order probe, compute host profile, bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "step $name rc=$rc" | tee -a $OUT/session.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
run probe 300 python tools/probes/softmax_order_probe.py > $OUT/probe.json 2> $OUT/probe.err
cat $OUT/probe.json
run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -3 $OUT/pytest_gpu.log
run cprof 300 python tools/compute_profile.py > $OUT/compute_profile.txt 2>&1
run bench 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
run prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 > $OUT/prof.log 2>&1
echo done
