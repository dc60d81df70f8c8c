#!/bin/bash
# HBM-side bytes per headline update: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (TCC counter budget)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -s KILL "$@"; local rc=$?; echo "step $name rc=$rc" >&2; if [ $rc -ne 0 ]; then exit $rc; fi; }
run pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 5 --warmup 1 > $OUT/pmc_fetch.log 2>&1
run pmc_write 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 5 --warmup 1 > $OUT/pmc_write.log 2>&1
find $OUT/pmc_fetch $OUT/pmc_write -name "*counter_collection.csv"
