#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "step $name rc=$rc" >&2; if [ $rc -ne 0 ]; then exit $rc; fi; }
run graph_bench 300 python -u tools/graph_bench.py > $OUT/graph_bench.json 2> $OUT/graph_bench.err
tail -1 $OUT/graph_bench.json
