#!/bin/bash
# secondary BASELINE configs at their real shapes (bench.py --config map|image|bert), one timeout each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "step $name rc=$rc" >&2; if [ $rc -ne 0 ]; then exit $rc; fi; }
run map 400 python bench.py --config map --steps 5 --warmup 1 > $OUT/cfg_map.json 2> $OUT/cfg_map.err
cat $OUT/cfg_map.json
run bert 500 python bench.py --config bert --steps 3 --warmup 1 > $OUT/cfg_bert.json 2> $OUT/cfg_bert.err
cat $OUT/cfg_bert.json
run image 600 python bench.py --config image --steps 2 --warmup 1 > $OUT/cfg_image.json 2> $OUT/cfg_image.err
cat $OUT/cfg_image.json
