#!/bin/bash
# Same-shape reference comparisons (secondary configs + headline reference rate), one timeout per GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "step $name rc=$rc" >&2; if [ $rc -ne 0 ]; then exit $rc; fi; }
run refcfg 600 python -u tools/ref_config_bench.py --which ${WHICH:-bert,image} --steps 2 > $OUT/ref_config_bench.json 2> $OUT/ref_config_bench.err
cat $OUT/ref_config_bench.json
run refhead 400 python -u tools/ref_bench.py --steps 10 --warmup 2 > $OUT/ref_bench.json 2> $OUT/ref_bench.err
cat $OUT/ref_bench.json
if [ "${LPIPS_EXP:-1}" = 1 ]; then
  run lpips_exp 400 python -u tools/lpips_trunk_exp.py > $OUT/lpips_trunk_exp.json 2> $OUT/lpips_trunk_exp.err
  cat $OUT/lpips_trunk_exp.json
fi
