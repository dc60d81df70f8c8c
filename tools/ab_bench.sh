#!/bin/bash
# Same-box A/B of two builds of the native library on the headline (alternating runs): build/ab_old/_tmx_native.so
# (TMX_NATIVE_LIB) vs the in-tree library.  usage: gpurun -- bash tools/ab_bench.sh <out-subdir> [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ab}; mkdir -p "$OUT"
for r in $(seq 1 "${2:-3}"); do
  for v in old new; do
    if [ $v = old ]; then export TMX_NATIVE_LIB=$PWD/build/ab_old/_tmx_native.so; else unset TMX_NATIVE_LIB; fi
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 > "$OUT/$v.$r.json" 2>/dev/null
    rc=$?; if [ $rc -ne 0 ]; then echo "bench $v rc=$rc"; exit $rc; fi
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['update_only_ms_per_step'], d['compute_incl_sync_ms'])" "$OUT/$v.$r.json" $v
  done
done
