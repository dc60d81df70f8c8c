#!/bin/bash
# A/B: row-pass code stores plain vs non-temporal (tools/kexp harness built with -DTMX_ROWPASS_NT_STORE=0/1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "step $name rc=$rc" >&2; if [ $rc -ne 0 ]; then exit $rc; fi; }
for i in 1 2; do
  run store0_$i 120 ./build/kexp_store0 > $OUT/kexp_store0_$i.json
  run store1_$i 120 ./build/kexp_store1 > $OUT/kexp_store1_$i.json
done
for f in $OUT/kexp_store*.json; do echo $f; python3 -c "import json,sys; d=json.load(open('$f')); print({k: d[k] for k in ('rowpass_logits_record_us','fixup_noop_us','class_pass_us','update_sequence_us')}, d['logits']['hist_l1'], d['logits_misspeculated']['confmat_diffs'])"; done
