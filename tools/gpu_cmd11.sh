#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "step $name rc=$rc" >&2; if [ $rc -ne 0 ]; then exit $rc; fi; }
run hun_tests 300 python -u -m pytest tests/unittests/audio/test_hungarian_native.py tests/unittests/audio/test_audio.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/hun_tests.log 2>&1
tail -2 $OUT/hun_tests.log
run hun_bench 120 python -u -c "
import time, json, torch, torchmetrics_forked_amd
from torchmetrics_forked_amd import ops; ops.require()
res = {}
for S in (4, 8, 16, 32):
    m = torch.randn(4096, S, S, dtype=torch.float64)
    t0 = time.perf_counter(); h = torch.ops.tmx.linear_assignment(m, True); th = time.perf_counter() - t0
    md = m.cuda(); torch.ops.tmx.linear_assignment_gpu(md, True); torch.cuda.synchronize()
    t0 = time.perf_counter(); d = torch.ops.tmx.linear_assignment_gpu(md, True); torch.cuda.synchronize(); td = time.perf_counter() - t0
    assert torch.equal(h, d.cpu())
    res[f'B4096_S{S}'] = {'host_ms': round(th * 1e3, 2), 'gpu_ms': round(td * 1e3, 3)}
print(json.dumps(res), flush=True)
" > $OUT/hun_bench.json 2> $OUT/hun_bench.err
cat $OUT/hun_bench.json
