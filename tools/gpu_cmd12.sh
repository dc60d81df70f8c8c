#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "step $name rc=$rc" >&2; if [ $rc -ne 0 ]; then exit $rc; fi; }
run bleu_tests 300 python -u -m pytest tests/unittests/text/test_bleu_gpu.py tests/unittests/text -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/bleu_tests.log 2>&1
tail -2 $OUT/bleu_tests.log
run bleu_bench 200 python -u -c "
import time, json, random, torch
from torchmetrics_forked_amd import ops; ops.require()
from torchmetrics_forked_amd.functional.text.helper import _pack, _Vocab
rng = random.Random(0); W = [f'w{i}' for i in range(5000)]
hyps = [[rng.choice(W) for _ in range(rng.randint(10, 60))] for _ in range(20000)]
refs = [[[rng.choice(W) for _ in range(rng.randint(10, 60))] for _ in range(4)] for _ in range(20000)]
v = _Vocab(); h, ho = _pack(hyps, v); r, ro = _pack([x for rs in refs for x in rs], v)
g = torch.tensor([0] + [4] * len(refs)).cumsum(0)
t0 = time.perf_counter(); host = torch.ops.tmx.bleu_stats(h, ho, r, ro, g, 4); th = time.perf_counter() - t0
d = [x.cuda() for x in (h, ho, r, ro, g)]; torch.ops.tmx.bleu_stats_gpu(*d, 4, 60); torch.cuda.synchronize()
t0 = time.perf_counter(); dev = torch.ops.tmx.bleu_stats_gpu(*d, 4, 60); torch.cuda.synchronize(); td = time.perf_counter() - t0
assert all(torch.equal(a, b.cpu()) for a, b in zip(host, dev))
print(json.dumps({'sentences': 20000, 'refs_per_sentence': 4, 'tokens': '10-60', 'host_ms': round(th * 1e3, 2), 'gpu_ms': round(td * 1e3, 3)}), flush=True)
" > $OUT/bleu_bench.json 2> $OUT/bleu_bench.err
cat $OUT/bleu_bench.json
