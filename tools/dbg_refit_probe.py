import sys, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
from test_curve_refit_gpu import _batch, _run
from torchmetrics_forked_amd import ops
ops.require()
for dtype in (torch.float16, torch.bfloat16):
    for C in (10, 64, 250):
        x, t = _batch(3001, C, False, dtype, seed=C)
        good = _run(x, t, 1); bad = _run(x, t, 0)
        d = (good[0] - bad[0]).nonzero()
        print(dtype, C, 'hist diffs', d.shape[0], 'cm equal', torch.equal(good[1], bad[1]))
        for c, lab, code in d[:12].tolist():
            print('  class', c, 'label', lab, 'code', hex(code), 'good', int(good[0][c, lab, code]), 'bad', int(bad[0][c, lab, code]))
