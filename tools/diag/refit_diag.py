"""Where does the refit differ from a correct prediction (fp16, small-class route)?  Prints differing bins."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_curve_refit_gpu import _batch, _run  # noqa: E402

for dtype in (torch.float16, torch.bfloat16):
    for C in (10, 64, 520):
        x, t = _batch(3001, C, False, dtype, seed=C)
        good = _run(x, t, speculated=1)
        bad = _run(x, t, speculated=0)
        d = (good[0] != bad[0]).nonzero()
        print(dtype, C, "diff bins", d.shape[0], "good sum", int(good[0].sum()), "bad sum", int(bad[0].sum()),
              "pos good/bad", int(good[0][:, 1].sum()), int(bad[0][:, 1].sum()))
        for row in d[:12].tolist():
            c, k, b = row
            print("   class", c, "pos" if k else "neg", "bin", hex(b), "good", int(good[0][c, k, b]), "bad", int(bad[0][c, k, b]))
