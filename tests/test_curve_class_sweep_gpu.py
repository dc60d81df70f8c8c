"""Independent oracle for every multiclass histogram route at the class counts of the round-5 sweep
(``tools/mc_small_probe.py``): the exact (class, label, 16-bit code) histogram built by the fused row + class passes vs
the one built from ATen's GPU softmax of the same logits, the fused confusion matrix vs ATen's arg-max, and AUROC / AP
from the histogram vs the sort-based computation on ATen's scores.

Routes covered: the small-class row pass (C <= 256: DIRECT 16-B loads for C % 8 == 0, LDS staging otherwise) with
the partial class pass; the tile row pass with rows read in place at
stride C for C % 8 != 0 (UNALIGNED, no padding copy: C = 300, 999, 1001); and the round-4 u16 class pass
(``TMX_CLASS_PASS_U16=1``, whole 65,536-row chunks whose 16-bit counters can wrap) in a child process.
The row pass sums exp(x - max) in a different fp32 order than ATen's softmax, so a quotient within an ulp of a 16-bit
rounding boundary may land one code away: per shape at most 2e-5 of the elements move, each by one code."""
import os
import subprocess
import sys

import pytest
import torch

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.ops import classification as K

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


def _hist_from_scores(scores, target, C):
    codes = scores.view(torch.int16).long() & 0x7FFF
    codes = torch.where(codes > 0x3FFF, torch.zeros_like(codes), codes)
    lab = (torch.arange(C, device=scores.device)[None, :] == target[:, None]).long()
    flat = (torch.arange(C, device=scores.device)[None, :] * 2 + lab) * K.N_CODES + codes
    h = torch.zeros(C, 2, K.N_CODES, dtype=torch.long, device=scores.device)
    h.view(-1).index_add_(0, flat.reshape(-1), torch.ones_like(flat.reshape(-1)))
    return h


def check_shape(C, N, seed=0, offset=0):
    """Fused histogram / confusion matrix / scores vs the ATen oracle; ``offset`` > 0 reads the logits from a view
    that starts ``offset`` elements into its storage (not 16-B aligned)."""
    from torchmetrics_forked_amd.functional.classification import _curve_engine as eng

    g = torch.Generator(device="cuda").manual_seed(1000 + C + seed)
    base = torch.randn(N * C + offset, device="cuda", generator=g).bfloat16()
    x = base[offset:].view(N, C)
    t = torch.randint(0, C, (N,), device="cuda", generator=g)
    t[::37] = -1  # ignored rows
    hist = torch.zeros(C, 2, K.N_CODES, dtype=torch.long, device="cuda")
    cm = torch.zeros(C, C, dtype=torch.long, device="cuda")
    K.curve_hist_update(x, t, hist, "multiclass", -1, cm)
    keep = t != -1
    ref = torch.softmax(x[keep].float(), dim=1).bfloat16()
    tk = t[keep]
    href = _hist_from_scores(ref, tk, C)
    moved = int((hist - href).abs().sum()) // 2
    assert moved <= max(4, int(2e-5 * N * C)), moved
    assert int(hist.sum()) == int(href.sum()) == int(keep.sum()) * C
    cm_ref = torch.zeros(C, C, dtype=torch.long, device="cuda")
    cm_ref.view(-1).index_add_(0, tk * C + x[keep].float().argmax(1), torch.ones_like(tk))
    assert torch.equal(cm, cm_ref)
    red = K.curve_hist_reduce(hist)
    labels = torch.nn.functional.one_hot(tk, C).bool()
    auc_s, ap_s, _, _ = eng.samples_scores(ref, labels)
    assert abs(red[:, 0].mean().item() - auc_s.mean().item()) <= 1e-6
    assert abs(red[:, 1].mean().item() - ap_s.mean().item()) <= 1e-6
    same = ((hist - href).abs().sum((1, 2)) == 0)  # classes without a moved score: exactly the sort-based result
    torch.testing.assert_close(red[same, 0], auc_s[same], rtol=0, atol=1e-12)
    torch.testing.assert_close(red[same, 1], ap_s[same], rtol=0, atol=1e-12)


@pytest.mark.parametrize(("C", "N"), [(10, 1 << 20), (64, 1 << 20), (100, 262_144), (104, 262_144), (256, 262_144),
                                      (300, 65_536 + 77), (999, 70_001), (1001, 65_536 + 123)])
def test_class_sweep_vs_aten_softmax_and_sort(C, N):
    check_shape(C, N)


@pytest.mark.parametrize(("C", "N", "offset"), [(1001, 65_536, 3), (100, 65_536, 1), (1000, 65_536, 5)])
def test_unaligned_logit_views_vs_aten(C, N, offset):
    """Logits whose storage offset breaks 16-B alignment: C % 8 != 0 reads rows in place; a C % 8 == 0 view that is
    not 16-B aligned takes the generic kernel (the two-pass routes need aligned vectors)."""
    check_shape(C, N, seed=1, offset=offset)


def test_u16_class_pass_wrap_vs_aten():
    """The round-4 u16 class pass (``TMX_CLASS_PASS_U16=1``; read once per process) counts whole 65,536-row chunks in
    16-bit LDS counters that wrap when every row of a chunk lands in one bin: one class whose codes are all equal over
    131,072 rows (two full chunks), beside softmax classes, against the ATen oracle -- in a child process."""
    code = (
        "import sys, torch; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
        "from test_curve_class_sweep_gpu import check_shape\n"
        "from torchmetrics_forked_amd.ops import classification as K\n"
        "from torchmetrics_forked_amd import ops; ops.require()\n"
        "check_shape(1000, 65_536 + 11)\n"
        "N, C = 131_072, 1000\n"
        "x = torch.full((N, C), -1.0, device='cuda').bfloat16()\n"  # logits (outside [0, 1]): every score 1/C, one code
        "t = torch.randint(0, C, (N,), device='cuda')\n"
        "hist = torch.zeros(C, 2, K.N_CODES, dtype=torch.long, device='cuda')\n"
        "K.curve_hist_update(x, t, hist, 'multiclass', None)\n"
        "ref = torch.softmax(x.float(), 1).bfloat16()\n"
        "code = int(ref[0, 0].view(torch.int16)) & 0x7FFF\n"
        "pos = torch.bincount(t, minlength=C)\n"
        "assert torch.equal(hist[:, 1, code], pos) and torch.equal(hist[:, 0, code], N - pos), 'u16 wrap'\n"
        "assert int(hist.sum()) == N * C\n"
        "print('ok')\n"
    ) % (os.path.dirname(os.path.abspath(__file__)), os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, TMX_CLASS_PASS_U16="1")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.strip().endswith("ok"), out.stdout[-2000:] + out.stderr[-4000:]
