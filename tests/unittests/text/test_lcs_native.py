"""ROUGE-L LCS kernels: host multi-word bit-parallel (tmx::lcs_batch) and the GPU wave kernel (tmx::lcs_gpu) against
a plain O(n m) dynamic program."""
import random

import pytest
import torch

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.functional.text.helper import _pack, _Vocab

pytestmark = pytest.mark.skipif(not ops.load(), reason="native library not built")


def _lcs_dp(a, b):
    prev = [0] * (len(b) + 1)
    for x in a:
        cur = [0] * (len(b) + 1)
        for j, y in enumerate(b, 1):
            cur[j] = prev[j - 1] + 1 if x == y else max(prev[j], cur[j - 1])
        prev = cur
    return prev[-1]


def _pairs(seed, n=60, vocab=12, max_len=300):
    rng = random.Random(seed)
    out = []
    for i in range(n):
        la, lb = rng.randint(0, max_len), rng.choice([0, 1, 63, 64, 65, 127, 128, 129, rng.randint(1, max_len)])
        out.append(([f"w{rng.randrange(vocab)}" for _ in range(la)], [f"w{rng.randrange(vocab)}" for _ in range(lb)]))
    return out


def _packed(pairs):
    v = _Vocab()
    a, a_off = _pack([p for p, _ in pairs], v)
    b, b_off = _pack([t for _, t in pairs], v)
    return a, a_off, b, b_off


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_host_lcs_matches_dp(seed):
    pairs = _pairs(seed)
    got = torch.ops.tmx.lcs_batch(*_packed(pairs)).tolist()
    assert got == [_lcs_dp(a, b) for a, b in pairs]


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
@pytest.mark.parametrize("seed", [0, 1])
def test_gpu_lcs_matches_host(seed):
    pairs = _pairs(seed, n=200, vocab=8, max_len=1024)
    packed = _packed(pairs)
    host = torch.ops.tmx.lcs_batch(*packed)
    max_ref = max(len(t) for _, t in pairs)
    dev = torch.ops.tmx.lcs_gpu(*[x.cuda() for x in packed], max_ref)
    assert torch.equal(dev.cpu(), host)
    small = pairs[:20]
    assert dev[:20].tolist() == [_lcs_dp(a, b) for a, b in small]


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_rouge_l_on_gpu_matches_cpu():
    from torchmetrics_forked_amd.text import ROUGEScore

    rng = random.Random(5)
    words = [f"tok{i}" for i in range(30)]
    preds = [" ".join(rng.choice(words) for _ in range(rng.randint(200, 600))) for _ in range(40)]
    target = [" ".join(rng.choice(words) for _ in range(rng.randint(200, 900))) for _ in range(40)]
    cpu, gpu = ROUGEScore(rouge_keys=("rougeL",)), ROUGEScore(rouge_keys=("rougeL",)).cuda()
    cpu.update(preds, target)
    gpu.update(preds, target)
    a, b = cpu.compute(), gpu.compute()
    for k in a:
        assert torch.allclose(a[k], b[k].cpu()), k
