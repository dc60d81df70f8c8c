"""GPU text DPs (csrc/text_dp.hip) vs their host ops: extended edit distance (one thread per pair, bit-identical
fp64) and clipped n-gram overlap (one wave per hypothesis, 128-bit keys); module-level EED / chrF / ROUGE-N with
GPU states equal the CPU metrics."""
import random

import pytest
import torch

from torchmetrics_forked_amd import ops

pytestmark = pytest.mark.gpu

_WORDS = "the a cat sat on mat dog ran far away home blue sky today , . ! ? and of to in it is was".split()


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


def _sent(rnd, lo=3, hi=30):
    return " ".join(rnd.choice(_WORDS) for _ in range(rnd.randint(lo, hi)))


def _pack(strings):
    from torchmetrics_forked_amd.functional.text.helper import _pack_codepoints

    return _pack_codepoints(strings)


@pytest.mark.parametrize("n_pairs", [1, 37, 700])
def test_eed_gpu_bit_identical_to_host(n_pairs):
    rnd = random.Random(n_pairs)
    hyps = [" " + _sent(rnd) + " " for _ in range(n_pairs)]
    refs = [" " + _sent(rnd) + " " for _ in range(n_pairs)]
    hyps[0] = " "  # degenerate rows
    h, ho = _pack(hyps)
    r, ro = _pack(refs)
    args = (ord(" "), 2.0, 0.3, 0.2, 1.0)
    host = torch.ops.tmx.eed_batch(h, ho, r, ro, *args)
    dev = torch.ops.tmx.eed_gpu(h.cuda(), ho.cuda(), r.cuda(), ro.cuda(), *args, max(len(x) for x in hyps))
    assert torch.equal(dev.cpu(), host)


@pytest.mark.parametrize("n_order,tok", [(6, "char"), (2, "word"), (4, "word"), (9, "word")])
def test_ngram_overlap_gpu_equals_host(n_order, tok):
    from torchmetrics_forked_amd.functional.text.helper import _pack as pack_ids
    from torchmetrics_forked_amd.functional.text.helper import _Vocab

    rnd = random.Random(n_order)
    hyps, groups, refs = [], [0], []
    for _ in range(300):
        s = _sent(rnd)
        hyps.append(list(s) if tok == "char" else s.split())
        k = rnd.randint(1, 3)
        for _ in range(k):
            t = _sent(rnd)
            refs.append(list(t) if tok == "char" else t.split())
        groups.append(groups[-1] + k)
    vocab = _Vocab()
    h, ho = pack_ids(hyps, vocab)
    r, ro = pack_ids(refs, vocab)
    g = torch.tensor(groups)
    host = torch.ops.tmx.ngram_overlap(h, ho, r, ro, g, n_order)
    bits = max(1, len(vocab._ids).bit_length())
    if n_order * bits > 128:
        pytest.skip("keys do not fit 128 bits")
    dev = torch.ops.tmx.ngram_overlap_gpu(h.cuda(), ho.cuda(), r.cuda(), ro.cuda(), g.cuda(), n_order, bits, max(len(x) for x in hyps))
    for a, b in zip(dev, host):
        assert torch.equal(a.cpu(), b)


def test_text_modules_gpu_equal_cpu():
    import torchmetrics_forked_amd.text as T

    rnd = random.Random(5)
    preds = [_sent(rnd, 10, 40) for _ in range(200)]
    target = [[_sent(rnd, 10, 40), _sent(rnd, 10, 40)] for _ in range(200)]
    for make in (lambda: T.ExtendedEditDistance(), lambda: T.CHRFScore(), lambda: T.CHRFScore(n_word_order=0),
                 lambda: T.ROUGEScore(rouge_keys=("rouge1", "rouge2", "rougeL"))):
        cpu, gpu = make(), make().cuda()
        cpu.update(preds, target)
        gpu.update(preds, target)
        a, b = cpu.compute(), gpu.compute()
        if isinstance(a, dict):
            for k in a:
                assert torch.allclose(a[k].float(), b[k].float().cpu(), atol=1e-6), k
        else:
            assert torch.allclose(a.float(), b.float().cpu(), atol=1e-6)
