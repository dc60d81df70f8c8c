"""Randomised edge-case drive of the native host (C++) ops — empty and single-token sequences, sequences longer
than one 64-bit word (multi-word bit-parallel paths), repeated tokens, degenerate assignment / filter inputs.
Exact ops are checked against small Python DPs; the rest for shape / finiteness.  ``tools/sanitize_host.py`` runs
this module (and the text / audio / detection suites) against an ASan + UBSan build of the same sources."""
import random

import pytest
import torch

from torchmetrics_forked_amd import ops


def _lev(a, b):
    prev = list(range(len(b) + 1))
    for i, x in enumerate(a, 1):
        cur = [i] + [0] * len(b)
        for j, y in enumerate(b, 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (x != y))
        prev = cur
    return prev[-1]


def _lcs(a, b):
    prev = [0] * (len(b) + 1)
    for x in a:
        cur = [0]
        for j, y in enumerate(b, 1):
            cur.append(prev[j - 1] + 1 if x == y else max(prev[j], cur[j - 1]))
        prev = cur
    return prev[-1]


def _flat(seqs):
    data, off = [], [0]
    for s in seqs:
        data.extend(s)
        off.append(len(data))
    return torch.tensor(data, dtype=torch.long), torch.tensor(off, dtype=torch.long)


def _seqs(rng, n, max_len, vocab):
    lens = [0, 1, 63, 64, 65, 130] + [rng.randint(0, max_len) for _ in range(n - 6)]
    return [[rng.randrange(vocab) for _ in range(k)] for k in lens]


@pytest.fixture(scope="module", autouse=True)
def _native():
    if not ops.load():
        pytest.skip("native library not built")


@pytest.mark.parametrize("seed", range(3))
def test_levenshtein_and_lcs_exact(seed):
    rng = random.Random(seed)
    a = _seqs(rng, 24, 150, 5 + seed * 10)
    b = list(reversed(_seqs(rng, 24, 150, 5 + seed * 10)))
    fa, oa = _flat(a)
    fb, ob = _flat(b)
    lev = torch.ops.tmx.levenshtein_batch(fa, oa, fb, ob).tolist()
    lcs = torch.ops.tmx.lcs_batch(fa, oa, fb, ob).tolist()
    assert lev == [_lev(x, y) for x, y in zip(a, b)]
    assert lcs == [_lcs(x, y) for x, y in zip(a, b)]


def test_text_metrics_edge_cases():
    from torchmetrics_forked_amd.functional.text import (
        bleu_score,
        char_error_rate,
        chrf_score,
        edit_distance,
        extended_edit_distance,
        rouge_score,
        translation_edit_rate,
        word_error_rate,
    )

    rng = random.Random(7)
    words = ["a", "b", "c", "the", "cat", "sat", "on", "mat"]
    preds = ["", "a", " ".join(rng.choice(words) for _ in range(90)), "the cat sat on the mat " * 12]
    refs = ["a b", "", " ".join(rng.choice(words) for _ in range(70)), "the cat sat on a mat " * 11]
    for fn in (word_error_rate, char_error_rate):
        assert torch.isfinite(fn(preds[2:], refs[2:]))
    assert edit_distance(preds, refs).shape == ()
    assert torch.isfinite(translation_edit_rate(preds[2:], [[r] for r in refs[2:]]))
    assert torch.isfinite(extended_edit_distance(preds[2:], [[r] for r in refs[2:]]))
    assert torch.isfinite(bleu_score(preds[2:], [[r] for r in refs[2:]], n_gram=4))
    assert torch.isfinite(chrf_score(preds[2:], [[r] for r in refs[2:]]))
    assert all(torch.isfinite(v) for v in rouge_score(preds[2:], refs[2:]).values())


@pytest.mark.parametrize("n", [1, 2, 5, 9])
def test_linear_assignment_degenerate(n):
    for metric in (torch.zeros(n, n), torch.ones(n, n), torch.randn(n, n), torch.arange(n * n, dtype=torch.float).reshape(n, n)):
        for maximize in (False, True):
            perm = torch.ops.tmx.linear_assignment(metric.double().unsqueeze(0), maximize)[0]
            assert sorted(perm.tolist()) == list(range(n))


def test_levinson_and_iir():
    r = torch.rand(3, 16, dtype=torch.float64)
    r[:, 0] += 16.0  # diagonally dominant Toeplitz systems
    b = torch.randn(3, 16, dtype=torch.float64)
    x = torch.ops.tmx.toeplitz_solve(r, b)
    idx = (torch.arange(16)[:, None] - torch.arange(16)[None, :]).abs()
    for k in range(3):
        torch.testing.assert_close(r[k][idx] @ x[k], b[k], rtol=1e-8, atol=1e-8)
    sig = torch.randn(2, 500, dtype=torch.float64)
    coef_b = torch.tensor([[0.2, 0.3]], dtype=torch.float64).repeat(2, 1)
    coef_a = torch.tensor([[1.0, -0.5]], dtype=torch.float64).repeat(2, 1)
    y = torch.ops.tmx.iir_filter(sig, coef_b, coef_a)
    assert y.shape == sig.shape and torch.isfinite(y).all()


def test_coco_eval_degenerate_images():
    from torchmetrics_forked_amd.detection import MeanAveragePrecision

    m = MeanAveragePrecision(iou_type="bbox")
    boxes = torch.tensor([[0.0, 0.0, 10.0, 10.0], [5.0, 5.0, 20.0, 20.0]])
    m.update([dict(boxes=torch.zeros(0, 4), scores=torch.zeros(0), labels=torch.zeros(0, dtype=torch.long))],
             [dict(boxes=boxes, labels=torch.tensor([1, 2]))])
    m.update([dict(boxes=boxes, scores=torch.tensor([0.9, 0.1]), labels=torch.tensor([1, 1]))],
             [dict(boxes=torch.zeros(0, 4), labels=torch.zeros(0, dtype=torch.long))])
    m.update([dict(boxes=boxes.repeat(60, 1), scores=torch.rand(120), labels=torch.randint(0, 3, (120,)))],
             [dict(boxes=boxes.repeat(5, 1), labels=torch.randint(0, 3, (10,)), iscrowd=torch.randint(0, 2, (10,)))])
    out = m.compute()
    assert all(torch.isfinite(v).all() or (v == -1).all() for k, v in out.items() if k != "classes")
