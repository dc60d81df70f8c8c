"""Rank-local (sharded) BERTScore compute under DDP (gloo, 2 ranks): every rank embeds only its own pairs and the
per-pair scores are all-gathered; equals the replicated compute (token states gathered, full forward per rank)."""
import os
import tempfile

import pytest
import torch

from tests.helpers.multirank import run_multirank

_WORDS = "the cat sat on a mat while dog ran far away from home under blue sky today".split()


def _tiny():
    import transformers

    d = tempfile.mkdtemp()
    vocab = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"] + sorted(set(_WORDS))
    with open(os.path.join(d, "vocab.txt"), "w") as f:
        f.write("\n".join(vocab) + "\n")
    tok = transformers.BertTokenizer(os.path.join(d, "vocab.txt"))
    cfg = transformers.BertConfig(vocab_size=len(vocab), hidden_size=32, num_hidden_layers=2, num_attention_heads=2,
                                  intermediate_size=64, max_position_embeddings=64)
    torch.manual_seed(0)
    return tok, transformers.BertModel(cfg).eval()


def _pairs(r, n):
    import random

    rnd = random.Random(10 + r)
    p = [" ".join(rnd.choice(_WORDS) for _ in range(rnd.randint(2, 8))) for _ in range(n)]
    t = [" ".join(rnd.choice(_WORDS) for _ in range(rnd.randint(2, 8))) for _ in range(n)]
    return p, t


def check_sharded_bert(rank, world, device):
    from torchmetrics_forked_amd.text import BERTScore

    tok, model = _tiny()
    p, t = _pairs(rank, 3 + 2 * rank)
    kw = dict(model=model, user_tokenizer=tok, max_length=24)
    sharded, replicated = BERTScore(sharded_compute=True, **kw), BERTScore(**kw)
    sharded.update(p[:2], t[:2])
    sharded.update(p[2:], t[2:])
    replicated.update(p, t)
    a, b = sharded.compute(), replicated.compute()
    assert a["f1"].numel() == sum(3 + 2 * r for r in range(world))
    for k in ("precision", "recall", "f1"):
        torch.testing.assert_close(a[k].cpu(), b[k].cpu(), atol=1e-6, rtol=0)


def test_sharded_bert_score_gloo():
    pytest.importorskip("transformers")
    run_multirank(check_sharded_bert, 2, "gloo")
