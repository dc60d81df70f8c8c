"""Text metrics vs the reference implementation (pure-Python string metrics run directly; BERTScore / InfoLM
with a tiny random-init BERT built locally — no downloads).  ROUGE-Lsum and the Porter stemmer need nltk, which
is not installed: those paths are parity-unpinned here."""
import random

import pytest
import torch

import torchmetrics_forked_amd.functional.text as F
import torchmetrics_forked_amd.text as T

_WORDS = "the cat dog sat on a mat is big small red blue and or it was there here . , ! ?".split()


def _sentences(seed, n, lo=0, hi=14, words=_WORDS):
    rnd = random.Random(seed)
    return [" ".join(rnd.choice(words) for _ in range(rnd.randint(lo, hi))) for _ in range(n)]


def _refs(seed, n, k=3):
    rnd = random.Random(seed + 1000)
    return [_sentences(seed * 7 + i, rnd.randint(1, k), 1, 14) for i in range(n)]


def _close(a, b, atol=1e-6):
    if isinstance(a, (tuple, list)):
        for x, y in zip(a, b):
            _close(x, y, atol)
        return
    if isinstance(a, dict):
        assert set(a) == set(b), (set(a), set(b))
        for k in a:
            _close(a[k], b[k], atol)
        return
    a = torch.as_tensor(a).double()
    b = torch.as_tensor(b).double()
    torch.testing.assert_close(a.reshape(b.shape) if a.numel() == b.numel() else a, b, atol=atol, rtol=0, equal_nan=True)


@pytest.mark.parametrize("name", ["word_error_rate", "char_error_rate", "match_error_rate", "word_information_lost", "word_information_preserved"])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_asr_functional(reference, name, seed):
    import torchmetrics.functional.text as R

    p, t = _sentences(seed, 20, 1), _sentences(seed + 50, 20, 1)
    _close(getattr(F, name)(p, t), getattr(R, name)(p, t))
    _close(getattr(F, name)(p[0], t[0]), getattr(R, name)(p[0], t[0]))


def test_long_sequences_use_dp_path(reference):
    import torchmetrics.functional.text as R

    p = _sentences(3, 6, 70, 140)
    t = _sentences(4, 6, 70, 140)
    _close(F.word_error_rate(p, t), R.word_error_rate(p, t))
    _close(F.char_error_rate(p, t), R.char_error_rate(p, t))


@pytest.mark.parametrize("sub", [1, 2, 0])
@pytest.mark.parametrize("reduction", ["mean", "sum", "none"])
def test_edit_distance(reference, sub, reduction):
    import torchmetrics.functional.text as R

    p = _sentences(5, 12, 0, 30) + ["x" * 120, "abc"]
    t = _sentences(6, 12, 0, 30) + ["y" * 3 + "x" * 40, "a" * 90]  # very different lengths exercise the beam band
    _close(F.edit_distance(p, t, substitution_cost=sub, reduction=reduction), R.edit_distance(p, t, substitution_cost=sub, reduction=reduction))


@pytest.mark.parametrize("language", ["en", "ja"])
def test_eed(reference, language):
    import torchmetrics.functional.text as R

    p, t = _sentences(7, 10, 1), _refs(7, 10)
    a = F.extended_edit_distance(p, t, language=language, return_sentence_level_score=True)
    b = R.extended_edit_distance(p, t, language=language, return_sentence_level_score=True)
    _close(a, b)
    _close(F.extended_edit_distance(p, t, alpha=1.0, rho=0.5, deletion=0.3, insertion=0.7), R.extended_edit_distance(p, t, alpha=1.0, rho=0.5, deletion=0.3, insertion=0.7))


@pytest.mark.parametrize("kw", [{}, {"normalize": True}, {"no_punctuation": True}, {"lowercase": False}, {"normalize": True, "asian_support": True}])
def test_ter(reference, kw):
    import torchmetrics.functional.text as R

    p, t = _sentences(8, 15, 0, 25), _refs(8, 15)
    a = F.translation_edit_rate(p, t, return_sentence_level_score=True, **kw)
    b = R.translation_edit_rate(p, t, return_sentence_level_score=True, **kw)
    _close(a[0], b[0])
    _close(torch.cat(a[1]), torch.cat(b[1]))


def test_ter_long_shift_search(reference):
    import torchmetrics.functional.text as R

    rnd = random.Random(9)
    base = [rnd.choice(_WORDS) for _ in range(60)]
    shuffled = base[30:] + base[:30]
    p = [" ".join(shuffled), " ".join(base[::-1])]
    t = [[" ".join(base)], [" ".join(base), " ".join(shuffled)]]
    _close(F.translation_edit_rate(p, t), R.translation_edit_rate(p, t))


@pytest.mark.parametrize("n_gram", [1, 2, 4])
@pytest.mark.parametrize("smooth", [False, True])
def test_bleu(reference, n_gram, smooth):
    import torchmetrics.functional.text as R

    p, t = _sentences(10, 12, 3), _refs(10, 12)
    _close(F.bleu_score(p, t, n_gram=n_gram, smooth=smooth), R.bleu_score(p, t, n_gram=n_gram, smooth=smooth))


@pytest.mark.parametrize("tokenize", ["none", "13a", "zh", "intl", "char"])
@pytest.mark.parametrize("lowercase", [False, True])
def test_sacre_bleu(reference, tokenize, lowercase):
    import torchmetrics.functional.text as R

    words = _WORDS + ["The", "Cat", "中文", "测试", "3.5", "A-1", "&amp;", "x/y"]
    p = _sentences(11, 10, 3, 14, words)
    t = [_sentences(12 + i, 2, 3, 14, words) for i in range(10)]
    _close(F.sacre_bleu_score(p, t, tokenize=tokenize, lowercase=lowercase), R.sacre_bleu_score(p, t, tokenize=tokenize, lowercase=lowercase))


@pytest.mark.parametrize("kw", [{}, {"n_word_order": 0}, {"n_char_order": 3, "n_word_order": 1, "beta": 1.0}, {"lowercase": True, "whitespace": True}])
def test_chrf(reference, kw):
    import torchmetrics.functional.text as R

    p, t = _sentences(13, 12, 0, 14), _refs(13, 12)
    a = F.chrf_score(p, t, return_sentence_level_score=True, **kw)
    b = R.chrf_score(p, t, return_sentence_level_score=True, **kw)
    _close(a, b)


@pytest.mark.parametrize("accumulate", ["best", "avg"])
@pytest.mark.parametrize("keys", [("rouge1", "rouge2", "rougeL"), ("rouge3", "rougeL", "rouge1")])
def test_rouge(reference, accumulate, keys):
    import torchmetrics.functional.text as R

    p, t = _sentences(14, 10, 0, 14), _refs(14, 10)
    _close(F.rouge_score(p, t, accumulate=accumulate, rouge_keys=keys), R.rouge_score(p, t, accumulate=accumulate, rouge_keys=keys))


def test_rouge_lsum_runs_without_nltk():
    r = F.rouge_score(["The cat sat. It was big."], [["A cat sat. It is big!"]], rouge_keys=("rougeLsum",))
    assert 0 < float(r["rougeLsum_fmeasure"]) <= 1


def test_squad(reference):
    import torchmetrics.functional.text as R

    preds = [{"prediction_text": s, "id": str(i)} for i, s in enumerate(_sentences(15, 8, 0, 6))]
    target = [{"answers": {"answer_start": [0, 0], "text": a}, "id": str(i)} for i, a in enumerate(_refs(15, 8))]
    _close(F.squad(preds, target), R.squad(preds, target))


@pytest.mark.parametrize("ignore_index", [None, 1])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_perplexity(reference, ignore_index, dtype):
    import torchmetrics.functional.text as R

    g = torch.Generator().manual_seed(0)
    preds = torch.randn(3, 7, 11, generator=g, dtype=dtype)
    target = torch.randint(0, 11, (3, 7), generator=g)
    _close(F.perplexity(preds, target, ignore_index=ignore_index), R.perplexity(preds, target, ignore_index=ignore_index), atol=1e-5)


# ---------------------------------------------------------------------------------------------------------------
# modules
# ---------------------------------------------------------------------------------------------------------------
@pytest.mark.parametrize(
    ("cls", "kw"),
    [
        ("WordErrorRate", {}), ("CharErrorRate", {}), ("MatchErrorRate", {}), ("WordInfoLost", {}), ("WordInfoPreserved", {}),
        ("BLEUScore", {"n_gram": 3}), ("SacreBLEUScore", {"tokenize": "13a"}), ("CHRFScore", {}),
        ("TranslationEditRate", {}), ("ExtendedEditDistance", {}), ("EditDistance", {}), ("EditDistance", {"reduction": "none"}),
        ("ROUGEScore", {"rouge_keys": ("rouge1", "rougeL")}),
    ],
)
def test_modules_vs_reference(reference, cls, kw):
    import torchmetrics.text as R

    ours, theirs = getattr(T, cls)(**kw), getattr(R, cls)(**kw)
    multi_ref = cls in ("BLEUScore", "SacreBLEUScore", "CHRFScore", "TranslationEditRate", "ExtendedEditDistance", "ROUGEScore")
    for b in range(3):
        p = _sentences(20 + b, 6, 1)
        t = _refs(20 + b, 6) if multi_ref else _sentences(40 + b, 6, 1)
        ours.update(p, t)
        theirs.update(p, t)
    _close(ours.compute(), theirs.compute())


def _ddp_wer(rank, world):
    m = T.WordErrorRate()
    for b in range(rank, 4, world):
        m.update(_sentences(60 + b, 5, 1), _sentences(80 + b, 5, 1))
    return float(m.compute())


def _ddp_bleu(rank, world):
    m = T.BLEUScore()
    for b in range(rank, 4, world):
        m.update(_sentences(60 + b, 5, 3), _refs(60 + b, 5))
    return float(m.compute())


@pytest.mark.parametrize(("fn", "ref"), [("_ddp_wer", "wer"), ("_ddp_bleu", "bleu")])
def test_text_ddp(fn, ref):
    from tests.helpers.ddp import run_ddp

    got = run_ddp(globals()[fn])
    if ref == "wer":
        m = T.WordErrorRate()
        for b in range(4):
            m.update(_sentences(60 + b, 5, 1), _sentences(80 + b, 5, 1))
    else:
        m = T.BLEUScore()
        for b in range(4):
            m.update(_sentences(60 + b, 5, 3), _refs(60 + b, 5))
    assert all(abs(g - float(m.compute())) < 1e-6 for g in got)


# ---------------------------------------------------------------------------------------------------------------
# model-based metrics with a tiny local BERT
# ---------------------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def tiny_bert(tmp_path_factory):
    transformers = pytest.importorskip("transformers")
    d = tmp_path_factory.mktemp("tinybert")
    vocab = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"] + sorted(set(w.lower() for w in _WORDS))
    (d / "vocab.txt").write_text("\n".join(vocab) + "\n")
    tok = transformers.BertTokenizer(str(d / "vocab.txt"))
    cfg = transformers.BertConfig(vocab_size=len(vocab), hidden_size=32, num_hidden_layers=2, num_attention_heads=2,
                                  intermediate_size=64, max_position_embeddings=64)
    torch.manual_seed(0)
    mlm = transformers.BertForMaskedLM(cfg).eval()
    mlm.save_pretrained(str(d))
    tok.save_pretrained(str(d))
    return str(d), tok, mlm


def _ordered_pairs(n):
    # strictly increasing lengths on both sides: the reference's independent length sorts are then the identity,
    # so its pairing coincides with the correct one and the two implementations are comparable
    rnd = random.Random(3)
    p = [" ".join(rnd.choice(_WORDS[:18]) for _ in range(2 + i)) for i in range(n)]
    t = [" ".join(rnd.choice(_WORDS[:18]) for _ in range(3 + i)) for i in range(n)]
    return p, t


@pytest.mark.parametrize("kw", [{}, {"idf": True}, {"num_layers": 1}, {"all_layers": True}])
def test_bert_score_vs_reference(reference, tiny_bert, kw):
    from torchmetrics.functional.text import bert_score as ref_bs

    path, tok, mlm = tiny_bert
    model = mlm.bert
    p, t = _ordered_pairs(6)
    a = F.bert_score(p, t, model=model, user_tokenizer=tok, max_length=32, batch_size=4, **kw)
    b = ref_bs(p, t, model=model, user_tokenizer=tok, max_length=32, batch_size=4, **kw)
    for k in ("precision", "recall", "f1"):
        _close(a[k].cpu(), b[k], atol=1e-5)


def test_bert_score_module_and_correct_pairing(tiny_bert):
    path, tok, mlm = tiny_bert
    p, t = _ordered_pairs(5)
    # shuffled order: every prediction must still be scored against its own reference
    perm = [3, 0, 4, 1, 2]
    a = F.bert_score(p, t, model=mlm.bert, user_tokenizer=tok, max_length=32)
    b = F.bert_score([p[i] for i in perm], [t[i] for i in perm], model=mlm.bert, user_tokenizer=tok, max_length=32)
    _close(b["f1"], a["f1"][perm], atol=1e-6)
    m = T.BERTScore(model=mlm.bert, user_tokenizer=tok, max_length=32)
    m.update(p[:2], t[:2])
    m.update(p[2:], t[2:])
    _close(m.compute()["f1"], a["f1"], atol=1e-6)


@pytest.mark.parametrize("measure,kw", [("kl_divergence", {}), ("alpha_divergence", {"alpha": 0.5}), ("l2_distance", {}),
                                        ("fisher_rao_distance", {}), ("ab_divergence", {"alpha": 0.5, "beta": 0.5}),
                                        ("renyi_divergence", {"alpha": 0.5}), ("beta_divergence", {"beta": 0.5})])
@pytest.mark.parametrize("idf", [False, True])
def test_infolm_vs_reference(reference, tiny_bert, measure, kw, idf):
    from torchmetrics.functional.text import infolm as ref_infolm

    path, _, _ = tiny_bert
    p, t = _ordered_pairs(4)
    a = F.infolm(p, t, model_name_or_path=path, information_measure=measure, idf=idf, max_length=32, verbose=False,
                 return_sentence_level_score=True, **kw)
    b = ref_infolm(p, t, model_name_or_path=path, information_measure=measure, idf=idf, max_length=32, verbose=False,
                   return_sentence_level_score=True, **kw)
    _close(a[1], b[1], atol=1e-4)
