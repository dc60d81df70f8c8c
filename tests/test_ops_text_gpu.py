"""gfx950 text kernels vs PyTorch references: fused token NLL (Perplexity) and MFMA BERTScore greedy matching."""
import pytest
import torch

from torchmetrics_forked_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


@pytest.mark.parametrize("shape", [(2, 5, 7), (4, 128, 30522), (1, 3, 50257), (8, 64, 1000)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.bfloat16])
@pytest.mark.parametrize("ignore_index", [None, 0])
def test_token_nll_kernel(shape, dtype, ignore_index):
    g = torch.Generator().manual_seed(shape[-1])
    logits = (torch.randn(*shape, generator=g) * 3).to(dtype)
    target = torch.randint(0, shape[-1], shape[:2], generator=g)
    nll = torch.ops.tmx.token_nll(logits.reshape(-1, shape[-1]).cuda(), target.reshape(-1).cuda(),
                                  0 if ignore_index is None else ignore_index, ignore_index is not None)
    ref = -torch.log_softmax(logits.double().reshape(-1, shape[-1]), 1).gather(1, target.reshape(-1, 1)).squeeze(1)
    if ignore_index is not None:
        ref = torch.where(target.reshape(-1) == ignore_index, torch.zeros_like(ref), ref)
    tol = 1e-9 if dtype == torch.float64 else 2e-4
    torch.testing.assert_close(nll.double().cpu(), ref, atol=tol, rtol=tol)


def test_perplexity_gpu_matches_cpu():
    from torchmetrics_forked_amd.functional.text import perplexity

    g = torch.Generator().manual_seed(1)
    preds = torch.randn(4, 33, 517, generator=g)
    target = torch.randint(0, 517, (4, 33), generator=g)
    torch.testing.assert_close(perplexity(preds.cuda(), target.cuda(), ignore_index=3).cpu(), perplexity(preds, target, ignore_index=3),
                               atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("shape", [(3, 40, 50, 32), (2, 1000, 1024, 40), (1, 256, 768, 776), (3, 512, 512, 64), (2, 128, 64, 768), (5, 17, 33, 24), (64, 512, 512, 768), (2, 300, 129, 72), (2, 130, 257, 20)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_bert_greedy_match_kernel(shape, dtype):
    b, lp, lr, d = shape
    g = torch.Generator().manual_seed(lp * lr)
    p = torch.nn.functional.normalize(torch.randn(b, lp, d, generator=g), dim=-1)
    r = torch.nn.functional.normalize(torch.randn(b, lr, d, generator=g), dim=-1)
    p[:, 0] = 0  # masked special token
    pq, rq = p.to(dtype), r.to(dtype)
    rowmax, colmax = torch.ops.tmx.bert_greedy_match(pq.cuda(), rq.cuda())
    sim = torch.bmm(pq.double(), rq.double().transpose(1, 2))
    tol = 1e-5 if dtype == torch.float32 else 2e-3
    torch.testing.assert_close(rowmax.cpu().double(), sim.max(2).values, atol=tol, rtol=0)
    torch.testing.assert_close(colmax.cpu().double(), sim.max(1).values, atol=tol, rtol=0)


def test_bert_score_gpu_matches_cpu():
    transformers = pytest.importorskip("transformers")
    from torchmetrics_forked_amd.functional.text import bert_score

    cfg = transformers.BertConfig(vocab_size=100, hidden_size=64, num_hidden_layers=2, num_attention_heads=2, intermediate_size=128)
    torch.manual_seed(0)
    model = transformers.BertModel(cfg).eval()
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(5, 100, (6, 24), generator=g)
    mask = torch.ones_like(ids)
    mask[:, 18:] = 0
    tids = torch.randint(5, 100, (6, 24), generator=g)
    preds, target = {"input_ids": ids, "attention_mask": mask}, {"input_ids": tids, "attention_mask": torch.ones_like(tids)}
    cpu = bert_score(preds, target, model=model, idf=True)
    gpu = bert_score(preds, target, model=model.cuda(), idf=True, device="cuda")
    for k in ("precision", "recall", "f1"):
        torch.testing.assert_close(gpu[k].cpu(), cpu[k], atol=1e-4, rtol=0)


@pytest.mark.parametrize("max_len,vocab,n", [(20, 6, 500), (64, 3, 300), (65, 4, 200), (300, 5, 64), (1024, 8, 16), (200, 1000, 50)])
def test_levenshtein_gpu_matches_host(max_len, vocab, n):
    """One wave per pair, multi-word bit-parallel DP (csrc/text_gpu.hip) vs the host kernel (Myers / two-row DP)."""
    from torchmetrics_forked_amd.functional.text.helper import _levenshtein_many

    g = torch.Generator().manual_seed(max_len * 7 + vocab)
    preds = [torch.randint(0, vocab, (int(torch.randint(0, max_len + 1, (1,), generator=g)),), generator=g).tolist() for _ in range(n)]
    target = [torch.randint(0, vocab, (int(torch.randint(0, max_len + 1, (1,), generator=g)),), generator=g).tolist() for _ in range(n)]
    target[0], preds[1] = [], []  # empty sides
    host = _levenshtein_many(preds, target)
    dev = _levenshtein_many(preds, target, torch.device("cuda"), force_gpu=True)
    assert dev.is_cuda
    assert torch.equal(dev.cpu(), host)


def test_wer_family_gpu_states_large_batch_matches_cpu():
    import torchmetrics_forked_amd.text as T

    g = torch.Generator().manual_seed(0)
    words = ["w%d" % i for i in range(30)]
    mk = lambda k: " ".join(words[int(i)] for i in torch.randint(0, 30, (k,), generator=g))  # noqa: E731
    preds = [mk(int(torch.randint(1, 90, (1,), generator=g))) for _ in range(3000)]
    target = [mk(int(torch.randint(1, 90, (1,), generator=g))) for _ in range(3000)]
    for cls in (T.WordErrorRate, T.CharErrorRate, T.MatchErrorRate, T.WordInfoLost, T.WordInfoPreserved):
        gpu, cpu = cls().cuda(), cls()
        gpu.update(preds, target)
        cpu.update(preds, target)
        torch.testing.assert_close(gpu.compute().cpu(), cpu.compute(), atol=1e-6, rtol=1e-6)
