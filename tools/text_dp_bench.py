"""GPU text kernels of csrc/text_dp.hip vs their host ops (one MI355X + the box's CPU cores):
  * EED pair DPs: ``tmx::eed_gpu`` (one thread per pair, bit-identical) vs ``tmx::eed_batch`` (parallel host);
  * EditDistance beam DPs: ``tmx::levenshtein_beam_gpu`` vs ``tmx::levenshtein_beam_batch``;
  * chrF character n-gram overlap (order 6) and ROUGE-2 word overlap: ``tmx::ngram_overlap_gpu`` vs ``tmx::ngram_overlap``.
GPU times include the host-to-device copies of the packed ids and the copy back.  Prints one JSON line."""
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from torchmetrics_forked_amd import ops  # noqa: E402
from torchmetrics_forked_amd.functional.text.helper import _pack, _pack_codepoints, _Vocab  # noqa: E402

WORDS = "the a cat sat on mat dog ran far away home blue sky today , . ! ? and of to in it is was model data".split()


def sent(rnd, lo, hi):
    return " ".join(rnd.choice(WORDS) for _ in range(rnd.randint(lo, hi)))


def best_of(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return 1e3 * best


def main() -> None:
    ops.require()
    dev = torch.device("cuda", 0)
    rnd = random.Random(0)
    out = {"host_threads": torch.get_num_threads()}
    # EED
    n = 4096
    hyps = [" " + sent(rnd, 15, 40) + " " for _ in range(n)]
    refs = [" " + sent(rnd, 15, 40) + " " for _ in range(n)]
    h, ho = _pack_codepoints(hyps)
    r, ro = _pack_codepoints(refs)
    args = (ord(" "), 2.0, 0.3, 0.2, 1.0)
    mx = max(len(x) for x in hyps)
    out["eed_pairs"] = n
    out["eed_mean_chars"] = round(h.numel() / n, 1)
    out["eed_host_ms"] = round(best_of(lambda: torch.ops.tmx.eed_batch(h, ho, r, ro, *args)), 2)
    out["eed_gpu_ms"] = round(best_of(lambda: torch.ops.tmx.eed_gpu(h.to(dev), ho.to(dev), r.to(dev), ro.to(dev), *args, mx).cpu()), 2)
    a = torch.ops.tmx.eed_batch(h, ho, r, ro, *args)
    b = torch.ops.tmx.eed_gpu(h.to(dev), ho.to(dev), r.to(dev), ro.to(dev), *args, mx).cpu()
    out["eed_identical"] = bool(torch.equal(a, b))
    # EditDistance beam DP (substitution cost 2)
    preds = [sent(rnd, 15, 40) for _ in range(n)]
    tgts = [sent(rnd, 15, 40) for _ in range(n)]
    p, po = _pack_codepoints(preds)
    t, to = _pack_codepoints(tgts)
    mr = max(len(x) for x in tgts)
    out["edit_pairs"] = n
    out["edit_host_ms"] = round(best_of(lambda: torch.ops.tmx.levenshtein_beam_batch(p, po, t, to, 1, 1, 2)), 2)
    out["edit_gpu_ms"] = round(best_of(lambda: torch.ops.tmx.levenshtein_beam_gpu(p.to(dev), po.to(dev), t.to(dev), to.to(dev), 1, 1, 2, mr).cpu()), 2)
    out["edit_identical"] = bool(torch.equal(torch.ops.tmx.levenshtein_beam_batch(p, po, t, to, 1, 1, 2),
                                             torch.ops.tmx.levenshtein_beam_gpu(p.to(dev), po.to(dev), t.to(dev), to.to(dev), 1, 1, 2, mr).cpu()))
    # TER shift search (one reference per hypothesis, block moves + substitutions)
    nt = 4096
    refs_w, hyps_w = [], []
    for _ in range(nt):
        r = sent(rnd, 10, 30).split()
        h = list(r)
        s0 = rnd.randrange(len(h) - 2)
        blk = h[s0:s0 + 3]
        del h[s0:s0 + 3]
        t0 = rnd.randrange(len(h) + 1)
        h[t0:t0] = blk
        h[rnd.randrange(len(h))] = rnd.choice(WORDS)
        refs_w.append(r)
        hyps_w.append(h)
    vocab_t = _Vocab()
    ta, tao = _pack(refs_w, vocab_t)
    tb, tbo = _pack(hyps_w, vocab_t)
    tg = torch.arange(nt + 1)
    ma, mb = max(map(len, refs_w)), max(map(len, hyps_w))
    out["ter_pairs"] = nt
    out["ter_host_ms"] = round(best_of(lambda: torch.ops.tmx.ter_batch(tb, tbo, ta, tao, tg)), 2)
    out["ter_gpu_ms"] = round(best_of(lambda: torch.ops.tmx.ter_gpu(ta.int().to(dev), tao.to(dev), tb.int().to(dev), tbo.to(dev), ma, mb).cpu()), 2)
    out["ter_identical"] = bool(torch.equal(torch.ops.tmx.ter_batch(tb, tbo, ta, tao, tg)[0],
                                            torch.ops.tmx.ter_gpu(ta.int().to(dev), tao.to(dev), tb.int().to(dev), tbo.to(dev), ma, mb).cpu()))
    # n-gram overlap
    for name, tok, order, nh in (("chrf_char6", list, 6, 20000), ("rouge2_word", str.split, 2, 50000)):
        hs, rs, groups = [], [], [0]
        for _ in range(nh):
            hs.append(tok(sent(rnd, 10, 30)))
            for _ in range(2):
                rs.append(tok(sent(rnd, 10, 30)))
            groups.append(groups[-1] + 2)
        vocab = _Vocab()
        hh, hho = _pack(hs, vocab)
        rr, rro = _pack(rs, vocab)
        g = torch.tensor(groups)
        bits = max(1, len(vocab._ids).bit_length())
        mh = max(len(x) for x in hs)
        out[f"{name}_hyps"] = nh
        out[f"{name}_host_ms"] = round(best_of(lambda: torch.ops.tmx.ngram_overlap(hh, hho, rr, rro, g, order)), 2)

        def gpu():
            d = [x.to(dev) for x in (hh, hho, rr, rro, g)]
            return [t.cpu() for t in torch.ops.tmx.ngram_overlap_gpu(*d, order, bits, mh)]

        out[f"{name}_gpu_ms"] = round(best_of(gpu), 2)
        host = torch.ops.tmx.ngram_overlap(hh, hho, rr, rro, g, order)
        out[f"{name}_identical"] = all(torch.equal(x, y) for x, y in zip(gpu(), host))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
