"""Per-kernel microbenchmark at the headline shape (bf16 logits [65536, 1000]); times with HIP events."""
import json
import sys

import torch

sys.path.insert(0, ".")
from torchmetrics_forked_amd.ops import classification as K  # noqa: E402


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1000.0  # us


def main():
    N, C = 65536, 1000
    dev = torch.device("cuda")
    x = torch.randn(N, C, device=dev).bfloat16()
    t = torch.randint(0, C, (N,), device=dev)
    hist = torch.zeros(C, 2, K.N_CODES, dtype=torch.long, device=dev)
    cm = torch.zeros(C, C, dtype=torch.long, device=dev)
    res = {
        "range_flag_us": timeit(lambda: K.range_flag(x)),
        "curve_hist_update_us": timeit(lambda: K.curve_hist_update(x, t, hist, "multiclass", None)),
        "curve_hist_update_fused_confmat_us": timeit(lambda: K.curve_hist_update(x, t, hist, "multiclass", None, cm)),
        "curve_hist_reduce_us": timeit(lambda: K.curve_hist_reduce(hist)),
        "mc_confmat_update_us": timeit(lambda: K.mc_confmat_update(x, t, cm, None)),
        "aten_softmax_us": timeit(lambda: x.softmax(1)),
        "hbm_copy_131MB_us": timeit(lambda: x.clone()),
    }
    print(json.dumps({k: round(v, 1) for k, v in res.items()}))


if __name__ == "__main__":
    main()
