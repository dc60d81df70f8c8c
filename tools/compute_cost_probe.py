"""Where does the headline's ``compute_incl_sync_ms`` go?  (bench.py: elapsed wall time of 20 updates + compute +
synchronize, minus the GPU time of the 20 updates.)

Per window (the bench's exact sequence, repeated ``--reps`` times in one process) this records:
  * ``incl_sync_us``      -- bench.py's quantity;
  * ``gpu_compute_kernels_us`` -- GPU time from the end of the last update to the end of compute()'s kernels (an
                             event recorded just before compute's one flag read);
  * ``gpu_compute_us``    -- the same to an event recorded after compute() returned (adds the host's share);
  * ``compute_host_us``   -- host time inside compute() (it ends with the one flag read, i.e. a stream sync);
  * ``host_after_gpu_us`` -- incl_sync minus gpu_compute: launch-from-idle latency + sync wake-ups + Python after
                             the device finished;
and, once per process, the round trip of an empty kernel + synchronize on an idle GPU.
Variant (argv[1]): ``base`` or ``spin`` (hipSetDeviceFlags(hipDeviceScheduleSpin) before the HIP context exists:
synchronize busy-waits instead of yielding / sleeping).  One JSON line.

    python tools/compute_cost_probe.py [base|spin] [--reps 6]
"""
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    variant = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "base"
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 6
    flags_rc = None
    if variant == "spin":
        hip = ctypes.CDLL("libamdhip64.so")
        flags_rc = int(hip.hipSetDeviceFlags(ctypes.c_uint(1)))  # hipDeviceScheduleSpin
    import torch

    import torchmetrics_forked_amd as tm
    from torchmetrics_forked_amd import ops

    ops.require()
    dev = torch.device("cuda", 0)
    C, B, steps = 1000, 65536, 20
    g = torch.Generator(device=dev).manual_seed(1234)
    pool = [(torch.randn(B, C, device=dev, generator=g).bfloat16(), torch.randint(0, C, (B,), device=dev, generator=g)) for _ in range(4)]
    coll = tm.MetricCollection({"auroc": tm.MulticlassAUROC(num_classes=C), "confmat": tm.MulticlassConfusionMatrix(num_classes=C)}).to(dev)

    # an event just before compute()'s one flag read: the GPU time of compute's kernels without the host's share
    from torchmetrics_forked_amd.utilities import validation

    orig_read = validation.HostCheckBatch._read
    marks = []

    def read_marked(items):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        marks.append((ev, time.perf_counter()))
        return orig_read(items)

    validation.HostCheckBatch._read = staticmethod(read_marked)

    # idle round trip: one tiny kernel + synchronize
    x = torch.zeros(1, device=dev)
    rts = []
    for _ in range(50):
        torch.cuda.synchronize(dev)
        time.sleep(0.002)
        t0 = time.perf_counter()
        x.add_(1)
        torch.cuda.synchronize(dev)
        rts.append((time.perf_counter() - t0) * 1e6)

    out = {"variant": variant, "set_flags_rc": flags_rc, "idle_kernel_roundtrip_us": round(statistics.median(rts), 1), "windows": []}
    for _ in range(reps):
        for i in range(5):
            coll.update(*pool[i % 4])
        coll.compute()
        coll.reset()
        torch.cuda.synchronize(dev)
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        t0 = time.perf_counter()
        e0.record()
        for i in range(steps):
            coll.update(*pool[i % 4])
        e1.record()
        t1 = time.perf_counter()
        marks.clear()
        coll.compute()
        t2 = time.perf_counter()
        e2.record()
        torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        upd = e0.elapsed_time(e1) * 1e3
        gpu_c = e1.elapsed_time(e2) * 1e3
        gpu_k = e1.elapsed_time(marks[0][0]) * 1e3 if marks else float("nan")
        incl = (t3 - t0) * 1e6 - upd
        out["windows"].append({"incl_sync_us": round(incl, 1), "gpu_compute_kernels_us": round(gpu_k, 1), "gpu_compute_us": round(gpu_c, 1),
                               "compute_host_us": round((t2 - t1) * 1e6, 1), "n_reads": len(marks),
                               "host_to_read_us": round((marks[0][1] - t1) * 1e6, 1) if marks else None,
                               "read_to_return_us": round((t2 - marks[0][1]) * 1e6, 1) if marks else None,
                               "final_sync_us": round((t3 - t2) * 1e6, 1), "host_after_gpu_us": round(incl - gpu_c, 1),
                               "enqueue_us": round((t1 - t0) * 1e6, 1), "gpu_update_us_per_step": round(upd / steps, 2)})
    w = out["windows"]
    out["median"] = {k: round(statistics.median(d[k] for d in w), 1) for k in w[0]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
