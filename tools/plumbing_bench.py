"""BASELINE config 1 ("plumbing"): ``MulticlassAccuracy(num_classes=5)``, batch 10, CPU, gloo world 2 -- this framework
and the unmodified reference timed by the same harness (the reference's own DDP test pool is 2 gloo processes on
localhost, ``/root/reference/tests/unittests/conftest.py:28-73``).

Per rank: a pool of synthetic batches (fp32 logits ``[10, 5]`` + int64 labels), ``--warmup`` untimed steps + one
compute, ``reset()``, then the timed window of exactly ``--steps`` steps and ONE ``compute()`` (gloo all-reduce /
all-gather sync included), bracketed by barriers; max over ranks.  ``value`` = world * steps / seconds.
Modes: ``update`` (K updates + compute) and ``forward`` (K forward calls -- per-batch value + accumulation -- + compute).
One thread per rank (``torch.set_num_threads(1)``), as the reference's test pool.

Usage::

    python tools/plumbing_bench.py --impl tmx|ref [--steps 2000] [--warmup 50] [--world 2] [--mode update|forward|both]

Prints one JSON line per mode (rank 0).  ``bench.py --config plumbing`` runs the ``tmx`` side in the bench.py format.
"""
import argparse
import json
import os
import socket
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF_SRC = "/root/reference/src"


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _metric_cls(impl: str):
    if impl == "ref":
        for p in (os.path.join(REPO, "tests", "_oracle"), REF_SRC):
            if p not in sys.path:
                sys.path.append(p)
        import warnings

        warnings.filterwarnings("ignore")
        from torchmetrics.classification import MulticlassAccuracy
    else:
        if REPO not in sys.path:
            sys.path.insert(0, REPO)
        from torchmetrics_forked_amd.classification import MulticlassAccuracy
    return MulticlassAccuracy


def run_rank(impl: str, mode: str, steps: int, warmup: int, world: int, rank: int, num_classes: int = 5, batch: int = 10) -> dict:
    """One rank of the timed window (process group already initialised when world > 1)."""
    import torch
    import torch.distributed as dist

    torch.set_num_threads(1)
    cls = _metric_cls(impl)
    g = torch.Generator().manual_seed(1234 + rank)
    pool = [(torch.randn(batch, num_classes, generator=g), torch.randint(0, num_classes, (batch,), generator=g)) for _ in range(64)]
    metric = cls(num_classes=num_classes)
    step = metric.update if mode == "update" else metric.__call__

    for i in range(warmup):
        step(*pool[i % 64])
    if warmup:
        metric.compute()
    metric.reset()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        step(*pool[i % 64])
    t1 = time.perf_counter()
    res = metric.compute()
    t2 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # per-rank pieces, reduced separately (round 6): a rank whose loop finishes early waits inside compute()'s
    # collective for the slow one -- that wait is the loop skew, not compute work.  compute_own_s = this rank's
    # compute() call minus the time it spent waiting for the slowest rank's loop to end.
    upd, comp = t1 - t0, t2 - t1
    t = torch.tensor([elapsed, upd, upd, comp], dtype=torch.float64)
    if world > 1:
        tmax, tmin = t.clone(), t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(tmin, op=dist.ReduceOp.MIN)
        wait = float(tmax[1]) - upd  # how long this rank's compute waited for the slowest loop (lower bound)
        own = torch.tensor([max(comp - wait, 0.0)], dtype=torch.float64)
        dist.all_reduce(own, op=dist.ReduceOp.MAX)
        return {"elapsed": float(tmax[0]), "update_s": float(tmax[1]), "update_min_s": float(tmin[2]), "compute_s": float(tmax[3]),
                "compute_own_s": float(own[0]), "value_result": float(res)}
    return {"elapsed": elapsed, "update_s": upd, "update_min_s": upd, "compute_s": comp, "compute_own_s": comp, "value_result": float(res)}


def _report(impl: str, mode: str, steps: int, warmup: int, world: int, r: dict) -> dict:
    return {
        "metric": f"metric-updates/sec (whole job), MulticlassAccuracy 5-cls bs=10, {mode}",
        "impl": "torchmetrics_forked_amd" if impl == "tmx" else "reference (unmodified, /root/reference/src)",
        "value": round(world * steps / r["elapsed"], 1),
        "unit": "updates/s",
        "n_ranks": world,
        "backend": "gloo" if world > 1 else None,
        "steps": steps,
        "warmup": warmup,
        "us_per_step_incl_compute": round(1e6 * r["elapsed"] / steps, 2),
        "us_per_step_loop_only": round(1e6 * r["update_s"] / steps, 2),
        "compute_incl_sync_us": round(1e6 * (r["elapsed"] - r["update_s"]), 1),
        "compute_call_us_max_rank": round(1e6 * r["compute_s"], 1),
        "compute_own_us": round(1e6 * r["compute_own_s"], 1),
        "loop_skew_us": round(1e6 * (r["update_s"] - r["update_min_s"]), 1),
        "result": r["value_result"],
        "threads_per_rank": 1,
        "data": "synthetic fp32 logits [10, 5] + int64 labels, 64-batch pool per rank",
    }


def _entry(rank: int, args: argparse.Namespace, port: int, outdir: str) -> None:
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(args.world))
    if args.world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=args.world)
    try:
        lines = []
        for mode in (["update", "forward"] if args.mode == "both" else [args.mode]):
            r = run_rank(args.impl, mode, args.steps, args.warmup, args.world, rank)
            lines.append(json.dumps(_report(args.impl, mode, args.steps, args.warmup, args.world, r)))
        if rank == 0:
            with open(os.path.join(outdir, "out.jsonl"), "w") as f:
                f.write("\n".join(lines) + "\n")
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--impl", choices=["tmx", "ref"], default="tmx")
    ap.add_argument("--mode", choices=["update", "forward", "both"], default="both")
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--world", type=int, default=2)
    args = ap.parse_args(argv)
    import torch.multiprocessing as mp

    with tempfile.TemporaryDirectory() as outdir:
        mp.start_processes(_entry, args=(args, _free_port(), outdir), nprocs=args.world, join=True, start_method="spawn")
        print(open(os.path.join(outdir, "out.jsonl")).read(), end="", flush=True)


if __name__ == "__main__":
    main()
