"""Headline benchmark: metric-updates/sec of MulticlassAUROC + MulticlassConfusionMatrix (C=1000, bs=65536, bf16).

BASELINE.json config 2: "MulticlassAUROC + ConfusionMatrix num_classes=1000 bs=65536 bf16, 8xMI355X DDP sync".

One *step* = one ``MetricCollection.update(preds, target)`` on a fresh synthetic batch (bf16 logits
``[65536, 1000]`` + int64 labels, pre-generated in HBM and cycled, i.e. what a prefetching loader hands over).
The timed window is exactly K steps followed by ONE ``compute()`` (cross-rank RCCL sync + final AUROC over all
classes + confusion matrix), bracketed by barrier + device synchronize on both sides; the max over ranks is
reported.  ``value`` = world_size * K / max_rank_seconds (whole-job aggregate, weak scaling: per-GPU batch fixed).

Usage::

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config auroc|map|image|bert|plumbing]

* ``--gpus 1`` (default): one process.
* ``--gpus N`` without ``WORLD_SIZE`` in the environment: this process launches ``torch.distributed.run`` with N
  ranks on 127.0.0.1 as a child and exits with its code.  The launcher never touches the GPU itself.
* under ``torch.distributed.run`` (``WORLD_SIZE``/``RANK``/``LOCAL_RANK`` set): one rank per GPU, RCCL
  (``nccl`` backend) when a GPU is visible, gloo on CPU-only hosts.

Secondary BASELINE configs (``--config map|image|bert``) are implemented in ``tools/config_bench.py`` and print one
JSON line in the same format.  ``--config plumbing`` is BASELINE config 1 (``MulticlassAccuracy(num_classes=5)``,
batch 10, CPU, 2 gloo ranks, one thread each): ``tools/plumbing_bench.py`` times K ``update`` calls + one ``compute``
and, on a second line, K ``forward`` calls + one ``compute`` (``--impl ref`` there runs the unmodified reference).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _launch_ranks(n: int, argv: list) -> int:
    """Run this script under ``torch.distributed.run`` with ``n`` local ranks (child process; no exec, no GPU)."""
    cmd = [
        sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
        "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv,
    ]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "4")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def _baseline() -> "float | None":
    """BASELINE.json publishes no number.  BASELINE.md's config-2 row holds a builder-measured rate of the
    unmodified reference on one MI355X under this same harness (``profiles/reference_baseline_mi355x.json``, per-GPU
    updates/s).  Weak scaling: the whole-node baseline for N GPUs is N x that rate."""
    here = os.path.dirname(os.path.abspath(__file__))
    try:
        with open(os.path.join(here, "BASELINE.json")) as f:
            pub = json.load(f).get("published", {})
        if isinstance(pub, dict) and pub.get("metric_updates_per_sec_1gpu"):
            return float(pub["metric_updates_per_sec_1gpu"])
    except Exception:
        pass
    try:
        with open(os.path.join(here, "profiles", "reference_baseline_mi355x.json")) as f:
            return float(json.load(f)["ref_updates_per_sec"])
    except Exception:
        # profiles/ does not travel to the GPU box (.gpurunignore): the same measured rate, K = 50 updates + compute
        return _REF_MEASURED_UPDATES_PER_SEC


_REF_MEASURED_UPDATES_PER_SEC = 54.227  # profiles/reference_baseline_mi355x.json["ref_updates_per_sec"]


def _parse(argv: list) -> argparse.Namespace:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="auroc", choices=["auroc", "map", "image", "bert", "plumbing"])
    ap.add_argument("--num-classes", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--pool", type=int, default=4, help="distinct synthetic batches cycled through")
    ap.add_argument("--no-fuse", action="store_true", help="disable the fused collection update plan (A/B)")
    ap.add_argument("--replicated-compute", action="store_true",
                    help="all-reduce the full histogram and compute every class on every rank (A/B against the default"
                         " class-sharded compute: reduce-scatter by class + all-gather of per-class AUROC)")
    ap.add_argument("--small", action="store_true", help="(secondary configs) reduced shapes for CPU smoke runs")
    return ap.parse_args(argv)


def _worker(args: argparse.Namespace) -> None:
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: reporting the launched world size", file=sys.stderr)
    use_cuda = torch.cuda.is_available()
    if use_cuda:
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)
    else:
        device = torch.device("cpu")
    if world > 1:
        dist.init_process_group("nccl" if use_cuda else "gloo", device_id=device if use_cuda else None)

    if args.config != "auroc":
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
        from config_bench import run_config

        out = run_config(args, device, world, rank)
        if rank == 0 and out is not None:
            print(json.dumps(out), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    import torchmetrics_forked_amd as tm
    from torchmetrics_forked_amd import ops

    if use_cuda:
        ops.require()

    C, B = args.num_classes, args.batch
    coll = tm.MetricCollection(
        {
            "auroc": tm.MulticlassAUROC(num_classes=C, sharded_compute=world > 1 and not args.replicated_compute),
            "confmat": tm.MulticlassConfusionMatrix(num_classes=C),
        }
    ).to(device)
    if args.no_fuse:
        coll._fused_plans = []

    gen = torch.Generator(device=device).manual_seed(1234 + rank)
    pool = []
    for _ in range(args.pool):
        logits = torch.randn(B, C, device=device, generator=gen, dtype=torch.float32).to(torch.bfloat16)
        target = torch.randint(0, C, (B,), device=device, generator=gen)
        pool.append((logits, target))

    def sync() -> None:
        if use_cuda:
            torch.cuda.synchronize(device)

    def barrier() -> None:
        if world > 1:
            dist.barrier()

    # warmup (includes one compute so every kernel / collective path is initialised)
    for i in range(args.warmup):
        coll.update(*pool[i % args.pool])
    if args.warmup:
        coll.compute()
    coll.reset()
    sync()
    barrier()
    sync()

    # the timing events are created (and the runtime's event machinery initialised by one record) before the clock
    # starts: the first timing event of a process costs ~70 us of host time, which is measurement apparatus, not metric
    # work (tools/compute_cost_probe.py, profiles/compute_cost_r6.json)
    ev_start = torch.cuda.Event(enable_timing=True) if use_cuda else None
    ev_upd = torch.cuda.Event(enable_timing=True) if use_cuda else None
    if use_cuda:
        ev_upd.record()
        sync()
    t0 = time.perf_counter()
    if use_cuda:
        ev_start.record()
    for i in range(args.steps):
        coll.update(*pool[i % args.pool])
    if use_cuda:
        # (diagnostic split only: the updates' side-stream work -- the curve update lanes -- is joined into this stream
        # so the event closes the update share; compute would join it first anyway, the total is unaffected)
        for m in coll.values(copy_state=False):
            m._join_side_work()
        ev_upd.record()
    res = coll.compute()
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    upd_ms = ev_start.elapsed_time(ev_upd) if use_cuda else float("nan")

    t = torch.tensor([elapsed, upd_ms], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, upd_ms = float(t[0]), float(t[1])

    if rank == 0:
        value = world * args.steps / elapsed
        base = _baseline()
        out = {
            "metric": f"metric-updates/sec (whole node), MulticlassAUROC {C}-cls bs={B}",
            "value": round(value, 3),
            "unit": "updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / (base * world), 3) if base else None,
            "dtype": "bf16",
            "data": f"synthetic (randn bf16 logits [{B},{C}] + uniform int64 labels, pre-generated pool in HBM)",
            "config": {
                "model": f"MulticlassAUROC(num_classes={C})+MulticlassConfusionMatrix(num_classes={C})",
                "global_batch": B * world,
                "seq_len": 1,
                "parallelism": f"dp{world}",
            },
            "update_only_ms_per_step": round(upd_ms / args.steps, 4) if use_cuda else None,
            "compute_incl_sync_ms": round(1000.0 * elapsed - (upd_ms if use_cuda else 0.0), 3) if use_cuda else None,
            "auroc": float(res["auroc"]),
            "fused_update": not args.no_fuse,
            "sharded_compute": world > 1 and not args.replicated_compute,
            "backend": (dist.get_backend() if world > 1 else None),
            "device": torch.cuda.get_device_name(device) if use_cuda else "cpu",
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _plumbing(args: argparse.Namespace) -> None:
    """BASELINE config 1 on the CPU: 2 gloo ranks (spawned here; no GPU is touched), update and forward modes."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
    import contextlib
    import io

    import plumbing_bench

    steps = args.steps if args.steps != 50 else 2000  # the default K of the GPU configs is too short a CPU window
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        plumbing_bench.main(["--impl", "tmx", "--mode", "both", "--steps", str(steps), "--warmup", str(max(args.warmup, 50)), "--world", "2"])
    for line in buf.getvalue().splitlines():
        r = json.loads(line)
        out = {
            "metric": r["metric"], "value": r["value"], "unit": "updates/s", "n_gpus": 0, "n_ranks": r["n_ranks"],
            "steps": r["steps"], "warmup": r["warmup"], "ms_per_step": round(r["us_per_step_incl_compute"] / 1000.0, 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": r["data"],
            "config": {"model": "MulticlassAccuracy(num_classes=5)", "global_batch": 10 * r["n_ranks"], "seq_len": 1,
                       "parallelism": "gloo dp2 (CPU)"},
            "us_per_step_loop_only": r["us_per_step_loop_only"], "compute_incl_sync_us": r["compute_incl_sync_us"],
        }
        print(json.dumps(out), flush=True)


def main() -> None:
    argv = sys.argv[1:]
    args = _parse(argv)
    if args.config == "plumbing":
        _plumbing(args)
        return
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # launcher: N ranks as a child process group; this process never initialises the GPU
        sys.exit(_launch_ranks(args.gpus, argv))
    _worker(args)


if __name__ == "__main__":
    main()
