"""Spawn ``world`` fresh processes joined in one process group (gloo on CPU, nccl = RCCL on MI355X) and run a
module-level check function on every rank.

Unlike ``tests/helpers/ddp.py`` (a session-wide 2-process gloo pool) this starts a new group per call, so the same
check bodies run at any world size and on either backend: the gloo runs here rehearse exactly the collective call
pattern the RCCL runs issue on a GPU node (one process per GPU, ``cuda:rank``).
"""
import os
import socket
import tempfile
import traceback
from typing import Any, Callable, List


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _entry(rank: int, fn: Callable, world: int, backend: str, port: int, outdir: str) -> None:
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.set_num_threads(2)
    status = "ok"
    try:
        if backend == "nccl":
            torch.cuda.set_device(rank)
            device = torch.device("cuda", rank)
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)
        elif backend == "gloo_cuda":  # gloo collectives (host), metric states on the one visible GPU
            device = torch.device("cuda", 0)
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            device = torch.device("cpu")
            dist.init_process_group("gloo", rank=rank, world_size=world)
        fn(rank, world, device)
        dist.barrier()
    except BaseException:  # noqa: BLE001 - reported to the parent
        status = traceback.format_exc()
    finally:
        with open(os.path.join(outdir, f"rank{rank}.txt"), "w") as f:
            f.write(status)
        if dist.is_initialized():
            dist.destroy_process_group()


def run_multirank(fn: Callable, world: int, backend: str = "gloo", timeout: float = 240.0) -> List[str]:
    """Run ``fn(rank, world, device)`` on ``world`` spawned ranks; raises with every failing rank's traceback."""
    import torch.multiprocessing as mp

    with tempfile.TemporaryDirectory() as outdir:
        ctx = mp.start_processes(
            _entry, args=(fn, world, backend, _free_port(), outdir), nprocs=world, join=False, start_method="spawn"
        )
        import time

        t0 = time.time()
        while not ctx.join(timeout=5):
            if time.time() - t0 > timeout:
                for p in ctx.processes:
                    if p.is_alive():
                        p.terminate()
                raise TimeoutError(f"multirank run of {fn.__name__} (world={world}, {backend}) exceeded {timeout}s")
        out: List[Any] = []
        for r in range(world):
            path = os.path.join(outdir, f"rank{r}.txt")
            out.append(open(path).read() if os.path.exists(path) else "no result file")
    bad = [f"rank {r}:\n{s}" for r, s in enumerate(out) if s != "ok"]
    if bad:
        raise AssertionError("\n".join(bad))
    return out
