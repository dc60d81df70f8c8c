"""Session-wide pool of 2 spawned processes joined in a gloo process group on 127.0.0.1.

Mirrors the reference's test strategy (reference ``tests/unittests/conftest.py:28-73``): multi-process
synchronisation is exercised without a cluster.  Functions sent to the pool must be importable (module level).
"""
import os
import socket
from typing import Any, Callable, List

from multiprocessing import TimeoutError as mp_TimeoutError

NUM_PROCESSES = 2
DDP_TIMEOUT_S = float(os.environ.get("TMX_TEST_DDP_TIMEOUT", "90"))
_POOL = None


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _init_worker(port: int, counter: Any) -> None:
    import torch
    import torch.distributed as dist

    with counter.get_lock():
        rank = counter.value
        counter.value += 1
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(NUM_PROCESSES)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=NUM_PROCESSES)


def _rank() -> int:
    import torch.distributed as dist

    return dist.get_rank()


def _call(fn: Callable, args: tuple) -> Any:
    import torch.distributed as dist

    r = dist.get_rank()
    out = fn(r, NUM_PROCESSES, *args)
    # a test body without collectives could finish before the other worker picks up its task, letting one worker
    # run both; the barrier holds each task until both ranks are in one, so the two tasks land on distinct ranks
    dist.barrier()
    return r, out


def get_pool():
    global _POOL
    if _POOL is None:
        import torch.multiprocessing as mp

        ctx = mp.get_context("spawn")
        counter = ctx.Value("i", 0)
        _POOL = ctx.Pool(NUM_PROCESSES, initializer=_init_worker, initargs=(_free_port(), counter))
        # make sure every worker joined the group (each task lands on a distinct worker only if they block)
    return _POOL


def run_ddp(fn: Callable, *args: Any) -> List[Any]:
    """Run ``fn(rank, world, *args)`` on both workers concurrently; returns results ordered by rank."""
    global _POOL
    pool = get_pool()
    try:
        # bounded: a rank that raised while its peer waits in a collective would otherwise hang the whole session
        res = pool.starmap_async(_call, [(fn, args)] * NUM_PROCESSES, chunksize=1).get(timeout=DDP_TIMEOUT_S)
    except mp_TimeoutError:
        pool.terminate()
        pool.join()
        _POOL = None
        raise AssertionError(f"ddp test body did not finish within {DDP_TIMEOUT_S} s (a rank hung in a collective)") from None
    assert sorted(r for r, _ in res) == list(range(NUM_PROCESSES)), "pool tasks did not land on distinct ranks"
    return [v for _, v in sorted(res, key=lambda x: x[0])]


def close_pool() -> None:
    global _POOL
    if _POOL is not None:
        _POOL.close()
        _POOL.join()
        _POOL = None
