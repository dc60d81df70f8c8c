"""``bench.py --gpus N`` launches N ranks itself (torch.distributed.run child; gloo on a CPU-only host) and reports
the launched world size — the contract the driver's 1/2/4/8-GPU scaling runs rely on."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def _run(args):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                         timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_bench_spawns_requested_ranks():
    res = _run(["--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "512", "--num-classes", "16"])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2"
    assert res["config"]["global_batch"] == 1024 and res["steps"] == 2 and res["warmup"] == 1
    assert res["backend"] == "gloo" and res["sharded_compute"] is True
    assert 0.0 <= res["auroc"] <= 1.0 and res["value"] > 0


def test_bench_single_process_default():
    res = _run(["--steps", "2", "--warmup", "1", "--batch", "256", "--num-classes", "16"])
    assert res["n_gpus"] == 1 and res["config"]["parallelism"] == "dp1"
