"""Where does the headline collection's compute() block on the GPU?  After 20 queued updates (the bench window's
backlog), trace every Python / C call of compute() with sys.setprofile and print the calls that took > 10 us of wall
time (self + children), plus the total.  A call that waits for the update backlog shows up as ~1.5 ms."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import torchmetrics_forked_amd as tm  # noqa: E402
from torchmetrics_forked_amd import ops  # noqa: E402

ops.require()
dev = torch.device("cuda", 0)
C, B = 1000, 65536
coll = tm.MetricCollection({"auroc": tm.MulticlassAUROC(num_classes=C), "confmat": tm.MulticlassConfusionMatrix(num_classes=C)}).to(dev)
pool = [(torch.randn(B, C, device=dev).bfloat16(), torch.randint(0, C, (B,), device=dev)) for _ in range(4)]
for i in range(5):
    coll.update(*pool[i % 4])
coll.compute()
coll.reset()
torch.cuda.synchronize()

stack, events = [], []


def prof(frame, event, arg):  # noqa: ANN001
    if event in ("call", "c_call"):
        name = f"{os.path.basename(frame.f_code.co_filename)}:{frame.f_lineno}:{frame.f_code.co_name}" if event == "call" else f"C:{getattr(arg, '__qualname__', arg)}"
        stack.append((name, time.perf_counter(), len(stack)))
    elif event in ("return", "c_return", "c_exception"):
        if stack:
            name, t0, depth = stack.pop()
            events.append((t0, time.perf_counter() - t0, depth, name))


for i in range(20):
    coll.update(*pool[i % 4])
t0 = time.perf_counter()
sys.setprofile(prof)
coll.compute()
sys.setprofile(None)
t1 = time.perf_counter()
torch.cuda.synchronize()
print(f"compute wall (traced) {1e3 * (t1 - t0):.3f} ms")
for start, dur, depth, name in sorted(events):
    if dur > 10e-6:
        print(f"{1e6 * (start - t0):9.1f} us  {1e6 * dur:9.1f} us  {'  ' * depth}{name}")
