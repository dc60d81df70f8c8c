"""Per-config kernel times from a rocprofv3 kernel trace of tools/mc_small_probe.py: the probe generates each config's
logits (an ATen normal kernel) right before timing it, so the trace splits into one segment per config at those
kernels.  Prints the top kernels of each segment (calls, mean us, grid / block / VGPRs).

    python tools/trace_segments.py <kernel_trace.csv> [top]
"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 5
segs, cur = [], []
for r in rows:
    if "distribution" in r["Kernel_Name"] or "normal" in r["Kernel_Name"]:
        if cur:
            segs.append(cur)
        cur = []
        continue
    cur.append(r)
segs.append(cur)
for i, seg in enumerate(segs):
    agg = collections.defaultdict(lambda: [0, 0])
    for r in seg:
        k = f"{r['Kernel_Name'][:72]} g{r['Grid_Size_X']} b{r['Workgroup_Size_X']} v{r['VGPR_Count']} s{r['SGPR_Count']}"
        agg[k][0] += 1
        agg[k][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    print(f"=== segment {i}")
    for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{c:4d} {t / c / 1000:8.2f} us  {k}")
