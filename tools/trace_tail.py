"""Print the kernel timeline after the last update kernel of a rocprofv3 kernel trace (the compute() window)."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
marker = sys.argv[2] if len(sys.argv) > 2 else "class_hist"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = max(i for i, r in enumerate(rows) if marker in r["Kernel_Name"])
t0 = int(rows[idx]["End_Timestamp"])
busy = 0
for r in rows[idx - 2 :]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s >= t0:
        busy += e - s
    print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:8.1f}  {r['Kernel_Name'][:100]}")
print(f"kernel-busy after marker: {busy / 1000:.1f} us; span {(int(rows[-1]['End_Timestamp']) - t0) / 1000:.1f} us")
