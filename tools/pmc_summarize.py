"""Summarise tools/pmc_headline.sh passes: mean per dispatch of every counter, per headline kernel (row pass
mc_codes_kernel, class pass class_hist_hi_kernel), as one JSON object.

    python tools/pmc_summarize.py gpurun_out/<dir> > profiles/pmc_headline_rNN.json
"""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        kind = "row_pass" if "mc_codes_kernel" in name else ("class_pass" if "class_hist" in name else None)
        if kind:
            acc[kind][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: {c: round(sum(v) / len(v), 1) for c, v in sorted(d.items())} for k, d in acc.items()}
print(json.dumps(out, indent=1))
