"""Per-kernel PMC summary of a rocprofv3 rocpd database: mean counter value per dispatch and mean duration.

Usage: python tools/rocpd_pmc.py <results.db> [name-substring ...]
"""
import json
import sqlite3
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.split("(")[0] if not name.startswith("void at::") else name[:90]
    return name.replace("void ", "")[:90]


def main(path: str, filters) -> None:
    c = sqlite3.connect(path)
    rows = c.execute("select kernel_name, dispatch_id, counter_name, value, duration from counters_collection").fetchall()
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    dur = defaultdict(dict)
    for name, did, cname, val, d in rows:
        k = short(name)
        if filters and not any(f in k for f in filters):
            continue
        agg[k][cname] += val
        disp[k].add(did)
        dur[k][did] = d
    out = {}
    for k, counters in agg.items():
        n = len(disp[k])
        out[k] = {"dispatches": n, "mean_duration_us": round(sum(dur[k].values()) / n / 1e3, 2),
                  **{cn: round(v / n, 1) for cn, v in sorted(counters.items())}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
