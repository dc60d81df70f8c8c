"""Per-kernel summary (calls, mean/total us, grid, VGPRs, LDS) from a rocprofv3 rocpd SQLite database."""
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    return name[-110:]


def main(path: str, top: int = 40) -> None:
    c = sqlite3.connect(path)
    rows = c.execute(
        "select name, count(*), avg(duration), sum(duration), max(grid_x), max(workgroup_x), max(vgpr_count), max(lds_size)"
        " from kernels group by name order by sum(duration) desc"
    ).fetchall()
    print(f"{'kernel':110s} {'calls':>6s} {'mean_us':>9s} {'total_us':>10s} {'grid':>9s} {'wg':>5s} {'vgpr':>5s} {'lds':>7s}")
    for name, n, avg, tot, gx, wx, vg, lds in rows[:top]:
        print(f"{short(name):110s} {n:6d} {avg / 1e3:9.1f} {tot / 1e3:10.1f} {gx:9d} {wx:5d} {vg:5d} {lds:7d}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
