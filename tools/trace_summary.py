"""Summarise a rocprofv3 kernel trace (…_kernel_trace.csv) per kernel and launch shape: count, average and total
duration.  The shape (grid, workgroup, LDS) tells the levels of one kernel apart.

    python tools/trace_summary.py <kernel_trace.csv> [--skip N]   (skip the first N dispatches: warm-up)"""
import csv
import re
import sys
from collections import OrderedDict


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("ofdis::", "")
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"\(ofdis::TvArgs.*$|\(ofdis::\w+Args.*$|\([A-Za-z]+Args.*$", "", n)
    return n


def main():
    path = sys.argv[1]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 0
    rows = list(csv.DictReader(open(path)))[skip:]
    agg = OrderedDict()
    for r in rows:
        grid = "x".join(g for g in (r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Grid_Size_Y", ""),
                                       r.get("Grid_Size_Z", "")) if g not in ("", "1"))
        key = (short(r["Kernel_Name"]), grid, r.get("Workgroup_Size_X", ""), r.get("LDS_Block_Size", r.get("Lds_Size", "")))
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        a = agg.setdefault(key, [0, 0.0])
        a[0] += 1
        a[1] += d
    tot = sum(v[1] for v in agg.values())
    print(f"{'kernel':60s} {'grid':>16s} {'wg':>5s} {'lds':>7s} {'n':>6s} {'avg us':>9s} {'total us':>10s} {'%':>5s}")
    for (k, g, wg, lds), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k[:60]:60s} {g:>16s} {wg:>5s} {lds:>7s} {n:6d} {t / n:9.2f} {t:10.1f} {100 * t / tot:5.1f}")


if __name__ == "__main__":
    main()
