#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc passes: SQ ratios (per SQ_WAVE_CYCLES), instruction counts per wave,
and FETCH_SIZE / WRITE_SIZE bytes per launch (FETCH x 2 for gfx950, MI355X_MICROARCH.md HBM section).
Usage: python tools/pmc_summary.py DIR [kernel-regex]   (DIR holds one sub-directory per pass)"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    m = re.search(r"(k_\w+(<[^>]*>)?)", name)
    return m.group(1) if m else name[:40]


def main():
    d = sys.argv[1]
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
    out = {}
    for k, v in sorted(agg.items()):
        if pat and not pat.search(k):
            continue
        n = max((len(disp[(k, c)]) for c in v), default=1)
        row = {"launches": n}
        wc = v.get("SQ_WAVE_CYCLES")
        waves = v.get("SQ_WAVES")
        for c, x in v.items():
            nl = len(disp[(k, c)]) or 1
            if wc and (c.startswith("SQ_WAIT") or c.startswith("SQ_ACTIVE")):
                row[c + "/wave_cycles"] = round(x / wc, 3)
            elif c.startswith("SQ_INSTS") and waves:
                row[c + "/wave"] = round(x / waves, 1)
            elif c == "FETCH_SIZE":
                row["fetch_bytes_per_launch"] = round(x * 1024 * 2 / nl)
            elif c == "WRITE_SIZE":
                row["write_bytes_per_launch"] = round(x * 1024 / nl)
            else:
                row[c] = round(x / nl, 1)
        out[k] = row
        print(k, row)
    return out


if __name__ == "__main__":
    main()
