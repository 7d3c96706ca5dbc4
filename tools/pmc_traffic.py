#!/usr/bin/env python3
"""Per-launch HBM traffic of each kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Usage:  python tools/pmc_traffic.py FETCH_DIR WRITE_DIR KEY_SUFFIX [OUT_JSON [SOURCE]]
  FETCH_DIR / WRITE_DIR: the -d directories of the two passes (each holds *counter_collection.csv)
  KEY_SUFFIX: workload tag, e.g. "1920x1080:op2:b256" (bench.py looks up "<kernel>:<suffix>")
  SOURCE: where the passes are kept (recorded in every entry this run writes)

Per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of wide coalesced reads, so it is doubled; WRITE_SIZE is taken as is.
Kernels are grouped under the logical names bench.py / the C-ABI timer use.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

LOGICAL = [
    (r"k_pyr_base", "pyr_base"), (r"k_pyr_down", "pyr_down"), (r"k_pyr_pad_grad", "pyr_pad_grad"),
    (r"k_patch", "patch"), (r"k_aggregate", "aggregate"), (r"k_tv_prep", "tv_prep"),
    (r"k_tv_deriv", "tv_deriv"), (r"k_tv_smooth|k_tv_system|k_tv_smsys", "tv_system"), (r"k_tv_level", "tv_level"),
    (r"k_tv_sor", "tv_sor"),
    (r"k_tv_final", "tv_final"), (r"k_upsample", "upsample"),
]


def logical(name):
    for pat, lg in LOGICAL:
        if re.search(pat, name):
            return lg
    return None


def per_dispatch(d, counter):
    """{dispatch_id: (kernel_name, value)} summed over the counter's instances."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    out = {}
    for fn in files:
        with open(fn) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                key = (fn, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                name, v = out.get(key, (row["Kernel_Name"], 0.0))
                out[key] = (name, v + float(row["Counter_Value"]))
    return out


def main():
    fdir, wdir, suffix = sys.argv[1:4]
    out_json = sys.argv[4] if len(sys.argv) > 4 else os.path.join("profiles", "traffic.json")
    source = sys.argv[5] if len(sys.argv) > 5 else f"{fdir} + {wdir}"
    res = {}
    for d, counter, scale in ((fdir, "FETCH_SIZE", 2.0), (wdir, "WRITE_SIZE", 1.0)):
        acc = defaultdict(lambda: [0.0, 0])
        for name, v in per_dispatch(d, counter).values():
            lg = logical(name)
            if lg:
                acc[lg][0] += v * 1024.0 * scale
                acc[lg][1] += 1
        for lg, (tot, n) in acc.items():
            res.setdefault(lg, {})[counter] = tot / n
            res[lg]["launches_" + counter] = n
    table = json.load(open(out_json)) if os.path.exists(out_json) else {}
    for lg, r in sorted(res.items()):
        b = r.get("FETCH_SIZE", 0.0) + r.get("WRITE_SIZE", 0.0)
        table[f"{lg}:{suffix}"] = {"bytes_per_launch": b, "fetch_bytes_x2": r.get("FETCH_SIZE"),
                                   "write_bytes": r.get("WRITE_SIZE"), "launches": r.get("launches_FETCH_SIZE"),
                                   "source": source}
        print(f"{lg:14s} {b / 1e6:12.3f} MB/launch  (fetch x2 {r.get('FETCH_SIZE', 0) / 1e6:.3f}, "
              f"write {r.get('WRITE_SIZE', 0) / 1e6:.3f})")
    os.makedirs(os.path.dirname(out_json) or ".", exist_ok=True)
    json.dump(table, open(out_json, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
