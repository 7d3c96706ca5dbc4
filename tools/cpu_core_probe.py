#!/usr/bin/env python3
"""The port's OFClass core (oracle/ofdis_oracle.c) against SURVEY's probe of the reference core.

BASELINE.md §2 lists the reference's own `TIME (O.Flow Run-Time)` (oflow.cpp:333-337: OFClass only) per
config, measured single-threaded in the survey container with an Eigen-subset shim (upper bounds).  This
times the port's stages in THIS container, single-threaded, on the same configs -- pad, pyramid, OFClass
and upsample separately (ofo_run_u8_stages) -- and writes the ratio port / probe for the OFClass core
(the "DIS-core ratio"; the FDF half alone is pinned by tools/cpu_fairness.py against the reference's own
compiled FDF code).

    python tools/cpu_core_probe.py [out.json]     (container-only: pins itself to one core)
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (CONFIGS, params_of, oracle_params)
import of_dis_amd as od  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

# BASELINE.md:30-34 (probe of the reference core, ms)
PROBE_MS = {"A": (2.8, 4.0), "B": (5.1, 6.7), "C": (487.0, 487.0), "C2": (645.0, 645.0), "E": (4297.0, 4297.0)}


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r03", "cpu_core_vs_probe.json")
    try:
        os.sched_setaffinity(0, {min(os.sched_getaffinity(0))})
    except (AttributeError, OSError):
        pass
    res = {"what": "port stages, 1 thread, min / median over reps (ms); ratio = port OFClass / reference probe",
           "cpu_model": bench.cpu_model(), "configs": {}}
    for name in ("A", "B", "C", "C2", "E"):
        cfg = bench.CONFIGS[name]
        _, W, H, noc, mode, *_ = cfg
        q = bench.oracle_params(O, bench.params_of(od, cfg))
        a, b = od.synth_pair(W, H, noc, 0, mode)
        reps = 15 if W * H * noc <= 2_100_000 and name in ("A", "B") else 3
        st = [O.run_u8_stages(a, b, q)[1] for _ in range(reps)]
        mins = {k: round(min(s[k] for s in st) * 1e3, 3) for k in st[0]}
        meds = {k: round(statistics.median(s[k] for s in st) * 1e3, 3) for k in st[0]}
        lo, hi = PROBE_MS[name]
        total = sum(mins.values())
        res["configs"][name] = {
            "stages_min_ms": mins, "stages_median_ms": meds, "reps": reps,
            "probe_ofclass_ms": [lo, hi],
            "ofclass_ratio_vs_probe": [round(mins["ofclass"] / hi, 3), round(mins["ofclass"] / lo, 3)],
            "pyramid_upsample_share": round((mins["pyramid"] + mins["upsample"]) / total, 3),
        }
        print(name, res["configs"][name], flush=True)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
