#!/usr/bin/env python3
"""CPU-baseline fairness check: the oracle port (oracle/liboracle.so, the CPU baseline
bench.py times on the GPU box) against the reference's own FDF1.0.1 code compiled here (oracle/_ref, the
reference's default-build flags -O3 -msse4.1 with its SSE intrinsics), on identical inputs, single thread.

Container-only (needs /root/reference for oracle/_ref).  Times the two functions that dominate the
refinement -- compute_data (opticalflow_aux.c:408-594) and sor_coupled (solver.c:83-433) -- at the sizes of
config B's finest TV level (120x68) and config E's (960x544), and checks the outputs are bit-identical.
The DIS half (patch.cpp / patchgrid.cpp) needs Eigen, absent from this image: no reference timing exists
for it here.  Writes profiles/cpu_fairness.json (read by bench.py into cpu_baseline).

Usage: python tools/cpu_fairness.py [OUT_JSON]
"""
import ctypes as C
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import pyoracle as O  # noqa: E402


def rnd(rng, *shape, scale=1.0):
    return (rng.standard_normal(shape) * scale).astype(np.float32)


_raw = None


def raw_port():
    """liboracle.so with void-pointer argument types: the port's calls then cost what the reference's (byref image
    structs) cost, not 9-13 ndpointer dtype / flag validations per call (~30 us at 120x68, where one call is 50 us)."""
    global _raw
    if _raw is None:
        _raw = C.CDLL(os.path.join(O.HERE, "liboracle.so"))
        vp = C.c_void_p
        _raw.ofo_sor_coupled.argtypes = [vp] * 9 + [C.c_int, C.c_int, C.c_int, C.c_float]
        _raw.ofo_compute_data.argtypes = [vp] * 16 + [C.c_int, C.c_int, C.c_int, C.c_float, C.c_float]
    return _raw


def best_of(fn, seconds=1.5):
    fn()
    best, t_end = float("inf"), time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        t0 = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t0)
    return best


def sor_case(w, h, iters=3):
    rng = np.random.default_rng(w + h)
    du, dv = rnd(rng, h, w, scale=0.3), rnd(rng, h, w, scale=0.3)
    a11 = np.abs(rnd(rng, h, w)) + 1.0
    a22 = np.abs(rnd(rng, h, w)) + 1.0
    a12 = rnd(rng, h, w, scale=0.2)
    b1, b2 = rnd(rng, h, w), rnd(rng, h, w)
    sh, sv = np.abs(rnd(rng, h, w, scale=0.5)), np.abs(rnd(rng, h, w, scale=0.5))
    arrs = [du, dv, a11, a12, a22, b1, b2, sh, sv]
    R = O.ref(1)
    refs = []
    for a in arrs:
        r = O.RefImage(w, h)
        r.set(a)
        refs.append(r)
    snap = [r.buf.copy() for r in refs]

    def run_ref():
        for r, s in zip(refs, snap):
            r.buf[:] = s
        R.sor_coupled(*[r.ptr for r in refs], iters, C.c_float(1.6))

    mine = [a.copy() for a in arrs]
    mine_p = [m.ctypes.data for m in mine]
    L = raw_port()

    def run_port():
        for m, a in zip(mine, arrs):
            m[:] = a
        L.ofo_sor_coupled(*mine_p, w, h, iters, 1.6)

    t_ref, t_port = best_of(run_ref), best_of(run_port)
    same = all(np.array_equal(refs[k].get().view(np.uint32), mine[k].view(np.uint32)) for k in range(5))
    return t_ref, t_port, same


def data_case(w, h, noc=1):
    rng = np.random.default_rng(3 * w + h)
    I = [rnd(rng, noc, h, w, scale=s) for s in (5, 5, 8, 2, 2, 2, 3, 3)]
    mask = (rng.random((h, w)) > 0.1).astype(np.float32)
    du, dv = rnd(rng, h, w, scale=0.5), rnd(rng, h, w, scale=0.5)
    wx, wy, uu, vv = (rnd(rng, h, w) for _ in range(4))
    R = O.ref(noc)
    refs_in = []
    for arr, c in [(mask, 1), (wx, 1), (wy, 1), (du, 1), (dv, 1), (uu, 1), (vv, 1)] + [(a, noc) for a in I]:
        r = O.RefImage(w, h, c)
        r.set(arr)
        refs_in.append(r)
    outs = [O.RefImage(w, h) for _ in range(5)]
    hdo3 = np.float32(5.0) * np.float32(0.5) / np.float32(3.0)
    hgo3 = np.float32(10.0) * np.float32(0.5) / np.float32(3.0)
    mine = [np.zeros((h, w), np.float32) for _ in range(5)]
    Ic = [np.ascontiguousarray(a) for a in I]
    ptrs = [a.ctypes.data for a in mine + [mask, du, dv] + Ic]
    L = raw_port()

    def run_ref():
        R.compute_data(*[o.ptr for o in outs], *[r.ptr for r in refs_in], C.c_float(hdo3), C.c_float(0.0),
                       C.c_float(hgo3))

    def run_port():
        L.ofo_compute_data(*ptrs, w, h, noc, hdo3, hgo3)

    t_ref, t_port = best_of(run_ref), best_of(run_port)
    same = all(np.array_equal(outs[k].get().view(np.uint32), mine[k].view(np.uint32)) for k in range(5))
    return t_ref, t_port, same


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "cpu_fairness.json")
    O.build()
    rows = {}
    for name, (w, h) in {"B_level4_120x68": (120, 68), "E_level2_960x544": (960, 544)}.items():
        tr, tp, same = sor_case(w, h)
        rows[f"sor_coupled:{name}"] = {"ref_ms": tr * 1e3, "port_ms": tp * 1e3, "port_over_ref": tp / tr,
                                        "bitexact": same}
        tr, tp, same = data_case(w, h)
        rows[f"compute_data:{name}"] = {"ref_ms": tr * 1e3, "port_ms": tp * 1e3, "port_over_ref": tp / tr,
                                         "bitexact": same}
    ratio = float(np.exp(np.mean([np.log(r["port_over_ref"]) for r in rows.values()])))
    res = {"what": "oracle port (liboracle.so) vs the reference's FDF1.0.1 (oracle/_ref, -O3 -msse4.1 SSE), "
                   "1 thread, best-of timings, identical inputs",
           "port_over_ref_geomean": ratio, "cases": rows, "cpu_model": open("/proc/cpuinfo").read().split(
               "model name")[1].split("\n")[0].strip(": \t") if os.path.exists("/proc/cpuinfo") else platform.processor(),
           "dis_part": "not timed: patch.cpp / patchgrid.cpp need Eigen (absent); no reference build exists"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
