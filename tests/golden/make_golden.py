#!/usr/bin/env python3
"""Generate the committed golden vectors under tests/golden/ (container-only; needs /root/reference).

Two kinds of fixture, each an .npz of inputs + expected outputs (data only, no reference source):

* ``fdf_*.npz`` -- REFERENCE outputs.  Produced by the reference's own FDF1.0.1 sources
  (opticalflow_aux.c, solver.c, image.cpp) compiled where they lie by ``oracle/Makefile`` into
  ``oracle/_ref/`` and driven exactly like refine_variational.cpp:152-342 does
  (``oracle.pyoracle.ref_refine_level``), or by calling one reference function directly.
  These pin the oracle's FDF restatement (tests/test_golden.py) on machines without the reference.

* ``pipe_*.npz`` -- ORACLE regression vectors for the whole run_dense pipeline (pyramid -> OFClass ->
  upsample).  The DIS half of the reference (patch.cpp / patchgrid.cpp / oflow.cpp) needs Eigen and the
  pyramid/upsample need OpenCV, neither present in this image, so these outputs come from the oracle's
  restatement (DESIGN.md §5 "parity pinning"); the GPU tests compare the HIP path against them too.

Run:  python tests/golden/make_golden.py
"""
import ctypes as C
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import pyoracle as O  # noqa: E402


def rnd(rng, *shape, scale=1.0):
    return (rng.standard_normal(shape) * scale).astype(np.float32)


def refine_cases():
    """(mode, noc, w, h, level, oppoint) -- odd sizes exercise the FDF stride padding."""
    return [(1, 1, 30, 17, 6, 2), (1, 3, 41, 23, 2, 3), (2, 1, 37, 19, 3, 4), (2, 3, 24, 16, 1, 2)]


def make_refine(mode, noc, w, h, level, op):
    rng = np.random.default_rng(1000 * mode + 100 * noc + w)
    p = O.oppoint(op, 1920, mode, noc)
    nop = 2 if mode == 1 else 1
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    base = 128 + 60 * np.sin(0.31 * xx + 0.7 * np.sin(0.2 * yy)) * np.cos(0.27 * yy)
    im1 = np.stack([base + 10 * c for c in range(noc)]).astype(np.float32) + rnd(rng, noc, h, w, scale=3)
    im2 = np.roll(im1, 1, axis=-1) + rnd(rng, noc, h, w, scale=2)
    flow = rnd(rng, h, w, nop, scale=1.2)
    if mode == 2:
        flow = -np.abs(flow)
    out = O.ref_refine_level(noc, mode, im1, im2, flow, level, p.as_dict())
    np.savez_compressed(os.path.join(HERE, f"fdf_refine_m{mode}_c{noc}_{w}x{h}.npz"),
                        im1=im1, im2=im2, flow=flow, level=level, oppoint=op, mode=mode, noc=noc, out=out,
                        tv=np.array([p.tv_alpha, p.tv_gamma, p.tv_delta, p.tv_innerit, p.tv_solverit, p.tv_sor],
                                    np.float32))


def make_sor():
    """sor_coupled (solver.c:83-433) and sor_coupled_slow_but_readable_DE (solver.c:439-471)."""
    w, h, iters, omega = 37, 23, 3, 1.6
    rng = np.random.default_rng(77)
    a11 = np.abs(rnd(rng, h, w)) * 5 + 0.5
    a22 = np.abs(rnd(rng, h, w)) * 5 + 0.5
    a12 = rnd(rng, h, w, scale=0.3)
    b1, b2 = rnd(rng, h, w), rnd(rng, h, w)
    hh = np.abs(rnd(rng, h, w)); hh[:, -1] = 0
    vv = np.abs(rnd(rng, h, w)); vv[-1, :] = 0
    du, dv = rnd(rng, h, w, scale=0.1), rnd(rng, h, w, scale=0.1)
    ins = [du, dv, a11.astype(np.float32), a12, a22.astype(np.float32), b1, b2, hh, vv]
    R = O.ref(1)
    refs = []
    for a in ins:
        r = O.RefImage(w, h); r.set(a); refs.append(r)
    R.sor_coupled(*[r.ptr for r in refs], iters, C.c_float(omega))
    np.savez_compressed(os.path.join(HERE, "fdf_sor_coupled.npz"), du=ins[0], dv=ins[1], a11=ins[2], a12=ins[3],
                        a22=ins[4], b1=ins[5], b2=ins[6], h=ins[7], v=ins[8], iters=iters, omega=np.float32(omega),
                        out_du=refs[0].get(), out_dv=refs[1].get(), out_a11=refs[2].get(), out_a12=refs[3].get(),
                        out_a22=refs[4].get())
    refs = []
    for a in (ins[0], ins[2], ins[5], ins[7], ins[8]):
        r = O.RefImage(w, h); r.set(a); refs.append(r)
    R.sor_coupled_slow_but_readable_DE(*[r.ptr for r in refs], iters, C.c_float(omega))
    np.savez_compressed(os.path.join(HERE, "fdf_sor_de.npz"), du=ins[0], a11=ins[2], b1=ins[5], h=ins[7], v=ins[8],
                        iters=iters, omega=np.float32(omega), out_du=refs[0].get())


def make_sor_point_of():
    """sor_coupled_slow_but_readable (solver.c:34-78): the USE_OPENMP build's OF solver."""
    w, h, iters, omega = 29, 21, 3, 1.6
    rng = np.random.default_rng(78)
    a11 = (np.abs(rnd(rng, h, w)) * 5 + 0.5).astype(np.float32)
    a22 = (np.abs(rnd(rng, h, w)) * 5 + 0.5).astype(np.float32)
    a12 = rnd(rng, h, w, scale=0.3)
    b1, b2 = rnd(rng, h, w), rnd(rng, h, w)
    hh = np.abs(rnd(rng, h, w)); hh[:, -1] = 0
    vv = np.abs(rnd(rng, h, w)); vv[-1, :] = 0
    du, dv = rnd(rng, h, w, scale=0.1), rnd(rng, h, w, scale=0.1)
    ins = [du, dv, a11, a12, a22, b1, b2, hh, vv]
    R = O.ref(1)
    refs = []
    for a in ins:
        r = O.RefImage(w, h); r.set(a); refs.append(r)
    R.sor_coupled_slow_but_readable(*[r.ptr for r in refs], iters, C.c_float(omega))
    np.savez_compressed(os.path.join(HERE, "fdf_sor_point_of.npz"), du=du, dv=dv, a11=a11, a12=a12, a22=a22,
                        b1=b1, b2=b2, h=hh, v=vv, iters=iters, omega=np.float32(omega), out_du=refs[0].get(),
                        out_dv=refs[1].get())


def pipe_cases():
    """(w, h, noc, mode, oppoint, overrides) -- small whole-pipeline regression vectors."""
    return [(160, 120, 1, 1, 2, {}), (173, 97, 1, 1, 2, {}), (96, 64, 3, 1, 3, {"costfct": 1}),
            (120, 64, 1, 2, 4, {}), (128, 96, 1, 1, 2, {"usefbcon": 1})] + variant_pipe_cases()


def variant_pipe_cases():
    """Build variants: USE_OPENMP semantics (point SOR) and SELECTCHANNEL 2 (gradient-magnitude input)."""
    return [(128, 96, 1, 1, 2, {"omp_build": 1}), (136, 88, 1, 1, 2, {"gradmag": 1})]


def pipe_name(w, h, noc, mode, op, over=None):
    over = over or {}
    tag = "".join(t for k, t in (("usefbcon", "_fb"), ("omp_build", "_omp"), ("gradmag", "_grad")) if over.get(k))
    return os.path.join(HERE, f"pipe_m{mode}_c{noc}_op{op}_{w}x{h}{tag}.npz")


def make_pipe(w, h, noc, mode, op, over):
    import of_dis_amd as od  # host-only entry points (synthetic generator), no GPU needed
    a, b = od.synth_pair(w, h, noc, 11, mode)
    q = O.oppoint(op, w, mode, noc)
    for k, v in over.items():
        setattr(q, k, v)
    out = O.run_u8(a, b, q)
    np.savez_compressed(pipe_name(w, h, noc, mode, op, over), a=a, b=b, out=out, mode=mode, noc=noc, oppoint=op,
                        overrides=json.dumps(over))


def main():
    O.build()
    if not O.ref_available():
        sys.exit("oracle/_ref is not built (needs /root/reference): cannot make reference vectors")
    for c in refine_cases():
        make_refine(*c)
    make_sor()
    make_sor_point_of()
    for c in pipe_cases():
        make_pipe(*c)
    print("golden vectors written to", HERE)


if __name__ == "__main__":
    main()
