"""Pin the oracle's FDF1.0.1 restatement bit-for-bit against the reference's own sources.

oracle/_ref/libfdf_ref_c{1,3}.so are the reference files FDF1.0.1/{opticalflow_aux.c,solver.c,image.cpp}
compiled where they lie (oracle/Makefile).  Inputs are random; the reference's stride-padding columns are
filled with garbage so the tests also prove that garbage never reaches valid pixels.
"""
import ctypes as C

import numpy as np
import pytest

from oracle import pyoracle as O

pytestmark = pytest.mark.skipif(not O.ref_available() and not __import__("os").path.isdir("/root/reference"),
                                reason="reference FDF1.0.1 build unavailable")

SIZES = [(37, 23), (40, 17), (9, 5), (64, 48), (2, 2), (3, 7)]


def rnd(rng, *shape, scale=1.0):
    return (rng.standard_normal(shape) * scale).astype(np.float32)


def bits_equal(a, b):
    a = np.ascontiguousarray(a, np.float32).view(np.uint32)
    b = np.ascontiguousarray(b, np.float32).view(np.uint32)
    return np.array_equal(a, b)


@pytest.mark.parametrize("w,h", SIZES)
@pytest.mark.parametrize("noc", [1, 3])
def test_image_warp(oracle, w, h, noc):
    rng = np.random.default_rng(w * 100 + h + noc)
    R = O.ref(noc)
    src = rnd(rng, noc, h, w, scale=50)
    wx, wy = rnd(rng, h, w, scale=3), rnd(rng, h, w, scale=3)
    rs, rwx, rwy = O.RefImage(w, h, noc), O.RefImage(w, h), O.RefImage(w, h)
    rs.set(src); rwx.set(wx); rwy.set(wy)
    rd, rm = O.RefImage(w, h, noc), O.RefImage(w, h)
    R.image_warp(rd.ptr, rm.ptr, rs.ptr, rwx.ptr, rwy.ptr)
    dst = np.zeros((noc, h, w), np.float32); mask = np.zeros((h, w), np.float32)
    O.lib().ofo_image_warp(dst, mask, np.ascontiguousarray(src), wx, wy, w, h, noc)
    assert bits_equal(rm.get(), mask)
    assert bits_equal(rd.get().reshape(noc, h, w), dst)


@pytest.mark.parametrize("w,h", SIZES)
@pytest.mark.parametrize("noc", [1, 3])
def test_get_derivatives(oracle, w, h, noc):
    if h < 2:
        pytest.skip("reference vertical 5-tap needs h >= 2")
    rng = np.random.default_rng(7 + w + h)
    R = O.ref(noc)
    im1, im2 = rnd(rng, noc, h, w, scale=40), rnd(rng, noc, h, w, scale=40)
    r1, r2 = O.RefImage(w, h, noc), O.RefImage(w, h, noc)
    r1.set(im1); r2.set(im2)
    outs = [O.RefImage(w, h, noc) for _ in range(8)]
    R.get_derivatives(r1.ptr, r2.ptr, O.ref_conv(R, 2), *[o.ptr for o in outs])
    mine = [np.zeros((noc, h, w), np.float32) for _ in range(8)]
    O.lib().ofo_get_derivatives(np.ascontiguousarray(im1), np.ascontiguousarray(im2), w, h, noc, *mine)
    for k, (o, m) in enumerate(zip(outs, mine)):
        assert bits_equal(o.get().reshape(noc, h, w), m), f"derivative {k}"


@pytest.mark.parametrize("w,h", SIZES)
def test_compute_smoothness(oracle, w, h):
    rng = np.random.default_rng(11 + w * h)
    R = O.ref(1)
    uu, vv = rnd(rng, h, w, scale=2), rnd(rng, h, w, scale=2)
    ru, rv, rh, rvv = O.RefImage(w, h), O.RefImage(w, h), O.RefImage(w, h), O.RefImage(w, h)
    ru.set(uu); rv.set(vv)
    R.compute_smoothness(rh.ptr, rvv.ptr, ru.ptr, rv.ptr, O.ref_conv(R, 1), C.c_float(2.5))
    hh, vvv = np.zeros((h, w), np.float32), np.zeros((h, w), np.float32)
    O.lib().ofo_compute_smoothness(hh, vvv, uu, vv, w, h, 2.5)
    assert bits_equal(rh.get(), hh)
    assert bits_equal(rvv.get(), vvv)


@pytest.mark.parametrize("w,h", SIZES)
def test_sub_laplacian(oracle, w, h):
    rng = np.random.default_rng(5 + w)
    R = O.ref(1)
    dst, src, wh, wv = (rnd(rng, h, w) for _ in range(4))
    rd, rs, rh, rv = (O.RefImage(w, h) for _ in range(4))
    rd.set(dst); rs.set(src); rh.set(wh); rv.set(wv)
    R.sub_laplacian(rd.ptr, rs.ptr, rh.ptr, rv.ptr)
    mine = dst.copy()
    O.lib().ofo_sub_laplacian(mine, src, wh, wv, w, h)
    assert bits_equal(rd.get(), mine)


def _derivs(rng, noc, h, w):
    return [rnd(rng, noc, h, w, scale=s) for s in (3, 3, 5, 1, 1, 1, 2, 2)]


@pytest.mark.parametrize("w,h", SIZES)
@pytest.mark.parametrize("noc", [1, 3])
def test_compute_data(oracle, w, h, noc):
    rng = np.random.default_rng(17 + w + noc)
    R = O.ref(noc)
    I = _derivs(rng, noc, h, w)
    mask = (rng.random((h, w)) > 0.2).astype(np.float32)
    du, dv = rnd(rng, h, w, scale=0.5), rnd(rng, h, w, scale=0.5)
    wx, wy, uu, vv = (rnd(rng, h, w) for _ in range(4))
    refs_in = []
    for arr, c in [(mask, 1), (wx, 1), (wy, 1), (du, 1), (dv, 1), (uu, 1), (vv, 1)] + [(a, noc) for a in I]:
        r = O.RefImage(w, h, c); r.set(arr); refs_in.append(r)
    outs = [O.RefImage(w, h) for _ in range(5)]
    hdo3, hgo3 = np.float32(5.0) * np.float32(0.5) / np.float32(3.0), np.float32(10.0) * np.float32(0.5) / np.float32(3.0)
    R.compute_data(*[o.ptr for o in outs], *[r.ptr for r in refs_in], C.c_float(hdo3), C.c_float(0.0), C.c_float(hgo3))
    mine = [np.zeros((h, w), np.float32) for _ in range(5)]
    O.lib().ofo_compute_data(*mine, mask, du, dv, *[np.ascontiguousarray(a) for a in I], w, h, noc, hdo3, hgo3)
    for k in range(5):
        assert bits_equal(outs[k].get(), mine[k]), f"output {k}"


@pytest.mark.parametrize("w,h", SIZES)
@pytest.mark.parametrize("noc", [1, 3])
def test_compute_data_de(oracle, w, h, noc):
    rng = np.random.default_rng(23 + w + noc)
    R = O.ref(noc)
    I = _derivs(rng, noc, h, w)
    mask = (rng.random((h, w)) > 0.2).astype(np.float32)
    du = rnd(rng, h, w, scale=0.5)
    wx, uu = rnd(rng, h, w), rnd(rng, h, w)
    refs_in = []
    for arr, c in [(mask, 1), (wx, 1), (du, 1), (uu, 1)] + [(a, noc) for a in I]:
        r = O.RefImage(w, h, c); r.set(arr); refs_in.append(r)
    outs = [O.RefImage(w, h) for _ in range(2)]
    hdo3, hgo3 = np.float32(5.0) * np.float32(0.5) / np.float32(3.0), np.float32(10.0) * np.float32(0.5) / np.float32(3.0)
    R.compute_data_DE(*[o.ptr for o in outs], *[r.ptr for r in refs_in], C.c_float(hdo3), C.c_float(0.0), C.c_float(hgo3))
    mine = [np.zeros((h, w), np.float32) for _ in range(2)]
    O.lib().ofo_compute_data_de(*mine, mask, du, *[np.ascontiguousarray(a) for a in I], w, h, noc, hdo3, hgo3)
    for k in range(2):
        assert bits_equal(outs[k].get(), mine[k]), f"output {k}"


def _sor_inputs(rng, h, w):
    a11 = (np.abs(rnd(rng, h, w)) * 5 + 0.5).astype(np.float32)
    a22 = (np.abs(rnd(rng, h, w)) * 5 + 0.5).astype(np.float32)
    a12 = rnd(rng, h, w, scale=0.3)
    b1, b2 = rnd(rng, h, w), rnd(rng, h, w)
    hh = np.abs(rnd(rng, h, w)); hh[:, -1] = 0
    vv = np.abs(rnd(rng, h, w)); vv[-1, :] = 0
    du, dv = rnd(rng, h, w, scale=0.1), rnd(rng, h, w, scale=0.1)
    return du, dv, a11, a12, a22, b1, b2, hh, vv


@pytest.mark.parametrize("w,h", SIZES + [(1, 5), (6, 1)])
@pytest.mark.parametrize("iters", [1, 3, 5])
def test_sor_coupled(oracle, w, h, iters):
    rng = np.random.default_rng(31 + w * 7 + h + iters)
    R = O.ref(1)
    arrs = _sor_inputs(rng, h, w)
    refs = []
    for a in arrs:
        r = O.RefImage(w, h); r.set(a); refs.append(r)
    R.sor_coupled(*[r.ptr for r in refs], iters, C.c_float(1.6))
    mine = [a.copy() for a in arrs]
    O.lib().ofo_sor_coupled(*mine, w, h, iters, 1.6)
    for k in (0, 1, 2, 3, 4):
        assert bits_equal(refs[k].get(), mine[k]), f"array {k}"


@pytest.mark.parametrize("w,h", SIZES + [(1, 5), (6, 1)])
def test_sor_point_of(oracle, w, h):
    """sor_coupled_slow_but_readable (solver.c:34-78): the OpenMP build's OF solver, single-thread order."""
    rng = np.random.default_rng(53 + w * 3 + h)
    R = O.ref(1)
    arrs = _sor_inputs(rng, h, w)
    refs = []
    for a in arrs:
        r = O.RefImage(w, h); r.set(a); refs.append(r)
    R.sor_coupled_slow_but_readable(*[r.ptr for r in refs], 3, C.c_float(1.6))
    mine = [a.copy() for a in arrs]
    O.lib().ofo_sor_point_of(*mine, w, h, 3, 1.6)
    for k in (0, 1):
        assert bits_equal(refs[k].get(), mine[k]), f"array {k}"


@pytest.mark.parametrize("w,h", SIZES)
def test_sor_point_de(oracle, w, h):
    rng = np.random.default_rng(41 + w)
    R = O.ref(1)
    du, _, a11, _, _, b1, _, hh, vv = _sor_inputs(rng, h, w)
    refs = []
    for a in (du, a11, b1, hh, vv):
        r = O.RefImage(w, h); r.set(a); refs.append(r)
    R.sor_coupled_slow_but_readable_DE(*[r.ptr for r in refs], 3, C.c_float(1.6))
    mine = du.copy()
    O.lib().ofo_sor_point_de(mine, a11, b1, hh, vv, w, h, 3, 1.6)
    assert bits_equal(refs[0].get(), mine)


@pytest.mark.parametrize("mode,noc,omp", [(1, 1, 0), (1, 3, 0), (2, 1, 0), (2, 3, 0), (1, 1, 1), (1, 3, 1)])
@pytest.mark.parametrize("w,h,level", [(30, 17, 6), (41, 23, 2), (16, 12, 0)])
def test_refine_level(oracle, mode, noc, omp, w, h, level):
    """One VarRefClass level; omp = 1: the USE_OPENMP build's solver (refine_variational.cpp:202-203)."""
    rng = np.random.default_rng(100 + w + noc + mode)
    pad = 8
    p = O.oppoint(2, 1920, mode, noc)
    p.omp_build = omp
    nop = 2 if mode == 1 else 1
    im1 = (rng.random((noc, h, w)) * 255).astype(np.float32)
    im2 = np.roll(im1, 1, axis=-1) + rnd(rng, noc, h, w, scale=2)
    flow = rnd(rng, h, w, nop, scale=1.5)
    if mode == 2:
        flow = -np.abs(flow)
    ref = O.ref_refine_level(noc, mode, im1, im2, flow, level, p.as_dict())
    # oracle takes padded interleaved level images
    def padded(im):
        inter = np.transpose(im, (1, 2, 0))
        return np.ascontiguousarray(np.pad(inter, ((pad, pad), (pad, pad), (0, 0)), mode="edge"), np.float32)
    mine = np.ascontiguousarray(flow.copy())
    rc = O.lib().ofo_refine_level(padded(im1), padded(im2), w, h, pad, level, C.byref(p), mine)
    assert rc == 0
    assert bits_equal(ref, mine)
