"""CPU checks of the oracle's red-black SOR restatement (ofo_sor_rb_of / ofo_sor_rb_de), the checker of the GPU's
latency mode (option sor_mode = 1; tests/test_gpu_redblack.py compares the GPU against it bit for bit).

* against an independent float32 restatement in Python, written from solver.c's per-pixel expressions (:83-433 OF
  block form with the in-place inverse of :122-190, :439-471 DE point form) visited in red-black order;
* as an iteration: red-black and lexicographic SOR converge to the same solution of the same system;
* the order switch (oracle.sor_order) is scoped and the default stays solver.c's order (the golden vectors)."""
import ctypes as C

import numpy as np
import pytest

f32 = np.float32


def _system(rng, w, h):
    a11 = (np.abs(rng.standard_normal((h, w))) + 1.0).astype(f32)
    a22 = (np.abs(rng.standard_normal((h, w))) + 1.0).astype(f32)
    a12 = (0.2 * rng.standard_normal((h, w))).astype(f32)
    b1, b2 = (rng.standard_normal((h, w)).astype(f32) for _ in range(2))
    s = (np.abs(rng.standard_normal((h, w))) * 0.5 + 0.05).astype(f32)
    hh = np.zeros((h, w), f32)
    vv = np.zeros((h, w), f32)
    hh[:, :-1] = s[:, :-1] + s[:, 1:]  # compute_smoothness's horizontal / vertical diffusivities
    vv[:-1, :] = s[:-1, :] + s[1:, :]
    du, dv = (0.3 * rng.standard_normal((h, w))).astype(f32), (0.3 * rng.standard_normal((h, w))).astype(f32)
    return du, dv, a11, a12, a22, b1, b2, hh, vv


def _py_rb_of(du, dv, a11, a12, a22, b1, b2, hh, vv, its, om):
    h, w = du.shape
    du, dv = du.copy(), dv.copy()
    i11, i12, i22 = np.zeros_like(a11), np.zeros_like(a11), np.zeros_like(a11)
    for y in range(h):
        for x in range(w):
            hl = hh[y, x - 1] if x > 0 else f32(0)
            hr = hh[y, x]
            if y == 0:
                dp = hl + (hr + vv[y, x])
            elif y < h - 1:
                dp = (hl + hr) + (vv[y - 1, x] + vv[y, x])
            else:
                dp = hl + (hr + vv[y - 1, x])
            A11, A22, m = a22[y, x] + dp, a11[y, x] + dp, a12[y, x]
            det = A11 * A22 - m * m
            i11[y, x], i22[y, x], i12[y, x] = A11 / det, A22 / det, m / (f32(0) - det)
    for _ in range(its):
        for col in (0, 1):
            for y in range(h):
                for x in range(w):
                    if (x + y) % 2 != col:
                        continue
                    hl = hh[y, x - 1] if x > 0 else f32(0)
                    hr = hh[y, x]
                    ur = du[y, x + 1] if x < w - 1 else f32(0)
                    vr = dv[y, x + 1] if x < w - 1 else f32(0)
                    if y == 0:
                        s1 = (b1[y, x] + hr * ur) + vv[y, x] * du[y + 1, x]
                        s2 = (b2[y, x] + hr * vr) + vv[y, x] * dv[y + 1, x]
                    elif y < h - 1:
                        vt = vv[y - 1, x]
                        s1 = ((hr * ur) + vt * du[y - 1, x]) + (b1[y, x] + vv[y, x] * du[y + 1, x])
                        s2 = ((hr * vr) + vt * dv[y - 1, x]) + (b2[y, x] + vv[y, x] * dv[y + 1, x])
                    else:
                        vt = vv[y - 1, x]
                        s1 = (b1[y, x] + hr * ur) + vt * du[y - 1, x]
                        s2 = (b2[y, x] + hr * vr) + vt * dv[y - 1, x]
                    B1 = s1 if x == 0 else hl * du[y, x - 1] + s1
                    B2 = s2 if x == 0 else hl * dv[y, x - 1] + s2
                    u0, v0 = du[y, x], dv[y, x]
                    du[y, x] = u0 + om * ((i11[y, x] * B1 + i12[y, x] * B2) - u0)
                    dv[y, x] = v0 + om * ((i12[y, x] * B1 + i22[y, x] * B2) - v0)
    return du, dv


def _py_rb_de(du, a11, b1, hh, vv, its, om):
    h, w = du.shape
    du = du.copy()
    for _ in range(its):
        for col in (0, 1):
            for y in range(h):
                for x in range(w):
                    if (x + y) % 2 != col:
                        continue
                    su, sd = f32(0), f32(0)
                    if y > 0:
                        su = su - vv[y - 1, x] * du[y - 1, x]; sd = sd + vv[y - 1, x]
                    if x > 0:
                        su = su - hh[y, x - 1] * du[y, x - 1]; sd = sd + hh[y, x - 1]
                    if y < h - 1:
                        su = su - vv[y, x] * du[y + 1, x]; sd = sd + vv[y, x]
                    if x < w - 1:
                        su = su - hh[y, x] * du[y, x + 1]; sd = sd + hh[y, x]
                    A, B = a11[y, x] + sd, b1[y, x] - su
                    du[y, x] = (f32(1) - om) * du[y, x] + om * (B / A)
    return du


def _bits(x):
    return np.ascontiguousarray(x, f32).view(np.uint32)


@pytest.mark.parametrize("w,h,its", [(9, 7, 3), (8, 6, 2), (13, 2, 4), (2, 9, 1), (11, 11, 3)])
def test_sor_rb_of_matches_python(oracle, w, h, its):
    rng = np.random.default_rng(w * 31 + h)
    du, dv, a11, a12, a22, b1, b2, hh, vv = _system(rng, w, h)
    om = f32(1.6)
    want_u, want_v = _py_rb_of(du, dv, a11, a12, a22, b1, b2, hh, vv, its, om)
    got = [x.copy() for x in (du, dv, a11, a12, a22)]
    oracle.lib().ofo_sor_rb_of(*got, b1, b2, hh, vv, w, h, its, C.c_float(om))
    assert np.array_equal(_bits(got[0]), _bits(want_u)) and np.array_equal(_bits(got[1]), _bits(want_v))


@pytest.mark.parametrize("w,h,its", [(9, 7, 3), (1, 5, 2), (6, 1, 3), (12, 10, 4)])
def test_sor_rb_de_matches_python(oracle, w, h, its):
    rng = np.random.default_rng(w * 7 + h)
    du, _, a11, _, _, b1, _, hh, vv = _system(rng, w, h)
    om = f32(1.3)
    want = _py_rb_de(du, a11, b1, hh, vv, its, om)
    got = du.copy()
    oracle.lib().ofo_sor_rb_de(got, a11, b1, hh, vv, w, h, its, C.c_float(om))
    assert np.array_equal(_bits(got), _bits(want))


def test_rb_and_lexicographic_reach_one_solution(oracle):
    """Both orders are SOR on the same linear system: after many sweeps they agree (and differ after three)."""
    w, h = 24, 17
    rng = np.random.default_rng(5)
    du, dv, a11, a12, a22, b1, b2, hh, vv = _system(rng, w, h)
    du[:], dv[:] = 0, 0
    outs = {}
    for name, fn in (("rb", oracle.lib().ofo_sor_rb_of), ("lex", oracle.lib().ofo_sor_coupled)):
        for its in (3, 400):
            got = [x.copy() for x in (du, dv, a11, a12, a22)]
            fn(*got, b1, b2, hh, vv, w, h, its, C.c_float(1.6))
            outs[(name, its)] = np.stack(got[:2])
    assert not np.array_equal(outs[("rb", 3)], outs[("lex", 3)])
    assert np.abs(outs[("rb", 400)] - outs[("lex", 400)]).max() < 1e-4


def test_sor_order_switch_is_scoped(oracle):
    assert oracle.lib().ofo_get_sor_order() == 0
    with oracle.sor_order(1):
        assert oracle.lib().ofo_get_sor_order() == 1
    assert oracle.lib().ofo_get_sor_order() == 0
