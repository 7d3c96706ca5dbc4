"""Golden vectors (tests/golden/, made by tests/golden/make_golden.py).

CPU: the oracle reproduces the REFERENCE FDF1.0.1 outputs (fdf_*.npz) bit-for-bit -- this pins the
restatement without needing /root/reference -- and its whole-pipeline outputs still match the committed
regression vectors (pipe_*.npz).  GPU: the HIP path through the C-ABI matches the same pipeline vectors.
"""
import ctypes as C
import glob
import json
import os

import numpy as np
import pytest

from oracle import pyoracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _bits(x):
    return np.ascontiguousarray(x, np.float32).view(np.uint32)


def _load(path):
    return dict(np.load(path, allow_pickle=False))


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "fdf_refine_*.npz"))), ids=os.path.basename)
def test_refine_level_matches_reference_vectors(oracle, path):
    g = _load(path)
    mode, noc, level, op = int(g["mode"]), int(g["noc"]), int(g["level"]), int(g["oppoint"])
    im1, im2, flow = g["im1"], g["im2"], g["flow"]
    h, w = im1.shape[-2:]
    p = O.oppoint(op, 1920, mode, noc)
    tv = g["tv"]
    assert np.allclose([p.tv_alpha, p.tv_gamma, p.tv_delta, p.tv_innerit, p.tv_solverit, p.tv_sor], tv)
    pad = 8

    def padded(im):
        inter = np.transpose(im, (1, 2, 0))
        return np.ascontiguousarray(np.pad(inter, ((pad, pad), (pad, pad), (0, 0)), mode="edge"), np.float32)

    mine = np.ascontiguousarray(flow.copy())
    assert O.lib().ofo_refine_level(padded(im1), padded(im2), w, h, pad, level, C.byref(p), mine) == 0
    assert np.array_equal(_bits(mine), _bits(g["out"]))


def test_sor_coupled_matches_reference_vectors(oracle):
    g = _load(os.path.join(GOLD, "fdf_sor_coupled.npz"))
    h, w = g["du"].shape
    arrs = [g[k].copy() for k in ("du", "dv", "a11", "a12", "a22", "b1", "b2", "h", "v")]
    O.lib().ofo_sor_coupled(*arrs, w, h, int(g["iters"]), float(g["omega"]))
    for k, name in enumerate(("du", "dv", "a11", "a12", "a22")):
        assert np.array_equal(_bits(arrs[k]), _bits(g["out_" + name])), name


def test_sor_point_of_matches_reference_vectors(oracle):
    """The USE_OPENMP build's solver, sor_coupled_slow_but_readable (solver.c:34-78)."""
    g = _load(os.path.join(GOLD, "fdf_sor_point_of.npz"))
    h, w = g["du"].shape
    arrs = [g[k].copy() for k in ("du", "dv", "a11", "a12", "a22", "b1", "b2", "h", "v")]
    O.lib().ofo_sor_point_of(*arrs, w, h, int(g["iters"]), float(g["omega"]))
    assert np.array_equal(_bits(arrs[0]), _bits(g["out_du"])) and np.array_equal(_bits(arrs[1]), _bits(g["out_dv"]))


def test_sor_de_matches_reference_vectors(oracle):
    g = _load(os.path.join(GOLD, "fdf_sor_de.npz"))
    h, w = g["du"].shape
    du = g["du"].copy()
    O.lib().ofo_sor_point_de(du, g["a11"], g["b1"], g["h"], g["v"], w, h, int(g["iters"]), float(g["omega"]))
    assert np.array_equal(_bits(du), _bits(g["out_du"]))


PIPES = sorted(glob.glob(os.path.join(GOLD, "pipe_*.npz")))


def _pipe_params(mod, g):
    w = g["a"].shape[1]
    p = mod.oppoint(int(g["oppoint"]), w, int(g["mode"]), int(g["noc"]))
    for k, v in json.loads(str(g["overrides"])).items():
        setattr(p, k, v)
    return p


@pytest.mark.parametrize("path", PIPES, ids=os.path.basename)
def test_oracle_pipeline_regression(oracle, path):
    g = _load(path)
    out = O.run_u8(g["a"], g["b"], _pipe_params(O, g))
    assert np.array_equal(_bits(out), _bits(g["out"]))


@pytest.mark.gpu
@pytest.mark.parametrize("path", PIPES, ids=os.path.basename)
def test_hip_pipeline_matches_golden(path):
    import of_dis_amd as od
    g = _load(path)
    ctx = od.Context(0)
    try:
        out = ctx.run_host(g["a"], g["b"], _pipe_params(od, g))
    finally:
        ctx.close()
    assert np.array_equal(_bits(out), _bits(g["out"]))


@pytest.mark.parametrize("mode,op,noc", [(1, 2, 1), (1, 1, 1), (1, 3, 3), (2, 4, 1)])
def test_oracle_known_answer(oracle, mode, op, noc):
    """Known-answer check of the restated DIS+TV path (the part without a buildable reference): the
    synthetic pair moves by (6.5, 2.25) (+ <=0.5 deg rotation, <=1 % zoom) for flow and by a pure
    horizontal 6.5 px for depth; the median recovered motion must be within 0.25 px of it."""
    import of_dis_amd as od
    a, b = od.synth_pair(320, 240, noc, 0, mode)
    out = O.run_u8(a, b, O.oppoint(op, 320, mode, noc))
    med = np.median(out[40:-40, 40:-40].reshape(-1, out.shape[-1]), 0)
    want = [6.5, 2.25] if mode == 1 else [-6.5]
    assert np.all(np.abs(med - want) < 0.25), med


def test_oracle_gradmag_base_level(oracle):
    """SELECTCHANNEL 2 (run_dense.cpp:139-148): the finest pyramid level is sqrt(dx^2 + dy^2) of the Sobel
    (ksize 3, x 1/8, reflect-101) derivatives -- exact in fp32 up to the rounded sqrt, so an independent
    numpy computation must agree bit for bit."""
    import of_dis_amd as od
    a, _ = od.synth_pair(64, 48, 1, 2, 1)
    p = O.oppoint(2, 64, 1, 1)
    p.sc_f, p.sc_l, p.gradmag = 1, 0, 1
    lev = O.build_pyramid(a, p, 8)
    f = a[..., 0].astype(np.float64)
    fp = np.pad(f, 1, mode="reflect")  # numpy "reflect" == OpenCV BORDER_REFLECT_101
    dx = (fp[:-2, 2:] - fp[:-2, :-2] + fp[2:, 2:] - fp[2:, :-2]) / 8 + (fp[1:-1, 2:] - fp[1:-1, :-2]) / 4
    dy = (fp[2:, :-2] + fp[2:, 2:] - fp[:-2, :-2] - fp[:-2, 2:]) / 8 + (fp[2:, 1:-1] - fp[:-2, 1:-1]) / 4
    want = np.sqrt((dx * dx + dy * dy).astype(np.float32))  # squares exact; fp32 sqrt correctly rounded
    got = lev[0][0][8:-8, 8:-8, 0]
    assert np.array_equal(_bits(got), _bits(want))
