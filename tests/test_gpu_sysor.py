"""GPU parity of the fused system + SOR launch (option "sysor", k_tv_sysor in ofdis_tvsysor.hip).

One launch per TV inner iteration of a level of at most 128 rows: compute_smoothness, compute_data, sub_laplacian
and sor_coupled's inverse (FDF1.0.1/opticalflow_aux.c:138-223,408-594, solver.c:122-128) are produced four
anti-diagonals ahead of the exact-order SOR wavefront (solver.c:83-433) inside the same workgroup.  Same functions,
same order: the bar is the oracle's bits, per scale and at full resolution, at every size class the kernel
distinguishes (one or two row groups, h = 2 .. 128, folded and unfolded skew layouts, 2 and 3 sweeps, the first
inner iteration, the data term's colour half off).
"""
import numpy as np
import pytest

from test_gpu_parity import CASES, _params, assert_bitexact

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def od():
    import of_dis_amd
    return of_dis_amd


@pytest.fixture(scope="module")
def ctx(od):
    c = od.Context(0)
    c.set_option("sysor", 1)
    yield c
    c.close()


def _run_capture(O, ctx, a, b, p, q):
    ref, cap_d, cap_t = O.run_u8(a, b, q, capture=True)
    dis = {s: np.zeros_like(v) for s, v in cap_d.items()}
    tv = {s: np.zeros_like(v) for s, v in cap_t.items()}
    ctx.set_capture(dis, tv)
    try:
        got = ctx.run_host(a, b, p)
    finally:
        ctx.set_capture(None, None)
    for s in sorted(cap_d, reverse=True):
        assert_bitexact(dis[s], cap_d[s], f"scale {s} after aggregation")
        assert_bitexact(tv[s], cap_t[s], f"scale {s} after TV refinement")
    assert_bitexact(got, ref, "full-resolution flow")


SIZES = [
    # (w, h, noc, mode, op, overrides): levels below 128 rows take the fused launch
    (160, 120, 1, 1, 2, {}),                                   # 15 / 30 rows: one row group
    (640, 480, 1, 1, 2, {}),                                   # config A: 15, 30, 60 rows
    (173, 97, 1, 1, 2, {}),                                    # divisibility padding, odd sizes
    (400, 300, 1, 1, 2, {"sc_l": 1, "sc_f": 2}),               # 75 / 150 rows: two row groups, then the two launches
    (256, 256, 1, 1, 2, {"sc_l": 1, "sc_f": 2}),               # 64 rows exactly (one group), then 128 (two full groups)
    (260, 260, 1, 1, 2, {"sc_l": 1, "sc_f": 2}),               # 65 rows: the second group holds one row
    (96, 300, 1, 1, 2, {"sc_l": 1, "sc_f": 2}),                # tall levels (h > w): the unfolded skew layout
    (240, 200, 1, 1, 2, {"sc_l": 1, "sc_f": 2, "tv_solverit": 2}),  # 2 sweeps
    (160, 120, 1, 1, 2, {"tv_delta": 0.0}),                    # colour half of the data term off (hdo3 == 0)
    (160, 120, 1, 1, 2, {"tv_innerit": 1}),                    # the first inner iteration only
    (160, 120, 1, 1, 2, {"patnorm": 0, "tv_innerit": 2, "tv_solverit": 3, "tv_sor": 1.3}),
    (192, 128, 1, 1, 3, {}),                                   # op3 (p = 12), 4 scales
    (64, 16, 1, 1, 2, {"sc_l": 0, "sc_f": 2}),                 # 4 .. 16 rows, 16-column levels
    (40, 8, 1, 1, 2, {"sc_l": 0, "sc_f": 1, "p_samp_s": 4}),   # 4 / 8 rows
]


@pytest.mark.parametrize("w,h,noc,mode,op,over", SIZES)
def test_sysor_pipeline_bitexact(oracle, od, ctx, w, h, noc, mode, op, over):
    a, b = od.synth_pair(w, h, noc, 3, mode)
    p, q = _params(od, oracle, w, noc, mode, op, over)
    _run_capture(oracle, ctx, a, b, p, q)


@pytest.mark.parametrize("w,h,noc,mode,op,over", [c for c in CASES if c[0] <= 256])
def test_sysor_parity_cases(oracle, od, ctx, w, h, noc, mode, op, over):
    """The parity matrix's cases with the option on (those it does not apply to run the two launches)."""
    a, b = od.synth_pair(w, h, noc, 5, mode)
    p, q = _params(od, oracle, w, noc, mode, op, over)
    assert_bitexact(ctx.run_host(a, b, p), oracle.run_u8(a, b, q), "sysor")


def test_sysor_full_1080p(oracle, od, ctx):
    """BASELINE config B (1920 x 1080 op-point 2: 17 / 34 / 68-row levels, all fused), per scale."""
    a, b = od.synth_pair(1920, 1080, 1, 0, 1)
    p, q = _params(od, oracle, 1920, 1, 1, 2, {})
    _run_capture(oracle, ctx, a, b, p, q)


def test_sysor_batch(oracle, od, ctx):
    """A multi-frame launch (several frames per CU resident at once): every frame is the oracle's."""
    import torch
    w, h, n, nd = 640, 480, 600, 3
    pairs = [od.synth_pair(w, h, 1, 21 + f, 1) for f in range(nd)]
    a = torch.from_numpy(np.stack([pairs[i % nd][0] for i in range(n)])).cuda()
    b = torch.from_numpy(np.stack([pairs[i % nd][1] for i in range(n)])).cuda()
    p = od.oppoint(2, w, 1, 1)
    out = ctx.run(a, b, p)
    torch.cuda.synchronize()
    out = out.cpu().numpy()
    for i in range(nd):
        ref = oracle.run_u8(pairs[i][0], pairs[i][1], oracle.oppoint(2, w, 1, 1))
        assert_bitexact(out[i], ref, f"frame {i}")
    for f in range(nd, n):
        assert_bitexact(out[f], out[f % nd], f"frame {f}")
