"""GPU parity for every patch shape the reference accepts, not only the op-points' p = 8 / 12.

The reference takes any even patch size whose p*p*noc is a multiple of 4 (`run_dense.cpp:280`,
`oflow.cpp:80-91`, `patch.cpp:221-273`: LossComputeErrorImage walks novals/4 packets).  The library runs
them on four kernel families, chosen by shape (`launch_patch`, ofdis_kernels.hip):

* `k_patchq`  -- LDS-windowed four-lane form, gray p = 8 / 12 (round 3; `patch_quad=0` for the next one);
* `k_patchw`  -- LDS-windowed eight-lane form, RGB p = 8 / 12 (and gray with `patch_quad=0`);
* `k_patch8`  -- eight lanes per patch, values in registers: gray p = 2 / 4 / 6 / 10, p = 8 / 12 with
  `patch_window=0`;
* `k_patch`   -- one wave per patch (p*p*noc <= 448): gray p = 14..20, RGB p = 4 / 6 / 10, and every
  shape <= 448 with `wave_per_patch=1`;
* `k_patchg`  -- any shape, runtime value loops: p*p*noc > 448 (gray p >= 22, RGB p >= 14), and every
  shape with `patch_generic=1`.

Each case is compared bit for bit with the oracle per scale (after aggregation, after refinement) and at
full resolution.  The scales follow the CLI's op-point rule for the chosen patch size (sc_f from
`run_dense.cpp:181-184`, two or more finer scales kept) so that every level carries a real patch grid.
"""
import numpy as np
import pytest

from test_gpu_parity import _bits, assert_bitexact

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def od():
    import of_dis_amd
    return of_dis_amd


@pytest.fixture(scope="module")
def ctx(od):
    c = od.Context(0)
    yield c
    c.close()


def shape_params(od, O, w, noc, mode, op, p, over=None):
    """op-point `op` with patch size p, the coarsest scale recomputed for p like the CLI (fratio 5)."""
    a = od.oppoint(op, w, mode, noc)
    b = O.oppoint(op, w, mode, noc)
    keep = a.sc_f - a.sc_l
    sc_f = od.auto_first_scale(w, 5, p)
    for q in (a, b):
        q.p_samp_s = p
        q.sc_f = sc_f
        q.sc_l = max(0, sc_f - keep)
        for k, v in (over or {}).items():
            setattr(q, k, v)
    return a, b


def run_and_check(od, O, ctx, w, h, noc, mode, op, p, over=None, option=None, frame=3):
    a, b = od.synth_pair(w, h, noc, frame, mode)
    pg, pq = shape_params(od, O, w, noc, mode, op, p, over)
    assert od.validate(pg) == 0
    ref, cap_d, cap_t = O.run_u8(a, b, pq, capture=True)
    dis = {s: np.zeros_like(v) for s, v in cap_d.items()}
    tv = {s: np.zeros_like(v) for s, v in cap_t.items()}
    if option:
        ctx.set_option(*option)
    ctx.set_capture(dis, tv)
    try:
        got = ctx.run_host(a, b, pg)
    finally:
        ctx.set_capture(None, None)
        if option:
            ctx.set_option(option[0], 1 - option[1])
    tag = f"p={p} noc={noc} mode={mode}" + (f" {option[0]}={option[1]}" if option else "")
    for s in sorted(cap_d, reverse=True):
        assert_bitexact(dis[s], cap_d[s], f"{tag}: scale {s} after aggregation")
        assert_bitexact(tv[s], cap_t[s], f"{tag}: scale {s} after TV refinement")
    assert_bitexact(got, ref, f"{tag}: full-resolution flow")


GRAY = [2, 4, 6, 10, 14, 16, 20, 22, 24, 32]
RGB = [4, 6, 10, 14, 16, 20, 32]


@pytest.mark.parametrize("p", GRAY)
def test_gray_flow_patch_sizes(oracle, od, ctx, p):
    run_and_check(od, oracle, ctx, 320, 240, 1, 1, 2, p)


@pytest.mark.parametrize("p", RGB)
def test_rgb_flow_patch_sizes(oracle, od, ctx, p):
    # the L1 cost (config C's) on the RGB shapes, L2 for the largest (both cost paths on k_patchg)
    run_and_check(od, oracle, ctx, 288, 224, 3, 1, 3, p, {"costfct": 1 if p < 32 else 0})


@pytest.mark.parametrize("p,noc", [(10, 1), (14, 1), (24, 1), (6, 3), (14, 3)])
def test_depth_patch_sizes(oracle, od, ctx, p, noc):
    run_and_check(od, oracle, ctx, 320, 160, noc, 2, 4, p, {"max_iter": 16, "min_iter": 16})


@pytest.mark.parametrize("p,noc,over", [(24, 1, {"costfct": 2}), (16, 3, {"costfct": 2}),
                                        (22, 1, {"patnorm": 0}),
                                        (26, 1, {"min_iter": 2, "dp_thresh": 0.3, "dr_thresh": 0.9}),
                                        (22, 1, {"usefbcon": 1}), (14, 3, {"usefbcon": 1, "costfct": 1})])
def test_large_patch_options(oracle, od, ctx, p, noc, over):
    """k_patchg with the pseudo-Huber cost, without normalisation, with early stopping and with
    forward-backward merging (its weights feed the backward splat)."""
    run_and_check(od, oracle, ctx, 320, 240, noc, 1, 2, p, over)


@pytest.mark.parametrize("p,noc,mode,op", [(8, 1, 1, 2), (12, 1, 1, 3), (8, 3, 1, 2), (12, 3, 1, 3),
                                           (12, 1, 2, 4), (4, 3, 1, 2)])
def test_generic_kernel_on_small_shapes(oracle, od, ctx, p, noc, mode, op):
    """The any-shape kernel forced on the op-point shapes (option patch_generic): the same bits."""
    over = {"max_iter": 16, "min_iter": 16} if op == 4 else None
    run_and_check(od, oracle, ctx, 256, 192, noc, mode, op, p, over, option=("patch_generic", 1))


@pytest.mark.parametrize("p,noc,mode,op", [(8, 1, 1, 2), (12, 1, 1, 3), (12, 1, 2, 4)])
def test_unwindowed_eight_lane_kernel(oracle, od, ctx, p, noc, mode, op):
    """patch_window=0: p = 8 / 12 gray on k_patch8 (L1 gathers) instead of the LDS-windowed k_patchw."""
    over = {"max_iter": 16, "min_iter": 16} if op == 4 else None
    run_and_check(od, oracle, ctx, 256, 192, noc, mode, op, p, over, option=("patch_window", 0))


def test_oflow_imgpadding_larger_than_patch(oracle, od):
    """OFC::OFClass with imgpadding > p_samp_s (oflow.h:99-106 allows any padding >= p): caller pyramids
    padded by 14 for 8-pixel patches, and by 20 for 12-pixel RGB patches."""
    O = oracle
    for (w, h, noc, op, pad, costfct) in ((320, 240, 1, 2, 14, 0), (256, 192, 3, 3, 20, 1)):
        a, b = od.synth_pair(w, h, noc, 6, 1)
        q = O.oppoint(op, w, 1, noc)
        q.costfct = costfct
        pa, pb = O.build_pyramid(a, q, pad), O.build_pyramid(b, q, pad)
        lists = []
        for pyr in (pa, pb):
            for k in range(3):
                lst = [None] * 32
                for s, v in pyr.items():
                    lst[s] = v[k]
                lists.append(lst)
        out = np.zeros((h >> q.sc_l) * (w >> q.sc_l) * 2, np.float32)
        od.OFClass(*lists, pad, out, None, w, h, q.sc_f, q.sc_l, q.max_iter, q.min_iter, q.dp_thresh,
                   q.dr_thresh, q.res_thresh, q.p_samp_s, q.patove, False, q.costfct, noc, q.patnorm, True,
                   q.tv_alpha, q.tv_gamma, q.tv_delta, q.tv_innerit, q.tv_solverit, q.tv_sor, 0)
        want = O.oflow(pa, pb, w, h, q, pad)
        assert_bitexact(out.reshape(want.shape), want, f"OFClass imgpadding {pad} > p {q.p_samp_s} (noc {noc})")
        assert np.isfinite(_bits(out).view(np.float32)).all()
