"""Latency mode (option sor_mode = 1): red-black SOR order, levels of up to 8192 pixels run the
whole inner loop in one launch per frame (k_tv_level_rb, of_dis_amd/csrc/ofdis_tvrb.hip), larger ones the system
kernels and global-memory half-sweeps (k_tv_sor_rb).

Two gates:
* bit-exactness against the oracle's red-black restatement (oracle.sor_order(1): ofo_sor_rb_of / ofo_sor_rb_de --
  the same per-pixel updates as solver.c:83-433 / :439-471, red pixels then black ones), stage by stage: every
  system is the reference's bits and the order is the only difference;
* end-point difference against the exact path (the reference's lexicographic order, the CPU oracle), as SURVEY
  §8(c) and BASELINE.md §3 set it: average <= 0.05 px at configs A, B and a config-D shard; max and p99 reported.
(The reference itself measured 0.025 / 0.020 px average for a red-black substitute)"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def od():
    import of_dis_amd
    return of_dis_amd


@pytest.fixture(scope="module")
def rbctx(od):
    c = od.Context(0)
    c.set_option("sor_mode", 1)
    yield c
    c.close()


def _epe(got, ref):
    d = got.astype(np.float64) - ref
    return np.sqrt((d ** 2).sum(-1))


def _bits(x):
    return np.ascontiguousarray(x, np.float32).view(np.uint32)


def _assert_bitexact(got, want, what):
    assert got.shape == want.shape, (what, got.shape, want.shape)
    if not np.array_equal(_bits(got), _bits(want)):
        bad = np.argwhere(_bits(got) != _bits(want))
        d = np.abs(got.astype(np.float64) - want.astype(np.float64))
        raise AssertionError(f"{what}: {len(bad)} / {got.size} differ, max |d| {np.nanmax(d):.3g}, first at "
                             f"{tuple(bad[0])}: got {got[tuple(bad[0])]!r} want {want[tuple(bad[0])]!r}")


def _params(od, O, w, noc, mode, op, over):
    p, q = od.oppoint(op, w, mode, noc), O.oppoint(op, w, mode, noc)
    for k, v in over.items():
        setattr(p, k, v)
        setattr(q, k, v)
    return p, q


# (w, h, noc, mode, op, overrides): the configs' op-points and the level geometries the colour-split layout has to
# get right -- odd widths (colour = p & 1), odd heights, odd pixel counts, tall (h > w) levels, exactly 8192 pixels
# (four entries per colour and thread, the LDS full), one entry per thread, 2 x 2, levels over 8192 pixels
# (global half-sweeps), 2 and 4 sweeps, forward-backward, depth and colour images
RB_CASES = [
    (640, 480, 1, 1, 2, {}),                                  # config A
    (1920, 1080, 1, 1, 2, {}),                                # config B / D (120x68, 60x34, 30x17)
    (640, 480, 3, 1, 3, {}),                                  # RGB op3 (levels up to 160x120: global form)
    (480, 256, 1, 2, 4, {}),                                  # depth op4
    (240, 120, 3, 2, 2, {}),                                  # RGB depth
    (128, 64, 1, 1, 2, {"sc_l": 0, "sc_f": 1}),               # 128x64 = 8192 pixels: CPT 4, LDS 160 KB
    (128, 64, 1, 2, 2, {"sc_l": 0, "sc_f": 1}),               # ... depth
    (130, 63, 1, 1, 2, {"sc_l": 0, "sc_f": 0}),               # 130x63 = 8190: odd height, even width
    (127, 63, 1, 1, 2, {"sc_l": 0, "sc_f": 0}),               # 127x63: odd width and odd pixel count
    (45, 181, 1, 1, 2, {"sc_l": 0, "sc_f": 0}),               # tall, odd x odd
    (33, 21, 1, 2, 2, {"sc_l": 0, "sc_f": 0}),                # depth, odd x odd, one entry per thread
    (100, 90, 3, 1, 2, {"sc_l": 0, "sc_f": 1}),               # RGB: 9000 pixels at scale 0 (global), 50x45 fused
    (90, 90, 3, 1, 2, {"sc_l": 0, "sc_f": 1}),                # RGB, 8100 pixels (CPT 4)
    (160, 120, 1, 1, 2, {"tv_solverit": 2, "tv_innerit": 2}),  # 2 sweeps, more inner iterations
    (160, 120, 1, 1, 2, {"tv_solverit": 4, "tv_sor": 1.3}),   # 4 sweeps
    (160, 120, 1, 1, 2, {"usefbcon": 1}),                     # forward-backward: the backward refinement too
    (160, 120, 1, 1, 2, {"sc_l": 0, "sc_f": 2}),              # 160x120 = 19200 pixels at scale 0: global form
    (8, 8, 1, 1, 2, {"sc_l": 2, "sc_f": 2, "p_samp_s": 2}),   # 2 x 2 level
]


@pytest.mark.parametrize("w,h,noc,mode,op,over", RB_CASES)
def test_redblack_bitexact_vs_oracle_rb(oracle, od, rbctx, w, h, noc, mode, op, over):
    a, b = od.synth_pair(w, h, noc, 1, mode)
    p, q = _params(od, oracle, w, noc, mode, op, over)
    with oracle.sor_order(1):
        ref, cap_d, cap_t = oracle.run_u8(a, b, q, capture=True)
    dis = {s: np.zeros_like(v) for s, v in cap_d.items()}
    tv = {s: np.zeros_like(v) for s, v in cap_t.items()}
    rbctx.set_capture(dis, tv)
    try:
        got = rbctx.run_host(a, b, p)
    finally:
        rbctx.set_capture(None, None)
    for s in sorted(cap_d, reverse=True):
        _assert_bitexact(dis[s], cap_d[s], f"scale {s} after aggregation")
        _assert_bitexact(tv[s], cap_t[s], f"scale {s} after TV refinement")
    _assert_bitexact(got, ref, "full-resolution flow")


@pytest.mark.parametrize("w,h,noc,mode,op,over", RB_CASES)
def test_redblack_uncaptured_bitexact(oracle, od, rbctx, w, h, noc, mode, op, over):
    """The same geometries without a stage capture (the path the CLI and batches take): the full-resolution flow is
    the oracle's red-black bits for another synthetic scene."""
    a, b = od.synth_pair(w, h, noc, 2, mode)
    p, q = _params(od, oracle, w, noc, mode, op, over)
    with oracle.sor_order(1):
        ref = oracle.run_u8(a, b, q)
    _assert_bitexact(rbctx.run_host(a, b, p), ref, "full-resolution flow (no capture)")


# (W, H, noc, mode, op, frame, gate): the 0.05 px gate of SURVEY §8(c) at the op-point-2 configs (A, B / D);
# the finer op-points 3 / 4 (more levels, finest scale 1 or 2) are reported against a looser 0.1 px ceiling
# (measured round 2: 640x480 RGB op3 0.054 px average).
@pytest.mark.parametrize("W,H,noc,mode,op,frame,gate", [(640, 480, 1, 1, 2, 0, 0.05), (1920, 1080, 1, 1, 2, 0, 0.05),
                                                        (1920, 1080, 1, 1, 2, 3, 0.05), (640, 480, 3, 1, 3, 1, 0.1),
                                                        (480, 256, 1, 2, 4, 0, 0.1)])
def test_redblack_epe_gate(oracle, od, rbctx, W, H, noc, mode, op, frame, gate):
    a, b = od.synth_pair(W, H, noc, frame, mode)
    p = od.oppoint(op, W, mode, noc)
    ref = oracle.run_u8(a, b, oracle.oppoint(op, W, mode, noc))
    got = rbctx.run_host(a, b, p)
    e = _epe(got, ref)
    print(f"red-black vs exact {W}x{H} noc {noc} mode {mode} op {op}: avg {e.mean():.4f} p99 "
          f"{np.percentile(e, 99):.4f} max {e.max():.4f} px")
    assert np.isfinite(got).all()
    assert e.mean() <= gate, (e.mean(), np.percentile(e, 99), e.max())


def test_redblack_d_shard_epe(oracle, od, rbctx):
    """A config-D shard (32 pairs of BASELINE's 256, one GPU of eight) in one device call: every frame within the
    0.05 px average gate against the exact path, and bit-exact against the oracle's red-black order."""
    import torch
    W, H, n = 1920, 1080, 32
    pairs = [od.synth_pair(W, H, 1, f, 1) for f in range(n)]
    p = od.oppoint(2, W, 1, 1)
    a = torch.from_numpy(np.stack([x[0] for x in pairs])).cuda()
    b = torch.from_numpy(np.stack([x[1] for x in pairs])).cuda()
    out = rbctx.run(a, b, p)
    torch.cuda.synchronize()
    out = out.cpu().numpy()
    q = oracle.oppoint(2, W, 1, 1)
    avgs, p99s, maxs = [], [], []
    for f in (0, 7, 8, 31):  # the eight synth scenes repeat: frames f and f + 8 share a scene
        exact = oracle.run_u8(pairs[f][0], pairs[f][1], q)
        with oracle.sor_order(1):
            rb = oracle.run_u8(pairs[f][0], pairs[f][1], q)
        _assert_bitexact(out[f], rb, f"frame {f}")
        e = _epe(out[f], exact)
        avgs.append(e.mean()); p99s.append(np.percentile(e, 99)); maxs.append(e.max())
    print(f"D shard red-black vs exact: avg {np.mean(avgs):.4f} (max over frames {max(avgs):.4f}) "
          f"p99 {max(p99s):.4f} max {max(maxs):.4f} px")
    assert max(avgs) <= 0.05, avgs


def test_redblack_batch_equals_singles(od, rbctx):
    """Frames stay independent in red-black mode (fused and global forms), and the mode is deterministic."""
    import torch
    for w, h, sc_l in ((320, 240, 0), (320, 240, 2)):  # 76800 px (global half-sweeps) / 80x60 (fused level launch)
        n = 3
        pairs = [od.synth_pair(w, h, 1, f, 1) for f in range(n)]
        p = od.oppoint(2, w, 1, 1)
        p.sc_l = sc_l
        a = torch.from_numpy(np.stack([x[0] for x in pairs])).cuda()
        b = torch.from_numpy(np.stack([x[1] for x in pairs])).cuda()
        out = rbctx.run(a, b, p)
        torch.cuda.synchronize()
        out = out.cpu().numpy()
        for f in range(n):
            single = rbctx.run_host(pairs[f][0], pairs[f][1], p)
            assert np.array_equal(out[f].view(np.uint32), single.view(np.uint32)), (w, h, sc_l, f)
