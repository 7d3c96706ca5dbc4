"""Opt-in red-black SOR (option sor_mode = 1): a different iteration from sor_coupled's
lexicographic order, so it is gated by end-point difference against the exact path (the CPU oracle), as
SURVEY §8(c) and BASELINE.md §3 set it: average <= 0.05 px at configs A and B; max and p99 are reported.
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


# (W, H, noc, mode, op, frame, gate): the 0.05 px gate of SURVEY §8(c) at the op-point-2 configs (A, B / D);
# the finer op-points 3 / 4 (more levels, finest scale 1 or 2) are reported against a looser 0.1 px ceiling
# (measured: 640x480 RGB op3 0.054 px average).
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


def test_redblack_batch_equals_singles(od, rbctx):
    """Frames stay independent in red-black mode (LDS and global forms), and the mode is deterministic."""
    import torch
    w, h, n = 320, 240, 3
    pairs = [od.synth_pair(w, h, 1, f, 1) for f in range(n)]
    p = od.oppoint(2, w, 1, 1)
    p.sc_l = 0  # 320x240 at scale 0: 76800 px, the global-memory half-sweep form
    a = torch.from_numpy(np.stack([x[0] for x in pairs])).cuda()
    b = torch.from_numpy(np.stack([x[1] for x in pairs])).cuda()
    out = rbctx.run(a, b, p)
    torch.cuda.synchronize()
    out = out.cpu().numpy()
    for f in range(n):
        single = rbctx.run_host(pairs[f][0], pairs[f][1], p)
        assert np.array_equal(out[f].view(np.uint32), single.view(np.uint32)), f
