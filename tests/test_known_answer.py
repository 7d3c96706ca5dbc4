"""Known-answer anchor for the DIS half (patch.cpp / patchgrid.cpp / oflow.cpp), whose reference code cannot
be built here (no Eigen): pure translations of the synthetic texture, the setups SURVEY §4 probed the
reference on -- 640x480 shifted by (3.3, -1.7), 1080p shifted by (6.5, 2.25) -- where the reference's
average end-point error against the true shift measured 0.10 px and 0.15 px (SURVEY.md:214-216).

Gates: average EPE <= 0.12 px at 640x480 and <= 0.18 px at 1080p over the image with a
16-pixel border excluded (the probe's border handling is not recorded; the whole-image means are reported
beside it and gated at 0.15 / 0.18).  The CPU test pins the oracle; the GPU test shows the HIP path gives
the oracle's bits, hence the same EPE, and prints both.
"""
import numpy as np
import pytest

SETUPS = [  # (W, H, shift, gate with a 16 px border excluded, whole-image gate, probe EPE of the reference)
    (640, 480, (3.3, -1.7), 0.12, 0.15, 0.10),
    (1920, 1080, (6.5, 2.25), 0.18, 0.18, 0.15),
]


def epe_stats(flow, shift):
    e = np.sqrt(((flow.astype(np.float64) - np.array(shift, np.float64)) ** 2).sum(-1))
    return {"whole": float(e.mean()), "b16": float(e[16:-16, 16:-16].mean()),
            "b40": float(e[40:-40, 40:-40].mean()), "p99": float(np.percentile(e, 99))}


@pytest.fixture(scope="module")
def od():
    import of_dis_amd
    return of_dis_amd


@pytest.mark.parametrize("W,H,shift,gate,gate_whole,probe", SETUPS)
@pytest.mark.parametrize("frame", [0, 1])
def test_oracle_pure_shift_epe(oracle, od, W, H, shift, gate, gate_whole, probe, frame):
    a, b = od.synth_shift_pair(W, H, shift, 1, frame)
    flow = oracle.run_u8(a, b, oracle.oppoint(2, W, 1, 1))
    st = epe_stats(flow, shift)
    print(f"oracle {W}x{H} shift {shift} frame {frame}: {st} (reference probe {probe})")
    assert st["b16"] <= gate and st["whole"] <= gate_whole, st


def test_shift_pair_is_a_translation(od):
    """Frame b is frame a moved by the shift: an integer shift makes b an exact copy of a's texture
    (the noise is independent per frame, sigma 2)."""
    a, b = od.synth_shift_pair(200, 100, (3.0, -2.0), 1, 0)
    d = b[10:-10, 10:-10].astype(np.float64) - a[12:-8, 7:-13].astype(np.float64)  # b(x, y) = a(x - 3, y + 2)
    assert abs(d.mean()) < 0.2 and 2.0 < d.std() < 3.5


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,shift,gate,gate_whole,probe", SETUPS)
def test_gpu_pure_shift_epe(oracle, od, W, H, shift, gate, gate_whole, probe):
    ctx = od.Context(0)
    try:
        for frame in (0, 1):
            a, b = od.synth_shift_pair(W, H, shift, 1, frame)
            got = ctx.run_host(a, b, od.oppoint(2, W, od.MODE_OF, 1))
            ref = oracle.run_u8(a, b, oracle.oppoint(2, W, 1, 1))
            g, r = epe_stats(got, shift), epe_stats(ref, shift)
            print(f"{W}x{H} shift {shift} frame {frame}: GPU {g}  oracle {r}  reference probe {probe}")
            assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
            assert g["b16"] <= gate and g["whole"] <= gate_whole, g
    finally:
        ctx.close()
