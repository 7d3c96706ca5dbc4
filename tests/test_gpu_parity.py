"""GPU parity: the HIP path (libofdis.so through its C-ABI) against the CPU oracle on identical inputs.

The kernels keep the reference evaluation order, so the bar is bit-exactness (compared as uint32 bit
patterns), stage by stage: pyramid, flow after patch aggregation per scale, flow after TV refinement per
scale, and the full-resolution output.  At BASELINE's full 1080p size the check is the same (the oracle
finishes in well under a second per pair).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(x):
    return np.ascontiguousarray(x, np.float32).view(np.uint32)


def assert_bitexact(got, want, what):
    got, want = np.asarray(got, np.float32), np.asarray(want, np.float32)
    assert got.shape == want.shape, (what, got.shape, want.shape)
    if not np.array_equal(_bits(got), _bits(want)):
        d = np.abs(got.astype(np.float64) - want.astype(np.float64))
        bad = np.argwhere(_bits(got) != _bits(want))
        raise AssertionError(f"{what}: {len(bad)} / {got.size} values differ; max |d| = {np.nanmax(d):.3g}; "
                             f"first at {tuple(bad[0])}: got {got[tuple(bad[0])]!r} want {want[tuple(bad[0])]!r}")


@pytest.fixture(scope="module")
def od():
    import of_dis_amd
    return of_dis_amd


@pytest.fixture(scope="module")
def ctx(od):
    c = od.Context(0)
    yield c
    c.close()


CASES = [
    # (w, h, noc, mode, oppoint, overrides)
    (160, 120, 1, 1, 2, {}),
    (640, 480, 1, 1, 2, {}),
    (200, 150, 1, 1, 1, {}),                                  # op1: no TV refinement, overlap .3
    (173, 97, 1, 1, 2, {}),                                   # divisibility padding on both axes
    (192, 128, 3, 1, 3, {}),                                  # RGB op3 (p = 12, L2 as defined)
    (192, 128, 3, 1, 3, {"costfct": 1}),                      # RGB op3 with the L1 cost of BASELINE config C
    (192, 128, 1, 1, 3, {}),                                  # gray op3: p = 12 flow on four lanes per patch
    (192, 128, 1, 1, 4, {"costfct": 1, "max_iter": 16, "min_iter": 16}),  # ... L1 cost
    (240, 120, 1, 2, 4, {"costfct": 2, "max_iter": 16, "min_iter": 16}),  # depth p = 12, pseudo-Huber
    (192, 128, 1, 1, 3, {"usefbcon": 1, "costfct": 1}),       # four-lane p = 12 flow with forward-backward
    (176, 140, 1, 1, 3, {"patnorm": 0, "min_iter": 4, "dp_thresh": 0.3, "dr_thresh": 0.9}),  # ... no norm., stops
    (160, 120, 1, 1, 2, {"costfct": 2}),                      # pseudo-Huber
    (160, 120, 1, 1, 2, {"min_iter": 2, "dp_thresh": 0.3, "dr_thresh": 0.9}),  # early stopping active
    (160, 120, 1, 1, 2, {"patnorm": 0, "tv_innerit": 2, "tv_solverit": 4, "tv_sor": 1.3}),
    (240, 120, 1, 2, 4, {"max_iter": 16, "min_iter": 16}),    # depth from stereo, op4
    (240, 120, 3, 2, 2, {}),                                  # RGB depth
    (240, 120, 3, 2, 4, {"max_iter": 16, "min_iter": 16}),    # RGB depth, p = 12 (samples kept, L2 cost)
    (160, 120, 1, 1, 2, {"usefbcon": 1}),                     # forward-backward merging (patchgrid.cpp:277-375)
    (200, 150, 1, 1, 1, {"usefbcon": 1}),                     # ... without TV refinement
    (192, 128, 3, 1, 3, {"usefbcon": 1, "costfct": 1}),       # ... RGB (weight-pointer quirk, bounds [1, w-1))
    (240, 120, 1, 2, 4, {"usefbcon": 1, "max_iter": 16, "min_iter": 16}),  # ... depth (right camera clamp)
    (400, 300, 1, 1, 2, {"sc_l": 0, "sc_f": 2}),              # 300 rows: 5 row groups x 3 sweep waves
    (320, 600, 1, 2, 2, {"sc_l": 0, "sc_f": 1}),              # 600 rows, 3 sweeps: two rows per lane (R = 2)
    (320, 600, 1, 1, 2, {"sc_l": 0, "sc_f": 1, "tv_solverit": 2}),  # 2 sweeps, 513..1024 rows: R = 2, 1024 threads
    (256, 1000, 1, 2, 2, {"sc_l": 0, "sc_f": 1, "tv_solverit": 2}),  # ... depth, 1000 rows (8 row-pair groups)
    (256, 704, 1, 1, 2, {"sc_l": 0, "sc_f": 1}),              # 3 sweeps, 641..1024 rows: register pipeline
    (300, 280, 3, 1, 2, {"sc_l": 0, "sc_f": 1}),              # RGB, 280 rows: streaming smoothness + system
    (200, 300, 3, 2, 2, {"sc_l": 0, "sc_f": 1}),              # ... RGB depth, tall (unfolded) layout
    (160, 120, 1, 1, 2, {"omp_build": 1}),                    # USE_OPENMP build: point SOR (solver.c:34-78)
    (240, 200, 1, 1, 2, {"sc_l": 1, "sc_f": 2, "tv_solverit": 2}),  # fused system + SOR: 2 sweeps, 2 row groups
    (248, 232, 1, 2, 2, {"sc_l": 1, "sc_f": 2}),              # ... depth, 116 rows (2 row groups)
    (192, 128, 3, 1, 3, {"omp_build": 1, "usefbcon": 1}),     # ... RGB, forward-backward
    (173, 97, 1, 1, 2, {"gradmag": 1}),                       # SELECTCHANNEL 2: gradient-magnitude pyramid
    (240, 120, 1, 2, 4, {"gradmag": 1, "max_iter": 16, "min_iter": 16}),  # ... depth
    (160, 120, 1, 1, 2, {"gradmag": 1, "sc_l": 0, "sc_f": 2}),             # ... finest scale 0
]


def _params(od, O, w, noc, mode, op, over):
    p = od.oppoint(op, w, mode, noc)
    q = O.oppoint(op, w, mode, noc)
    for k, v in over.items():
        setattr(p, k, v)
        setattr(q, k, v)
    return p, q


@pytest.mark.parametrize("w,h,noc,mode,op,over", CASES)
def test_pipeline_bitexact(oracle, od, ctx, w, h, noc, mode, op, over):
    O = oracle
    a, b = od.synth_pair(w, h, noc, 3, mode)
    p, q = _params(od, O, w, noc, mode, op, over)
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


VARIANTS = [  # (option, value, default): non-default kernels
    ("sor_pipe", 1, 0),        # one-wave register-pipeline SOR (the default only for tall levels)
    ("sor_generic", 1, 0),     # generic global-memory SOR
    ("wave_per_patch", 1, 0),  # one wave per DIS patch instead of eight lanes
    ("sor_cring", 0, 2),       # sweep-per-wave SOR without the LDS coefficient ring
    ("sor_cring", 1, 2),       # the coefficient ring sized to the workgroup limit instead of the level
    ("sor_cring", 3, 2),       # the clamped in-frame load form (the oversubscribed launches' loads) on every launch
    ("smsys", 0, 1),           # smoothness and system as two launches (s through memory)
    ("sor_rows2", 0, 1),       # 321..640-row levels on the register pipeline instead of two rows per lane
    ("smsys_prefetch", 0, 1),  # fused smoothness + system: derivative images loaded in phase 2
    ("smsys_small", 0, 1),     # latency regime: the throughput row blocks (4 pixels per thread)
    ("pyr_rgb", 0, 1),         # colour pyramid base by the byte loop (k_pyr_base) instead of dword loads + SAD
    ("pad_grad_v", 0, 1),      # colour pyramid pad + gradients one thread per pixel (the channels in the thread)
    ("agg_stage", 0, 1),       # aggregation gathering every patch displacement from p_iter (no LDS staging)
    ("smsys_deriv", 0, 1),     # fused launch reads all eight derivative planes (prepd writes them)
    ("prepd_df", 0, 1),        # smsys_deriv levels: k_tv_prepd (4-pixel halo, per channel) writes Ix, Iy, Iz
    ("smsys_march", 0, 1),     # tall levels: the 2-D tiled fused launch (smsys2d auto: on below 512 pairs)
    (("smsys_march", "smsys2d"), (0, 0), (1, 2)),  # tall levels: two launches (smoothness, then system)
    ("prepd", 0, 2),           # prep and the derivative filters as three launches (t, It, Ix, Iy through memory)
    ("prepd", 1, 2),           # ... three launches for colour images only
    ("patch_generic", 1, 0),   # every patch shape on the any-shape kernel k_patchg
    ("patch_quad", 0, 1),      # gray p = 8 / 12 on eight lanes per patch (k_patchw) instead of four (k_patchq)
    ("patch_x16", 0, 1),       # RGB p = 12 on eight lanes per patch (k_patchw) instead of sixteen (k_patchx)
    ("patch_x16", 2, 1),       # k_patchx on its exact square-root evaluation (the fallback of the scaled fast one)
    ("patch_absw", 0, 1),      # loss weights to the aggregation instead of the aggregation-weight slot planes
    ("patch_buf", 0, 1),       # gray p = 12 windows by global loads instead of buffer loads
    ("patch_fdiv", 0, 1),      # LLT solves by IEEE divisions instead of the FMA-corrected pivot reciprocals
    ("patch_maxres", 0, 1),    # op-point stopping test on the mean |w| instead of the largest |w|
    ("up_form", 0, 3),         # flow upsample with the horizontal taps once per output row (round 4's kernel)
    ("up_form", 1, 3),         # ... once per source row, 4-row blocks
    ("up_form", 2, 3),         # ... once per source row, 8-row blocks
]


@pytest.mark.parametrize("variant", VARIANTS, ids=lambda v: f"{v[0]}={v[1]}" if isinstance(v[0], str)
                         else "+".join(f"{k}={x}" for k, x in zip(v[0], v[1])))
@pytest.mark.parametrize("w,h,noc,mode,op,over", [c for c in CASES if c[0] <= 200 or c[1] > 256])
def test_kernel_variants_bitexact(oracle, od, ctx, variant, w, h, noc, mode, op, over):
    """Every kernel variant (TV / SOR / DIS patch) gives the same bits as the default path and the oracle."""
    key, val, default = variant
    keys, vals, defaults = ((key,), (val,), (default,)) if isinstance(key, str) else (key, val, default)
    a, b = od.synth_pair(w, h, noc, 4, mode)
    p, q = _params(od, oracle, w, noc, mode, op, over)
    ref = oracle.run_u8(a, b, q)
    for k, v in zip(keys, vals):
        ctx.set_option(k, v)
    try:
        got = ctx.run_host(a, b, p)
    finally:
        for k, d in zip(keys, defaults):
            ctx.set_option(k, d)
    assert_bitexact(got, ref, f"{keys}={vals}")


def _flat_pair(od, w, h, noc, mode):
    """The synthetic pair with constant blocks (zero gradients: regularised Hessians, zero residuals and
    right-hand sides) and a saturated stripe: the patch solves' fallback divisions run beside the fast ones."""
    a, b = od.synth_pair(w, h, noc, 6, mode)
    a, b = a.copy(), b.copy()
    for img in (a, b):
        img[: h // 3, : w // 3] = 0
        img[h // 2:, w // 2: w // 2 + w // 5] = 128
        img[h // 4: h // 4 + 6, :] = 255
    b[: h // 3 + 4, : w // 3 + 4] = 0
    return a, b


@pytest.mark.parametrize("fdiv", [1, 0])
@pytest.mark.parametrize("w,h,noc,mode,op,over", [(160, 120, 1, 1, 2, {}), (192, 128, 1, 1, 3, {}),
                                                  (192, 128, 3, 1, 3, {"costfct": 1}), (240, 120, 1, 2, 4, {}),
                                                  (176, 140, 1, 1, 3, {"patnorm": 0})])
def test_flat_regions_bitexact(oracle, od, ctx, fdiv, w, h, noc, mode, op, over):
    """Constant image blocks: the LLT solves' reciprocal-and-FMA divisions hand zero / out-of-range numerators
    to the IEEE division (patch_fdiv), and every flow value is still the oracle's."""
    a, b = _flat_pair(od, w, h, noc, mode)
    p, q = _params(od, oracle, w, noc, mode, op, over)
    ctx.set_option("patch_fdiv", fdiv)
    try:
        got = ctx.run_host(a, b, p)
    finally:
        ctx.set_option("patch_fdiv", 1)
    assert_bitexact(got, oracle.run_u8(a, b, q), f"flat blocks, patch_fdiv={fdiv}")


@pytest.mark.parametrize("w,h,noc,op,over", [(160, 120, 1, 2, {}), (173, 97, 1, 2, {}), (192, 128, 3, 3, {}),
                                              (1920, 1080, 1, 2, {}), (640, 480, 1, 2, {}), (330, 250, 1, 2, {}),
                                              (2000, 1000, 1, 2, {}), (173, 97, 1, 2, {"gradmag": 1}),
                                              (640, 480, 1, 2, {"gradmag": 1}),
                                              (96, 64, 1, 2, {"gradmag": 1, "sc_l": 0, "sc_f": 1})])
def test_pyramid_bitexact(oracle, od, ctx, w, h, noc, op, over):
    O = oracle
    a, _ = od.synth_pair(w, h, noc, 1, 1)
    p, q = _params(od, O, w, noc, 1, op, over)
    pw, ph = O.divisibility_pad(w, h, q.sc_f)
    padded = np.pad(a, ((ph // 2, ph - ph // 2), (pw // 2, pw - pw // 2), (0, 0)), mode="edge")
    want = O.build_pyramid(padded, q, q.p_samp_s)
    got = ctx.pyramid_host(a, p)
    for s in want:
        for k, name in enumerate(("img", "dx", "dy")):
            assert_bitexact(got[s][k], want[s][k], f"level {s} {name}")


def test_ofclass_host_api_bitexact(oracle, od):
    """OFC::OFClass mirror (oflow.h:99-126) with caller-built pyramids, incl. an initflow."""
    O = oracle
    w, h = 320, 240
    a, b = od.synth_pair(w, h, 1, 5, 1)
    q = O.oppoint(2, w, 1, 1)
    pa, pb = O.build_pyramid(a, q, 8), O.build_pyramid(b, q, 8)
    L = [None] * 32
    lists = []
    for pyr in (pa, pb):
        for k in range(3):
            lst = list(L)
            for s, v in pyr.items():
                lst[s] = v[k]
            lists.append(lst)
    rng = np.random.default_rng(0)
    init = (rng.standard_normal(((h >> (q.sc_f + 1)), (w >> (q.sc_f + 1)), 2)) * 0.5).astype(np.float32)
    for initflow, fb in ((None, 0), (init, 0), (init, 1)):
        out = np.zeros((h >> q.sc_l) * (w >> q.sc_l) * 2, np.float32)
        od.OFClass(*lists, 8, out, initflow, w, h, q.sc_f, q.sc_l, q.max_iter, q.min_iter, q.dp_thresh,
                   q.dr_thresh, q.res_thresh, q.p_samp_s, q.patove, bool(fb), q.costfct, 1, q.patnorm, True,
                   q.tv_alpha, q.tv_gamma, q.tv_delta, q.tv_innerit, q.tv_solverit, q.tv_sor, 0)
        q.usefbcon = fb
        want = O.oflow(pa, pb, w, h, q, 8, initflow=initflow)
        q.usefbcon = 0
        assert_bitexact(out.reshape(want.shape), want, f"OFClass initflow={initflow is not None} usefbcon={fb}")


def test_batch_equals_singles(od, ctx):
    """Frame i of a batch equals the same pair run alone (no cross-frame leakage)."""
    import torch
    w, h, n = 320, 240, 5
    pairs = [od.synth_pair(w, h, 1, f, 1) for f in range(n)]
    a = torch.from_numpy(np.stack([x[0] for x in pairs])).cuda()
    b = torch.from_numpy(np.stack([x[1] for x in pairs])).cuda()
    p = od.oppoint(2, w, 1, 1)
    outs = []
    configs = ((1, 0, 1), (1, 0, 1), (1, 0, 0), (3, 2, 1), (4, 1, 1), (3, 2, 2), (3, 2, 2), (2, 1, 0), (2, 3, 2),
               (1, 2, 1), (1, 2, 0))
    for streams, chunk, graph in configs:
        # whole batch on one stream (graph captured, then replayed; eager launches); chunks round-robin over
        # streams (also captured with their fork / join: graph 2); chunks one after another on one stream
        ctx.set_option("streams", streams)
        ctx.set_option("chunk", chunk)
        ctx.set_option("graph", graph)
        o = ctx.run(a, b, p)
        torch.cuda.synchronize()
        outs.append(o.cpu().numpy())
    ctx.set_option("graph", 1)
    ctx.set_option("streams", 0)
    ctx.set_option("chunk", 0)
    for f in range(n):
        single = ctx.run_host(pairs[f][0], pairs[f][1], p)
        for k, out in enumerate(outs):
            assert_bitexact(out[f], single, f"batch frame {f} (config {k})")


def test_bad_batch_arguments_enqueue_nothing(od, ctx):
    """An empty or malformed batch is refused with OFDIS_ERR_INVALID_ARGUMENT (ofdis.h, ofdis_run_batch_u8)
    before anything is enqueued: the output buffer is untouched and the context runs the next batch bit-exact."""
    import torch
    from of_dis_amd import _lib
    w, h = 160, 120
    pa, pb = od.synth_pair(w, h, 1, 0, 1)
    p = od.oppoint(2, w, 1, 1)
    want = ctx.run_host(pa, pb, p)
    a = torch.from_numpy(pa[None]).cuda().unsqueeze(-1)
    b = torch.from_numpy(pb[None]).cuda().unsqueeze(-1)
    out = torch.full((1, h, w, 2), 7.0, device="cuda")
    torch.cuda.synchronize()
    ap, bp, op = a.data_ptr(), b.data_ptr(), out.data_ptr()
    for n, ww, hh, x, y, z in ((0, w, h, ap, bp, op), (-1, w, h, ap, bp, op), (1, 0, h, ap, bp, op),
                               (1, w, -h, ap, bp, op), (1, w, h, 0, bp, op), (1, w, h, ap, 0, op), (1, w, h, ap, bp, 0)):
        with pytest.raises(_lib.OfdisError) as e:
            ctx.run_ptr(x, y, n, ww, hh, p, z)
        assert e.value.code == _lib.ERR_INVALID_ARGUMENT, (n, ww, hh)
    torch.cuda.synchronize()
    assert bool((out == 7.0).all()), "a refused call wrote the output"
    ctx.run_ptr(ap, bp, 1, w, h, p, op)
    torch.cuda.synchronize()
    assert_bitexact(out[0].cpu().numpy(), want, "batch after refused calls")


def test_default_stream_inputs_are_ordered(od, ctx):
    """Inputs produced by kernels on torch's default (legacy NULL) stream right before the call -- here the
    copy kernel of .contiguous() on permuted views -- are complete when the flow kernels read them, and the
    flow is complete for the next kernel on that stream, with no host synchronisation in between."""
    import torch
    w, h, n = 320, 240, 4
    pairs = [od.synth_pair(w, h, 1, f, 1) for f in range(n)]
    p = od.oppoint(2, w, 1, 1)
    want = np.stack([ctx.run_host(x[0], x[1], p) for x in pairs])
    at = torch.from_numpy(np.stack([x[0] for x in pairs])).cuda()
    bt = torch.from_numpy(np.stack([x[1] for x in pairs])).cuda()
    torch.cuda.synchronize()
    assert torch.cuda.current_stream().cuda_stream == 0
    for rep in range(3):
        # a permuted view: .contiguous() inside Context.run launches a copy kernel on the default stream
        a = (at.permute(0, 2, 1, 3).contiguous() + 0).permute(0, 2, 1, 3)
        b = (bt.permute(0, 2, 1, 3).contiguous() + 0).permute(0, 2, 1, 3)
        assert not a.is_contiguous()
        out = ctx.run(a, b, p)
        got = (out * 1.0).cpu().numpy()  # a default-stream kernel consumes the flow
        assert_bitexact(got, want, f"default-stream round {rep}")


def test_full_1080p_bitexact(oracle, od, ctx):
    """BASELINE config B size (1920x1080, op-point 2): GPU == oracle bit-for-bit."""
    a, b = od.synth_pair(1920, 1080, 1, 0, 1)
    p = od.oppoint(2, 1920, 1, 1)
    got = ctx.run_host(a, b, p)
    ref = oracle.run_u8(a, b, oracle.oppoint(2, 1920, 1, 1))
    assert_bitexact(got, ref, "1080p op2")


@pytest.mark.parametrize("form", [0, 1, 2])
@pytest.mark.parametrize("w,h,op,over", [(1920, 1080, 2, {}), (1000, 562, 2, {}), (330, 250, 1, {}),
                                         (640, 480, 2, {"sc_l": 2}), (2100, 70, 2, {"sc_l": 1, "sc_f": 2})])
def test_upsample_forms_bitexact(oracle, od, ctx, form, w, h, op, over):
    """Every optical-flow upsample kernel (up_form) at 2^l = 2 / 4 / 8, cropped divisibility padding, several
    1024-column blocks and a partial last one: the full-resolution flow is the oracle's."""
    a, b = od.synth_pair(w, h, 1, 9, 1)
    p, q = _params(od, oracle, w, 1, 1, op, over)
    ctx.set_option("up_form", form)
    try:
        got = ctx.run_host(a, b, p)
    finally:
        ctx.set_option("up_form", 3)
    assert_bitexact(got, oracle.run_u8(a, b, q), f"up_form={form}")


def test_lanes_capture_native(od, tmp_path):
    """The multi-lane round robin captured as a HIP graph (option graph=2) in a process of its own, i.e. under the
    ROCm runtime libofdis.so links: captured, replayed, bit-identical to its eager issue."""
    import subprocess
    from test_host_abi import ROOT
    libdir = os.path.dirname(od._lib.LIB_PATH)
    exe = str(tmp_path / "lanes_capture")
    subprocess.run(["g++", "-std=c++14", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "lanes_capture.cpp"), "-L", libdir, "-lofdis",
                    f"-Wl,-rpath,{libdir}", "-o", exe], check=True, capture_output=True, timeout=300)
    r = subprocess.run([exe, "2"], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, OFDIS_TRACE="1"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("same 1") == 2, r.stdout
    assert "graph: capture (kind 1" in r.stderr and "graph: captured rc 0 end 0" in r.stderr, r.stderr[-2000:]


def test_oflow_hpp_dropin_program(oracle, od, tmp_path):
    """A C++ program written against include/ofdis_oflow.hpp (reference signature of OFC::OFClass) gives
    the oracle's flow bit-for-bit."""
    import subprocess
    from test_host_abi import build_dropin
    w, h = 256, 128
    a, b = od.synth_pair(w, h, 1, 9, 1)
    for name, im in (("a.pgm", a), ("b.pgm", b)):
        (tmp_path / name).write_bytes(f"P5\n{w} {h}\n255\n".encode() + im.tobytes())
    exe = build_dropin(tmp_path)
    out = tmp_path / "o.flo"
    r = subprocess.run([exe, str(tmp_path / "a.pgm"), str(tmp_path / "b.pgm"), str(out)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    q = oracle.oppoint(2, w, 1, 1)
    want = oracle.oflow(oracle.build_pyramid(a, q, 8), oracle.build_pyramid(b, q, 8), w, h, q, 8)
    assert_bitexact(od.read_flo(str(out)), want, "OFC::OFClass drop-in program")


@pytest.mark.parametrize("exe_name,noc,mode,over", [("run_OF_INT", 1, 1, {}), ("run_OF_RGB", 3, 1, {}),
                                                     ("run_DE_INT", 1, 2, {}), ("run_DE_RGB", 3, 2, {}),
                                                     ("run_OF_GRAD", 1, 1, {"gradmag": 1}),
                                                     ("run_DE_GRAD", 1, 2, {"gradmag": 1}),
                                                     ("run_OF_INT_OMP", 1, 1, {"omp_build": 1})])
def test_cli_png_inputs(oracle, od, tmp_path, exe_name, noc, mode, over):
    """The CLI reads colour PNGs with cv::imread's semantics (GRAYSCALE conversion for *_INT) and writes
    the oracle's flow (.flo) / depth (.pfm) for the decoded pixels, bit for bit."""
    import os
    import subprocess
    from test_image_io import encode_png
    w, h = 176, 112
    a3, b3 = od.synth_pair(w, h, 3, 4, mode)  # BGR
    for name, im in (("a.png", a3), ("b.png", b3)):
        (tmp_path / name).write_bytes(encode_png(im[..., ::-1].astype(np.int64), 2, 8, interlace=name == "b.png"))
    a = od.read_image(str(tmp_path / "a.png"), noc)
    b = od.read_image(str(tmp_path / "b.png"), noc)
    if noc == 3:
        assert np.array_equal(a, a3) and np.array_equal(b, b3)
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "of_dis_amd", "bin", exe_name)
    out = tmp_path / ("o.flo" if mode == 1 else "o.pfm")
    r = subprocess.run([exe, str(tmp_path / "a.png"), str(tmp_path / "b.png"), str(out), "2"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    q = oracle.oppoint(2, w, mode, noc)
    for k, v in over.items():
        setattr(q, k, v)
    want = oracle.run_u8(a, b, q)
    if mode == 1:
        got = od.read_flo(str(out))
    else:
        raw = out.read_bytes()
        head = f"Pf\n{w} {h}\n-1.000000\n".encode()
        assert raw.startswith(head)
        got = -np.frombuffer(raw[len(head):], np.float32).reshape(h, w)[::-1][..., None]
    assert_bitexact(got, want, f"{exe_name} on PNG inputs")


@pytest.mark.parametrize("n", [300, 520])
def test_auto_two_streams_bitexact(oracle, od, ctx, n):
    """From 256 pairs the library splits the batch over two streams by default (ofdis_runtime.cpp
    stream_count): every frame equals the one-stream whole-batch result, and frames of both chunks equal
    the oracle."""
    import torch
    w, h, nd = 96, 64, 4
    pairs = [od.synth_pair(w, h, 1, f, 1) for f in range(nd)]
    a = torch.from_numpy(np.stack([pairs[i % nd][0] for i in range(n)])).cuda()
    b = torch.from_numpy(np.stack([pairs[i % nd][1] for i in range(n)])).cuda()
    p = od.oppoint(2, w, 1, 1)
    ctx.set_option("streams", 0)
    ctx.set_option("chunk", 0)
    auto = ctx.run(a, b, p)
    torch.cuda.synchronize()
    auto = auto.cpu().numpy()
    ctx.set_option("streams", 1)
    try:
        one = ctx.run(a, b, p)
        torch.cuda.synchronize()
        one = one.cpu().numpy()
    finally:
        ctx.set_option("streams", 0)
    assert_bitexact(auto, one, "two-stream chunks vs one stream")
    q = oracle.oppoint(2, w, 1, 1)
    half = (n + 1) // 2
    for f in (0, half - 1, half, n - 1):  # first / last frame of each chunk
        ref = oracle.run_u8(pairs[f % nd][0], pairs[f % nd][1], q)
        assert_bitexact(auto[f], ref, f"frame {f}")


def test_cli_stdout_timers(od, tmp_path):
    """run_OF_INT at the default verbosity 2 prints the reference's stdout timers in its order
    (run_dense.cpp:319,352,428; oflow.cpp:177,297,336), with the per-scale patch counts."""
    import os
    import re
    import subprocess
    w, h = 640, 480
    a, b = od.synth_pair(w, h, 1, 2, 1)
    for name, im in (("a.pgm", a), ("b.pgm", b)):
        (tmp_path / name).write_bytes(f"P5\n{w} {h}\n255\n".encode() + im.tobytes())
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "of_dis_amd", "bin", "run_OF_INT")
    r = subprocess.run([exe, str(tmp_path / "a.pgm"), str(tmp_path / "b.pgm"), str(tmp_path / "o.flo")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("TIME")]
    heads = [re.match(r"TIME \(([^)]*)\)", ln).group(1).split(",")[0].strip() for ln in lines]
    assert heads[:3] == ["Image loading", "Pyramide+Gradients", "Grid Memo. Alloc."], heads
    assert heads[-2:] == ["O.Flow Run-Time", "Saving flow file"], heads
    scales = [ln for ln in lines if ln.startswith("TIME (Sc:")]
    p = od.oppoint(2, w, 1, 1)
    assert len(scales) == p.sc_f - p.sc_l + 1
    for ln, s in zip(scales, range(p.sc_f, p.sc_l - 1, -1)):
        m = re.match(r"TIME \(Sc: (\d+), #p:\s*(\d+), pconst, pinit, poptim, cflow, tvopt, total\):"
                     r"\s+([\d.]+)\s+([\d.]+)\s+([\d.]+)\s+([\d.]+)\s+([\d.]+) ->\s+([\d.]+) ms\.", ln)
        assert m, ln
        assert int(m.group(1)) == s
        ws, hs = w >> s, h >> s
        assert int(m.group(2)) == -(-ws // 4) * -(-hs // 4)  # nopw * noph, steps 4 (patchgrid.cpp:43-46)


def test_capture_on_large_batch(oracle, od, ctx):
    """A stage capture on a batch that would be chunked over two streams (>= 256 pairs, and with explicit
    stream / chunk options) runs as one launch and captures frame 0 exactly."""
    import torch
    w, h, n = 96, 64, 520
    pa, pb = od.synth_pair(w, h, 1, 0, 1)
    a = torch.from_numpy(np.stack([pa] * n)).cuda()
    b = torch.from_numpy(np.stack([pb] * n)).cuda()
    p = od.oppoint(2, w, 1, 1)
    q = oracle.oppoint(2, w, 1, 1)
    ref, cap_d, cap_t = oracle.run_u8(pa, pb, q, capture=True)
    for streams, chunk in ((0, 0), (3, 100)):
        dis = {s: np.zeros_like(v) for s, v in cap_d.items()}
        tv = {s: np.zeros_like(v) for s, v in cap_t.items()}
        ctx.set_option("streams", streams)
        ctx.set_option("chunk", chunk)
        ctx.set_capture(dis, tv)
        try:
            out = ctx.run(a, b, p)
            torch.cuda.synchronize()
        finally:
            ctx.set_capture(None, None)
            ctx.set_option("streams", 0)
            ctx.set_option("chunk", 0)
        for s in cap_d:
            assert_bitexact(dis[s], cap_d[s], f"streams={streams} chunk={chunk}: scale {s} after aggregation")
            assert_bitexact(tv[s], cap_t[s], f"streams={streams} chunk={chunk}: scale {s} after TV refinement")
        o = out.cpu().numpy()
        assert_bitexact(o[0], ref, "frame 0")
        assert_bitexact(o[n - 1], ref, "last frame")


def test_large_batch_1080p_first_middle_last(oracle, od, ctx):
    """2048 pairs of a 1080p op-point-2 pair in one call (the library's two 1024-pair chunks on two streams,
    34 GB of output): the first, middle (both chunk edges) and last frames equal the oracle bit for bit, and
    every frame equals frame 0 on the device (late-frame indexing and chunking at the bench's output size)."""
    import torch
    w, h, n = 1920, 1080, 2048
    pa, pb = od.synth_pair(w, h, 1, 7, 1)
    a = torch.from_numpy(pa).cuda().unsqueeze(0).expand(n, -1, -1, -1).contiguous()
    b = torch.from_numpy(pb).cuda().unsqueeze(0).expand(n, -1, -1, -1).contiguous()
    p = od.oppoint(2, w, 1, 1)
    ctx.set_option("streams", 0)
    ctx.set_option("chunk", 0)
    out = ctx.run(a, b, p)
    torch.cuda.synchronize()
    del a, b
    ref = oracle.run_u8(pa, pb, oracle.oppoint(2, w, 1, 1))
    for f in (0, n // 2 - 1, n // 2, n - 1):
        assert_bitexact(out[f].cpu().numpy(), ref, f"frame {f} of {n}")
    ov = out.view(n, -1).view(torch.int32)
    same = [int(torch.equal(ov[f], ov[0])) for f in range(n)]
    assert sum(same) == n, [f for f in range(n) if not same[f]][:10]
    del out, ov
    torch.cuda.empty_cache()


@pytest.mark.parametrize("deriv", [0, 1])
def test_throughput_row_blocks_bitexact(oracle, od, ctx, deriv):
    """A batch large enough that the fused system kernel takes its throughput row blocks (frames x row blocks
    >= 4096: 1400 pairs of 160 x 120) with smsys_deriv on and off: every frame equals the oracle's bits (the
    single-pair tests only ever see the latency-regime row blocks)."""
    import torch
    w, h, n, nd = 160, 120, 1400, 4
    pairs = [od.synth_pair(w, h, 1, 11 + f, 1) for f in range(nd)]
    a = torch.from_numpy(np.stack([pairs[i % nd][0] for i in range(n)])).cuda()
    b = torch.from_numpy(np.stack([pairs[i % nd][1] for i in range(n)])).cuda()
    p = od.oppoint(2, w, 1, 1)
    q = oracle.oppoint(2, w, 1, 1)
    ctx.set_option("smsys_deriv", deriv)
    ctx.set_option("streams", 1)
    try:
        out = ctx.run(a, b, p)
        torch.cuda.synchronize()
        out = out.cpu().numpy()
    finally:
        ctx.set_option("smsys_deriv", 1)
        ctx.set_option("streams", 0)
    for i in range(nd):
        ref = oracle.run_u8(pairs[i][0], pairs[i][1], q)
        assert_bitexact(out[i], ref, f"frame {i}")
    for f in range(nd, n):
        assert_bitexact(out[f], out[f % nd], f"frame {f}")
