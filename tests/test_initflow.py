"""Initial-flow input: OFClass's initflow (oflow.h:106, oflow.cpp:215-217) fed the way
run_dense.cpp's commented-out plumbing prepares it (:293-294 hasinfile/infile, :302 divisibility
2^(sc_f+1), :356-379 replicate pad, x 2^-(sc_f+1), cv::resize INTER_AREA).

CPU part: the oracle's INTER_AREA restatement against an independent numpy float32 loop of OpenCV's
resizeAreaFast order (k x k block row-major, summed four at a time, x 1/k^2).  OpenCV is absent, so the
order itself is unpinned; exactness checks (constant fields, powers of two) anchor the arithmetic.
GPU part (marked gpu): the HIP path with an initial flow against the oracle, bit for bit.
"""
import ctypes as C

import numpy as np
import pytest


@pytest.fixture(scope="module")
def O():
    from oracle import pyoracle
    pyoracle.build()
    return pyoracle


def area_numpy(init, padw, padh, sc_f):
    h, w, nop = init.shape
    k = 1 << (sc_f + 1)
    l, t = padw // 2, padh // 2
    ys = np.clip(np.arange(h + padh) - t, 0, h - 1)
    xs = np.clip(np.arange(w + padw) - l, 0, w - 1)
    padded = init[ys][:, xs] * np.float32(2.0 ** (-sc_f - 1))
    ho, wo = (h + padh) // k, (w + padw) // k
    out = np.zeros((ho, wo, nop), np.float32)
    scale = np.float32(1.0 / (k * k))
    for y in range(ho):
        for x in range(wo):
            blk = padded[y * k:(y + 1) * k, x * k:(x + 1) * k].reshape(k * k, nop)  # row-major
            s = np.zeros(nop, np.float32)
            j = 0
            while j <= k * k - 4:
                s = s + (((blk[j] + blk[j + 1]) + blk[j + 2]) + blk[j + 3])
                j += 4
            while j < k * k:
                s = s + blk[j]
                j += 1
            out[y, x] = s * scale
    return out


@pytest.mark.parametrize("w,h,nop,sc_f", [(40, 24, 2, 1), (37, 29, 2, 2), (64, 48, 1, 2), (21, 13, 2, 0)])
def test_oracle_init_area_matches_numpy(O, w, h, nop, sc_f):
    rng = np.random.default_rng(w * h)
    init = (rng.standard_normal((h, w, nop)) * 7).astype(np.float32)
    padw, padh = O.divisibility_pad(w, h, sc_f + 1)
    k = 1 << (sc_f + 1)
    out = np.zeros(((h + padh) // k, (w + padw) // k, nop), np.float32)
    O.lib().ofo_init_flow_area(init, w, h, nop, padw, padh, sc_f, out)
    want = area_numpy(init, padw, padh, sc_f)
    assert np.array_equal(out.view(np.uint32), want.view(np.uint32))


def test_oracle_init_constant_field(O):
    """A constant full-resolution flow c arrives at the coarsest grid as c * 2^-(sc_f+1), exactly."""
    w, h, sc_f = 48, 40, 2
    init = np.empty((h, w, 2), np.float32)
    init[..., 0], init[..., 1] = 6.5, -2.25
    padw, padh = O.divisibility_pad(w, h, sc_f + 1)
    out = np.zeros(((h + padh) >> 3, (w + padw) >> 3, 2), np.float32)
    O.lib().ofo_init_flow_area(init, w, h, 2, padw, padh, sc_f, out)
    assert np.all(out[..., 0] == np.float32(6.5 / 8)) and np.all(out[..., 1] == np.float32(-2.25 / 8))


def test_oracle_init_changes_result_and_is_used(O):
    """The initial flow reaches OFClass: initialised with the pair's own flow the result stays near the
    uninitialised one; a wildly wrong initialisation moves it much further."""
    import of_dis_amd as od
    w, h = 160, 120
    a, b = od.synth_pair(w, h, 1, 3, 1)
    q = O.oppoint(2, w, 1, 1)
    base = O.run_u8(a, b, q)
    good = O.run_u8(a, b, q, init=base)
    bad = O.run_u8(a, b, q, init=np.full((h, w, 2), 40.0, np.float32))
    assert np.isfinite(good).all() and np.isfinite(bad).all()
    epe = lambda x, y: float(np.sqrt(((x - y) ** 2).sum(-1)).mean())  # noqa: E731
    assert 0 < epe(good, base) < 2.0
    assert epe(bad, base) > 5 * epe(good, base)


# ------------------------------------------------------------------------------------------- GPU

CASES = [
    (160, 120, 1, 1, 2, {}),
    (173, 97, 1, 1, 2, {}),        # divisibility padding by 2^(sc_f+1) on both axes
    (192, 128, 3, 1, 3, {}),
    (240, 120, 1, 2, 4, {"max_iter": 16, "min_iter": 16}),
    (160, 120, 1, 1, 2, {"usefbcon": 1}),
]


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,noc,mode,op,over", CASES)
def test_gpu_init_bitexact(O, w, h, noc, mode, op, over):
    import of_dis_amd as od
    a, b = od.synth_pair(w, h, noc, 5, mode)
    p, q = od.oppoint(op, w, mode, noc), O.oppoint(op, w, mode, noc)
    for k, v in over.items():
        setattr(p, k, v)
        setattr(q, k, v)
    rng = np.random.default_rng(1)
    nop = 2 if mode == 1 else 1
    init = (O.run_u8(a, b, q) + rng.standard_normal((h, w, nop)).astype(np.float32)).astype(np.float32)
    want = O.run_u8(a, b, q, init=init)
    ctx = od.Context(0)
    got = ctx.run_host(a, b, p, init=init)
    ctx.close()
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
def test_gpu_init_batch_paths(O):
    """Batch with per-frame initial flows: one stream (graph), eager, round-robin chunks (eager and captured)."""
    import torch
    import of_dis_amd as od
    w, h, n = 176, 96, 5
    pairs = [od.synth_pair(w, h, 1, f, 1) for f in range(n)]
    q = O.oppoint(2, w, 1, 1)
    inits = [O.run_u8(x[0], x[1], q) * np.float32(0.9) for x in pairs]
    want = [O.run_u8(x[0], x[1], q, init=i) for x, i in zip(pairs, inits)]
    a = torch.from_numpy(np.stack([x[0] for x in pairs])).cuda()
    b = torch.from_numpy(np.stack([x[1] for x in pairs])).cuda()
    ini = torch.from_numpy(np.stack(inits)).cuda()
    p = od.oppoint(2, w, 1, 1)
    ctx = od.Context(0)
    for streams, chunk, graph in ((1, 0, 1), (1, 0, 1), (1, 0, 0), (2, 2, 1), (2, 2, 2), (1, 2, 1)):
        ctx.set_option("streams", streams)
        ctx.set_option("chunk", chunk)
        ctx.set_option("graph", graph)
        out = ctx.run(a, b, p, init=ini)
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        for f in range(n):
            assert np.array_equal(o[f].view(np.uint32), want[f].view(np.uint32)), (streams, chunk, graph, f)
    ctx.close()


@pytest.mark.gpu
def test_gpu_cli_hasinfile(O, tmp_path):
    import os
    import subprocess
    import of_dis_amd as od
    w, h = 160, 112
    a, b = od.synth_pair(w, h, 1, 2, 1)
    for name, im in (("a.pgm", a), ("b.pgm", b)):
        (tmp_path / name).write_bytes(f"P5\n{w} {h}\n255\n".encode() + im.tobytes())
    q = O.oppoint(2, w, 1, 1)
    init = O.run_u8(a, b, q) + np.float32(0.5)
    od.write_flo(str(tmp_path / "init.flo"), init)
    params = [str(x) for x in (q.sc_f, q.sc_l, q.max_iter, q.min_iter)] + \
        ["0.05", "0.95", "0", "8", "0.4", "0", "1", "0", "1", "10", "10", "5", "1", "3", "1.6", "0"]
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "of_dis_amd", "bin", "run_OF_INT")
    for extra, init_used in (([], None), (["0"], None), (["1", str(tmp_path / "init.flo")], init)):
        out = tmp_path / "o.flo"
        r = subprocess.run([exe, str(tmp_path / "a.pgm"), str(tmp_path / "b.pgm"), str(out)] + params + extra,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        q2 = O.params_from_strings(params, 1, 1) if hasattr(O, "params_from_strings") else q
        want = O.run_u8(a, b, q2, init=init_used)
        assert np.array_equal(od.read_flo(str(out)).view(np.uint32), want.view(np.uint32)), extra
