"""CPU tests of the C-ABI library (no GPU): every header symbol is exported, host-only entry points
(parameters, validation, file formats, synthetic inputs) behave like the reference's, and the device
entry points fail loudly -- with a status code, never a silent CPU fallback -- when no GPU is visible.
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import of_dis_amd as od
from of_dis_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ofdis.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ofdis_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    L = od.lib()
    names = header_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # and the ctypes mirror binds exactly the header's set
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(re.findall(r"\bT (ofdis_[a-z0-9_]+)", nm.stdout))
    assert set(names) <= exported
    assert exported <= set(names), f"exported but undeclared: {sorted(exported - set(names))}"


def test_library_is_gfx950_code():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", _lib.LIB_PATH], capture_output=True, text=True)
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob or "gfx950" in out.stdout


def test_abi_version_and_status_strings():
    L = od.lib()
    assert L.ofdis_abi_version() == 2
    for code in range(7):
        assert L.ofdis_status_string(code)
    assert b"unknown" in L.ofdis_status_string(99).lower()


# op-point table of run_dense.cpp:226-268 (sc_f automatic, run_dense.cpp:181-184)
OPPOINTS = {
    1: dict(p_samp_s=8, patove=0.3, max_iter=16, min_iter=16, usetvref=0, keep=2),
    2: dict(p_samp_s=8, patove=0.4, max_iter=12, min_iter=12, usetvref=1, keep=2),
    3: dict(p_samp_s=12, patove=0.75, max_iter=16, min_iter=16, usetvref=1, keep=4),
    4: dict(p_samp_s=12, patove=0.75, max_iter=128, min_iter=128, usetvref=1, keep=5),
}


@pytest.mark.parametrize("op", [1, 2, 3, 4])
@pytest.mark.parametrize("width", [640, 1920, 3840, 100])
def test_oppoint_table(oracle, op, width):
    p = od.oppoint(op, width)
    e = OPPOINTS[op]
    sc_f = int(np.floor(np.log2(2.0 * width / (5.0 * e["p_samp_s"]))))
    assert p.sc_f == sc_f == od.auto_first_scale(width, 5, e["p_samp_s"])
    assert p.sc_l == max(0, sc_f - e["keep"])
    for k in ("p_samp_s", "max_iter", "min_iter", "usetvref"):
        assert getattr(p, k) == e[k], k
    assert np.float32(p.patove) == np.float32(e["patove"])
    assert (p.costfct, p.patnorm, p.usefbcon, p.tv_innerit, p.tv_solverit) == (0, 1, 0, 1, 3)
    assert np.float32(p.tv_sor) == np.float32(1.6) and p.tv_alpha == 10 and p.tv_gamma == 10 and p.tv_delta == 5
    # the oracle's table is the same
    q = oracle.oppoint(op, width, 1, 1)
    assert bytes(p) == bytes(q)


def test_baseline_shapes():
    """SURVEY §8 shapes table: coarsest/finest scales of configs A, B, C, E."""
    for (w, op, mode), (f, l) in {(640, 2, 1): (5, 3), (1920, 2, 1): (6, 4), (1920, 3, 1): (6, 2),
                                  (3840, 4, 2): (7, 2)}.items():
        p = od.oppoint(op, w, mode)
        assert (p.sc_f, p.sc_l) == (f, l)


def test_params_from_strings_matches_readme_order():
    vals = "7 2 128 128 0.05 0.95 0 12 0.75 0 1 0 1 10 10 5 10 3 1.6 2".split()
    p = od.params_from_strings(vals, od.MODE_DE, 1)
    assert (p.sc_f, p.sc_l, p.max_iter, p.min_iter, p.p_samp_s) == (7, 2, 128, 128, 12)
    assert (p.usefbcon, p.patnorm, p.costfct, p.usetvref, p.tv_innerit, p.tv_solverit, p.verbosity) == \
        (0, 1, 0, 1, 10, 3, 2)
    assert np.float32(p.dp_thresh) == np.float32(0.05) and np.float32(p.patove) == np.float32(0.75)
    with pytest.raises(od.OfdisError):
        od.params_from_strings(vals[:19])


@pytest.mark.parametrize("change,code", [
    ({"p_samp_s": 7}, _lib.ERR_INVALID_ARGUMENT),      # odd patch
    ({"p_samp_s": 0}, _lib.ERR_INVALID_ARGUMENT),
    ({"sc_l": 7}, _lib.ERR_INVALID_ARGUMENT),          # sc_l > sc_f
    ({"costfct": 10}, _lib.ERR_UNSUPPORTED),           # NCC: unimplemented upstream too
    ({"patove": 1.0}, _lib.ERR_INVALID_ARGUMENT),
    ({"mode": 3}, _lib.ERR_INVALID_ARGUMENT),
    ({"noc": 2}, _lib.ERR_INVALID_ARGUMENT),
])
def test_validation_rejects(change, code):
    p = od.oppoint(2, 1920).copy(**change)
    assert od.validate(p, 1920, 1088, 8) == code


@pytest.mark.parametrize("noc", [1, 3])
def test_every_even_patch_size_accepted(noc):
    """The reference takes any even p with p*p*noc a multiple of 4 (run_dense.cpp:280, patch.cpp:230): every
    such shape up to 32 validates; odd sizes do not."""
    for p_s in range(2, 34, 2):
        p = od.oppoint(2, 1920, od.MODE_OF, noc).copy(p_samp_s=p_s)
        assert od.validate(p, 1920, 1088, p_s) == 0, p_s
        assert od.validate(p, 1920, 1088, p_s + 6) == 0, p_s  # imgpadding > p
    for p_s in (3, 9, 15):
        assert od.validate(od.oppoint(2, 1920, od.MODE_OF, noc).copy(p_samp_s=p_s)) == _lib.ERR_INVALID_ARGUMENT


def test_validation_geometry():
    p = od.oppoint(2, 1920)
    assert od.validate(p, 1920, 1088, 8) == 0
    assert od.validate(p.copy(usefbcon=1), 1920, 1088, 8) == 0  # forward-backward merging is supported
    assert od.validate(p, 1920, 1080, 8) == _lib.ERR_INVALID_ARGUMENT  # not divisible by 2^6
    assert od.validate(p, 1920, 1088, 4) == _lib.ERR_INVALID_ARGUMENT  # imgpadding < p
    rgb = od.oppoint(3, 1920, od.MODE_OF, 3)
    assert od.validate(rgb, 1920, 1088, 12) == 0


def test_flo_roundtrip_and_layout(tmp_path):
    rng = np.random.default_rng(0)
    flow = rng.standard_normal((7, 5, 2)).astype(np.float32)
    path = str(tmp_path / "x.flo")
    od.write_flo(path, flow)
    raw = open(path, "rb").read()
    assert raw[:4] == b"PIEH"
    assert np.frombuffer(raw[4:12], np.int32).tolist() == [5, 7]
    assert np.array_equal(np.frombuffer(raw[12:], np.float32).reshape(7, 5, 2), flow)
    assert np.array_equal(od.read_flo(path), flow)


def test_pfm_layout(tmp_path):
    d = np.arange(12, dtype=np.float32).reshape(3, 4) - 5
    path = str(tmp_path / "x.pfm")
    od.write_pfm(path, d)
    raw = open(path, "rb").read()
    head = b"Pf\n4 3\n-1.000000\n"
    assert raw.startswith(head)
    body = np.frombuffer(raw[len(head):], np.float32).reshape(3, 4)
    assert np.array_equal(body, -d[::-1])  # rows bottom-up, values negated (run_dense.cpp:61-82)


def test_read_pnm_bgr(tmp_path):
    L = od.lib()
    rgb = np.arange(2 * 3 * 3, dtype=np.uint8).reshape(2, 3, 3)
    path = tmp_path / "x.ppm"
    path.write_bytes(b"P6\n3 2\n255\n" + rgb.tobytes())
    buf = np.zeros(18, np.uint8)
    w, h, c = C.c_int(), C.c_int(), C.c_int()
    assert L.ofdis_read_pnm(str(path).encode(), buf.ctypes.data, C.byref(w), C.byref(h), C.byref(c), 18) == 0
    assert (w.value, h.value, c.value) == (3, 2, 3)
    assert np.array_equal(buf.reshape(2, 3, 3), rgb[..., ::-1])  # cv::imread order
    assert L.ofdis_read_pnm(b"/nonexistent.pgm", None, C.byref(w), C.byref(h), C.byref(c), 0) == _lib.ERR_IO


def test_synth_pair_deterministic_and_moving():
    a1, b1 = od.synth_pair(96, 64, 1, 3)
    a2, b2 = od.synth_pair(96, 64, 1, 3)
    assert np.array_equal(a1, a2) and np.array_equal(b1, b2)
    a3, _ = od.synth_pair(96, 64, 1, 4)
    assert not np.array_equal(a1, a3)
    # frame b is frame a moved by about (+6.5, +2.25): the best integer shift is (6..7, 2)
    A, B = a1[..., 0].astype(np.float32), b1[..., 0].astype(np.float32)
    best = min(((np.abs(A[10:50, 10:80] - B[10 + dy:50 + dy, 10 + dx:80 + dx]).mean(), dx, dy)
                for dx in range(0, 9) for dy in range(0, 5)))
    assert best[1] in (6, 7) and best[2] == 2


def test_algorithmic_bytes_model():
    p = od.oppoint(2, 1920)
    up = od.algorithmic_bytes(p, 1920, 1080, "upsample")
    assert up == 1920 * 1080 * 2 * 4
    sor = od.algorithmic_bytes(p, 1920, 1080, "tv_sor")
    # 44 B/px/sweep over scales 6,5,4 with tv_innerit*(s+1) iterations of 3 sweeps
    want = sum(44 * (1920 >> s) * (1088 >> s) * 3 * (s + 1) for s in (6, 5, 4))
    assert sor == want
    with pytest.raises(od.OfdisError):
        od.algorithmic_bytes(p, 1920, 1080, "nope")


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(od.OfdisError) as e:
        od.Context(0)
    assert e.value.code in (_lib.ERR_NO_DEVICE, _lib.ERR_DEVICE)


def test_cli_usage_and_no_gpu(tmp_path):
    exe = os.path.join(ROOT, "of_dis_amd", "bin", "run_OF_INT")
    assert os.access(exe, os.X_OK)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "usage" in r.stderr
    a, b = od.synth_pair(64, 64, 1, 0)
    for name, im in (("a.pgm", a), ("b.pgm", b)):
        (tmp_path / name).write_bytes(b"P5\n64 64\n255\n" + im.tobytes())
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    r = subprocess.run([exe, str(tmp_path / "a.pgm"), str(tmp_path / "b.pgm"), str(tmp_path / "o.flo"), "2"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert not (tmp_path / "o.flo").exists()


def build_dropin(tmp_path):
    """Compile tests/cpp/dropin_ofclass.cpp against include/ofdis_oflow.hpp + libofdis.so."""
    exe = str(tmp_path / "dropin_ofclass")
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["g++", "-std=c++14", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "dropin_ofclass.cpp"), "-L", libdir, "-lofdis",
                    f"-Wl,-rpath,{libdir}", "-o", exe], check=True, capture_output=True, timeout=300)
    return exe


def test_oflow_hpp_dropin_compiles(tmp_path):
    """The reference-signature OFC::OFClass wrapper compiles and links as plain C++ (no HIP headers)."""
    assert os.access(build_dropin(tmp_path), os.X_OK)


@pytest.mark.parametrize("w,h,noc,op,sc_l", [(640, 480, 3, 2, 0), (960, 540, 1, 2, 0), (1920, 1080, 1, 2, None),
                                           (3840, 2160, 1, 4, None)])
def test_max_frames_per_launch_keeps_plane_groups_below_2_30(w, h, noc, op, sc_l):
    """The refinement kernels address a plane group (frames * noc * skewed plane floats) with 32-bit byte
    offsets; the runtime chunks a batch so that no launch exceeds 2^30 floats per group."""
    p = od.oppoint(op, w, 1, noc)
    if sc_l is not None:
        p.sc_l = sc_l
    cap = od.max_frames_per_launch(p, w, h)
    d = 1 << p.sc_f
    wp, hp = w + (-w) % d, h + (-h) % d
    plane = 0
    for s in range(p.sc_l, p.sc_f + 1):  # skewed plane of the largest level (ofdis_runtime.cpp skew_plane)
        lw, lh = wp >> s, hp >> s
        slots = lw * lh if lh <= lw else (lw + lh - 1) * lh
        plane = max(plane, (slots + 64 + 3) // 4 * 4)
    assert cap >= 1 and cap * noc * plane < 2 ** 30 <= (cap + 1) * noc * plane
    p.usetvref = 0
    assert od.max_frames_per_launch(p, w, h) == 2 ** 30
