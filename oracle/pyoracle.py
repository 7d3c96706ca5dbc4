"""TEST INFRASTRUCTURE ONLY: ctypes bindings to the CPU oracle and the reference FDF1.0.1 build.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
The product (of_dis_amd) never does.

* ``liboracle.so`` -- the clean-room CPU restatement (oracle/ofdis_oracle.c).
* ``_ref/libfdf_ref_c{1,3}.so`` -- the reference's own FDF1.0.1 sources compiled where they lie
  (oracle/Makefile); used to pin the restatement of the variational part bit-for-bit.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")


class Params(C.Structure):
    """Layout of ``ofdis_params`` (include/ofdis.h)."""

    _fields_ = [
        ("mode", C.c_int), ("noc", C.c_int), ("sc_f", C.c_int), ("sc_l", C.c_int),
        ("max_iter", C.c_int), ("min_iter", C.c_int),
        ("dp_thresh", C.c_float), ("dr_thresh", C.c_float), ("res_thresh", C.c_float),
        ("p_samp_s", C.c_int), ("patove", C.c_float), ("usefbcon", C.c_int), ("costfct", C.c_int),
        ("patnorm", C.c_int), ("usetvref", C.c_int),
        ("tv_alpha", C.c_float), ("tv_gamma", C.c_float), ("tv_delta", C.c_float),
        ("tv_innerit", C.c_int), ("tv_solverit", C.c_int), ("tv_sor", C.c_float), ("verbosity", C.c_int),
        ("omp_build", C.c_int), ("gradmag", C.c_int),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def build(quiet: bool = True) -> None:
    """Build liboracle.so and (when /root/reference exists) _ref/*.so."""
    targets = ["liboracle.so"]
    if os.path.isdir(os.environ.get("OFDIS_REFERENCE", "/root/reference")):
        targets.append("ref")
    subprocess.run(["make", "-s", "-C", HERE] + targets, check=True,
                   stdout=subprocess.DEVNULL if quiet else None)


_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        vp = C.c_void_p
        L.ofo_eigen_sum.argtypes = [_f32p, C.c_int]
        L.ofo_eigen_sum.restype = C.c_float
        L.ofo_auto_first_scale.argtypes = [C.c_int, C.c_int, C.c_int]
        L.ofo_params_oppoint.argtypes = [C.POINTER(Params), C.c_int, C.c_int, C.c_int, C.c_int]
        L.ofo_divisibility_pad.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.ofo_build_pyramid.argtypes = [_u8p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, vp]
        L.ofo_build_pyramid_ex.argtypes = [_u8p] + [C.c_int] * 7 + [vp, vp, vp]
        L.ofo_oflow.argtypes = [vp] * 6 + [C.c_int, _f32p, vp, C.c_int, C.c_int, C.POINTER(Params), vp, vp]
        L.ofo_upsample_crop.argtypes = [_f32p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                        C.c_int, C.c_int, _f32p]
        L.ofo_run_u8.argtypes = [_u8p, _u8p, C.c_int, C.c_int, C.POINTER(Params), _f32p, vp, vp]
        L.ofo_run_u8_init.argtypes = [_u8p, _u8p, vp, C.c_int, C.c_int, C.POINTER(Params), _f32p, vp, vp]
        L.ofo_run_u8_stages.argtypes = [_u8p, _u8p, vp, C.c_int, C.c_int, C.POINTER(Params), _f32p, vp, vp,
                                        C.POINTER(C.c_double)]
        L.ofo_init_flow_area.argtypes = [_f32p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _f32p]
        L.ofo_refine_level.argtypes = [_f32p, _f32p, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(Params), _f32p]
        L.ofo_image_warp.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, C.c_int, C.c_int, C.c_int]
        L.ofo_get_derivatives.argtypes = [_f32p, _f32p, C.c_int, C.c_int, C.c_int] + [_f32p] * 8
        L.ofo_compute_smoothness.argtypes = [_f32p, _f32p, _f32p, _f32p, C.c_int, C.c_int, C.c_float]
        L.ofo_sub_laplacian.argtypes = [_f32p, _f32p, _f32p, _f32p, C.c_int, C.c_int]
        L.ofo_compute_data.argtypes = [_f32p] * 16 + [C.c_int, C.c_int, C.c_int, C.c_float, C.c_float]
        L.ofo_compute_data_de.argtypes = [_f32p] * 12 + [C.c_int, C.c_int, C.c_int, C.c_float, C.c_float]
        L.ofo_sor_coupled.argtypes = [_f32p] * 9 + [C.c_int, C.c_int, C.c_int, C.c_float]
        L.ofo_sor_point_de.argtypes = [_f32p] * 5 + [C.c_int, C.c_int, C.c_int, C.c_float]
        L.ofo_sor_point_of.argtypes = [_f32p] * 9 + [C.c_int, C.c_int, C.c_int, C.c_float]
        L.ofo_sor_rb_of.argtypes = [_f32p] * 9 + [C.c_int, C.c_int, C.c_int, C.c_float]
        L.ofo_sor_rb_de.argtypes = [_f32p] * 5 + [C.c_int, C.c_int, C.c_int, C.c_float]
        L.ofo_set_sor_order.argtypes = [C.c_int]
        L.ofo_get_sor_order.restype = C.c_int
        for f in ("ofo_params_oppoint", "ofo_build_pyramid", "ofo_build_pyramid_ex", "ofo_oflow", "ofo_upsample_crop", "ofo_run_u8",
                  "ofo_run_u8_init", "ofo_refine_level"):
            getattr(L, f).restype = C.c_int
        _lib = L
    return _lib


class sor_order:
    """Context manager: the oracle's refinements use red-black SOR order (1; the GPU's opt-in sor_mode = 1) or
    solver.c's lexicographic order (0, the default) inside the block."""

    def __init__(self, order: int):
        self.order = order

    def __enter__(self):
        self.prev = lib().ofo_get_sor_order()
        lib().ofo_set_sor_order(self.order)
        return self

    def __exit__(self, *exc):
        lib().ofo_set_sor_order(self.prev)
        return False


def oppoint(op: int, width: int, mode: int = 1, noc: int = 1) -> Params:
    p = Params()
    lib().ofo_params_oppoint(C.byref(p), op, width, mode, noc)
    return p


def divisibility_pad(w, h, sc_f):
    pw, ph = C.c_int(), C.c_int()
    lib().ofo_divisibility_pad(w, h, sc_f, C.byref(pw), C.byref(ph))
    return pw.value, ph.value


def _ptr_array(arrs, n=32):
    out = (C.c_void_p * n)()
    for s, a in arrs.items():
        out[s] = a.ctypes.data
    return out


def build_pyramid(img: np.ndarray, p: Params, imgpadding: int):
    """img: divisibility-padded u8 [h][w][noc] -> dict level -> (img, dx, dy) padded float arrays."""
    h, w = img.shape[:2]
    noc = p.noc
    lev = {}
    for s in range(p.sc_l, p.sc_f + 1):
        shp = ((h >> s) + 2 * imgpadding, (w >> s) + 2 * imgpadding, noc)
        lev[s] = tuple(np.zeros(shp, np.float32) for _ in range(3))
    rc = lib().ofo_build_pyramid_ex(np.ascontiguousarray(img, dtype=np.uint8), w, h, noc, p.sc_f, p.sc_l,
                                    imgpadding, p.gradmag,
                                    _ptr_array({s: v[0] for s, v in lev.items()}),
                                    _ptr_array({s: v[1] for s, v in lev.items()}),
                                    _ptr_array({s: v[2] for s, v in lev.items()}))
    assert rc == 0, rc
    return lev


def nop_of(p: Params) -> int:
    return 2 if p.mode == 1 else 1


def oflow(pyr_a, pyr_b, width, height, p: Params, imgpadding: int, initflow=None, capture=False):
    """OFClass restatement.  pyr_a/pyr_b: dict level -> (img, dx, dy).  Returns flow at sc_l (and captures)."""
    nop = nop_of(p)
    out = np.zeros(((height >> p.sc_l), (width >> p.sc_l), nop), np.float32)
    cap_d, cap_t = {}, {}
    if capture:
        for s in range(p.sc_l, p.sc_f + 1):
            cap_d[s] = np.zeros(((height >> s), (width >> s), nop), np.float32)
            cap_t[s] = np.zeros_like(cap_d[s])
    arrs = [_ptr_array({s: v[k] for s, v in pyr.items()}) for pyr in (pyr_a, pyr_b) for k in range(3)]
    init = None if initflow is None else np.ascontiguousarray(initflow, dtype=np.float32)
    rc = lib().ofo_oflow(*arrs, imgpadding, out, None if init is None else init.ctypes.data, width, height,
                         C.byref(p), _ptr_array(cap_d) if capture else None, _ptr_array(cap_t) if capture else None)
    if rc != 0:
        raise RuntimeError(f"ofo_oflow failed: {rc}")
    return (out, cap_d, cap_t) if capture else out


def run_u8(a: np.ndarray, b: np.ndarray, p: Params, capture=False, init=None):
    """Whole run_dense pipeline for one pair of u8 [h][w][noc] images -> flow [h][w][nop].
    init: optional full-resolution initial flow [h][w][nop] (run_dense.cpp:293-294, 356-379)."""
    h, w = a.shape[:2]
    nop = nop_of(p)
    out = np.zeros((h, w, nop), np.float32)
    cap_d, cap_t = {}, {}
    if capture:
        pw, ph = divisibility_pad(w, h, p.sc_f + (init is not None))
        for s in range(p.sc_l, p.sc_f + 1):
            cap_d[s] = np.zeros((((h + ph) >> s), ((w + pw) >> s), nop), np.float32)
            cap_t[s] = np.zeros_like(cap_d[s])
    ini = None if init is None else np.ascontiguousarray(init, np.float32).reshape(h, w, nop)
    rc = lib().ofo_run_u8_init(np.ascontiguousarray(a, np.uint8), np.ascontiguousarray(b, np.uint8),
                               None if ini is None else ini.ctypes.data, w, h, C.byref(p), out,
                               _ptr_array(cap_d) if capture else None, _ptr_array(cap_t) if capture else None)
    if rc != 0:
        raise RuntimeError(f"ofo_run_u8 failed: {rc}")
    return (out, cap_d, cap_t) if capture else out


def run_u8_stages(a: np.ndarray, b: np.ndarray, p: Params):
    """run_u8 plus the wall time (s) of its stages: pad, pyramid (both frames), OFClass, upsample + crop."""
    h, w = a.shape[:2]
    out = np.zeros((h, w, nop_of(p)), np.float32)
    st = (C.c_double * 4)()
    rc = lib().ofo_run_u8_stages(np.ascontiguousarray(a, np.uint8), np.ascontiguousarray(b, np.uint8), None, w, h,
                                 C.byref(p), out, None, None, st)
    if rc != 0:
        raise RuntimeError(f"ofo_run_u8_stages failed: {rc}")
    return out, {"pad": st[0], "pyramid": st[1], "ofclass": st[2], "upsample": st[3]}


# --------------------------------------------------------------------------- reference FDF1.0.1 (_ref)

class ImageT(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("stride", C.c_int), ("c1", C.c_void_p)]


class ColorImageT(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("stride", C.c_int),
                ("c1", C.c_void_p), ("c2", C.c_void_p), ("c3", C.c_void_p)]


def _aligned(n: int) -> np.ndarray:
    raw = np.empty(n + 16, np.float32)
    off = (-raw.ctypes.data % 64) // 4
    return raw[off:off + n]


class RefImage:
    """An FDF image_t / color_image_t backed by a 64-byte aligned numpy buffer with stride ceil4(w).

    Padding columns are filled with garbage on purpose (the reference leaves them uninitialised)."""

    def __init__(self, w, h, noc=1, rng=None):
        self.w, self.h, self.noc = w, h, noc
        self.stride = (w + 3) // 4 * 4
        self.buf = _aligned(self.stride * h * noc)
        rng = rng or np.random.default_rng(99)
        self.buf[:] = rng.standard_normal(self.buf.size).astype(np.float32) * 1e3
        if noc == 1:
            self.st = ImageT(w, h, self.stride, self.buf.ctypes.data)
        else:
            n = self.stride * h
            d = self.buf.ctypes.data
            self.st = ColorImageT(w, h, self.stride, d, d + 4 * n, d + 8 * n)

    @property
    def ptr(self):
        return C.byref(self.st)

    def set(self, planar: np.ndarray):
        """planar: [noc][h][w] or [h][w]."""
        v = self.view()
        v[...] = np.asarray(planar, np.float32).reshape(v.shape)

    def view(self):
        return self.buf.reshape(self.noc, self.h, self.stride)[:, :, : self.w].reshape(
            (self.noc, self.h, self.w) if self.noc > 1 else (self.h, self.w))

    def get(self):
        return np.ascontiguousarray(self.view())


_ref_libs = {}


def ref_available() -> bool:
    return all(os.path.exists(os.path.join(HERE, "_ref", f"libfdf_ref_c{c}.so")) for c in (1, 3))


def ref(noc: int = 1):
    """The reference's FDF1.0.1 compiled with SELECTCHANNEL = noc."""
    if noc not in _ref_libs:
        path = os.path.join(HERE, "_ref", f"libfdf_ref_c{noc}.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        vp = C.c_void_p
        L.image_new.restype = C.POINTER(ImageT)
        L.convolution_new.restype = vp
        L.convolution_new.argtypes = [C.c_int, C.POINTER(C.c_float), C.c_int]
        L.image_warp.argtypes = [vp] * 5
        L.get_derivatives.argtypes = [vp] * 11
        L.compute_smoothness.argtypes = [vp] * 5 + [C.c_float]
        L.sub_laplacian.argtypes = [vp] * 4
        L.compute_data.argtypes = [vp] * 20 + [C.c_float] * 3
        L.compute_data_DE.argtypes = [vp] * 14 + [C.c_float] * 3
        L.sor_coupled.argtypes = [vp] * 9 + [C.c_int, C.c_float]
        L.sor_coupled_slow_but_readable_DE.argtypes = [vp] * 5 + [C.c_int, C.c_float]
        L.sor_coupled_slow_but_readable.argtypes = [vp] * 9 + [C.c_int, C.c_float]
        _ref_libs[noc] = L
    return _ref_libs[noc]


def ref_conv(L, order: int):
    """deriv (order 2) and deriv_flow (order 1) filters exactly as refine_variational.cpp:45-48 builds them."""
    if order == 2:
        half = (C.c_float * 3)(0.0, np.float32(-8.0) / np.float32(12.0), np.float32(1.0) / np.float32(12.0))
    else:
        half = (C.c_float * 2)(0.0, -0.5)
    return L.convolution_new(order, half, 0)


def ref_refine_level(noc, mode, im1, im2, flow, level, p):
    """refine_variational.cpp:152-342 glue, driven through the reference FDF functions."""
    h, w = im1.shape[-2:]
    R = ref(noc)
    n_inner = p["tv_innerit"] * (level + 1)
    f32 = np.float32
    qa = f32(0.25) * f32(p["tv_alpha"])
    hgo3 = f32(p["tv_gamma"]) * f32(0.5) / f32(3.0)
    hdo3 = f32(p["tv_delta"]) * f32(0.5) / f32(3.0)
    img = lambda c=1: RefImage(w, h, c)
    rim1, rim2 = img(noc), img(noc)
    rim1.set(im1); rim2.set(im2)
    wx, wy = img(), img()
    wx.set(flow[..., 0])
    if mode == 1:
        wy.set(flow[..., 1])
    else:
        wy.buf[:] = 0  # image_erase(wy_dummy)
    du, dv, mask, sh, sv, uu, vv = (img() for _ in range(7))
    a11, a12, a22, b1, b2 = (img() for _ in range(5))
    wim2 = img(noc)
    I = [img(noc) for _ in range(8)]
    R.image_warp(wim2.ptr, mask.ptr, rim2.ptr, wx.ptr, wy.ptr)
    R.get_derivatives(rim1.ptr, wim2.ptr, ref_conv(R, 2), *[x.ptr for x in I])
    du.buf[:] = 0; dv.buf[:] = 0
    uu.buf[:] = wx.buf; vv.buf[:] = wy.buf
    dflow = ref_conv(R, 1)
    for _ in range(n_inner):
        R.compute_smoothness(sh.ptr, sv.ptr, uu.ptr, vv.ptr if mode == 1 else wy.ptr, dflow, C.c_float(qa))
        if mode == 1:
            R.compute_data(a11.ptr, a12.ptr, a22.ptr, b1.ptr, b2.ptr, mask.ptr, wx.ptr, wy.ptr, du.ptr, dv.ptr,
                           uu.ptr, vv.ptr, *[x.ptr for x in I], C.c_float(hdo3), C.c_float(0), C.c_float(hgo3))
            R.sub_laplacian(b1.ptr, wx.ptr, sh.ptr, sv.ptr)
            R.sub_laplacian(b2.ptr, wy.ptr, sh.ptr, sv.ptr)
            sor = R.sor_coupled_slow_but_readable if p.get("omp_build") else R.sor_coupled  # :202-205
            sor(du.ptr, dv.ptr, a11.ptr, a12.ptr, a22.ptr, b1.ptr, b2.ptr, sh.ptr, sv.ptr,
                p["tv_solverit"], C.c_float(p["tv_sor"]))
            uu.buf[:] = wx.buf + du.buf
            vv.buf[:] = wy.buf + dv.buf
        else:
            R.compute_data_DE(a11.ptr, b1.ptr, mask.ptr, wx.ptr, du.ptr, uu.ptr, *[x.ptr for x in I],
                              C.c_float(hdo3), C.c_float(0), C.c_float(hgo3))
            R.sub_laplacian(b1.ptr, wx.ptr, sh.ptr, sv.ptr)
            R.sor_coupled_slow_but_readable_DE(du.ptr, a11.ptr, b1.ptr, sh.ptr, sv.ptr, p["tv_solverit"],
                                               C.c_float(p["tv_sor"]))
            s = wx.buf + du.buf
            uu.buf[:] = np.where(s < 0, s, np.float32(0))  # _mm_min_ps(s, 0)
    out = np.stack([uu.get()] + ([vv.get()] if mode == 1 else []), axis=-1)
    return out
