"""Host-side mirror of the reference's operator interface for the hot path.

* ``OFClass`` -- same name, argument order and meaning as ``OFC::OFClass::OFClass`` (oflow.h:99-126):
  per-scale padded image/gradient pyramids in, flow at the finest computed scale out.  Computed on
  the GPU by libofdis.so (``ofdis_oflow_compute``).
* ``Context`` -- the batched device path (``ofdis_run_batch_u8``): u8 frame pairs already in HBM ->
  full-resolution flow, i.e. run_dense.cpp's main() minus image decode and file write.
* run_dense helpers: operating points, explicit parameters, .flo/.pfm I/O, synthetic pairs.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np

from ._lib import MODE_DE, MODE_OF, Params, check, lib

_f32 = np.float32


def auto_first_scale(width: int, fratio: int = 5, patchsize: int = 8) -> int:
    """AutoFirstScaleSelect (run_dense.cpp:181-184)."""
    return lib().ofdis_auto_first_scale(width, fratio, patchsize)


def oppoint(op: int, width: int, mode: int = MODE_OF, noc: int = 1) -> Params:
    """Operating point 1-4 (run_dense.cpp:226-268) for an image of the given (unpadded) width."""
    p = Params()
    check(lib().ofdis_params_oppoint(C.byref(p), op, width, mode, noc), "ofdis_params_oppoint")
    return p


def params_from_strings(values: Sequence[str], mode: int = MODE_OF, noc: int = 1) -> Params:
    """The 20 explicit positional CLI parameters (run_dense.cpp:270-295)."""
    arr = (C.c_char_p * len(values))(*[str(v).encode() for v in values])
    p = Params()
    check(lib().ofdis_params_from_strings(C.byref(p), len(values), arr, mode, noc), "ofdis_params_from_strings")
    return p


def validate(p: Params, width: int = -1, height: int = -1, imgpadding: int = -1) -> int:
    return lib().ofdis_params_validate(C.byref(p), width, height, imgpadding)


def synth_pair(width: int, height: int, noc: int = 1, frame: int = 0, mode: int = MODE_OF):
    """Deterministic synthetic u8 pair [h][w][noc]; frame b moves by a known flow."""
    a = np.empty((height, width, noc), np.uint8)
    b = np.empty_like(a)
    check(lib().ofdis_synth_pair_u8(a.ctypes.data, b.ctypes.data, width, height, noc, frame, mode), "synth")
    return a, b


def synth_shift_pair(width: int, height: int, shift, noc: int = 1, frame: int = 0):
    """The synth_pair texture with frame b a pure translation of frame a by shift = (sx, sy) (true flow)."""
    a = np.empty((height, width, noc), np.uint8)
    b = np.empty((height, width, noc), np.uint8)
    check(lib().ofdis_synth_shift_pair_u8(a.ctypes.data, b.ctypes.data, width, height, noc, frame,
                                          float(shift[0]), float(shift[1])), "synth")
    return a, b


def write_flo(path: str, flow: np.ndarray) -> None:
    """SaveFlowFile (run_dense.cpp:17-58)."""
    flow = np.ascontiguousarray(flow, _f32)
    h, w = flow.shape[:2]
    nc = 1 if flow.ndim == 2 else flow.shape[2]
    check(lib().ofdis_write_flo(path.encode(), flow.ctypes.data, w, h, nc), "write_flo")


def write_pfm(path: str, depth: np.ndarray) -> None:
    """SavePFMFile (run_dense.cpp:61-82)."""
    depth = np.ascontiguousarray(depth.reshape(depth.shape[0], depth.shape[1]), _f32)
    check(lib().ofdis_write_pfm(path.encode(), depth.ctypes.data, depth.shape[1], depth.shape[0]), "write_pfm")


def read_flo(path: str, nc: int = 2) -> np.ndarray:
    """ReadFlowFile (run_dense.cpp:85-129)."""
    w, h = C.c_int(), C.c_int()
    check(lib().ofdis_read_flo(path.encode(), None, C.byref(w), C.byref(h), nc), "read_flo")
    out = np.empty((h.value, w.value, nc), _f32)
    check(lib().ofdis_read_flo(path.encode(), out.ctypes.data, C.byref(w), C.byref(h), nc), "read_flo")
    return out


def read_image(path: str, noc: int = 1) -> np.ndarray:
    """cv::imread(path, GRAYSCALE if noc == 1 else COLOR) for PNG / Netpbm: u8 [h, w, noc], BGR for 3."""
    w, h = C.c_int(), C.c_int()
    check(lib().ofdis_read_image(path.encode(), None, C.byref(w), C.byref(h), noc, 0), "read_image")
    out = np.empty((h.value, w.value, noc), np.uint8)
    check(lib().ofdis_read_image(path.encode(), out.ctypes.data, C.byref(w), C.byref(h), noc, out.size),
          "read_image")
    return out


def _ptr_list(arrs, n=32):
    out = (C.c_void_p * n)()
    keep = []
    for s, a in enumerate(arrs):
        if a is None:
            continue
        a = np.ascontiguousarray(a, _f32)
        keep.append(a)
        out[s] = a.ctypes.data
    return out, keep


class OFClass:
    """``OFC::OFClass`` (oflow.h:99-126): constructing it computes the flow into ``outflow``.

    Image/gradient arguments are sequences indexed by scale (entries below sc_l may be None); each
    entry is the padded (h_s + 2*imgpadding, w_s + 2*imgpadding[, noc]) float32 array.  ``outflow``
    (float32, (height>>sc_l)*(width>>sc_l)*nop elements, interleaved) is written in place.  Extra
    keyword-only ``mode`` selects SELECTMODE (1 flow, 2 depth); ``noc`` is SELECTCHANNEL.
    """

    def __init__(self, im_ao_in, im_ao_dx_in, im_ao_dy_in, im_bo_in, im_bo_dx_in, im_bo_dy_in,
                 imgpadding_in: int, outflow: np.ndarray, initflow: Optional[np.ndarray],
                 width_in: int, height_in: int, sc_f_in: int, sc_l_in: int, max_iter_in: int, min_iter_in: int,
                 dp_thresh_in: float, dr_thresh_in: float, res_thresh_in: float, p_samp_s_in: int, patove_in: float,
                 usefbcon_in: bool, costfct_in: int, noc_in: int, patnorm_in: int, usetvref_in: bool,
                 tv_alpha_in: float, tv_gamma_in: float, tv_delta_in: float, tv_innerit_in: int,
                 tv_solverit_in: int, tv_sor_in: float, verbosity_in: int, *, mode: int = MODE_OF):
        p = Params(mode=mode, noc=noc_in, sc_f=sc_f_in, sc_l=sc_l_in, max_iter=max_iter_in, min_iter=min_iter_in,
                   dp_thresh=dp_thresh_in, dr_thresh=dr_thresh_in, res_thresh=res_thresh_in, p_samp_s=p_samp_s_in,
                   patove=patove_in, usefbcon=int(bool(usefbcon_in)), costfct=costfct_in, patnorm=patnorm_in,
                   usetvref=int(bool(usetvref_in)), tv_alpha=tv_alpha_in, tv_gamma=tv_gamma_in,
                   tv_delta=tv_delta_in, tv_innerit=tv_innerit_in, tv_solverit=tv_solverit_in, tv_sor=tv_sor_in,
                   verbosity=verbosity_in)
        self.params = p
        if not (isinstance(outflow, np.ndarray) and outflow.dtype == _f32 and outflow.flags.c_contiguous):
            raise TypeError("outflow must be a C-contiguous float32 numpy array (written in place)")
        need = (width_in >> sc_l_in) * (height_in >> sc_l_in) * p.nop
        if outflow.size != need:
            raise ValueError(f"outflow has {outflow.size} elements, expected {need}")
        arrays = [_ptr_list(x) for x in (im_ao_in, im_ao_dx_in, im_ao_dy_in, im_bo_in, im_bo_dx_in, im_bo_dy_in)]
        init = None if initflow is None else np.ascontiguousarray(initflow, _f32)
        rc = lib().ofdis_oflow_compute(*[a[0] for a in arrays], imgpadding_in, outflow.ctypes.data,
                                       None if init is None else init.ctypes.data, width_in, height_in, C.byref(p))
        check(rc, "OFClass")


class Context:
    """One MI355X: batched u8 frame pairs -> full-resolution flow (``ofdis_run_batch_u8``)."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        check(lib().ofdis_context_create(device, C.byref(h)), f"ofdis_context_create(device={device})")
        self._h = h
        self.device = device
        self._keep = []

    def close(self):
        if getattr(self, "_h", None):
            lib().ofdis_context_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run_ptr(self, a_ptr: int, b_ptr: int, n: int, width: int, height: int, p: Params, out_ptr: int,
                stream: int = 0, init_ptr: int = 0) -> None:
        """Device pointers in, device pointer out; asynchronous on `stream` (hipStream_t handle).
        init_ptr: optional device float [n, h, w, nop] initial flow (ofdis_run_batch_u8_init)."""
        check(lib().ofdis_run_batch_u8_init(self._h, a_ptr, b_ptr, init_ptr or None, n, width, height, C.byref(p),
                                            out_ptr, stream or None), "ofdis_run_batch_u8_init")

    def run(self, a, b, p: Params, out=None, init=None):
        """torch.uint8 CUDA tensors [n, h, w] or [n, h, w, noc] -> torch.float32 [n, h, w, nop].
        init: optional float32 CUDA tensor [n, h, w, nop], the initial flow at full resolution."""
        import torch
        if a.dim() == 3:
            a, b = a.unsqueeze(-1), b.unsqueeze(-1)
        n, h, w, noc = a.shape
        if noc != p.noc or a.dtype != torch.uint8 or not (a.is_cuda and b.is_cuda):
            raise ValueError("expected uint8 CUDA tensors with noc channels")
        a, b = a.contiguous(), b.contiguous()
        if out is None:
            out = torch.empty((n, h, w, p.nop), dtype=torch.float32, device=a.device)
        stream = torch.cuda.current_stream(a.device).cuda_stream
        if init is not None:
            if tuple(init.shape) != (n, h, w, p.nop) or init.dtype != torch.float32 or not init.is_cuda:
                raise ValueError("init must be a float32 CUDA tensor [n, h, w, nop]")
            init = init.contiguous()
        # stream 0 is torch's default (the legacy NULL stream): the C-ABI orders the call after the work queued
        # there (e.g. the copy kernels of .contiguous() above) and that stream's later work after the call
        self.run_ptr(a.data_ptr(), b.data_ptr(), n, w, h, p, out.data_ptr(), stream,
                     init.data_ptr() if init is not None else 0)
        return out

    def run_host(self, a: np.ndarray, b: np.ndarray, p: Params, init: Optional[np.ndarray] = None) -> np.ndarray:
        """numpy u8 [n,h,w,noc] (or a single [h,w,noc] pair) -> numpy float32 flow; synchronous.
        init: optional initial flow at full resolution, [n,h,w,nop] (or [h,w,nop] for a single pair)."""
        single = a.ndim == 3
        a4 = np.ascontiguousarray(a[None] if single else a, np.uint8)
        b4 = np.ascontiguousarray(b[None] if single else b, np.uint8)
        n, h, w = a4.shape[:3]
        out = np.empty((n, h, w, p.nop), _f32)
        i4 = None
        if init is not None:
            i4 = np.ascontiguousarray(init, _f32).reshape(n, h, w, p.nop)
        check(lib().ofdis_run_batch_u8_init_host(self._h, a4.ctypes.data, b4.ctypes.data,
                                                 None if i4 is None else i4.ctypes.data, n, w, h, C.byref(p),
                                                 out.ctypes.data), "ofdis_run_batch_u8_init_host")
        return out[0] if single else out

    def pyramid_host(self, img: np.ndarray, p: Params, imgpadding: Optional[int] = None):
        """Device pyramid of one u8 image -> {scale: (img, dx, dy)} padded float arrays."""
        h, w = img.shape[:2]
        pad = p.p_samp_s if imgpadding is None else imgpadding
        d = 1 << p.sc_f
        wp, hp = w + ((d - w % d) % d), h + ((d - h % d) % d)
        lev = {s: tuple(np.zeros(((hp >> s) + 2 * pad, (wp >> s) + 2 * pad, p.noc), _f32) for _ in range(3))
               for s in range(p.sc_l, p.sc_f + 1)}
        ptrs = []
        for k in range(3):
            arr = (C.c_void_p * 32)()
            for s, v in lev.items():
                arr[s] = v[k].ctypes.data
            ptrs.append(arr)
        img = np.ascontiguousarray(img, np.uint8)
        check(lib().ofdis_pyramid_u8_host(self._h, img.ctypes.data, w, h, C.byref(p), pad, *ptrs), "pyramid")
        return lev

    def set_capture(self, dis: Optional[dict], tv: Optional[dict], nscales: int = 32):
        """Capture frame 0's flow after aggregation / after TV per scale into the given arrays."""
        d = (C.c_void_p * nscales)()
        t = (C.c_void_p * nscales)()
        self._keep = []
        for src, dst in ((dis or {}, d), (tv or {}, t)):
            for s, a in src.items():
                assert a.dtype == _f32 and a.flags.c_contiguous
                dst[s] = a.ctypes.data
                self._keep.append(a)
        check(lib().ofdis_context_set_stage_capture(self._h, d, t, nscales), "capture")

    def set_option(self, key: str, value: int):
        check(lib().ofdis_context_set_option(self._h, key.encode(), int(value)), f"option {key}")

    def enable_kernel_timing(self, on: bool = True):
        check(lib().ofdis_context_enable_kernel_timing(self._h, int(on)), "timing")

    def kernel_time(self, name: str):
        ms, cnt = C.c_double(), C.c_long()
        check(lib().ofdis_context_kernel_time(self._h, name.encode(), C.byref(ms), C.byref(cnt)), "kernel_time")
        return ms.value, cnt.value


def kernel_names():
    return lib().ofdis_kernel_names().decode().split(",")


def max_frames_per_launch(p: Params, width: int, height: int) -> int:
    """Frames one launch of the refinement kernels takes at this size (32-bit plane-group offsets)."""
    v = C.c_int()
    check(lib().ofdis_max_frames_per_launch(C.byref(p), width, height, C.byref(v)), "max_frames_per_launch")
    return v.value


def algorithmic_bytes(p: Params, width: int, height: int, kernel: str) -> float:
    v = C.c_double()
    check(lib().ofdis_algorithmic_bytes(C.byref(p), width, height, kernel.encode(), C.byref(v)), "bytes")
    return v.value


__all__ = ["OFClass", "Context", "Params", "oppoint", "params_from_strings", "validate", "synth_pair", "synth_shift_pair",
           "write_flo", "write_pfm", "read_flo", "read_image", "auto_first_scale", "kernel_names", "algorithmic_bytes",
           "max_frames_per_launch",
           "MODE_OF", "MODE_DE"]
