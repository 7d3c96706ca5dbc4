"""ctypes bindings to of_dis_amd/libofdis.so (the C-ABI declared in include/ofdis.h).

The shared library is the product: HIP kernels for gfx950 plus the host runtime.  There is no CPU
fallback -- if the library is missing or no gfx950 device is visible, calls fail loudly.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# OFDIS_LIB: another build of the same library (A/B timing of kernel variants, tools/ab_session.sh)
LIB_PATH = os.environ.get("OFDIS_LIB") or os.path.join(PKG_DIR, "libofdis.so")
CSRC = os.path.join(PKG_DIR, "csrc")

OK = 0
ERR_INVALID_ARGUMENT = 1
ERR_UNSUPPORTED = 2
ERR_OUT_OF_MEMORY = 3
ERR_DEVICE = 4
ERR_NO_DEVICE = 5
ERR_IO = 6

MODE_OF = 1
MODE_DE = 2


class OfdisError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = lib().ofdis_status_string(code).decode() if _lib is not None else str(code)
        super().__init__(f"{what}: {msg} (status {code})" if what else f"{msg} (status {code})")


class Params(C.Structure):
    """ofdis_params (include/ofdis.h), mirroring OFC::optparam's explicit fields (oflow.h:45-66)."""

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

    def copy(self, **kw):
        q = Params()
        C.memmove(C.byref(q), C.byref(self), C.sizeof(Params))
        for k, v in kw.items():
            setattr(q, k, v)
        return q

    @property
    def nop(self) -> int:
        return 2 if self.mode == MODE_OF else 1

    def __repr__(self):
        return "Params(" + ", ".join(f"{k}={v!r}" for k, v in self.as_dict().items()) + ")"


def build(verbose: bool = False) -> None:
    """Compile libofdis.so (+ CLI binaries) for gfx950 with hipcc, in-tree."""
    jobs = os.environ.get("MAX_JOBS", "4")
    subprocess.run(["make", "-s", "-j", str(jobs), "-C", CSRC], check=True,
                   stdout=None if verbose else subprocess.DEVNULL)


_lib = None


def lib():
    """Load libofdis.so; raises if it has not been built (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    try:  # load torch's HIP runtime first: libofdis then binds to it (same SONAME) -> one runtime per process
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'` "
                          "or `make -C of_dis_amd/csrc` (hipcc, gfx950)")
    L = C.CDLL(LIB_PATH)
    vp, i, f = C.c_void_p, C.c_int, C.c_float
    P = C.POINTER(Params)
    sig = {
        "ofdis_abi_version": ([], i),
        "ofdis_status_string": ([i], C.c_char_p),
        "ofdis_auto_first_scale": ([i, i, i], i),
        "ofdis_params_oppoint": ([P, i, i, i, i], i),
        "ofdis_params_from_strings": ([P, i, C.POINTER(C.c_char_p), i, i], i),
        "ofdis_params_validate": ([P, i, i, i], i),
        "ofdis_oflow_compute": ([vp] * 6 + [i, vp, vp, i, i, P], i),
        "ofdis_context_create": ([i, C.POINTER(vp)], i),
        "ofdis_context_destroy": ([vp], None),
        "ofdis_run_batch_u8": ([vp, vp, vp, i, i, i, P, vp, vp], i),
        "ofdis_run_batch_u8_host": ([vp, vp, vp, i, i, i, P, vp], i),
        "ofdis_run_batch_u8_init": ([vp, vp, vp, vp, i, i, i, P, vp, vp], i),
        "ofdis_run_batch_u8_init_host": ([vp, vp, vp, vp, i, i, i, P, vp], i),
        "ofdis_pyramid_u8_host": ([vp, vp, i, i, P, i, vp, vp, vp], i),
        "ofdis_context_set_stage_capture": ([vp, vp, vp, i], i),
        "ofdis_context_set_option": ([vp, C.c_char_p, i], i),
        "ofdis_context_enable_kernel_timing": ([vp, i], i),
        "ofdis_context_kernel_time": ([vp, C.c_char_p, C.POINTER(C.c_double), C.POINTER(C.c_long)], i),
        "ofdis_kernel_names": ([], C.c_char_p),
        "ofdis_algorithmic_bytes": ([P, i, i, C.c_char_p, C.POINTER(C.c_double)], i),
        "ofdis_max_frames_per_launch": ([P, i, i, C.POINTER(i)], i),
        "ofdis_write_flo": ([C.c_char_p, vp, i, i, i], i),
        "ofdis_write_pfm": ([C.c_char_p, vp, i, i], i),
        "ofdis_read_flo": ([C.c_char_p, vp, C.POINTER(i), C.POINTER(i), i], i),
        "ofdis_read_pnm": ([C.c_char_p, vp, C.POINTER(i), C.POINTER(i), C.POINTER(i), C.c_size_t], i),
        "ofdis_read_image": ([C.c_char_p, vp, C.POINTER(i), C.POINTER(i), i, C.c_size_t], i),
        "ofdis_synth_pair_u8": ([vp, vp, i, i, i, i, i], i),
        "ofdis_synth_shift_pair_u8": ([vp, vp, i, i, i, i, C.c_float, C.c_float], i),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def check(rc: int, what: str = "") -> None:
    if rc != OK:
        raise OfdisError(rc, what)
