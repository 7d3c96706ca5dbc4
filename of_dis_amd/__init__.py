"""of_dis_amd -- MI355X-native (gfx950 HIP) DIS optical flow / stereo depth hot path.

Drop-in for lordnn/OF_DIS's OFClass / run_dense pipeline.  The compute lives in libofdis.so
(hand-written HIP kernels + C-ABI, include/ofdis.h); this package is a thin host-side mirror.
"""
from ._lib import MODE_DE, MODE_OF, OfdisError, Params, build, lib  # noqa: F401
from .ofclass import (Context, OFClass, algorithmic_bytes, auto_first_scale, kernel_names,  # noqa: F401
                      max_frames_per_launch, oppoint, params_from_strings, read_flo, read_image, synth_pair, synth_shift_pair, validate,
                      write_flo, write_pfm)

__version__ = "0.1.0"
