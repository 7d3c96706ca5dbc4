#!/usr/bin/env python3
"""tools/capture_repro.hip's probe inside a process that imported torch (its bundled HIP runtime serves the
process).  Usage: python tools/capture_repro_torch.py MODE [chunks]"""
import ctypes
import os
import sys

import torch  # noqa: F401  (loads torch/lib/libamdhip64.so first)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "bin", "libcapture_repro.so"))
print("hip runtime:", sorted({l.split()[-1] for l in open("/proc/self/maps") if "amdhip" in l}), flush=True)
sys.exit(lib.capture_repro(int(sys.argv[1]) if len(sys.argv) > 1 else 2, int(sys.argv[2]) if len(sys.argv) > 2 else 3))
