"""Single-pair (and small-batch) calls on the device, for rocprofv3 kernel traces of the latency regime.

    python tools/latency_calls.py [--config B] [--pairs 1] [--reps 20] [--option sor_mode=1 ...]

Prints the median wall time per call (device-resident input and output, synchronised per call)."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--noc", type=int, default=1)
    ap.add_argument("--mode", type=int, default=1)
    ap.add_argument("--op", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=1)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--option", action="append", default=[])
    a = ap.parse_args()
    import torch
    import of_dis_amd as od
    ctx = od.Context(0)
    for o in a.option:
        k, v = o.split("=")
        ctx.set_option(k, int(v))
    W, H, n = a.width, a.height, a.pairs
    pairs = [od.synth_pair(W, H, a.noc, f, a.mode) for f in range(min(n, 8))]
    A = torch.from_numpy(np.stack([pairs[f % len(pairs)][0] for f in range(n)])).cuda()
    B = torch.from_numpy(np.stack([pairs[f % len(pairs)][1] for f in range(n)])).cuda()
    p = od.oppoint(a.op, W, a.mode, a.noc)
    out = torch.empty((n, H, W, 2 if a.mode == 1 else 1), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        ctx.run_ptr(A.data_ptr(), B.data_ptr(), n, W, H, p, out.data_ptr(), s)
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        ctx.run_ptr(A.data_ptr(), B.data_ptr(), n, W, H, p, out.data_ptr(), s)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    print(f"{W}x{H} op{a.op} noc{a.noc} mode{a.mode} pairs {n} options {a.option}: median {np.median(ts) * 1e3:.3f} ms "
          f"min {min(ts) * 1e3:.3f} ms per call")
    ctx.close()


if __name__ == "__main__":
    main()
