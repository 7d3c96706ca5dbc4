"""Per-process wall time of the drop-in CLIs, the way the reference is used: one frame pair per process
(run_dense.cpp:186-431; its own timers at :315-353 and :424-429).

For each case: synthetic PNG pair written to a scratch directory, the CLI run `--reps` times as a fresh process,
its wall time measured around the process, its stdout TIME lines (the reference's timers) parsed, and its stderr
breakdown (OFDIS_CLI_TIMING=1: image load, context create = HIP runtime init + code-object load, the call = H2D +
path + D2H, context destroy, file write) recorded.  Beside it, the CPU port (oracle/ofdis_oracle.c, one thread) on
the same decoded pair in this process: the reference's CPU path has no GPU start-up to pay.

    python tools/cli_wall.py --out profiles/r06/cli_wall.json [--reps 5] [--cases B_OF_INT,...]
"""
import argparse
import json
import os
import re
import struct
import subprocess
import sys
import tempfile
import time
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = {  # name: (binary, width, height, noc, mode)
    "1080p_OF_INT": ("run_OF_INT", 1920, 1080, 1, 1),
    "1080p_OF_RGB": ("run_OF_RGB", 1920, 1080, 3, 1),
    "1080p_DE_INT": ("run_DE_INT", 1920, 1080, 1, 2),
    "4K_OF_INT": ("run_OF_INT", 3840, 2160, 1, 1),
    "4K_DE_INT": ("run_DE_INT", 3840, 2160, 1, 2),
}


def write_png(path, img):
    """Minimal PNG: 8-bit gray (h, w, 1) or BGR (h, w, 3) stored as RGB, filter 0, one IDAT."""
    h, w, c = img.shape
    px = img[..., ::-1] if c == 3 else img
    raw = b"".join(b"\x00" + px[y].tobytes() for y in range(h))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    ihdr = struct.pack(">IIBBBBB", w, h, 8, 2 if c == 3 else 0, 0, 0, 0)
    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + chunk(b"IDAT", zlib.compress(raw, 6)) +
                chunk(b"IEND", b""))


def parse(out, err):
    times = {}
    for line in out.splitlines():
        m = re.match(r"TIME \((.*?)\s*\) \(ms\): ([0-9.eE+-]+)", line)
        if m:
            times[m.group(1).strip()] = float(m.group(2))
    scales = [line for line in out.splitlines() if line.startswith("TIME (Sc:")]
    cli = {}
    m = re.search(r"cli_ms (.*)", err)
    if m:
        f = m.group(1).split()
        cli = {f[i]: float(f[i + 1]) for i in range(0, len(f) - 1, 2)}
    return times, scales, cli


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cases", default=",".join(CASES))
    ap.add_argument("--cpu", action="store_true", help="also time the CPU port on each pair")
    a = ap.parse_args()
    import of_dis_amd as od
    bindir = os.path.join(ROOT, "of_dis_amd", "bin")
    res = {"what": "one pair per process (the reference's usage): wall around the process, the reference's stdout "
                   "timers, and the stderr breakdown (OFDIS_CLI_TIMING=1); cpu_port_ms: the oracle port, 1 thread, "
                   "same decoded pair, in-process (no start-up)", "reps": a.reps, "cases": {}}
    tmp = tempfile.mkdtemp(prefix="cliwall_")
    for name in a.cases.split(","):
        exe, W, H, noc, mode = CASES[name]
        im_a, im_b = od.synth_pair(W, H, noc, 0, mode)
        pa, pb, po = (os.path.join(tmp, f"{name}_{x}") for x in ("a.png", "b.png", "out.flo" if mode == 1 else "out.pfm"))
        write_png(pa, im_a)
        write_png(pb, im_b)
        env = dict(os.environ, OFDIS_CLI_TIMING="1")
        runs = []
        for r in range(a.reps):
            t0 = time.perf_counter()
            p = subprocess.run([os.path.join(bindir, exe), pa, pb, po], capture_output=True, text=True, env=env,
                               timeout=120)
            wall = (time.perf_counter() - t0) * 1e3
            if p.returncode != 0:
                raise RuntimeError(f"{name}: rc {p.returncode}: {p.stderr[-500:]}")
            times, scales, cli = parse(p.stdout, p.stderr)
            runs.append({"wall_ms": round(wall, 3), "timers": times, "cli_ms": cli, "scales": scales})
            print(f"{name} rep {r}: wall {wall:.1f} ms  {cli}  O.Flow {times.get('O.Flow Run-Time')}", flush=True)
        med = lambda xs: float(np.median(xs))  # noqa: E731
        entry = {"binary": exe, "width": W, "height": H, "noc": noc, "mode": mode,
                 "wall_ms_median": round(med([r["wall_ms"] for r in runs]), 3),
                 "breakdown_ms_median": {k: round(med([r["cli_ms"][k] for r in runs]), 3)
                                         for k in runs[0]["cli_ms"]},
                 "reference_timers_ms_median": {k: round(med([r["timers"][k] for r in runs if k in r["timers"]]), 4)
                                                for k in runs[0]["timers"]},
                 "first_run": runs[0], "runs": runs}
        if a.cpu:
            from oracle import pyoracle as O
            q = O.oppoint(2, W, mode, noc)
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                O.run_u8(im_a, im_b, q)
                ts.append((time.perf_counter() - t0) * 1e3)
            entry["cpu_port_ms"] = round(min(ts), 3)
        res["cases"][name] = entry
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: {"wall": v["wall_ms_median"], **v["breakdown_ms_median"], "cpu": v.get("cpu_port_ms")}
                      for k, v in res["cases"].items()}, indent=1))


if __name__ == "__main__":
    main()
