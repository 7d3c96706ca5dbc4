#!/usr/bin/env python3
"""Headline benchmark: BASELINE.json metric "MPix/s (and frames/sec) 1080p op-point-2; avg EPE vs CPU ref".

Default workload (BASELINE configs[1], "B"): run_OF_INT 1920x1080 grayscale, operating point 2 (patch 8,
overlap 0.4, TV on), batches of synthetic frame pairs resident in HBM.  One step = the whole hot path
(pad + pyramid + DIS + aggregation + TV + upsample + crop) over one batch of `--batch` pairs per GPU.
`--config A|C|D|E` runs the other BASELINE configs (640x480 op2; 1080p RGB op3 with the L1 cost; B at
32 pairs per GPU = 256 over 8 GPUs; 4K stereo depth op4 with 10 TV outer iterations).
N > 1: one process per GPU (torch.distributed.run); frames are sharded, no data-path collective; the
only collectives are the barrier and the max-over-ranks of the elapsed time (RCCL, control traffic).

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md

# BASELINE.json configs -> (binary, width, height, noc, mode, oppoint, explicit 20 parameters or None, batch)
CONFIGS = {
    "A": ("run_OF_INT", 640, 480, 1, 1, 2, None, 1024),
    "B": ("run_OF_INT", 1920, 1080, 1, 1, 2, None, 1024),
    # op-point 3 as the config text states it ("finer scale, L1 cost"): op3 values with costfct = 1
    "C": ("run_OF_RGB", 1920, 1080, 3, 1, 3, "6 2 16 16 0.05 0.95 0 12 0.75 0 1 1 1 10 10 5 1 3 1.6 2", 64),
    "D": ("run_OF_INT", 1920, 1080, 1, 1, 2, None, 32),
    # op-point 4 values with tv_innerit = 10
    "E": ("run_DE_INT", 3840, 2160, 1, 2, 4, "7 2 128 128 0.05 0.95 0 12 0.75 0 1 0 1 10 10 5 10 3 1.6 2", 256),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="B", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="frame pairs per GPU per step (0 = the config's)")
    ap.add_argument("--distinct", type=int, default=8, help="distinct synthetic pairs tiled over the batch")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--streams", type=int, default=0,
                    help="HIP streams the batch's chunks round-robin over (0 = the library's auto: 2 from 512 pairs)")
    ap.add_argument("--chunk", type=int, default=0, help="frames per chunk (0 = the batch split over the streams)")
    ap.add_argument("--tv-fused", type=int, default=-1, help="1/0: force the fused TV level kernel on/off")
    ap.add_argument("--option", action="append", default=[], help="context option key=value (A/B runs)")
    ap.add_argument("--host-io", action="store_true",
                    help="also time the host-buffer entry point (PCIe-inclusive rate, reported separately)")
    ap.add_argument("--no-kernel-timing", action="store_true")
    return ap.parse_args()


def config_tag(cfg, B):
    """Workload key of profiles/traffic.json (tools/pmc_traffic.py)."""
    return f"{cfg[1]}x{cfg[2]}:op{cfg[5]}:b{B}" + ("" if cfg[3] == 1 else ":rgb")


def kernel_roofline(od, p, W, H, B, per_launch, cfg, steps, kernels, name):
    """HBM roofline of one kernel: algorithmic bytes per launch (SURVEY §8(d) byte model x the frames one
    launch processes) / its average launch time (HIP events on the launch stream); traffic = HBM bytes per
    launch from the rocprofv3 PMC passes (profiles/traffic.json, tools/pmc_traffic.py, keyed by the pairs
    per launch) when recorded."""
    k = kernels[name]
    bytes_frame = od.algorithmic_bytes(p, W, H, name)
    launches_per_step = k["launches"] / steps
    bytes_launch = bytes_frame * B / launches_per_step
    achieved = bytes_launch / (k["avg_us"] * 1e-6) / 1e9
    traffic = None
    tf = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tf):
        try:
            ent = json.load(open(tf)).get(f"{name}:{config_tag(cfg, per_launch)}")
            traffic = None if ent is None else round(ent["bytes_per_launch"])
        except Exception:
            traffic = None
    return {"kernel": name, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "algorithmic_bytes_per_launch": bytes_launch, "avg_launch_us": round(k["avg_us"], 2)}


def params_of(mod, cfg):
    """The config's parameters through a module's parameter API (of_dis_amd or the oracle mirror)."""
    _, W, H, noc, mode, op, explicit, _ = cfg
    if explicit:
        return mod.params_from_strings(explicit.split(), mode, noc)
    return mod.oppoint(op, W, mode, noc)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)

    import of_dis_amd as od
    from of_dis_amd import distributed as odd

    cfg = CONFIGS[args.config]
    binary, W, H, noc, mode, op, explicit, default_batch = cfg
    B = args.batch or default_batch
    p = params_of(od, cfg)
    p.verbosity = 0
    nop = p.nop
    ctx = od.Context(dev.index)
    ctx.set_option("streams", args.streams)
    ctx.set_option("chunk", args.chunk)
    # the library's chunking (ofdis_runtime.cpp stream_count): streams 0 = 2 from 512 pairs, else 1
    streams_eff = args.streams or (2 if B >= 512 else 1)
    chunk_eff = min(B, args.chunk or -(-B // streams_eff))
    if args.tv_fused >= 0:
        ctx.set_option("tv_fused", args.tv_fused)
    for kv in args.option:
        k, v = kv.split("=")
        ctx.set_option(k, int(v))

    # synthetic inputs, resident in HBM before timing: distinct pairs per rank, tiled over the batch
    first = odd.shard_range(B * world, rank, world)[0]
    nd = max(1, min(args.distinct, B))
    pairs = [od.synth_pair(W, H, noc, first + k, mode) for k in range(nd)]
    a = torch.empty((B, H, W, noc), dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    for i in range(B):
        a[i].copy_(torch.from_numpy(pairs[i % nd][0]))
        b[i].copy_(torch.from_numpy(pairs[i % nd][1]))
    out = torch.empty((B, H, W, nop), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step():
        ctx.run_ptr(a.data_ptr(), b.data_ptr(), B, W, H, p, out.data_ptr(), stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    elapsed = odd.max_over_ranks(elapsed, dev) if world > 1 else elapsed

    frames = B * world * args.steps
    mpix = W * H * frames / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3

    # ---- per-kernel device time with HIP events on the launch stream (a second pass of the same steps,
    # chunks serialised on one stream so that every kernel is timed alone on the GPU)
    kernels = {}
    roofline = None
    roofline_sor = None
    if not args.no_kernel_timing:
        # the same launches (chunk_eff pairs each), serialised on one stream: each kernel timed alone
        # (HIP events bracketing launches of two concurrent streams do not measure the kernels: they
        # measured 2x rocprofv3's kernel durations)
        ctx.set_option("streams", 1)
        ctx.set_option("chunk", chunk_eff)
        ctx.enable_kernel_timing(True)
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        for k in od.kernel_names():
            ms, cnt = ctx.kernel_time(k)
            if cnt:
                kernels[k] = {"total_ms": ms, "launches": cnt, "avg_us": ms / cnt * 1e3}
        ctx.enable_kernel_timing(False)
        ctx.set_option("streams", args.streams)
        ctx.set_option("chunk", args.chunk)
        dom = max(kernels, key=lambda k: kernels[k]["total_ms"])
        roofline = kernel_roofline(od, p, W, H, B, chunk_eff, cfg, args.steps, kernels, dom)
        if dom != "tv_sor" and "tv_sor" in kernels:  # the north-star kernel, reported beside the dominant one
            roofline_sor = kernel_roofline(od, p, W, H, B, chunk_eff, cfg, args.steps, kernels, "tv_sor")

    # ---- host-buffer entry point (PCIe-inclusive; never the headline value)
    host_io = None
    if args.host_io and rank == 0:
        ha = np.stack([pairs[i % nd][0] for i in range(B)])
        hb = np.stack([pairs[i % nd][1] for i in range(B)])
        ctx.run_host(ha, hb, p)
        reps = max(1, args.steps // 2)
        t0h = time.perf_counter()
        for _ in range(reps):
            ctx.run_host(ha, hb, p)
        th = time.perf_counter() - t0h
        host_io = {"value": round(W * H * B * reps / th / 1e6, 2), "unit": "MPix/s",
                   "what": "ofdis_run_batch_u8_host: u8 frames H2D + whole path + f32 flow D2H, pageable host memory"}

    # ---- CPU baseline (rank 0, N=1 only): the oracle port, single thread, bounded sample
    cpu = None
    parity = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        from oracle import pyoracle as O
        q = params_of(O, cfg) if hasattr(O, "params_from_strings") or not explicit else None
        if q is None:  # the oracle's mirror of ofdis_params: same fields, same meaning
            q = O.Params()
            for k, v in p.as_dict().items():
                setattr(q, k, v)
        done, t0c, max_epe, bitexact = 0, time.perf_counter(), 0.0, 0
        gpu_out = out.cpu().numpy()
        while True:
            k = done % nd
            ref = O.run_u8(pairs[k][0], pairs[k][1], q)
            done += 1
            if done <= nd:  # compare against the GPU output of the same pair
                g = gpu_out[k]
                epe = float(np.sqrt(((g - ref) ** 2).sum(-1)).mean())
                max_epe = max(max_epe, epe)
                bitexact += int(np.array_equal(g.view(np.uint32), ref.view(np.uint32)))
            if time.perf_counter() - t0c > args.cpu_seconds:
                break
        tc = time.perf_counter() - t0c
        cpu = {"value": round(W * H * done / tc / 1e6, 3), "unit": "MPix/s", "cores": 1, "kind": "port",
               "frames_per_sec": round(done / tc, 3),
               "sample": f"{done} synthetic {W}x{H} {binary} pairs (config {args.config}), oracle/ofdis_oracle.c "
                         f"single thread (pad+pyramid+OFClass+upsample), {tc:.1f} s"}
        parity = {"avg_epe_vs_cpu_ref_max": max_epe, "bitexact_frames": bitexact, "compared_frames": min(done, nd)}

    if rank == 0:
        line = {
            "metric": "MPix/s (and frames/sec) 1080p op-point-2; avg EPE vs CPU ref",
            "value": round(mpix, 2), "unit": "MPix/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "frames_per_sec": round(frames / elapsed, 2),
            "config": {"workload": f"{binary} {W}x{H} op-point {op}" + (f" ({explicit})" if explicit else "")
                                   + f", {B} pairs/GPU/step", "name": args.config,
                       "width": W, "height": H, "channels": noc, "oppoint": op, "batch_per_gpu": B,
                       "streams": streams_eff, "pairs_per_launch": chunk_eff, "tv_fused": args.tv_fused,
                       "options": args.option,
                       "parallelism": f"frame-sharded x{world}"},
            "roofline": roofline, "roofline_tv_sor": roofline_sor, "cpu_baseline": cpu, "parity": parity,
            "host_io": host_io, "kernels": kernels,
        }
        if cpu:
            line["speedup_vs_cpu_1core"] = round(mpix / cpu["value"], 1)
        print(json.dumps(line))
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
