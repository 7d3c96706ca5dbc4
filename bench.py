#!/usr/bin/env python3
"""Headline benchmark: BASELINE.json metric "MPix/s (and frames/sec) 1080p op-point-2; avg EPE vs CPU ref".

Workload (BASELINE configs[1]): run_OF_INT 1920x1080 grayscale, operating point 2 (patch 8, overlap 0.4,
TV on), batches of synthetic frame pairs resident in HBM.  One step = the whole hot path
(pad + pyramid + DIS + aggregation + TV + upsample + crop) over one batch of `--batch` pairs per GPU.
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="frame pairs per GPU per step")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--oppoint", type=int, default=2)
    ap.add_argument("--distinct", type=int, default=8, help="distinct synthetic pairs tiled over the batch")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--streams", type=int, default=1, help="HIP streams the batch's chunks round-robin over")
    ap.add_argument("--chunk", type=int, default=0, help="frames per chunk (0 = whole batch in one chunk)")
    ap.add_argument("--tv-fused", type=int, default=-1, help="1/0: force the fused TV level kernel on/off")
    ap.add_argument("--no-kernel-timing", action="store_true")
    return ap.parse_args()


def kernel_roofline(od, p, W, H, B, args, kernels, name):
    """HBM roofline of one kernel: algorithmic bytes per launch (SURVEY §8(d) byte model x the frames one
    launch processes) / its average launch time (HIP events on the launch stream); traffic = HBM bytes per
    launch from the rocprofv3 PMC passes (profiles/traffic.json, tools/pmc_traffic.py) when recorded."""
    k = kernels[name]
    bytes_frame = od.algorithmic_bytes(p, W, H, name)
    launches_per_step = k["launches"] / args.steps
    bytes_launch = bytes_frame * B / launches_per_step
    achieved = bytes_launch / (k["avg_us"] * 1e-6) / 1e9
    traffic = None
    tf = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tf):
        try:
            ent = json.load(open(tf)).get(f"{name}:{W}x{H}:op{args.oppoint}:b{B}")
            traffic = None if ent is None else round(ent["bytes_per_launch"])
        except Exception:
            traffic = None
    return {"kernel": name, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "algorithmic_bytes_per_launch": bytes_launch, "avg_launch_us": round(k["avg_us"], 2)}


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

    W, H, B = args.width, args.height, args.batch
    p = od.oppoint(args.oppoint, W, od.MODE_OF, 1)
    p.verbosity = 0
    ctx = od.Context(dev.index)
    ctx.set_option("streams", args.streams)
    ctx.set_option("chunk", args.chunk)
    if args.tv_fused >= 0:
        ctx.set_option("tv_fused", args.tv_fused)

    # synthetic inputs, resident in HBM before timing: distinct pairs per rank, tiled over the batch
    first = odd.shard_range(B * world, rank, world)[0]
    nd = max(1, min(args.distinct, B))
    pairs = [od.synth_pair(W, H, 1, first + k, od.MODE_OF) for k in range(nd)]
    a = torch.empty((B, H, W), dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    for i in range(B):
        a[i].copy_(torch.from_numpy(pairs[i % nd][0][..., 0]))
        b[i].copy_(torch.from_numpy(pairs[i % nd][1][..., 0]))
    out = torch.empty((B, H, W, 2), dtype=torch.float32, device=dev)
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
        ctx.set_option("streams", 1)
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
        dom = max(kernels, key=lambda k: kernels[k]["total_ms"])
        roofline = kernel_roofline(od, p, W, H, B, args, kernels, dom)
        if dom != "tv_sor" and "tv_sor" in kernels:  # the north-star kernel, reported beside the dominant one
            roofline_sor = kernel_roofline(od, p, W, H, B, args, kernels, "tv_sor")

    # ---- CPU baseline (rank 0, N=1 only): the oracle port, single thread, bounded sample
    cpu = None
    parity = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        from oracle import pyoracle as O
        q = O.oppoint(args.oppoint, W, 1, 1)
        O.run_u8(pairs[0][0], pairs[0][1], q)  # warm (allocations)
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
               "sample": f"{done} synthetic 1920x1080 op2 pairs, oracle/ofdis_oracle.c single thread "
                         f"(pad+pyramid+OFClass+upsample), {tc:.1f} s"}
        parity = {"avg_epe_vs_cpu_ref_max": max_epe, "bitexact_frames": bitexact, "compared_frames": min(done, nd)}

    if rank == 0:
        line = {
            "metric": "MPix/s (and frames/sec) 1080p op-point-2; avg EPE vs CPU ref",
            "value": round(mpix, 2), "unit": "MPix/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "frames_per_sec": round(frames / elapsed, 2),
            "config": {"workload": f"run_OF_INT {W}x{H} gray op-point {args.oppoint}, {B} pairs/GPU/step",
                       "width": W, "height": H, "oppoint": args.oppoint, "batch_per_gpu": B,
                       "streams": args.streams, "chunk": args.chunk, "tv_fused": args.tv_fused,
                       "parallelism": f"frame-sharded x{world}"},
            "roofline": roofline, "roofline_tv_sor": roofline_sor, "cpu_baseline": cpu, "parity": parity, "kernels": kernels,
        }
        if cpu:
            line["speedup_vs_cpu_1core"] = round(mpix / cpu["value"], 1)
        print(json.dumps(line))
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
