#!/usr/bin/env python3
"""Headline benchmark: BASELINE.json metric "MPix/s (and frames/sec) 1080p op-point-2; avg EPE vs CPU ref".

Default workload (BASELINE configs[1], "B"): run_OF_INT 1920x1080 grayscale, operating point 2 (patch 8,
overlap 0.4, TV on), batches of synthetic frame pairs resident in HBM.  One step = the whole hot path
(pad + pyramid + DIS + aggregation + TV + upsample + crop) over one batch of `--batch` pairs per GPU.
`--config A|C|C2|D|E` runs the other BASELINE configs (640x480 op2; 1080p RGB op3 with the L1 cost / as
op-point 3 defines it (L2); D = a batch of 256 1080p op2 pairs per step sharded over the GPUs (strong
scaling: 256 on one GPU, 32 per GPU on 8); 4K stereo depth op4 with 10 TV outer iterations).

Multi-GPU: `--gpus N` (N > 1) without a torch.distributed environment re-launches this script as N ranks
(`python -m torch.distributed.run --nproc-per-node N`, a child process -- this parent never touches a GPU)
and exits with its status.  Each rank owns a contiguous shard of frames (no data-path collective); the
control collectives are a broadcast of rank 0's parameters, the barrier + max-over-ranks of the timed
region, and a sum of counters (frames, parity, kernel time) -- RCCL on GPU.  `--dry-run` runs the same
rank logic on gloo without a GPU (CPU test of the launcher and the shard bookkeeping).

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md

# BASELINE.json configs -> (binary, width, height, noc, mode, oppoint, explicit 20 parameters or None, batch)
CONFIGS = {
    "A": ("run_OF_INT", 640, 480, 1, 1, 2, None, 2048),  # 1024: 110k, 2048: 113k MPix/s (profiles/r02/sweep6)
    # 4096 pairs per GPU per step = two 2048-pair chunks on two streams.  Round 3 (faster patch and TV kernels),
    # same box, ABAB (profiles/r03/batch): 2048 pairs 291-309k (bimodal: the lanes' phase alignment), 3072 308k,
    # 4096 312-316k MPix/s; round 2's sweep had 2048 best (profiles/r02/sweep3)
    "B": ("run_OF_INT", 1920, 1080, 1, 1, 2, None, 4096),
    # op-point 3 as the config text states it ("finer scale, L1 cost"): op3 values with costfct = 1.
    # 512 pairs = two 256-pair chunks on two streams (64: 6.9k, 128: 7.4k, 256: 7.8k, 512: 8.1k, 1024: 8.2k
    # MPix/s; profiles/r02/ab/ab_batch*)
    "C": ("run_OF_RGB", 1920, 1080, 3, 1, 3, "6 2 16 16 0.05 0.95 0 12 0.75 0 1 1 1 10 10 5 1 3 1.6 2", 512),
    # op-point 3 as run_dense.cpp:248-253 defines it (costfct 0, L2); SURVEY §8(d): report both
    "C2": ("run_OF_RGB", 1920, 1080, 3, 1, 3, None, 512),
    # BASELINE configs[3]: 256 pairs per step in total, sharded over the GPUs (strong scaling, STRONG below)
    "D": ("run_OF_INT", 1920, 1080, 1, 1, 2, None, 256),
    # op-point 4 values with tv_innerit = 10; 512 = two 256-pair chunks on two streams
    # (256: 6.85k, 512: 7.57k, 1024: 7.54k MPix/s; profiles/r02/ab/ab_batch*)
    "E": ("run_DE_INT", 3840, 2160, 1, 2, 4, "7 2 128 128 0.05 0.95 0 12 0.75 0 1 0 1 10 10 5 10 3 1.6 2", 512),
}
METRIC = "MPix/s (and frames/sec) 1080p op-point-2; avg EPE vs CPU ref"
# configs whose batch is the whole job's (sharded over the ranks) rather than each GPU's
STRONG = {"D"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10,
                    help="untimed steps first (the clocks and the caches settle: 3 left the first timed steps of a "
                         "fresh process up to 4 %% slower)")
    ap.add_argument("--config", default="B", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="frame pairs per GPU per step (0 = the config's)")
    ap.add_argument("--total", type=int, default=0,
                    help="frame pairs per step over ALL GPUs, sharded over the ranks (strong scaling; 0 = the "
                         "config's: D 256, the others weak scaling at --batch per GPU)")
    ap.add_argument("--distinct", type=int, default=8, help="distinct synthetic pairs tiled over the batch")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="bounded CPU-baseline sample per leg (1 core, all cores; 0 = skip)")
    ap.add_argument("--streams", type=int, default=0,
                    help="HIP streams the batch's chunks round-robin over (0 = the library's auto: 2 from 256 pairs)")
    ap.add_argument("--chunk", type=int, default=0, help="frames per chunk (0 = the batch split over the streams)")
    ap.add_argument("--option", action="append", default=[], help="context option key=value (A/B runs)")
    ap.add_argument("--host-io", action="store_true",
                    help="also time the host-buffer entry point (PCIe-inclusive rate, reported separately)")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--no-latency", action="store_true", help="skip the single-pair latency leg")
    ap.add_argument("--probe-regions", type=int, default=0,
                    help="diagnostic: time this many extra K-step regions before the reported one (stderr)")
    ap.add_argument("--dry-run", action="store_true", help="rank/shard bookkeeping on gloo, no GPU (CPU test)")
    ap.add_argument("--parity-frames", type=int, default=8,
                    help="distinct timed-pass frames re-checked against the CPU oracle on every rank (their tiles: "
                         "on the device)")
    return ap.parse_args()


def relaunch_as_ranks(args) -> int:
    """`--gpus N` outside a torch.distributed environment: run N ranks as a child torchrun job."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


def config_tag(cfg, B):
    """Workload key of profiles/traffic.json (tools/pmc_traffic.py)."""
    return f"{cfg[1]}x{cfg[2]}:op{cfg[5]}:b{B}" + ("" if cfg[3] == 1 else ":rgb") + (
        ":l1" if cfg[6] and cfg[3] == 3 else "")


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
    out = {"kernel": name, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
           "algorithmic_bytes_per_launch": bytes_launch, "avg_launch_us": round(k["avg_us"], 2)}
    if name == "tv_sor":
        # Three readings of one launch time.  The SURVEY §8(d) unit counts 44 (OF) / 24 (DE)
        # B per pixel PER SWEEP (a streaming sweep-by-sweep model); k_tv_sor_lanes runs all sweeps of a call in one
        # pass and reads each pixel's coefficients once, so that figure is a streaming-equivalent rate that can
        # exceed the peak -- it is not a roofline fraction.  The two roofline fractions: the once-per-launch
        # compulsory bytes (44 / 24 B per pixel, what a sweep-fused kernel must move) and the PMC bytes.
        sweeps = max(1, int(p.tv_solverit))
        comp = bytes_launch / sweeps
        comp_gbs = comp / (k["avg_us"] * 1e-6) / 1e9
        out["model_equiv_frac"] = out.pop("frac")
        out["model_equiv_gbs"] = out.pop("achieved")
        out["achieved"] = round(comp_gbs, 1)
        out["frac"] = out["frac_compulsory"] = round(comp_gbs / HBM_PEAK_GBS, 4)
        out["compulsory_bytes_per_launch"] = comp
        out["frac_counters"] = (None if traffic is None else
                                round(traffic / (k["avg_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4))
        out["counters_vs_compulsory"] = None if traffic is None else round(traffic / comp, 3)
        out["note"] = ("frac = frac_compulsory: 44 (OF) / 24 (DE) B/px once per launch / launch time / 8 TB/s; "
                       "frac_counters: PMC FETCH_SIZE x2 + WRITE_SIZE per launch (profiles/traffic.json) / launch "
                       "time; model_equiv_frac: the SURVEY 8(d) per-sweep unit x sweeps, a streaming-equivalent "
                       "rate of the sweep-fused kernel (may exceed 1, not a roofline fraction)")
    if name == "tv_level":
        # the fused red-black level launch of the latency mode (sor_mode = 1): every inner iteration of a level in one
        # workgroup per frame; bytes = wx, wy and the eight derivative planes in, the flow out, once per level.  Not an
        # HBM-bound kernel: 1 + 2 * solverit workgroup barriers per inner iteration on one CU per frame
        out["limiter"] = ("barrier / VALU latency of one workgroup per frame (latency mode; the later inner "
                          "iterations read the derivative planes from L2)")
    if name == "patch":  # not an HBM-bound kernel: say what bounds it
        out["limiter"] = ("VALU issue: SQ_ACTIVE_INST_VALU x waves/SIMD ~ 0.9-1.2 of SIMD cycles at configs C and E "
                          "(profiles/r02/pmc, profiles/r03/pmc); bytes = compulsory per patch (template, gradients, "
                          "one window, outputs)")
    return out


def params_of(mod, cfg):
    """The config's parameters through a module's parameter API (of_dis_amd or the oracle mirror)."""
    _, W, H, noc, mode, op, explicit, _ = cfg
    if explicit:
        return mod.params_from_strings(explicit.split(), mode, noc)
    return mod.oppoint(op, W, mode, noc)


def oracle_params(O, p):
    q = O.Params()
    for k, v in p.as_dict().items():
        setattr(q, k, v)
    return q


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores() -> int:
    """The host cores this process may use: the box's CPU share (OMP_NUM_THREADS, 16 per GPU on the
    GPU pool) capped by the affinity mask."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(aff, share) if share > 0 else aff)


def cpu_quota():
    """CPUs this process may use by its cgroup quota (cgroup v2 cpu.max), or None when unlimited."""
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if quota == "max" else round(int(quota) / int(period), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(O, q, pairs, W, H, seconds, binary, cfg_name):
    """The oracle port (oracle/ofdis_oracle.c, -O3 -msse4.1 -ffp-contract=off; the reference's default
    build semantics: lexicographic block SOR, no OpenMP) timed over whole pairs (pad + pyramid + OFClass
    + upsample, the reference's verbosity-2 timer scope): one core (with the stage breakdown), one
    single-threaded worker per core of this process's CPU share, and one per host CPU of the node (nproc;
    the cgroup quota is reported beside it -- on a shared box it caps that leg), frame-parallel (ctypes
    releases the GIL inside the oracle)."""
    from concurrent.futures import ThreadPoolExecutor
    nd = len(pairs)
    t0 = time.perf_counter()
    done = 0
    stages = []
    while True:
        stages.append(O.run_u8_stages(pairs[done % nd][0], pairs[done % nd][1], q)[1])
        done += 1
        if time.perf_counter() - t0 > seconds:
            break
    t1 = time.perf_counter() - t0

    def parallel(workers):
        deadline = time.perf_counter() + seconds

        def worker(k):
            n = 0
            while True:
                O.run_u8(pairs[(k + n) % nd][0], pairs[(k + n) % nd][1], q)
                n += 1
                if time.perf_counter() > deadline:
                    return n
        t0 = time.perf_counter()
        with ThreadPoolExecutor(workers) as ex:
            n = sum(ex.map(worker, range(workers)))
        return n, time.perf_counter() - t0

    cores = host_cores()
    done_all, t_all = parallel(cores) if cores > 1 else (0, 0.0)
    node = os.cpu_count() or 1
    quota = cpu_quota()
    # the node leg only where this process may use more CPUs than the all-cores leg: under a cgroup quota of <= cores
    # CPUs, nproc workers time-share the same CPUs (slower than the cores leg, not a node figure -- VERDICT r03)
    node_runs = node > cores and (quota is None or quota > cores)
    done_node, t_node = parallel(node) if node_runs else (0, 0.0)
    fair = None
    ff = os.path.join(ROOT, "profiles", "cpu_fairness.json")
    if os.path.exists(ff):
        try:
            fair = json.load(open(ff))
        except Exception:
            fair = None
    out = {"value": round(W * H * done / t1 / 1e6, 3), "unit": "MPix/s", "cores": 1, "kind": "port",
           "frames_per_sec": round(done / t1, 3),
           "sample": f"{done} synthetic {W}x{H} {binary} pairs (config {cfg_name}), oracle/ofdis_oracle.c -O3 "
                     f"-msse4.1, 1 thread (pad+pyramid+OFClass+upsample), {t1:.1f} s",
           "cores_all": cores, "nproc": os.cpu_count(), "cpu_quota": cpu_quota(), "cpu_model": cpu_model(),
           "stages_ms_1core_median": {k: round(float(np.median([s_[k] for s_ in stages])) * 1e3, 3)
                                      for k in stages[0]},
           "fairness_vs_reference": fair}
    st = out["stages_ms_1core_median"]
    out["pyramid_upsample_share"] = round((st["pyramid"] + st["upsample"]) / sum(st.values()), 3)
    probe = os.path.join(ROOT, "profiles", "r03", "cpu_core_vs_probe.json")
    if os.path.exists(probe):  # the port's OFClass core against SURVEY's probe of the reference (container)
        try:
            ent = json.load(open(probe))["configs"].get(cfg_name)
            if ent:
                out["dis_core_ratio_vs_reference_probe"] = {
                    "ratio": ent["ofclass_ratio_vs_probe"], "port_ofclass_ms": ent["stages_min_ms"]["ofclass"],
                    "reference_probe_ms": ent["probe_ofclass_ms"], "where": "survey container, 1 thread",
                    "source": "tools/cpu_core_probe.py -> profiles/r03/cpu_core_vs_probe.json (BASELINE.md:30-34)"}
        except Exception:
            pass
    if done_all:
        out["value_all_cores"] = round(W * H * done_all / t_all / 1e6, 3)
        out["frames_per_sec_all_cores"] = round(done_all / t_all, 3)
        out["sample_all_cores"] = f"{done_all} pairs over {cores} worker threads, {t_all:.1f} s"
    if node > cores and not node_runs:
        out["value_node"] = None
        out["node_leg"] = (f"skipped: nproc {node} CPUs, but the cgroup quota caps this process at {quota} CPUs "
                           f"(the {cores}-worker leg is this host share's figure)")
    if done_node:
        out["value_node"] = round(W * H * done_node / t_node / 1e6, 3)
        out["frames_per_sec_node"] = round(done_node / t_node, 3)
        out["cores_node"] = node
        out["sample_node"] = f"{done_node} pairs over {node} worker threads (nproc), {t_node:.1f} s"
    return out


def plan_shards(args, cfg, world, rank):
    """This rank's [first, stop) of the step's pairs, the whole job's pairs per step and the scaling kind:
    strong (--total, or config D's 256 pairs) shards one batch over the ranks; weak gives every rank
    --batch pairs of its own."""
    total = args.total or (cfg[7] if args.config in STRONG and not args.batch else 0)
    if total:
        if total < world:
            raise SystemExit(f"bench.py: --total {total} < {world} ranks")
        first, stop = shard_range_of(total, rank, world)
        return first, stop, total, "strong"
    B = args.batch or cfg[7]
    first, stop = shard_range_of(B * world, rank, world)
    return first, stop, B * world, "weak"


def shard_range_of(n, rank, world):
    from of_dis_amd.distributed import shard_range
    return shard_range(n, rank, world)


def dry_run(args, cfg):
    """The rank logic without a GPU: gloo, shard bookkeeping, the control collectives."""
    import torch.distributed as dist
    from of_dis_amd import distributed as odd
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    first, stop, total, scaling = plan_shards(args, cfg, world, rank)
    shard = (first, stop)
    t0 = time.perf_counter()
    time.sleep(0.01 * (rank + 1))
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = odd.max_over_ranks(elapsed)
        frames = odd.sum_over_ranks([shard[1] - shard[0]])[0]
        shards = odd.all_gather_objects(list(shard))
    else:
        frames, shards = shard[1] - shard[0], [list(shard)]
    if rank == 0:
        if world != args.gpus:
            raise SystemExit(f"world size {world} != --gpus {args.gpus}")
        print(json.dumps({"metric": METRIC, "dry_run": True, "n_gpus": world, "ranks": world, "steps": args.steps,
                          "scaling": scaling, "config": {"name": args.config, "pairs_per_step": total},
                          "shards": shards, "frames": int(frames), "elapsed_max_s": elapsed}))
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_as_ranks(args))
    cfg = CONFIGS[args.config]
    if args.dry_run:
        return dry_run(args, cfg)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE {world} != --gpus {args.gpus}")
    # OFDIS_BENCH_REHEARSAL=1: rehearse the multi-rank path on a box with fewer GPUs than ranks -- ranks share
    # the GPUs round robin and the control collectives go over gloo (RCCL refuses two ranks on one GPU)
    rehearsal = os.environ.get("OFDIS_BENCH_REHEARSAL") == "1"
    gpu = local % max(1, torch.cuda.device_count()) if rehearsal else local
    # physical devices in use (a rehearsal's ranks share them); one GPU per rank otherwise
    n_devices = min(world, max(1, torch.cuda.device_count())) if rehearsal else world
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(gpu)
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", gpu if world > 1 else 0)

    import of_dis_amd as od
    from of_dis_amd import distributed as odd

    binary, W, H, noc, mode, op, explicit, default_batch = cfg
    first, stop, total, scaling = plan_shards(args, cfg, world, rank)
    B = stop - first  # this rank's pairs per step
    p = params_of(od, cfg)
    p.verbosity = 0
    if world > 1:  # one configuration for every shard
        odd.broadcast_params(p, dev)
    nop = p.nop
    ctx = od.Context(dev.index)
    ctx.set_option("streams", args.streams)
    ctx.set_option("chunk", args.chunk)
    # the library's chunking (ofdis_runtime.cpp stream_count): streams 0 = 2 from 256 pairs, else 1
    streams_eff = args.streams or (2 if B >= 256 else 1)
    chunk_eff = min(B, args.chunk or -(-B // streams_eff))
    for kv in args.option:
        k, v = kv.split("=")
        ctx.set_option(k, int(v))

    # synthetic inputs, resident in HBM before timing: this rank's shard of frames, distinct pairs tiled
    nd = max(1, min(args.distinct, B))
    pairs = [od.synth_pair(W, H, noc, first + k, mode) for k in range(nd)]
    a = torch.empty((B, H, W, noc), dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    for i in range(nd):
        a[i].copy_(torch.from_numpy(pairs[i][0]))
        b[i].copy_(torch.from_numpy(pairs[i][1]))
    for i in range(nd, B):
        a[i].copy_(a[i % nd])
        b[i].copy_(b[i % nd])
    out = torch.empty((B, H, W, nop), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step():
        ctx.run_ptr(a.data_ptr(), b.data_ptr(), B, W, H, p, out.data_ptr(), stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    for r in range(args.probe_regions):  # diagnostic (stderr only): run-to-run spread inside one process
        t = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        print(f"probe region {r}: {(time.perf_counter() - t) / args.steps * 1e3:.3f} ms/step", file=sys.stderr)
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
    # the timed pass's output of the distinct pairs, for the parity check below
    timed_out = out[:nd].cpu().numpy()
    # every other frame of the timed pass is a tile of one of the nd distinct pairs: compare its bits on the device
    # with its tile source (frames nd.. against frames 0..nd-1, nd at a time), so the oracle check of the distinct
    # frames covers the whole batch
    tiles_equal = [0] * nd  # per distinct pair: the later frames equal to it bit for bit
    ov = out.view(B, -1).view(torch.int32)
    for j in range(nd, B, nd):
        m = min(nd, B - j)
        if torch.equal(ov[j:j + m], ov[:m]):
            for i in range(m):
                tiles_equal[i] += 1
        else:
            for i in range(m):
                tiles_equal[i] += int(torch.equal(ov[j + i], ov[i]))
    del ov

    frames = total * args.steps
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
        # the upsample kernel the timed region ran (up_form auto follows the call's lanes, which this pass changes)
        up_user = any(o.split("=")[0] == "up_form" for o in args.option)
        if not up_user:
            lanes_eff = min(streams_eff, -(-B // chunk_eff))
            ctx.set_option("up_form", 1 if W >= 1024 and (lanes_eff >= 2 or B < 1024) else 0)
        ctx.enable_kernel_timing(True)
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        names = [k for k in od.kernel_names()]
        raw = []
        for k in names:
            ms, cnt = ctx.kernel_time(k)
            raw += [ms, cnt]
        if world > 1:  # whole-job device time per kernel (every rank ran the same launches)
            raw = odd.sum_over_ranks(raw, dev)
        for i, k in enumerate(names):
            ms, cnt = raw[2 * i], int(raw[2 * i + 1])
            if cnt:
                kernels[k] = {"total_ms": ms / world, "launches": cnt // world, "avg_us": ms / cnt * 1e3}
        ctx.enable_kernel_timing(False)
        ctx.set_option("streams", args.streams)
        ctx.set_option("chunk", args.chunk)
        if not up_user:
            ctx.set_option("up_form", 3)
        dom = max(kernels, key=lambda k: kernels[k]["total_ms"])
        roofline = kernel_roofline(od, p, W, H, B, chunk_eff, cfg, args.steps, kernels, dom)
        if dom != "tv_sor" and "tv_sor" in kernels:  # the north-star kernel, reported beside the dominant one
            roofline_sor = kernel_roofline(od, p, W, H, B, chunk_eff, cfg, args.steps, kernels, "tv_sor")

    # ---- single-pair latency (the drop-in CLI's case: one pair per call), device-resident and host buffers
    latency = None
    if rank == 0 and world == 1 and not args.no_latency:
        latency = pair_latency(od, ctx, p, pairs[0], dev, torch)

    # ---- strong-scaling configs on one GPU: the per-GPU rate at the shard size 8 GPUs would run (config D: 32 of
    # the 256 pairs), so a 1-GPU D number is never read as the per-GPU throughput of the 8-GPU job
    shard8 = None
    if scaling == "strong" and world == 1 and total >= 8:
        n8 = total // 8
        ctx.set_option("streams", 0)
        ctx.set_option("chunk", 0)
        for _ in range(args.warmup):
            ctx.run_ptr(a.data_ptr(), b.data_ptr(), n8, W, H, p, out.data_ptr(), stream)
        torch.cuda.synchronize(dev)
        t0s = time.perf_counter()
        for _ in range(args.steps):
            ctx.run_ptr(a.data_ptr(), b.data_ptr(), n8, W, H, p, out.data_ptr(), stream)
        torch.cuda.synchronize(dev)
        ts8 = time.perf_counter() - t0s
        r8 = W * H * n8 * args.steps / ts8 / 1e6
        shard8 = {"pairs_per_gpu": n8, "mpix_s_per_gpu": round(r8, 2), "ms_per_step": round(ts8 / args.steps * 1e3, 3),
                  "projected_1to8_efficiency": round(r8 / mpix, 3),
                  "what": f"1 GPU running the {n8}-pair shard each of 8 GPUs gets of this config's {total} pairs"}
        ctx.set_option("streams", args.streams)
        ctx.set_option("chunk", args.chunk)

    # ---- the latency mode beside the exact default (sor_mode = 1: red-black SOR, each TV level's inner loop in one
    # launch per frame): one pair per call, and a config-D shard (32 pairs per call, the pairs
    # each of 8 GPUs gets of BASELINE's 256) -- its end-point difference against the exact path is in "parity" below
    latency_mode = None
    rb_out = None
    if rank == 0 and world == 1 and not args.no_latency and not any(o.startswith("sor_mode") for o in args.option):
        ctx.set_option("sor_mode", 1)
        lat_rb = pair_latency(od, ctx, p, pairs[0], dev, torch)
        n32 = min(32, B)
        ctx.set_option("streams", 0)
        ctx.set_option("chunk", 0)
        for _ in range(max(1, args.warmup)):
            ctx.run_ptr(a.data_ptr(), b.data_ptr(), n32, W, H, p, out.data_ptr(), stream)
        torch.cuda.synchronize(dev)
        t0s = time.perf_counter()
        for _ in range(args.steps):
            ctx.run_ptr(a.data_ptr(), b.data_ptr(), n32, W, H, p, out.data_ptr(), stream)
        torch.cuda.synchronize(dev)
        t32 = time.perf_counter() - t0s
        rb_out = out[:min(nd, n32)].cpu().numpy()
        # strong-scaling configs (D): the same mode on the whole job's batch on this one GPU, so the 1 -> 8 projection
        # can be read against either N = 1 figure (the exact path's `value`, or this mode's own full-batch rate)
        full_rb = None
        if scaling == "strong" and world == 1 and B > n32:
            ctx.set_option("streams", args.streams)
            ctx.set_option("chunk", args.chunk)
            step()
            torch.cuda.synchronize(dev)
            t0s = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize(dev)
            tf = time.perf_counter() - t0s
            rf = W * H * B * args.steps / tf / 1e6
            full_rb = {"pairs_per_call": B, "mpix_s": round(rf, 2), "ms_per_step": round(tf / args.steps * 1e3, 3)}
        ctx.set_option("sor_mode", 0)
        ctx.set_option("streams", args.streams)
        ctx.set_option("chunk", args.chunk)
        r32 = W * H * n32 * args.steps / t32 / 1e6
        latency_mode = {"option": "sor_mode=1", "single_pair": lat_rb,
                        "shard_32": {"pairs_per_call": n32, "mpix_s_per_gpu": round(r32, 2),
                                     "ms_per_call": round(t32 / args.steps * 1e3, 3)},
                        "exact_single_pair_device_ms_median": latency["device_ms_median"] if latency else None}
        if full_rb is not None:
            latency_mode["full_batch_1gpu"] = full_rb
            latency_mode["projected_1to8_efficiency"] = {
                "vs_exact_value": round(r32 / mpix, 3), "vs_same_mode_full_batch": round(r32 / full_rb["mpix_s"], 3),
                "what": f"the {n32}-pair shard's rate in this mode over the 1-GPU rate of all {B} pairs: the exact "
                        "path's value, or this mode's own"}

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

    # ---- parity of the timed pass vs the CPU oracle (every rank: its shard's first frames), and the CPU
    # baseline (rank 0, N = 1 only): the oracle port on this host's cores, bounded samples
    cpu = None
    parity = None
    # compared frames, sum of avg EPE, max avg EPE, bit-exact distinct frames, frames of the batch bit-exact (a
    # bit-exact distinct frame and every later tile of it that equals it on the device), frames in the batch
    sums = [0.0, 0.0, 0.0, 0.0, 0.0, float(B)]
    if args.cpu_seconds > 0:
        from oracle import pyoracle as O
        q = oracle_params(O, p)
        ncmp = max(1, min(nd, args.parity_frames))
        for k in range(ncmp):
            ref = O.run_u8(pairs[k][0], pairs[k][1], q)
            g = timed_out[k]
            epe = float(np.sqrt(((g.astype(np.float64) - ref) ** 2).sum(-1)).mean())
            sums[0] += 1
            sums[1] += epe
            sums[2] = max(sums[2], epe)
            exact = np.array_equal(g.view(np.uint32), ref.view(np.uint32))
            sums[3] += int(exact)
            sums[4] += (1 + tiles_equal[k]) if exact else 0
            if rb_out is not None and k < len(rb_out):  # the latency mode's output of the same pair vs the exact path
                e = np.sqrt(((rb_out[k].astype(np.float64) - ref) ** 2).sum(-1))
                latency_mode.setdefault("epe_vs_exact_cpu_ref", []).append(
                    {"pair": k, "avg": round(float(e.mean()), 5), "p99": round(float(np.percentile(e, 99)), 4),
                     "max": round(float(e.max()), 4)})
        if rank == 0 and world == 1:
            cpu = cpu_baseline(O, q, pairs, W, H, args.cpu_seconds, binary, args.config)
    if world > 1:
        tot = odd.sum_over_ranks([sums[0], sums[1], sums[3], sums[4], sums[5]], dev)
        sums = [tot[0], tot[1], odd.max_over_ranks(sums[2], dev), tot[2], tot[3], tot[4]]
    if sums[0]:
        parity = {"avg_epe_vs_cpu_ref": sums[1] / sums[0], "avg_epe_vs_cpu_ref_max": sums[2],
                  "bitexact_frames": int(sums[4]), "batch_frames": int(sums[5]),
                  "oracle_compared_frames": int(sums[0]), "oracle_bitexact_frames": int(sums[3]),
                  "checked": "timed pass output: the distinct pairs against the CPU oracle bit for bit, every other "
                             "frame of the batch against its tile source on the device (int32 views, torch.equal)"}

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(mpix, 2), "unit": "MPix/s", "n_gpus": n_devices, "ranks": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "frames_per_sec": round(frames / elapsed, 2),
            "per_gpu_mpix_s": round(mpix / n_devices, 2),
            "config": {"workload": f"{binary} {W}x{H} op-point {op}" + (f" ({explicit})" if explicit else "")
                                   + (f", {total} pairs/step over {world} GPU(s)" if scaling == "strong"
                                      else f", {B} pairs/GPU/step"), "name": args.config,
                       "width": W, "height": H, "channels": noc, "oppoint": op, "batch_per_gpu": B,
                       "pairs_per_step": total,
                       "streams": streams_eff, "pairs_per_launch": chunk_eff,
                       "options": args.option,
                       "parallelism": f"frame-sharded x{world}" + (" (rehearsal: ranks share the GPU)"
                                                                   if rehearsal else "")},
            "roofline": roofline, "roofline_tv_sor": roofline_sor, "cpu_baseline": cpu, "parity": parity,
            "latency": latency, "latency_mode": latency_mode, "host_io": host_io, "shard_of_8": shard8,
            "kernels": kernels,
        }
        if cpu:
            line["speedup_vs_cpu_1core"] = round(mpix / cpu["value"], 1)
            if cpu.get("value_all_cores"):
                line["speedup_vs_cpu_all_cores"] = round(mpix / cpu["value_all_cores"], 1)
            if cpu.get("value_node"):
                line["speedup_vs_cpu_node"] = round(mpix / cpu["value_node"], 1)
        print(json.dumps(line))
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def pair_latency(od, ctx, p, pair, dev, torch, reps=20):
    """One pair per call (run_dense.cpp's case): device-resident (u8 in HBM, flow out in HBM, synchronised
    per call) and through host buffers (ofdis_run_batch_u8_host: H2D + path + D2H), plus the per-kernel
    breakdown of one device-resident pair."""
    H, W, noc = pair[0].shape
    a = torch.from_numpy(pair[0][None]).to(dev)
    b = torch.from_numpy(pair[1][None]).to(dev)
    o = torch.empty((1, H, W, p.nop), dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    ctx.set_option("streams", 1)
    ctx.set_option("chunk", 0)
    for _ in range(3):
        ctx.run_ptr(a.data_ptr(), b.data_ptr(), 1, W, H, p, o.data_ptr(), s)
    torch.cuda.synchronize(dev)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ctx.run_ptr(a.data_ptr(), b.data_ptr(), 1, W, H, p, o.data_ptr(), s)
        torch.cuda.synchronize(dev)
        ts.append(time.perf_counter() - t0)
    th = []
    for _ in range(max(3, reps // 4)):
        t0 = time.perf_counter()
        ctx.run_host(pair[0], pair[1], p)
        th.append(time.perf_counter() - t0)
    ctx.enable_kernel_timing(True)
    ctx.run_ptr(a.data_ptr(), b.data_ptr(), 1, W, H, p, o.data_ptr(), s)
    torch.cuda.synchronize(dev)
    brk = {}
    for k in od.kernel_names():
        ms, cnt = ctx.kernel_time(k)
        if cnt:
            brk[k] = {"ms": round(ms, 4), "launches": cnt}
    ctx.enable_kernel_timing(False)
    ctx.set_option("streams", 0)
    return {"pairs_per_call": 1, "device_ms_median": round(float(np.median(ts)) * 1e3, 3),
            "device_ms_min": round(min(ts) * 1e3, 3), "host_ms_median": round(float(np.median(th)) * 1e3, 3),
            "kernels_one_pair": brk}


if __name__ == "__main__":
    main()
