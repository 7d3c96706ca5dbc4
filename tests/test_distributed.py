"""Frame sharding on CPU: world_size-2 gloo process groups stand in for RCCL ranks.

The data path has no collective; these tests cover the control collectives bench.py uses (barrier,
max of elapsed time, sum of counters) and that the shards tile the batch exactly once.
"""
import os
import socket

import pytest
import torch.multiprocessing as mp

from of_dis_amd.distributed import shard_range


@pytest.mark.parametrize("n,world", [(256, 8), (10, 3), (3, 4), (0, 2), (1, 1)])
def test_shards_tile_the_batch(n, world):
    seen = []
    sizes = []
    for r in range(world):
        a, b = shard_range(n, r, world)
        assert 0 <= a <= b <= n
        seen.extend(range(a, b))
        sizes.append(b - a)
    assert seen == list(range(n))
    assert max(sizes) - min(sizes) <= 1


def test_shard_range_rejects_bad_rank():
    with pytest.raises(ValueError):
        shard_range(8, 2, 2)
    with pytest.raises(ValueError):
        shard_range(8, 0, 0)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from of_dis_amd.distributed import max_over_ranks, shard_range, sum_over_ranks
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a, b = shard_range(64, rank, world)
        dist.barrier()
        t = max_over_ranks(0.5 + rank)           # per-rank "elapsed"
        tot = sum_over_ranks([b - a, 1.0])        # frames processed, ranks
        q.put((rank, a, b, t, tot))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_control_collectives():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [(r[1], r[2]) for r in res] == [(0, 32), (32, 64)]
    assert all(r[3] == 1.5 for r in res)          # max over ranks
    assert all(r[4] == [64.0, 2.0] for r in res)  # whole-job frames


def test_bench_launcher_dry_run_two_ranks():
    """`bench.py --gpus 2` outside torchrun re-launches itself as 2 ranks (a child torch.distributed.run
    job); with --dry-run the ranks run on gloo without a GPU and rank 0 reports n_gpus 2 and the disjoint
    shards of config D: BASELINE configs[3]'s 256-pair batch split over the ranks (strong scaling)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--config", "D",
                        "--dry-run"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["dry_run"] and d["scaling"] == "strong"
    assert d["shards"] == [[0, 128], [128, 256]]
    assert d["frames"] == 256


@pytest.mark.parametrize("argv,world,shards,scaling", [
    (["--config", "B", "--batch", "4"], 2, [[0, 4], [4, 8]], "weak"),          # weak: --batch per GPU
    (["--config", "B", "--total", "10"], 3, [[0, 4], [4, 7], [7, 10]], "strong"),  # ragged strong shards
    (["--config", "D"], 4, [[0, 64], [64, 128], [128, 192], [192, 256]], "strong"),
])
def test_bench_shard_plans(argv, world, shards, scaling):
    """Shard plans of bench.py at several world sizes: every pair of the step owned by exactly one rank."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(world), "--dry-run"] + argv,
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert d["shards"] == shards and d["scaling"] == scaling and d["frames"] == shards[-1][1]


def test_bench_rejects_world_mismatch():
    """A rank whose WORLD_SIZE disagrees with --gpus fails instead of reporting the wrong n_gpus."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0


def _bcast_worker(rank, world, port, q):
    import torch.distributed as dist
    import of_dis_amd as od
    from of_dis_amd.distributed import broadcast_params
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = od.Params(mode=1, noc=1, sc_f=6, sc_l=4, p_samp_s=8, tv_sor=1.6) if rank == 0 else od.Params()
        broadcast_params(p)
        q.put((rank, p.as_dict()))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_broadcast_params():
    """Rank 0's ofdis_params reach every rank unchanged (the one parameter collective)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bcast_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1] and res[1]["sc_f"] == 6 and abs(res[1]["tv_sor"] - 1.6) < 1e-6
