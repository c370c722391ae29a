"""Multi-process (world size 2, gloo, CPU) coverage of the N>1 paths.

* STREAM: index-range shards with global ids, stepped independently, all-gathered, equal
  the unsharded step bit for bit (no data-path collective needed).
* NBODY: each rank all-gathers the float2 positions (the exchange rps_step does with
  ncclAllGather) and computes forces for its own targets == the unsharded forces.
* STREAM stats over ranks: each shard's stats in the form librps all-reduces over RCCL
  (StatsGlobal, rps_device.hpp: MAX of {-x_min, x_max, -y_min, y_max}, SUM of KE, particles,
  respawns) combine to the unsharded stats.
* bench.Dist: barrier + max-over-ranks as used by bench.py under torchrun.
"""
import os
import socket
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(rank, world, port):
    for p in (HERE, ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "rust-particle-system_amd", "python")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _stream_worker(rank, world, port, n_per, q, n_global=0):
    _setup(rank, world, port)
    import types

    import bench
    import oracle as orc
    import rps_amd as rps
    from helpers import random_soa

    if n_global:  # bench.py's strong split: rank r owns [r*G/W, (r+1)*G/W)
        n_per, lo, g = bench.shard(types.SimpleNamespace(particles=0, global_particles=n_global),
                                   types.SimpleNamespace(rank=rank, world=world))
        assert g == n_global
    else:
        lo, n_global = rank * n_per, n_per * world
    cfg = rps.default_particle_config(n_global)
    ext = rps.headline_ext()
    full = random_soa(n_global, list(cfg.screen_bounds), seed=77, life=(-0.1, 0.5))
    mine = {k: v[lo:lo + n_per].copy() for k, v in full.items()}
    for s in range(7):
        orc.stream_step(cfg, ext, mine, s, id_offset=lo)
    ref = None
    if rank == 0:
        ref = {k: v.copy() for k, v in full.items()}
        for s in range(7):
            orc.stream_step(cfg, ext, ref, s, id_offset=0)
    ok = 1
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([n_per]))
    width = max(int(t.item()) for t in sizes)
    for k in ("x", "y", "vx", "vy", "life"):  # shards padded to the largest for all_gather
        parts = [torch.zeros(width, dtype=torch.float32) for _ in range(world)]
        mine_k = np.zeros(width, np.float32)
        mine_k[:n_per] = mine[k]
        dist.all_gather(parts, torch.from_numpy(mine_k))
        got = torch.cat([p[:int(n.item())] for p, n in zip(parts, sizes)]).numpy()
        if rank == 0 and (got.size != n_global or not np.array_equal(got.view(np.uint32), ref[k].view(np.uint32))):
            ok = 0
    if rank == 0:
        q.put(ok)
    dist.barrier()
    dist.destroy_process_group()


def _nbody_worker(rank, world, port, n_per, q):
    _setup(rank, world, port)
    import oracle as orc
    import rps_amd as rps

    ext = rps.make_ext(nbody_strength=3.0, nbody_softening=1.5)
    g = np.random.default_rng(rank + 10)
    x = g.uniform(-500, 500, n_per).astype(np.float32)
    y = g.uniform(-300, 300, n_per).astype(np.float32)
    pos = torch.from_numpy(np.stack([x, y], 1).copy())
    gathered = [torch.zeros_like(pos) for _ in range(world)]
    dist.all_gather(gathered, pos)  # == ncclAllGather of float2 positions in rps_step
    allpos = torch.cat(gathered).numpy()
    ax, ay = orc.nbody_accel(ext, allpos[:, 0], allpos[:, 1], t0=rank * n_per, nt=n_per)
    out = [torch.zeros(n_per, dtype=torch.float32) for _ in range(world)]
    dist.all_gather(out, torch.from_numpy(ax))
    if rank == 0:
        rx, _ = orc.nbody_accel(ext, allpos[:, 0], allpos[:, 1])
        q.put(int(np.array_equal(torch.cat(out).numpy().view(np.uint32), rx.view(np.uint32))))
    dist.barrier()
    dist.destroy_process_group()


def _stats_worker(rank, world, port, n_per, q):
    _setup(rank, world, port)
    import oracle as orc
    import rps_amd as rps
    from helpers import random_soa

    cfg = rps.default_particle_config(n_per * world)
    ext = rps.headline_ext(stats=True)
    full = random_soa(n_per * world, list(cfg.screen_bounds), seed=91, life=(-0.1, 0.5))
    lo = rank * n_per
    mine = {k: v[lo:lo + n_per].copy() for k, v in full.items()}
    for s in range(4):
        st = orc.stream_step(cfg, ext, mine, s, id_offset=lo, stats=(s == 3))
    mm = torch.tensor([-st.bbox[0], st.bbox[1], -st.bbox[2], st.bbox[3]], dtype=torch.float32)
    sums = torch.tensor([st.kinetic_energy, float(st.particles), float(st.respawned)], dtype=torch.float64)
    dist.all_reduce(mm, op=dist.ReduceOp.MAX)  # == the two in-place ncclAllReduce calls
    dist.all_reduce(sums, op=dist.ReduceOp.SUM)
    if rank == 0:
        ref = {k: v.copy() for k, v in full.items()}
        for s in range(4):
            rst = orc.stream_step(cfg, ext, ref, s, stats=(s == 3))
        bbox = np.array([-mm[0].item(), mm[1].item(), -mm[2].item(), mm[3].item()], np.float32)
        ok = (np.array_equal(bbox, np.array(list(rst.bbox), np.float32)) and int(sums[1].item()) == rst.particles
              and int(sums[2].item()) == rst.respawned and rst.respawned > 0
              and abs(sums[0].item() - rst.kinetic_energy) <= 1e-9 * abs(rst.kinetic_energy))
        q.put(int(ok))
    dist.barrier()
    dist.destroy_process_group()


def _bench_dist_worker(rank, world, port, q):
    for p in (ROOT,):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import bench

    d = bench.Dist()
    assert d.world == world and d.backend == "gloo"
    d.barrier()
    m = d.max(float(rank) + 0.5)

    class St:  # one rank's last stats step (rps_stats)
        bbox = [-10.0 - rank, 20.0 + rank, -30.0 + rank, 40.0 - rank]
        kinetic_energy, particles, respawned, step = 1.5 * (rank + 1), 100 + rank, rank, 7

    g = bench.global_stats(d, St())
    ok = g == {"step": 7, "bbox": [-10.0 - (world - 1), 20.0 + world - 1, -30.0, 40.0], "ranks": world,
               "kinetic_energy": 1.5 * world * (world + 1) / 2, "particles": 100 * world + world * (world - 1) // 2,
               "respawned_last": world * (world - 1) // 2}
    if rank == 0:
        q.put(m if ok else -1.0)
    d.close()


def _run(fn, *args, world=2, extra=()):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.start_processes(fn, args=(world, _free_port(), *args, q, *extra), nprocs=world, join=True,
                       start_method="spawn")
    return q.get()


def test_stream_shards_equal_unsharded_gloo():
    assert _run(_stream_worker, 3001) == 1


def test_stream_strong_split_equals_unsharded_gloo():
    """bench.py's default (strong) split of one global count, ragged across the two ranks,
    equals the unsharded step bit for bit."""
    assert _run(_stream_worker, 0, extra=(6003,)) == 1


def test_nbody_allgather_shards_equal_unsharded_gloo():
    assert _run(_nbody_worker, 700) == 1


def test_stream_stats_allreduce_form_gloo():
    assert _run(_stats_worker, 5003) == 1


def test_bench_dist_barrier_and_max_gloo():
    assert _run(_bench_dist_worker) == 1.5
