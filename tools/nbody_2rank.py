"""Two processes on ONE GPU running the sharded all-pairs step through librps's own RCCL
communicator (rps_comm_init + in-place ncclAllGather): each rank owns half the particles,
rank 0 checks its shard's accelerations against the unsharded oracle.  Probe of whether the
multi-rank N-body data path runs here (RCCL may refuse two ranks on one device)."""
import os
import socket
import sys

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker(rank, world, port, n_per, q):
    for p in (os.path.join(ROOT, "rust-particle-system_amd", "python"), os.path.join(ROOT, "oracle"),
              os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as orc
    import rps_amd as rps

    n = n_per * world
    cfg = rps.default_particle_config(n, gravity=0.0)
    ext = rps.make_ext(nbody_strength=10.0, nbody_softening=1.0, shader_delay=0)
    g = np.random.default_rng(5)
    x = g.uniform(-900, 900, n).astype(np.float32)
    y = g.uniform(-500, 500, n).astype(np.float32)
    lo = rank * n_per
    obj = [rps.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    try:
        with rps.Context(n_per, rps.MODE_NBODY, device=0, id_offset=lo, global_count=n) as ctx:
            ctx.set_config(cfg, ext)
            ctx.comm_init(rank, world, obj[0])
            ctx.upload_soa(dict(x=x[lo:lo + n_per], y=y[lo:lo + n_per], vx=np.zeros(n_per, np.float32),
                                vy=np.zeros(n_per, np.float32)))
            ctx.step(1)
            ax = ctx.read_debug(rps.DEBUG_ACCEL_X)
            ay = ctx.read_debug(rps.DEBUG_ACCEL_Y)
        rx, ry = orc.nbody_accel(ext, x, y, t0=lo, nt=n_per)
        mag = np.hypot(rx, ry)
        err = np.hypot(ax - rx, ay - ry) / np.maximum(mag, 1e-30)
        res = f"rank {rank}: median rel err {np.median(err):.2e}, max {err.max():.2e}"
    except Exception as e:  # report RCCL refusing two ranks on one device
        res = f"rank {rank}: {type(e).__name__}: {e}"
    q.put(res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, 2, port, 4096, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    while not q.empty():
        print(q.get())
    sys.exit(max(abs(p.exitcode or 0) for p in procs))
