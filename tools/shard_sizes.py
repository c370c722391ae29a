"""The headline's per-rank shard sizes on one GPU: the metric is 1e8
particles at 1/2/4/8 GPUs, split into contiguous shards, so a rank of the N-GPU curve steps
1e8/N particles.  Each size runs as the LAST rank's shard of the 1e8 system (id_offset, global
count 1e8: the same attractors, respawn keys and config as in the N-GPU run), with the bench's
warmup and one HIP event pair around K launches.

    python tools/shard_sizes.py [K] [W]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-particle-system_amd", "python"))
import rps_amd as rps  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 500
W = int(sys.argv[2]) if len(sys.argv) > 2 else 100
G = 100_000_000
cfg = rps.default_particle_config(G, gravity=0.0)
ext = rps.headline_ext(stats=True)
ext.shader_delay = 0
for world in (1, 2, 4, 8, 16):
    lo, hi = G * (world - 1) // world, G
    n = hi - lo
    with rps.Context(n, rps.MODE_STREAM, id_offset=lo, global_count=G) as ctx:
        ctx.set_config(cfg, ext)
        ctx.init_scatter(0x5EED)
        ctx.step(W)
        ctx.sync()
        ms = ctx.time_steps(K) / K
        moved, _ = ctx.step_cost()
    print(json.dumps({"gpus": world, "particles_per_rank": n, "state_mb": round(moved / 2 / 1e6, 1),
                      "ms_per_step": round(ms, 5), "updates_per_s_per_gpu": n / (ms * 1e-3),
                      "moved_gbps": moved / (ms * 1e-3) / 1e9, "moved_frac_of_8tbps": moved / (ms * 1e-3) / 8e12,
                      "ideal_curve_updates_per_s": world * n / (ms * 1e-3)}), flush=True)
