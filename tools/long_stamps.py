"""Diagnostic for the SPH long-scan kernels (not a product tool): runs N particles of the bench's
SPH workload on a librps built with per-slot s_memtime stamps written into the offsets buffer
(a variant build), and prints the per-phase cycle distribution.

    python tools/long_stamps.py LIB N FRAMES"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-particle-system_amd", "python"))
import rps_amd as rps  # noqa: E402

lib, n, frames = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rps.LIB_PATH = os.path.abspath(lib)
scale = max(1.0, (n / 50000) ** 0.5)
cfg = rps.default_particle_config(n, screen_bounds=rps.screen_bounds_for(1920.0 * scale, 1080.0 * scale))
parts = rps.setup_particles_scatter(cfg, n, seed=1)
with rps.Context(n, rps.MODE_SPH) as ctx:
    ctx.set_config(cfg, rps.make_ext(shader_delay=0))
    ctx.upload(parts)
    ctx.step(frames)
    ctx.sync()
    o = ctx.read_debug(rps.DEBUG_LOOKUP_OFFSETS)
print("raw head:", o[:16].tolist(), " tags:", int(((o >> 16) == 0xABCD).sum()))
a = o[: (len(o) // 8) * 8].reshape(-1, 8).astype(np.int64)
a = a[(a[:, 7] >> 16) == 0xABCD]
names = ["total", "within", "queue", "runs", "own", "pressure", "viscosity"]
print(f"{len(a)} slots stamped (cycles)")
for i, nm in enumerate(names):
    v = a[:, i]
    print(f"{nm:10s} median {np.median(v):9.0f}  p90 {np.percentile(v, 90):9.0f}  max {v.max():9.0f}")
tot = a[:, 2:7].sum(1)
print(f"slot total median {np.median(tot):.0f}  p90 {np.percentile(tot, 90):.0f}  max {tot.max()}")
