import os, sys
sys.path.insert(0, "rust-particle-system_amd/python")
import numpy as np
import rps_amd as rps
for n in (50000, 300000):
    scale = max(1.0, (n / 50000) ** 0.5)
    cfg = rps.default_particle_config(n, screen_bounds=rps.screen_bounds_for(1920.0 * scale, 1080.0 * scale))
    parts = rps.setup_particles_scatter(cfg, n, seed=1)
    with rps.Context(n, rps.MODE_SPH) as ctx:
        ctx.set_config(cfg, rps.make_ext())
        ctx.upload(parts)
        for f in (6, 10, 30, 60):
            ctx.step(f - (0 if f == 6 else prev)) if False else None
        done = 0
        for f in (6, 10, 30, 60):
            ctx.step(f - done); done = f
            s = ctx.download_soa()
            lk = ctx.read_debug(rps.DEBUG_SPATIAL_LOOKUP).reshape(-1, 2)
            k0 = int((lk[:n, 0] == 0).sum())
            print(n, "frame", f, "NaN particles", int(np.isnan(s["x"]).sum()), "key-0 entries in [0,N)", k0, flush=True)
