"""Workload of the SPH traffic passes (tools/pmc_sph_traffic.sh): first a calibration stream --
STREAM mode, 2^24 particles, no lifetime/attractors/stats, 4 steps, so each stream launch reads
exactly 16 B and writes 16 B per particle (x, y, vx, vy) -- then the bench's SPH workload
(2^22 particles of the reference scatter over the scaled viewport, every frame active) for
`frames` frames.  The stream launches give the bytes per TCP->TCC request of 16-B accesses."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-particle-system_amd", "python"))
import rps_amd as rps  # noqa: E402

ns = 1 << 24
with rps.Context(ns, rps.MODE_STREAM) as ctx:
    cfg = rps.default_particle_config(ns, gravity=9.8)
    ctx.set_config(cfg, rps.make_ext(shader_delay=0))
    ctx.init_scatter(1)
    ctx.step(4)
    ctx.sync()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 22
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 12
scale = max(1.0, (n / 50000) ** 0.5)
cfg = rps.default_particle_config(n, screen_bounds=rps.screen_bounds_for(1920.0 * scale, 1080.0 * scale))
parts = rps.setup_particles_scatter(cfg, n, seed=0x5EED)
with rps.Context(n, rps.MODE_SPH) as ctx:
    ctx.set_config(cfg, rps.make_ext(shader_delay=0))
    ctx.upload(parts)
    ctx.step(frames)
    ctx.sync()
print(f"stream {ns} x 4 steps, SPH {n} x {frames} frames")
