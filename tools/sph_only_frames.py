"""Active SPH frames of one librps build for kernel traces (run on the GPU box), including
timing-only builds (their results are not checked):  python3 tools/sph_only_frames.py LIB N FRAMES"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-particle-system_amd", "python"))
import rps_amd as rps  # noqa: E402

lib, n, frames = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rps.LIB_PATH = os.path.abspath(lib)
scale = max(1.0, (n / 50000) ** 0.5)
cfg = rps.default_particle_config(n, screen_bounds=rps.screen_bounds_for(1920.0 * scale, 1080.0 * scale))
parts = rps.setup_particles_scatter(cfg, n, seed=0x5EED)
with rps.Context(n, rps.MODE_SPH) as ctx:
    ctx.set_config(cfg, rps.make_ext(shader_delay=0))
    ctx.upload(parts)
    ctx.step(5)
    ctx.sync()
    ms = ctx.time_steps(frames) / frames
print(f"{lib}: {ms:.4f} ms per frame", flush=True)
