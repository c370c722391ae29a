"""SPH frames for profiling (rocprofv3 --kernel-trace --stats -- python3 tools/sph_frames.py N FRAMES)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-particle-system_amd", "python"))
import rps_amd as rps  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 50
scale = max(1.0, (n / 50000) ** 0.5)
cfg = rps.default_particle_config(n, screen_bounds=rps.screen_bounds_for(1920.0 * scale, 1080.0 * scale))
parts = rps.setup_particles_scatter(cfg, n, seed=1)
with rps.Context(n, rps.MODE_SPH) as ctx:
    ctx.set_config(cfg, rps.make_ext())
    ctx.upload(parts)
    ms = ctx.time_steps(frames)
    print(f"SPH n={n}: {ms / frames:.4f} ms/frame over {frames} frames (first 4 gated)")
