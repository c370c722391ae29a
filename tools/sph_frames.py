"""SPH frames for profiling (rocprofv3 --kernel-trace --stats -- python3 tools/sph_frames.py N FRAMES).

Every frame is active (shader_delay 0: the reference's passes 4-5 run from the first frame,
as they do after SHADER_DELAY, wgsl:420-453), so ms/frame is an active frame's cost.  Ten
untimed frames first (the pad hazard of non-power-of-two N develops over the first frames)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-particle-system_amd", "python"))
import rps_amd as rps  # noqa: E402

if os.environ.get("AB_LIB"):  # a variant build (tools/build_variant.sh) for A/B traces
    rps.LIB_PATH = os.path.abspath(os.environ["AB_LIB"])

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 50
warm = int(sys.argv[3]) if len(sys.argv) > 3 else 10
scale = max(1.0, (n / 50000) ** 0.5) if n > 65536 else 1.0  # bench.py: reference viewport up to 65 536
cfg = rps.default_particle_config(n, screen_bounds=rps.screen_bounds_for(1920.0 * scale, 1080.0 * scale))
parts = rps.setup_particles_scatter(cfg, n, seed=1)
with rps.Context(n, rps.MODE_SPH) as ctx:
    ctx.set_config(cfg, rps.make_ext(shader_delay=0))
    ctx.upload(parts)
    ctx.step(warm)
    ctx.sync()
    ms = ctx.time_steps(frames)
    print(f"SPH n={n}: {ms / frames:.4f} ms/frame over {frames} active frames (after {warm} warm frames)")
