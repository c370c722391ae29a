"""Cost of the live parameter path: frames with a config upload each frame
(rps_set_config then rps_step(1): what the host mirrors' prepare_particle_buffers does on every
change, and what the reference's write_buffer does every frame) against frames without one,
on the GPU box.  The uploaded values do not change, so both runs simulate the same work.

    python tools/config_upload_bench.py [LIB ...]

Prints one JSON line per library and mode: wall ms per frame over 2000 frames after 200 warm
ones, for STREAM (C1: 65 536 particles, one attractor) and SPH (65 536 particles)."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(lib, mode):
    sys.path[:0] = [os.path.join(ROOT, "rust-particle-system_amd", "python"), os.path.join(ROOT, "tests")]
    import rps_amd as rps
    from helpers import ext_c1_attractor

    rps.LIB_PATH = os.path.abspath(lib)
    n = 65536
    if mode == "stream":
        cfg = rps.default_particle_config(n, gravity=9.8)
        ext = ext_c1_attractor(rps)
        ctx = rps.Context(n)
    else:
        cfg = rps.default_particle_config(n, screen_bounds=rps.screen_bounds_for(1920.0 * 1.15, 1080.0 * 1.15))
        ext = rps.make_ext()
        ctx = rps.Context(n, rps.MODE_SPH)
    ext.shader_delay = 0
    ctx.set_config(cfg, ext)
    ctx.upload(rps.setup_particles_scatter(cfg, n, seed=3))
    out = {"lib": lib, "mode": mode}
    for upload in (False, True):
        for phase, frames in (("warm", 200), ("timed", 2000)):
            ctx.sync()
            t0 = time.perf_counter()
            for f in range(frames):
                if upload:  # the config written every frame (the same values, so the
                    ctx.set_config(cfg, ext)  # simulated work is the same as without)
                ctx.step(1)
            ctx.sync()
            el = time.perf_counter() - t0
        out["ms_per_frame_upload" if upload else "ms_per_frame"] = el * 1e3 / frames
    ctx.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--one":
        one(sys.argv[2], sys.argv[3])
    else:
        libs = sys.argv[1:] or [os.path.join(ROOT, "rust-particle-system_amd", "lib", "librps.so")]
        for lib in libs:
            for mode in ("stream", "sph"):
                p = subprocess.run([sys.executable, __file__, "--one", lib, mode], capture_output=True, text=True,
                                   timeout=300)
                sys.stdout.write(p.stdout if p.returncode == 0 else p.stdout + p.stderr)
