"""Same-box A/B of librps builds on SPH frames (run on the GPU box).

    python tools/ab_sph.py [--n N] [--warm W] [--frames F] [--rounds R] LIB_A[@ENV=VAL...] LIB_B ...

Each variant runs in its own subprocess (one librps per process), in rounds A, B, A, B, ...
One run: N particles of the reference scatter, as bench.py places them: in the reference's
1920 x 1080 viewport up to N = 65 536 (its `sph.reference_sizes`), above that over a viewport
scaled to the default density (its 2^22 `sph` line); every frame active, W warm frames, F timed (HIP events).  The
default window is bench.py's (20 warm, 200 timed): at P != N the frame cost depends on the frame
index (the pad hazard's runs change from frame to frame, tools/sph_frame_curve.py), so tools that
time different windows report different numbers for the same build.
AB_MORTON=1 in a variant's environment uploads the particles in Morton order of their cells."""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(lib, n, frames, warm):
    sys.path.insert(0, os.path.join(ROOT, "rust-particle-system_amd", "python"))
    import rps_amd as rps

    rps.LIB_PATH = os.path.abspath(lib)
    scale = max(1.0, (n / 50000) ** 0.5) if n > 65536 else 1.0  # bench.py: reference viewport up to 65 536
    cfg = rps.default_particle_config(n, screen_bounds=rps.screen_bounds_for(1920.0 * scale, 1080.0 * scale))
    parts = rps.setup_particles_scatter(cfg, n, seed=0x5EED)
    if os.environ.get("AB_MORTON") == "1":  # upload in Morton order of the particles' cells
        import numpy as np

        r = float(cfg.smoothing_radius)
        cx = ((parts["position"][:, 0] - cfg.screen_bounds[0]) / r).astype(np.uint64) & 0xFFFF
        cy = ((parts["position"][:, 1] - cfg.screen_bounds[2]) / r).astype(np.uint64) & 0xFFFF

        def spread(v):
            v = (v | (v << 8)) & 0x00FF00FF
            v = (v | (v << 4)) & 0x0F0F0F0F
            v = (v | (v << 2)) & 0x33333333
            return (v | (v << 1)) & 0x55555555

        parts = parts[np.argsort(spread(cx) | (spread(cy) << np.uint64(1)), kind="stable")]
    with rps.Context(n, rps.MODE_SPH) as ctx:
        ctx.set_config(cfg, rps.make_ext(shader_delay=0))
        ctx.upload(parts)
        ctx.step(warm)
        ctx.sync()
        ms = ctx.time_steps(frames) / frames
    print(json.dumps({"lib": lib, "n": n, "ms_per_frame": ms}), flush=True)


def main():
    a = sys.argv[1:]
    if a and a[0] == "--one":
        one(a[1], int(a[2]), int(a[3]), int(a[4]))
        return
    n, frames, rounds, warm = 1 << 22, 200, 3, 20
    while a and a[0].startswith("--"):
        if a[0] == "--n":
            n = int(a[1])
        elif a[0] == "--frames":
            frames = int(a[1])
        elif a[0] == "--rounds":
            rounds = int(a[1])
        elif a[0] == "--warm":
            warm = int(a[1])
        a = a[2:]
    res = {v: [] for v in a}
    for _ in range(rounds):
        for v in a:
            lib, *envs = v.split("@")
            env = dict(os.environ)
            for e in envs:
                k, val = e.split("=", 1)
                env[k] = val
            p = subprocess.run([sys.executable, __file__, "--one", lib, str(n), str(frames), str(warm)], env=env,
                               capture_output=True, text=True, timeout=600)
            if p.returncode:
                print(p.stderr[-2000:], flush=True)
                sys.exit(p.returncode)
            res[v].append(json.loads(p.stdout.strip().splitlines()[-1])["ms_per_frame"])
    for v, ms in res.items():
        print(f"n={n} {v}: median {statistics.median(ms):.4f} ms/frame  (runs {', '.join(f'{m:.4f}' for m in ms)})")


if __name__ == "__main__":
    main()
