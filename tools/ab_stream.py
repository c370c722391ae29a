"""Same-box A/B of librps builds on the C3 headline step (run on the GPU box).

    python tools/ab_stream.py LIB_A LIB_B[@ENV=VAL[@ENV2=VAL2]] [...] [--rounds R] [--fuse K]

Each library runs in its own subprocess (one librps per process), in rounds A, B, A, B, ...
so drift of the box (clocks, temperature) hits every variant alike.  One run: the bench's
C3 workload (1e8 particles, headline_ext with stats, seeded scatter), 100 warm-up steps,
500 timed.  AB_ATTRACTORS / AB_LIFE in a variant's environment trim the workload, AB_N resizes it, AB_C2=1 runs
the C2 ext (one attractor, velocity-Verlet).  Prints one JSON line per run and the per-library medians."""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(lib, fuse, warm=100, steps=500):
    n = int(os.environ.get("AB_N", 100_000_000))
    sys.path.insert(0, os.path.join(ROOT, "rust-particle-system_amd", "python"))
    import rps_amd as rps

    rps.LIB_PATH = os.path.abspath(lib)
    cfg = rps.default_particle_config(n, gravity=0.0)
    ext = rps.headline_ext(stats=True)
    ext.shader_delay = 0
    ext.fuse_steps = fuse
    # Workload knobs for attributing the step's time (a variant's @ENV=VAL):
    # AB_ATTRACTORS=k keeps the first k attractors, AB_LIFE=0 turns the lifetime off.
    if os.environ.get("AB_C2") == "1":  # the C2 workload: one attractor, velocity-Verlet
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from helpers import ext_verlet_1att

        ext = ext_verlet_1att(rps)
        ext.shader_delay = 0
        ext.fuse_steps = fuse
    if "AB_ATTRACTORS" in os.environ:
        ext.num_attractors = min(ext.num_attractors, int(os.environ["AB_ATTRACTORS"]))
    if os.environ.get("AB_LIFE") == "0":
        ext.flags &= ~rps.EXT_LIFETIME
    with rps.Context(n) as ctx:
        ctx.set_config(cfg, ext)
        ctx.init_scatter(0x5EED)
        ctx.step(warm)
        ctx.sync()
        ms = ctx.time_steps(steps) / steps
    print(json.dumps({"lib": lib, "fuse": fuse, "ms_per_step": ms}), flush=True)


def main():
    args = sys.argv[1:]
    if args and args[0] == "--one":
        one(args[1], int(args[2]))
        return
    rounds, fuse, libs = 3, 1, []
    i = 0
    while i < len(args):
        if args[i] == "--rounds":
            rounds = int(args[i + 1])
            i += 2
        elif args[i] == "--fuse":
            fuse = int(args[i + 1])
            i += 2
        else:
            libs.append(args[i])
            i += 1
    res = {l: [] for l in libs}
    for _ in range(rounds):
        for l in libs:
            path, *envs = l.split("@")
            env = dict(os.environ, **dict(e.split("=", 1) for e in envs))
            p = subprocess.run([sys.executable, __file__, "--one", path, str(fuse)], capture_output=True,
                               text=True, timeout=300, env=env)
            if p.returncode != 0:
                print(p.stdout, p.stderr, flush=True)
                sys.exit(p.returncode)
            line = p.stdout.strip().splitlines()[-1]
            print(line, flush=True)
            res[l].append(json.loads(line)["ms_per_step"])
            print(json.dumps({"variant": l, "ms_per_step": res[l][-1]}), flush=True)
    print(json.dumps({"median_ms": {l: statistics.median(v) for l, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
