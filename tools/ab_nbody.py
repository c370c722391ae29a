"""Same-box A/B of librps builds on the all-pairs force kernel (run on the GPU box).

    python tools/ab_nbody.py [--n N] [--rounds R] LIB_A[@ENV=VAL...] LIB_B ...

Each variant runs in its own subprocess (one librps per process), in rounds A, B, A, B, ...
One run: N particles (default 2^21), the A11 scatter, 1 warm step, 2 timed steps; the force
kernel's HIP-event average.  Prints one JSON line per run and the per-variant medians."""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(lib, n):
    sys.path.insert(0, os.path.join(ROOT, "rust-particle-system_amd", "python"))
    import rps_amd as rps

    rps.LIB_PATH = os.path.abspath(lib)
    cfg = rps.default_particle_config(n, gravity=0.0)
    ext = rps.make_ext(nbody_strength=1.0e5, nbody_softening=1.0, shader_delay=0)
    with rps.Context(n, rps.MODE_NBODY) as ctx:
        ctx.set_config(cfg, ext)
        ctx.init_scatter(0x5EED)
        ctx.step(1)
        ctx.sync()
        ctx.set_profiling(1)
        ctx.step(2)
        ms, cnt = ctx.kernel_time()
    tf = 20.0 * n * n / (ms * 1e-3) / 1e12
    print(json.dumps({"lib": lib, "n": n, "force_ms": ms, "tflops": tf, "frac": tf / 157.3}), flush=True)


def main():
    a = sys.argv[1:]
    if a and a[0] == "--one":
        one(a[1], int(a[2]))
        return
    n, rounds = 1 << 21, 2
    while a and a[0].startswith("--"):
        if a[0] == "--n":
            n = int(a[1])
        elif a[0] == "--rounds":
            rounds = int(a[1])
        a = a[2:]
    res = {v: [] for v in a}
    for _ in range(rounds):
        for v in a:
            lib, *envs = v.split("@")
            env = dict(os.environ)
            for e in envs:
                k, val = e.split("=", 1)
                env[k] = val
            p = subprocess.run([sys.executable, __file__, "--one", lib, str(n)], env=env, capture_output=True,
                               text=True, timeout=600)
            if p.returncode:
                print(p.stderr[-2000:], flush=True)
                sys.exit(p.returncode)
            line = json.loads(p.stdout.strip().splitlines()[-1])
            print(json.dumps(dict(line, variant=v)), flush=True)
            res[v].append(line["force_ms"])
    for v, ms in res.items():
        m = statistics.median(ms)
        print(f"{v}: median force {m:.2f} ms = {20.0 * n * n / (m * 1e-3) / 1e12 / 157.3:.4f} of FP32 peak")


if __name__ == "__main__":
    main()
