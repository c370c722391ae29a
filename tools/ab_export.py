"""Same-box A/B of the render-interop export (rps_export_particles) between librps builds.

    python tools/ab_export.py [--n N] [--reps R] [--rounds K] LIB_A LIB_B ...

Each variant runs in its own subprocess (one librps per process), in rounds A, B, A, B, ...:
a 1e8-particle STREAM context (the headline state after its scatter), R exports into a
device buffer timed with HIP events (bench.py's export_side)."""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(lib, n, reps):
    sys.path.insert(0, os.path.join(ROOT, "rust-particle-system_amd", "python"))
    sys.path.insert(0, ROOT)
    import rps_amd as rps

    rps.LIB_PATH = os.path.abspath(lib)
    import bench

    cfg, ext = bench.workload(rps, n, 1)
    ctx = rps.Context(n, rps.MODE_STREAM, device=0)
    ctx.set_config(cfg, ext)
    ctx.init_scatter(0x5EED)
    ctx.step(5)
    ctx.sync()
    r = bench.export_side(ctx, n, reps)
    ctx.close()
    print(json.dumps({"lib": lib, "ms_per_export": r["ms_per_export"], "frac": r["roofline"]["frac"]}), flush=True)


def main():
    a = sys.argv[1:]
    if a and a[0] == "--one":
        one(a[1], int(a[2]), int(a[3]))
        return
    n, reps, rounds = 100_000_000, 40, 3
    while a and a[0].startswith("--"):
        if a[0] == "--n":
            n = int(a[1])
        elif a[0] == "--reps":
            reps = int(a[1])
        elif a[0] == "--rounds":
            rounds = int(a[1])
        a = a[2:]
    res = {v: [] for v in a}
    for _ in range(rounds):
        for v in a:
            p = subprocess.run([sys.executable, __file__, "--one", v, str(n), str(reps)], capture_output=True,
                               text=True, timeout=600)
            if p.returncode:
                print(p.stderr[-2000:], flush=True)
                sys.exit(p.returncode)
            res[v].append(json.loads(p.stdout.strip().splitlines()[-1])["ms_per_export"])
    for v, ms in res.items():
        print(f"n={n} {v}: median {statistics.median(ms):.4f} ms/export  (runs {', '.join(f'{m:.4f}' for m in ms)})")


if __name__ == "__main__":
    main()
