"""SPH ms/frame against the frame index (run on the GPU box).

    python tools/sph_frame_curve.py [--n 50000 65536] [--frames 300] [--window 10]

bench.py's `sph.reference_sizes` workload (default config at N, the reference scatter, seed
0x5EED, every frame active) stepped from frame 0 in windows of `window` frames, each timed with
one HIP event pair on the context stream (rps_time_steps).  Per window: ms/frame and, from
rps_sph_frame_cost of the window's last frame, the entries the reference's scans visit per
particle (E / N) and the sort launches.  At P != N (N = 50 000, P = 2^16) the pad hazard's stale
duplicates change the runs from frame to frame, so a frame's cost depends on which
frames a tool times; the summary lines give the mean over bench.py's window (frames 20..219)
and tools/ab_sph.py's old window (10..59)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-particle-system_amd", "python"))


def curve(rps, n, frames, window):
    cfg = rps.default_particle_config(n)
    parts = rps.setup_particles_scatter(cfg, n, seed=0x5EED)
    rows = []
    with rps.Context(n, rps.MODE_SPH) as ctx:
        ctx.set_config(cfg, rps.make_ext(shader_delay=0))
        ctx.upload(parts)
        ctx.step(1)  # code objects loaded, first frame's allocations touched (frame 0 not in a window)
        ctx.sync()
        f = 1
        while f + window <= frames:
            ms = ctx.time_steps(window) / window
            cost = ctx.sph_frame_cost()
            rows.append((f, f + window - 1, ms, cost["scanned_entries"] / n, cost["sort_launches"]))
            f += window
    return rows


def mean_over(rows, lo, hi):
    """Frame-weighted mean ms/frame of the windows inside frames [lo, hi]."""
    sel = [(b - a + 1, ms) for a, b, ms, _, _ in rows if a >= lo and b <= hi]
    return sum(k * ms for k, ms in sel) / sum(k for k, _ in sel) if sel else float("nan")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[50000, 65536])
    ap.add_argument("--frames", type=int, default=301)
    ap.add_argument("--window", type=int, default=10)
    args = ap.parse_args()
    import rps_amd as rps

    for n in args.n:
        rows = curve(rps, n, args.frames, args.window)
        print(f"# N = {n} (P = {1 << max(0, (n - 1).bit_length())}), windows of {args.window} active frames")
        print(f"{'frames':>11} {'ms/frame':>9} {'E/N':>7} {'sort launches':>13}")
        for a, b, ms, e, sl in rows:
            print(f"{a:>5}..{b:<5} {ms:9.4f} {e:7.2f} {sl:13d}")
        print(f"N={n}: frames 20..219 (bench.py window) {mean_over(rows, 20, 219):.4f} ms/frame (windows from 21); "
              f"frames 10..59 (ab_sph.py r05 window) {mean_over(rows, 10, 59):.4f} (windows from 11); "
              f"frames 1..10 {mean_over(rows, 1, 10):.4f}; last 50 {mean_over(rows, rows[-1][1] - 49, rows[-1][1]):.4f}",
              flush=True)


if __name__ == "__main__":
    main()
