"""How far the reference's own legal outcomes lie from the oracle's, one SPH frame at a time
(CPU only; the tolerance a comparison with a real wgpu run of compute_shader.wgsl must allow).

    python tools/wgsl_schedule_envelope.py [--n 4096 50000] [--warm 30] > profiles/<tag>_wgsl_schedule_envelope.txt

WGSL leaves three things to the implementation that change the SPH pass's results:
  * the intra-dispatch races: calculate_density reads other invocations'
    predicted_positions while pre_simulation_step writes them (wgsl:240 vs :430), and
    calculate_viscocity reads other particles' velocity while simulation_step writes it
    (:371 vs :410/:416/:452);
  * contraction of a*b+c into FMAs (WGSL permits it; the oracle and librps never contract).
From the same state (the oracle's after `warm` frames of bench.py's workload at N: the
reference scatter, every frame active), one frame is run under each of these outcomes and
compared with the oracle's frame (= librps's, bitwise):
  isolated pass 4     every density reads the other particles' predictions of the previous
                      frame (orc_sph_pre_stale; the interpreter's "isolated" schedule)
  lockstep pass 5     the viscosity scan sees the neighbours' post-pressure velocities
                      (orc_sph_sim_sched, one group; the interpreter's "lockstep")
  serial              one invocation after another in index order, as a serial CPU executor
  wg64 sequential     workgroups of 64 in lockstep, one after another in a random order
  fma                 the oracle's schedule with every a*b+c contracted (librps_oracle_fma.so)
The schedule restatements reproduce the interpreter's outcomes of the reference's shader bit
for bit (tests/test_wgsl_golden.py::test_oracle_schedule_restatements_match_reference_shader).
Reported per outcome, over the particles that are finite and not runaway (|v| <= 10x the 99th
percentile; at N != 2^k the pad hazard, SURVEY §0.5, sends some particles off to huge speeds):
particles whose state differs, |dv| over the 99th-percentile speed (median, 99th percentile,
max), max |dx| in smoothing radii, relative density difference (99th percentile, max)."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("rust-particle-system_amd/python", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))


def state(rps, orc, n, warm):
    cfg = rps.default_particle_config(n)
    parts = rps.setup_particles_scatter(cfg, n, seed=0x5EED)
    soa = dict(x=parts["position"][:, 0].copy(), y=parts["position"][:, 1].copy(),
               vx=parts["velocity"][:, 0].copy(), vy=parts["velocity"][:, 1].copy())
    st = orc.SphState(n, omp=True)
    for f in range(warm):
        cfg.frame_count = f + 1
        st.grid(cfg, soa)
        st.pre(cfg, soa)
        st.sim(cfg, soa)
    return cfg, soa, st


def one_frame(cfg, soa, st, mode, rng):
    from helpers import copy_soa

    s, c = copy_soa(soa), st.copy()
    c.omp = False
    c.grid(cfg, s)
    n = len(s["x"])
    if mode == "oracle":
        c.pre(cfg, s)
        c.sim(cfg, s)
    elif mode == "isolated pass 4":
        c.pre_stale(cfg, s)
        c.sim(cfg, s)
    elif mode == "lockstep pass 5":
        c.pre(cfg, s)
        c.sim_sched(cfg, s, [0], n)
    elif mode == "isolated 4 + lockstep 5":
        c.pre_stale(cfg, s)
        c.sim_sched(cfg, s, [0], n)
    elif mode == "serial":
        c.pre_sched(cfg, s, np.arange(n), 1)
        c.sim_sched(cfg, s, np.arange(n), 1)
    elif mode.startswith("wg64 sequential"):
        groups = (n + 63) // 64
        c.pre_sched(cfg, s, rng.permutation(groups), 64)
        c.sim_sched(cfg, s, rng.permutation(groups), 64)
    elif mode == "fma":
        c.pre(cfg, s, fma=True)
        c.sim(cfg, s, fma=True)
    else:
        raise ValueError(mode)
    return s, c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[4096, 65536, 50000])
    ap.add_argument("--warm", type=int, default=30)
    args = ap.parse_args()
    import oracle as orc
    import rps_amd as rps

    modes = ["isolated pass 4", "lockstep pass 5", "isolated 4 + lockstep 5", "serial", "wg64 sequential (1)",
             "wg64 sequential (2)", "wg64 sequential (3)", "fma"]
    print("# one SPH frame from the same state under the reference's other legal outcomes vs the oracle's "
          "(tools/wgsl_schedule_envelope.py)")
    for n in args.n:
        cfg, soa, st = state(rps, orc, n, args.warm)
        rng = np.random.default_rng(n)
        ref, rc = one_frame(cfg, soa, st, "oracle", rng)
        speed = np.hypot(ref["vx"], ref["vy"])
        fin = np.isfinite(speed) & np.isfinite(ref["x"]) & np.isfinite(ref["y"])
        vs = float(np.percentile(speed[fin], 99))  # the speed scale: runaway pad-hazard particles aside
        calm = fin & (speed <= 10.0 * vs)
        print(f"\n## N = {n}, after {args.warm} frames of the reference scatter (default config; 99th-percentile "
              f"|v| {vs:.1f}, smoothing radius {cfg.smoothing_radius}; {np.count_nonzero(~calm)} non-finite or runaway "
              f"(|v| > 10x that) particles excluded)")
        print(f"{'outcome':26} {'differ':>13} {'|dv|/v99: p50':>13} {'p99':>9} {'max':>9} {'max|dx|/r':>10} "
              f"{'drho/rho p99':>12} {'max':>9}")
        for mode in modes:
            s, c = one_frame(cfg, soa, st, mode, rng)
            ok = calm & np.isfinite(s["vx"]) & np.isfinite(s["vy"]) & np.isfinite(s["x"]) & np.isfinite(s["y"])
            differ = np.count_nonzero(((s["vx"] != ref["vx"]) | (s["vy"] != ref["vy"]) | (s["x"] != ref["x"])
                                       | (s["y"] != ref["y"])) & calm)
            dv = np.hypot(s["vx"][ok] - ref["vx"][ok], s["vy"][ok] - ref["vy"][ok]) / vs
            dx = np.hypot(s["x"][ok] - ref["x"][ok], s["y"][ok] - ref["y"][ok])
            d0, d1 = rc.dens[0::2][ok], c.dens[0::2][ok]
            rel = np.abs(d1 - d0) / np.maximum(np.abs(d0), 1e-30)
            print(f"{mode:26} {differ:>6}/{np.count_nonzero(calm):<6} {np.percentile(dv, 50):13.2e} "
                  f"{np.percentile(dv, 99):9.2e} {dv.max():9.2e} {dx.max() / cfg.smoothing_radius:10.2e} "
                  f"{np.percentile(rel, 99):12.2e} {rel.max():9.2e}", flush=True)

if __name__ == "__main__":
    main()
