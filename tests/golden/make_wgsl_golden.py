"""Golden fixtures from the reference's own shader: tests/golden/wgsl_*.npz.

    python tests/golden/make_wgsl_golden.py        (needs /root/reference; run in the dev container)

`assets/compute_shader.wgsl` of the reference is parsed and executed by tests/wgsl_interp.py
and driven by tests/wgsl_harness.py exactly as the reference's host code dispatches it (five
passes per frame, frame_count advanced first, SHADER_DELAY gating inside the shader).  The
shader source is read at generation time only; each file stores the inputs, the 144-B
ParticleConfig, and every frame's buffers after the frame: particles (x, y, vx, vy, colour),
spatial_lookup, spatial_lookup_offsets, and from the first active frame particle_densities
and predicted_positions.  Consumers: tests/test_wgsl_golden.py (the oracle, CPU) and
tests/test_gpu_golden.py (librps on the GPU).
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(ROOT, "rust-particle-system_amd", "python"), os.path.join(ROOT, "oracle"),
          os.path.dirname(HERE)):
    if p not in sys.path:
        sys.path.insert(0, p)

import rps_amd as rps  # noqa: E402
import wgsl_harness as H  # noqa: E402
from helpers import config_c1, random_soa  # noqa: E402

F = np.float32
ONLY = sys.argv[1:]  # regenerate just these fixtures (file names); default: all


def raw(struct):
    return np.frombuffer(ctypes.string_at(ctypes.addressof(struct), ctypes.sizeof(struct)), np.uint8).copy()


def blob(n, seed):
    g = np.random.default_rng(seed)
    s = max(20.0, np.sqrt(n) * 1.2)
    return dict(x=np.clip(g.normal(0, s, n), -955, 955).astype(F), y=np.clip(g.normal(0, s * 0.6, n), -535, 535).astype(F),
                vx=g.normal(0, 30, n).astype(F), vy=g.normal(0, 30, n).astype(F))


def case(name, cfg, soa, frames, schedules=None):
    """schedules: {frame: (pre, sim)} -- frames run under the interpreter's other schedules
    (stored as sched_pre / sched_sim per frame: 0 lockstep, 1 isolated)."""
    if ONLY and name not in ONLY:
        return
    out = H.run_reference(cfg, soa, frames, schedules=schedules)
    d = dict(cfg=raw(cfg), frames=np.array([frames]))
    code = {"lockstep": 0, "isolated": 1}
    sch = [(schedules or {}).get(f, ("lockstep", "isolated")) for f in range(1, frames + 1)]
    d["sched_pre"] = np.array([code[a] for a, _ in sch], np.uint8)
    d["sched_sim"] = np.array([code[b] for _, b in sch], np.uint8)
    for k in ("x", "y", "vx", "vy"):
        d["in_" + k] = soa[k]
    for f, buf in enumerate(out, start=1):
        for k in ("x", "y", "vx", "vy", "color", "lookup", "offsets"):
            d[f"f{f}_{k}"] = buf[k]
        if f >= 5:  # SHADER_DELAY (wgsl:66): densities / predictions exist from frame 5
            d[f"f{f}_dens"] = buf["dens"]
            d[f"f{f}_pred"] = buf["pred"]
    np.savez_compressed(os.path.join(HERE, name), **d)
    print(name, os.path.getsize(os.path.join(HERE, name)), "B", flush=True)


def main():
    if not H.available():
        sys.exit(f"{H.REF_SHADER} not found: the fixtures are generated in the dev container")
    # SPH, power-of-two N (no pads), gravity on: 7 frames, the last 3 active.
    case("wgsl_sph_n64.npz", rps.default_particle_config(64, gravity=100.0), blob(64, 5), 7)
    # SPH, non-pow2 N: the next_pow2 lookup's zero pad entries sort into [0, N).
    case("wgsl_sph_n100.npz", rps.default_particle_config(100, gravity=100.0), blob(100, 6), 7)
    # ... run until a particle pushed out of [0, N) has density 0 and its NaN spreads.
    case("wgsl_sph_n100_nan.npz", rps.default_particle_config(100, gravity=100.0), blob(100, 6), 11)
    # SPH at the reference defaults (gravity 0, default density), the reference scatter.
    n = 512
    scale = (n / 50000) ** 0.5
    cfg = rps.default_particle_config(n, screen_bounds=rps.screen_bounds_for(1920.0 * scale, 1080.0 * scale))
    parts = rps.setup_particles_scatter(cfg, n, seed=11)
    case("wgsl_sph_n512_default.npz", cfg,
         dict(x=parts["position"][:, 0].copy(), y=parts["position"][:, 1].copy(),
              vx=parts["velocity"][:, 0].copy(), vy=parts["velocity"][:, 1].copy()), 6)
    # SPH with particles far beyond the walls (cells off the grid, hashed like any other) and
    # a non-default radius and viewport.
    n = 200
    cfg = rps.default_particle_config(n, gravity=100.0, smoothing_radius=14.0,
                                      screen_bounds=rps.screen_bounds_for(2400.0, 1400.0))
    soa = blob(n, 8)
    soa["x"][:6] = F(2000.0)
    soa["y"][6:12] = F(-3000.0)
    case("wgsl_sph_n200_outside.npz", cfg, soa, 7)
    # Tiny N: P = 1 (no sort pass), 2, 4 (one pad) and 32 (15 pads); a lone particle is its
    # own only neighbour.
    for n, seed in ((1, 21), (2, 22), (3, 23), (17, 24)):
        soa = blob(n, seed)
        soa["x"] *= F(0.2)
        soa["y"] *= F(0.2)
        case(f"wgsl_sph_n{n}_tiny.npz", rps.default_particle_config(n, gravity=100.0), soa, 7)
    # The shader's other legal outcomes of its intra-dispatch races: frames
    # whose pass 4 runs "isolated" (every density reads the other particles' predictions of the
    # previous frame) and / or pass 5 "lockstep" (the viscosity scan sees the neighbours'
    # post-pressure velocities).  The oracle's schedule restatements (orc_sph_pre_stale,
    # orc_sph_sim_sched with one group) must reproduce them; tools/wgsl_schedule_envelope.py
    # measures how far these outcomes lie from the oracle's at larger N.
    sched = {5: ("isolated", "isolated"), 6: ("lockstep", "lockstep"), 7: ("isolated", "lockstep")}
    case("wgsl_sph_n64_sched.npz", rps.default_particle_config(64, gravity=100.0), blob(64, 5), 8, sched)
    case("wgsl_sph_n100_sched.npz", rps.default_particle_config(100, gravity=100.0), blob(100, 6), 8, sched)
    # The streaming reference subset (C1): pressure, near-pressure and viscosity multipliers
    # zero, so each active frame is gravity -> Euler -> walls -> colour; particles on and
    # beyond the walls.
    cfg = config_c1(rps, 128, gravity=9.8)
    case("wgsl_stream_c1_n128.npz", cfg, random_soa(128, list(cfg.screen_bounds), seed=107), 9)


if __name__ == "__main__":
    main()
