"""Generate the committed golden fixtures (tests/golden/*.npz) from the CPU oracle.

    python tests/golden/make_golden.py

The reference ships no tests or golden vectors and cannot run here, so these
fixtures are the oracle's outputs (oracle/rps_oracle.c, single-threaded, -ffp-contract=off)
on small seeded inputs, frozen: tests/test_golden.py checks that the oracle still reproduces
them bit for bit (no drift of the checker), tests/test_gpu_golden.py runs librps on the same
inputs and compares with the stored outputs directly.  Each file stores its inputs, the
144-B ParticleConfig and the ExtConfig as raw bytes, and the expected outputs.
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

import oracle as orc  # noqa: E402
import rps_amd as rps  # noqa: E402
from helpers import config_c1, copy_soa, ext_c1_attractor, ext_verlet_1att, random_soa  # noqa: E402

F = np.float32


def raw(struct):
    return np.frombuffer(ctypes.string_at(ctypes.addressof(struct), ctypes.sizeof(struct)), np.uint8).copy()


def blob(n, seed):
    g = np.random.default_rng(seed)
    s = max(20.0, np.sqrt(n) * 1.2)
    return dict(x=np.clip(g.normal(0, s, n), -955, 955).astype(F),
                y=np.clip(g.normal(0, s * 0.6, n), -535, 535).astype(F),
                vx=g.normal(0, 30, n).astype(F), vy=g.normal(0, 30, n).astype(F))


def stream_case(name, cfg, ext, soa, steps):
    """`steps` frames of rps_step: frame_count += 1, then an active step (index = active steps
    so far) once frame_count >= ext.shader_delay (wgsl:426)."""
    out = copy_soa(soa)
    stats = None
    act = 0
    for f in range(1, steps + 1):
        if f >= ext.shader_delay:
            stats = orc.stream_step(cfg, ext, out, act, stats=True)
            act += 1
    d = dict(cfg=raw(cfg), ext=raw(ext), steps=np.array([steps]))
    for k, v in soa.items():
        if v is not None:
            d["in_" + k] = v
    for k in ("x", "y", "vx", "vy"):
        d["out_" + k] = out[k]
    if out.get("exp") is not None:
        d["out_exp"] = out["exp"]
        d["out_life"] = out["life"]
    d["out_colour"] = orc.set_color_array(out["vx"], out["vy"], cfg.max_energy)
    d["out_stats_bbox"] = np.array(list(stats.bbox), F)
    d["out_stats_respawned"] = np.array([stats.respawned], np.uint64)
    np.savez_compressed(os.path.join(HERE, name), **d)


def sph_case(name, n, seed, frames):
    """SPH frames with SHADER_DELAY 5: per-pass buffers of every frame."""
    cfg = rps.default_particle_config(n, gravity=100.0)
    ext = rps.make_ext()
    soa = blob(n, seed)
    st = orc.SphState(n)
    ref = copy_soa(soa)
    d = dict(cfg=raw(cfg), ext=raw(ext), frames=np.array([frames]))
    for k, v in soa.items():
        d["in_" + k] = v
    for f in range(1, frames + 1):
        cfg.frame_count = f
        st.grid(cfg, ref)
        if f >= 5:
            st.pre(cfg, ref)
            d[f"f{f}_pred"] = st.pred.copy()
            d[f"f{f}_dens"] = st.dens.copy()
            st.sim(cfg, ref)
        d[f"f{f}_lookup"] = st.lookup.copy()
        d[f"f{f}_offsets"] = st.offsets.copy()
    for k in ("x", "y", "vx", "vy"):
        d["out_" + k] = ref[k]
    np.savez_compressed(os.path.join(HERE, name), **d)


def nbody_case(name, n, seed):
    cfg = config_c1(rps, n, gravity=9.8)
    ext = rps.make_ext(nbody_strength=50.0, nbody_softening=2.0, drag=0.1, shader_delay=0)
    g = np.random.default_rng(seed)
    soa = dict(x=g.uniform(-900, 900, n).astype(F), y=g.uniform(-500, 500, n).astype(F),
               vx=g.normal(0, 20, n).astype(F), vy=g.normal(0, 20, n).astype(F))
    ax, ay = orc.nbody_accel(ext, soa["x"], soa["y"])
    out = copy_soa(soa)
    orc.nbody_integrate(cfg, ext, ax, ay, out)
    d = dict(cfg=raw(cfg), ext=raw(ext), out_ax=ax, out_ay=ay)
    for k in ("x", "y", "vx", "vy"):
        d["in_" + k] = soa[k]
        d["out_" + k] = out[k]
    np.savez_compressed(os.path.join(HERE, name), **d)


def main():
    orc.lib()
    # C1 reference subset: gravity + Euler + walls (compute_shader.wgsl:392-400, :69-99).
    cfg = config_c1(rps, 4096, gravity=9.8)
    stream_case("stream_c1_subset.npz", cfg, rps.make_ext(shader_delay=0),
                random_soa(4096, list(cfg.screen_bounds), seed=101), 4)
    # C1 as BASELINE.json configs[0] states it: 65 536 particles of the reference scatter, one
    # point attractor at the origin, Euler, SHADER_DELAY 5 (12 frames = 8 active steps).
    cfg = config_c1(rps, 65536, gravity=9.8)
    ext = ext_c1_attractor(rps)
    ext.shader_delay = 5
    parts = rps.setup_particles_scatter(cfg, 65536, seed=7)
    stream_case("stream_c1_attractor.npz", cfg, ext,
                dict(x=parts["position"][:, 0].copy(), y=parts["position"][:, 1].copy(),
                     vx=parts["velocity"][:, 0].copy(), vy=parts["velocity"][:, 1].copy()), 12)
    # C2 shape: velocity-Verlet + one attractor.
    cfg = config_c1(rps, 2048, gravity=0.0)
    stream_case("stream_c2_verlet.npz", cfg, ext_verlet_1att(rps),
                random_soa(2048, list(cfg.screen_bounds), seed=102), 5)
    # C3 features: 4 moving attractors, drag, lifetime expiry + Philox respawn, ragged n.
    cfg = config_c1(rps, 4099, gravity=0.0)
    ext = rps.headline_ext()
    ext.shader_delay = 0
    stream_case("stream_c3_features.npz", cfg, ext,
                random_soa(4099, list(cfg.screen_bounds), seed=103, life=(-0.05, 0.3)), 20)
    # SPH: non-pow2 (pads) and pow2, 7 frames (5 gated by SHADER_DELAY).
    sph_case("sph_n1000.npz", 1000, 104, 7)
    sph_case("sph_n2048.npz", 2048, 105, 7)
    # All-pairs (oracle accumulates in f64: GPU compared within the N-body tolerance).
    nbody_case("nbody_n1024.npz", 1024, 106)
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)), "B")


if __name__ == "__main__":
    main()
