"""Test helpers: canonical configs, dict views for the numpy restatement, and
bitwise comparison utilities."""
import math

import numpy as np

F = np.float32


def config_c1(rps, n=65536, gravity=9.8):
    """C1: reference streaming subset at the 1920x1080 viewport (src/main.rs:136-153)."""
    return rps.default_particle_config(n, gravity=gravity, pressure_multiplier=0.0,
                                       near_density_multiplier=0.0, viscocity_strength=0.0)


def ext_reference(rps, shader_delay=5):
    return rps.make_ext(shader_delay=shader_delay)


def ext_verlet_1att(rps, seed=0x5EED):
    """C2: one attractor at the origin, velocity-Verlet."""
    return rps.make_ext(rps.VERLET, [dict(center=(0.0, 0.0), strength=1.0e5, softening=1.0)],
                        seed=seed, shader_delay=0)


def ext_c1_attractor(rps):
    return rps.make_ext(rps.EULER, [dict(center=(0.0, 0.0), strength=1.0e5, softening=1.0)],
                        shader_delay=0)


def cfg_dict(cfg):
    return dict(dt=cfg.fixed_delta_time, gravity=cfg.gravity, damping=cfg.damping_factor,
                bounds=list(cfg.screen_bounds), n=cfg.particle_count, radius=cfg.smoothing_radius,
                norms=(cfg.density_kernel_norm, cfg.near_density_kernel_norm, cfg.viscocity_kernel_norm),
                target_density=cfg.target_density, pressure_mult=cfg.pressure_multiplier,
                near_mult=cfg.near_density_multiplier, visc_strength=cfg.viscocity_strength,
                max_energy=cfg.max_energy)


def ext_dict(ext):
    d = dict(integrator=ext.integrator, drag=ext.drag, seed=ext.seed)
    d["attractors"] = [dict(center=(a.center[0], a.center[1]), orbit_radius=a.orbit_radius,
                            angular_velocity=a.angular_velocity, phase=a.phase, strength=a.strength,
                            softening=a.softening) for a in ext.attractors[: ext.num_attractors]]
    if ext.flags & 1:
        d["lifetime"] = (ext.life_min, ext.life_max)
        d["emitter"] = dict(center=(ext.emitter_center[0], ext.emitter_center[1]),
                            radius=ext.emitter_radius, speed=(ext.spawn_speed_min, ext.spawn_speed_max))
    return d


def random_soa(n, bounds, seed=1, vmax=200.0, life=None):
    """Seeded random state inside `bounds` (some particles on/over the walls)."""
    g = np.random.default_rng(seed)
    x0, x1, y0, y1 = bounds
    soa = dict(
        x=g.uniform(x0 - 5, x1 + 5, n).astype(F),
        y=g.uniform(y0 - 5, y1 + 5, n).astype(F),
        vx=g.uniform(-vmax, vmax, n).astype(F),
        vy=g.uniform(-vmax, vmax, n).astype(F),
    )
    if life is not None:
        soa["life"] = g.uniform(life[0], life[1], n).astype(F)
    return soa


def copy_soa(s):
    return {k: (None if v is None else v.copy()) for k, v in s.items()}


def assert_bitwise(a, b, what=""):
    """Bit-for-bit equality; for f32, any NaN equals any NaN.  IEEE 754 (and WGSL) leave NaN
    payloads and signs unspecified: the GPU's generated NaN is 0x7fc00000, x86's 0xffc00000,
    and a negate modifier flips a propagated NaN's sign on one side and not the other.  No
    non-NaN value on the path depends on a payload (comparisons, i32 casts and |v| ignore it),
    so every non-NaN bit still has to match."""
    a = np.ascontiguousarray(a).reshape(-1)
    b = np.ascontiguousarray(b).reshape(-1)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    ia = a.view(np.uint32) if a.dtype == np.float32 else a
    ib = b.view(np.uint32) if b.dtype == np.float32 else b
    diff = ia != ib
    if a.dtype == np.float32:
        diff &= ~(np.isnan(a) & np.isnan(b))
    bad = np.nonzero(diff)[0]
    if len(bad):
        i = bad[0]
        raise AssertionError(f"{what}: {len(bad)} of {a.size} differ; first at {i}: {a[i]!r} ({ia[i]:#010x}) "
                             f"vs {b[i]!r} ({ib[i]:#010x})")


def assert_soa_bitwise(a, b, keys=("x", "y", "vx", "vy"), what=""):
    for k in keys:
        assert_bitwise(a[k], b[k], f"{what}{k}")


def soa_to_particles(rps, soa):
    p = np.zeros(len(soa["x"]), dtype=rps.PARTICLE_DTYPE)
    p["position"][:, 0] = soa["x"]
    p["position"][:, 1] = soa["y"]
    p["velocity"][:, 0] = soa["vx"]
    p["velocity"][:, 1] = soa["vy"]
    p["color"] = 1.0
    return p
