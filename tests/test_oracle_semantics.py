"""The C oracle against the independent numpy restatement (bitwise), plus the
size-independent properties the path has (no GPU)."""
import numpy as np
import pytest

import ref_numpy as RN
from helpers import (F, assert_bitwise, assert_soa_bitwise, cfg_dict, config_c1, copy_soa,
                     ext_c1_attractor, ext_dict, ext_verlet_1att, random_soa)


def _run_both(orc, cfg, ext, soa, step=0, id_offset=0):
    a = copy_soa(soa)
    orc.stream_step(cfg, ext, a, step, id_offset)
    b = RN.stream_step(cfg_dict(cfg), ext_dict(ext), soa, step, id_offset)
    return a, b


@pytest.mark.parametrize("gravity", [0.0, 9.8, 1000.0])
def test_reference_subset_matches_numpy(rps, orc, gravity):
    # gravity -> Euler -> wall clamp (wgsl:397-400, :392-395, :69-99)
    cfg = config_c1(rps, 4096, gravity=gravity)
    ext = rps.make_ext(shader_delay=0)
    soa = random_soa(4096, list(cfg.screen_bounds), seed=11)
    a, b = _run_both(orc, cfg, ext, soa)
    assert_soa_bitwise(a, b)


def test_attractor_euler_and_drag_match_numpy(rps, orc):
    cfg = config_c1(rps, 4096)
    ext = rps.headline_ext()
    ext.flags = 0  # no lifetime: attractors + drag only
    soa = random_soa(4096, list(cfg.screen_bounds), seed=12)
    for step in (0, 1, 777):
        a, b = _run_both(orc, cfg, ext, soa, step)
        assert_soa_bitwise(a, b, what=f"step{step} ")


def test_verlet_matches_numpy(rps, orc):
    cfg = config_c1(rps, 4096, gravity=9.8)
    ext = ext_verlet_1att(rps)
    soa = random_soa(4096, list(cfg.screen_bounds), seed=13)
    a, b = _run_both(orc, cfg, ext, soa, 5)
    assert_soa_bitwise(a, b)


def test_lifetime_respawn_matches_numpy(rps, orc):
    cfg = config_c1(rps, 8192)
    ext = rps.headline_ext()
    soa = random_soa(8192, list(cfg.screen_bounds), seed=14, life=(-0.5, 0.5))
    a, b = _run_both(orc, cfg, ext, soa, step=42, id_offset=123456789)
    assert (b["life"] > 0).all()
    assert_soa_bitwise(a, b, keys=("x", "y", "vx", "vy", "exp", "life"))


def test_respawn_lands_in_emitter_disc(rps, orc):
    cfg = config_c1(rps, 4096)
    ext = rps.headline_ext()
    soa = random_soa(4096, list(cfg.screen_bounds), seed=15, life=(-1.0, -0.5))  # all die
    st = orc.stream_step(cfg, ext, soa, 3, stats=True)
    assert st.respawned == 4096
    r = np.hypot(soa["x"], soa["y"])
    assert (r <= 50.0 + 1e-3).all()
    # lifetimes U(1, 5) s quantised to whole steps: ceil(L / dt) * dt
    dt = cfg.fixed_delta_time
    assert ((soa["life"] >= 1.0) & (soa["life"] <= 5.0 + dt)).all()
    spd = np.hypot(soa["vx"], soa["vy"])
    assert (spd <= 100.0 + 1e-3).all()


def test_sharded_equals_unsharded(rps, orc):
    """Index-range sharding: rank r owns [r*N/R, (r+1)*N/R) with global ids, so
    the concatenated shards equal the unsharded step bit for bit."""
    cfg = config_c1(rps, 6000)
    ext = rps.headline_ext()
    soa = random_soa(6000, list(cfg.screen_bounds), seed=16, life=(-0.2, 3.0))
    whole = copy_soa(soa)
    orc.stream_step(cfg, ext, whole, 9, 0)
    parts = []
    for r in range(4):
        lo, hi = r * 1500, (r + 1) * 1500
        s = {k: v[lo:hi].copy() for k, v in soa.items()}
        orc.stream_step(cfg, ext, s, 9, lo)
        parts.append(s)
    for k in ("x", "y", "vx", "vy", "exp", "life"):
        assert_bitwise(np.concatenate([p[k] for p in parts]), whole[k], k)


def test_omp_build_equals_serial(rps, orc):
    cfg = config_c1(rps, 20000)
    ext = rps.headline_ext()
    soa = random_soa(20000, list(cfg.screen_bounds), seed=17, life=(-0.2, 3.0))
    a, b = copy_soa(soa), copy_soa(soa)
    orc.stream_step(cfg, ext, a, 4)
    orc.stream_step_omp(cfg, ext, b, 4, threads=4)
    assert_soa_bitwise(a, b, keys=("x", "y", "vx", "vy", "exp"))


@pytest.mark.parametrize("n", [20000, 1 << 15])
def test_omp_sph_equals_serial(rps, orc, n):
    """The OpenMP build of the five SPH passes (bench.py's SPH cpu_baseline) equals the serial
    checker bit for bit: lookup, offsets, densities, predictions and state over 3 frames
    (n = 20 000: non-pow2 pads)."""
    cfg = rps.default_particle_config(n, gravity=100.0)
    g = np.random.default_rng(n)
    soa = dict(x=np.clip(g.normal(0, 200, n), -955, 955).astype(F), y=np.clip(g.normal(0, 120, n), -535, 535).astype(F),
               vx=g.normal(0, 30, n).astype(F), vy=g.normal(0, 30, n).astype(F))
    a, b = copy_soa(soa), copy_soa(soa)
    sa, sb = orc.SphState(n), orc.SphState(n, omp=True, threads=4)
    ext = rps.make_ext(shader_delay=0)
    orc.run_steps(2, cfg, ext, a, 3, sph=sa)
    orc.run_steps(2, cfg, ext, b, 3, sph=sb)
    for name in ("lookup", "offsets", "dens", "pred"):
        assert_bitwise(getattr(sb, name), getattr(sa, name), name)
    assert_soa_bitwise(b, a)


def test_run_steps_gating(rps, orc):
    # frame_count < SHADER_DELAY (=5) gates passes 4-5 (wgsl:426, :442): 4 inert steps.
    cfg = config_c1(rps, 256, gravity=9.8)
    ext = rps.make_ext()
    soa = random_soa(256, list(cfg.screen_bounds), seed=18)
    ref = copy_soa(soa)
    fc, act = orc.run_steps(0, cfg, ext, soa, 4)
    assert (fc, act) == (4, 0)
    assert_soa_bitwise(soa, ref)
    fc, act = orc.run_steps(0, cfg, ext, soa, 1, fc, act)
    assert (fc, act) == (5, 1)
    orc.stream_step(cfg, ext, ref, 0)
    assert_soa_bitwise(soa, ref)


# ------------------------------------------------------------------------------------
# Bitonic network (wgsl:470-505 + src/particle_buffers.rs:108-138)
# ------------------------------------------------------------------------------------
@pytest.mark.parametrize("P", [2, 8, 64, 1024])
def test_bitonic_network_sorts_and_pairs_disjoint(P):
    g = np.random.default_rng(P)
    keys = list(g.integers(0, max(2, P // 3), P))
    for gw, flip in RN.bitonic_passes(P):
        seen = set()
        for l, r in RN.bitonic_pairs(P, gw, flip):
            assert r < P and l not in seen and r not in seen
            seen.update((l, r))
            if keys[l] > keys[r]:
                keys[l], keys[r] = keys[r], keys[l]
    assert keys == sorted(keys)


@pytest.mark.parametrize("n", [64, 1000])
def test_sph_oracle_matches_numpy(rps, orc, n):
    """Per-pass SPH restatements agree bitwise, incl. the non-pow2 pad hazard."""
    cfg = rps.default_particle_config(n, gravity=50.0)
    # A compact blob so cells hold several neighbours.
    g = np.random.default_rng(n)
    soa = dict(x=g.normal(0, 30, n).astype(F), y=g.normal(0, 30, n).astype(F),
               vx=g.normal(0, 20, n).astype(F), vy=g.normal(0, 20, n).astype(F))
    st = orc.SphState(n)
    a = copy_soa(soa)
    lookup_py = [[0, 0] for _ in range(st.P)]
    b = copy_soa(soa)
    cd = cfg_dict(cfg)
    for frame in range(1, 8):
        active = frame >= 5
        passes = st.grid(cfg, a)
        assert passes == (st.P.bit_length() - 1) * st.P.bit_length() // 2
        if active:
            st.pre(cfg, a)
        off_np, dens_np, pred_np = RN.sph_step(cd, b, lookup_py, active)
        assert_bitwise(st.lookup, np.array(lookup_py, np.uint32).reshape(-1), f"lookup f{frame}")
        assert_bitwise(st.offsets, np.array(off_np, np.uint32), f"offsets f{frame}")
        if active:
            assert_bitwise(st.dens, dens_np.reshape(-1), f"dens f{frame}")
            assert_bitwise(st.pred, pred_np.reshape(-1), f"pred f{frame}")
            st.sim(cfg, a)
            assert_soa_bitwise(a, b, what=f"f{frame} ")
    if n & (n - 1):
        # non-pow2: zero-initialised pads (key 0, idx 0) sort into the visible window.
        assert (st.lookup[: 2 * n : 2] == 0).sum() > 0


def test_nbody_oracle_matches_direct_sum(rps, orc):
    ext = rps.make_ext(nbody_strength=2.0, nbody_softening=0.5, shader_delay=0)
    g = np.random.default_rng(5)
    x = g.uniform(-100, 100, 300).astype(F)
    y = g.uniform(-100, 100, 300).astype(F)
    ax, ay = orc.nbody_accel(ext, x, y)
    dx = x[None, :].astype(np.float64) - x[:, None]
    dy = y[None, :].astype(np.float64) - y[:, None]
    inv3 = (dx * dx + dy * dy + 0.25) ** -1.5
    np.testing.assert_allclose(ax, 2.0 * (dx * inv3).sum(1), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(ay, 2.0 * (dy * inv3).sum(1), rtol=1e-5, atol=1e-6)
    sx, sy = orc.nbody_accel(ext, x, y, t0=100, nt=50)
    assert_bitwise(sx, ax[100:150])
    assert_bitwise(sy, ay[100:150])


def test_nbody_f32_baseline_port_close_to_oracle(rps, orc):
    """bench.py's all-pairs cpu_baseline computes the same force (f32, its own summation
    order): within f32 rounding of the f64-accumulated oracle."""
    ext = rps.make_ext(nbody_strength=1.0e5, nbody_softening=1.0, shader_delay=0)
    g = np.random.default_rng(9)
    x = g.uniform(-960, 960, 2000).astype(F)
    y = g.uniform(-540, 540, 2000).astype(F)
    ax, ay = orc.nbody_accel(ext, x, y)
    bx, by = orc.nbody_accel_f32_omp(ext, x, y, threads=2)
    err = np.hypot(bx - ax, by - ay) / np.hypot(ax, ay)
    assert float(np.median(err)) < 1e-5 and float(err.max()) < 1e-3
    tx, ty = orc.nbody_accel_f32_omp(ext, x, y, t0=500, nt=100, threads=2)
    assert_bitwise(tx, bx[500:600])
    assert_bitwise(ty, by[500:600])


def test_nbody_reference_with_abs_sum(rps, orc):
    """orc_nbody_accel_ref (the full-size N-body tests' checker, OpenMP over targets): the same
    accelerations as orc_nbody_accel bit for bit at any thread count, and G * sum_j |f_ij|
    equal to a numpy f64 direct sum."""
    ext = rps.make_ext(nbody_strength=3.0, nbody_softening=0.7, shader_delay=0)
    g = np.random.default_rng(12)
    x = g.uniform(-200, 200, 1500).astype(F)
    y = g.uniform(-100, 100, 1500).astype(F)
    ax, ay = orc.nbody_accel(ext, x, y, t0=200, nt=300)
    for threads in (1, 3):
        rx, ry, ab = orc.nbody_accel_ref(ext, x, y, t0=200, nt=300, threads=threads)
        assert_bitwise(rx, ax)
        assert_bitwise(ry, ay)
    dx = x[None, :].astype(np.float64) - x[200:500, None]
    dy = y[None, :].astype(np.float64) - y[200:500, None]
    d2 = dx * dx + dy * dy
    ref = 3.0 * (np.sqrt(d2) * (d2 + F(0.7) * F(0.7)) ** -1.5).sum(1)
    np.testing.assert_allclose(ab, ref, rtol=1e-12)
