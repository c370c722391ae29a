"""Known-answer tests pinning the CPU oracle (no GPU).

The reference ships no tests or golden vectors, so the oracle is pinned by
(a) values that follow directly from the reference's constants and formulas, computed here
independently of the oracle, (b) published Random123 Philox4x32-10 KAT vectors, and (c) a
second restatement in numpy (tests/ref_numpy.py, see test_oracle_semantics.py)."""
import math
import struct

import numpy as np
import pytest

import ref_numpy as RN

F = np.float32


def f32_bits(v):
    return struct.unpack("<I", struct.pack("<f", float(v)))[0]


def test_kernel_norms_match_reference_formula(rps):
    # src/main.rs:96-98 with SMOOTHING_RADIUS = 3*3 = 9 (src/main.rs:26-27), f32 arithmetic.
    d, nd, v = rps.kernel_norms(9.0)
    assert f32_bits(d) == 0x38621930  # 5.3906057e-05
    assert f32_bits(nd) == 0x3716BB75  # 8.9843425e-06
    assert f32_bits(v) == 0x32FE12E5  # 2.9578084e-08
    # 9^8 = 43046721 is not an f32; powf rounds it to 43046720.
    assert np.power(F(9.0), F(8.0), dtype=F) == F(43046720.0)


def test_hash_cell_known_answers(orc):
    # compute_shader.wgsl:132-142, u32 wrapping.
    assert orc.lib().orc_hash_cell(0, 1) == 9737333
    assert orc.lib().orc_cell_key(0, 1, 50000) == 37333
    assert orc.lib().orc_cell_key(0, 1, 65536) == 38005
    assert orc.lib().orc_hash_cell(-1, -1) == 4285214140
    assert orc.lib().orc_cell_key(-1, -1, 50000) == 14140
    assert orc.lib().orc_cell_key(-1, -1, 65536) == 11708
    assert orc.lib().orc_hash_cell(106, 60) == 585917218
    for cx, cy in [(0, 0), (5, -7), (-100000, 3), (2**31 - 1, -(2**31))]:
        assert orc.lib().orc_hash_cell(cx, cy) == RN.hash_cell(cx, cy)


def test_only_cell_00_maps_to_key0_at_default_viewport(orc):
    # at 1920x1080 / r=9 / N=50000 only cell (0,0) has key 0.
    hits = [(cx, cy) for cx in range(0, 1920 // 9 + 1) for cy in range(0, 1080 // 9 + 1)
            if orc.lib().orc_cell_key(cx, cy, 50000) == 0]
    assert hits == [(0, 0)]


@pytest.mark.parametrize("P,passes", [(2**16, 136), (2**20, 210), (2**24, 300), (2**27, 378)])
def test_bitonic_pass_counts(P, passes):
    # src/particle_compute.rs:117-149: S(S+1)/2 dispatches, S = log2 P.
    S = P.bit_length() - 1
    assert S * (S + 1) // 2 == passes


def test_f32_to_i32_semantics(orc):
    f = orc.lib().orc_f32_to_i32
    assert f(1.9) == 1 and f(-1.9) == -1 and f(-0.5) == 0
    assert f(3.0e9) == 2**31 - 1 and f(-3.0e9) == -(2**31)
    assert f(float("nan")) == 0


# Random123 kat_vectors for philox4x32-10 (counter, key -> output).
PHILOX_KAT = [
    ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
    ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
    ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
     [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
]


@pytest.mark.parametrize("ctr,key,out", PHILOX_KAT)
def test_philox_kat(orc, ctr, key, out):
    assert list(orc.philox(ctr, key)) == out
    got = RN.philox4x32_10(*[np.array([c], np.uint64) for c in ctr], key[0], key[1])
    assert [int(g[0]) for g in got] == out


def test_sincos_turns_accuracy_and_restatement(orc):
    u = (np.arange(0, 1 << 24, 997, dtype=np.uint32)).astype(F) * F(1.0 / 16777216.0)
    c_np, s_np = RN.sincos_turns(u)
    assert np.max(np.abs(c_np - np.cos(2 * np.pi * u.astype(np.float64)))) < 2e-6
    assert np.max(np.abs(s_np - np.sin(2 * np.pi * u.astype(np.float64)))) < 2e-6
    for k in range(0, len(u), 1013):
        c, s = orc.sincos_turns(float(u[k]))
        assert f32_bits(c) == f32_bits(c_np[k]) and f32_bits(s) == f32_bits(s_np[k])


def test_set_color_known_answers(orc):
    # compute_shader.wgsl:101-118 with max_energy = 2000 (src/main.rs:35).
    assert list(orc.set_color(0.0, 0.0, 2000.0)) == [0.0, 0.0, 1.0, 1.0]  # blue at rest
    v = math.sqrt(2000.0)  # E = 1000 = 0.5 * max -> t = 0 on the green->red ramp
    c = orc.set_color(v, 0.0, 2000.0)
    assert c[2] == 0.0 and c[3] == 1.0 and abs(c[1] - 1.0) < 1e-5
    assert list(orc.set_color(1000.0, 0.0, 2000.0)) == [1.0, 0.0, 0.0, 1.0]  # saturated red
    g = np.random.default_rng(3)
    vx = g.uniform(-100, 100, 2000).astype(F)
    vy = g.uniform(-100, 100, 2000).astype(F)
    vec = orc.set_color_array(vx, vy, 2000.0)
    for i in range(0, 2000, 97):
        assert np.array_equal(orc.set_color(float(vx[i]), float(vy[i]), 2000.0).view(np.uint32),
                              vec[i].view(np.uint32))


def test_attractor_inv_sqrt_accuracy(orc):
    """The attractor force's 1/sqrt (bit guess + 3 Newton steps) is within
    2.5 ulp of the exact value over 60 decades, and the C oracle equals the numpy restatement."""
    import ref_numpy as RN

    g = np.random.default_rng(3)
    r = np.exp(g.uniform(np.log(1e-30), np.log(1e30), 200_000)).astype(np.float32)
    y = RN.inv_sqrt(r)
    exact = 1.0 / np.sqrt(r.astype(np.float64))
    ulp = np.spacing(exact.astype(np.float32)).astype(np.float64)
    assert (np.abs(y.astype(np.float64) - exact) / ulp).max() <= 2.5
    for v in r[:2000]:
        assert np.float32(orc.inv_sqrt(float(v))).view(np.uint32) == RN.inv_sqrt(np.array([v], np.float32)).view(np.uint32)[0]


def test_life_steps_kat(orc):
    """Lifetime quantisation clamp(ceil(L/dt), 1, 65535)."""
    dt = np.float32(0.01)
    assert orc.life_steps(0.0, dt) == 1
    assert orc.life_steps(-3.0, dt) == 1
    assert orc.life_steps(float("nan"), dt) == 1
    assert orc.life_steps(1e9, dt) == 65535
    assert orc.life_steps(0.005, dt) == 1
    assert orc.life_steps(1.0, dt) == int(np.ceil(np.float32(1.0) / dt))
    assert orc.life_steps(5.0, dt) == int(np.ceil(np.float32(5.0) / dt))


def test_log_unit_accuracy_and_restatement(orc):
    """The initial scatter's fixed-op ln (orc_log_unit; device log_unit): within 2 ulp of the
    exact ln over every Box-Muller input u = k/2^24, k = 1..2^24, and the numpy restatement
    equals the C oracle bit for bit on a sample (incl. both ends and the sqrt(2) split)."""
    k = np.arange(1, (1 << 24) + 1, dtype=np.float64)
    u = (k / 16777216.0).astype(F)
    got = RN.log_unit(u)
    exact = np.log(u.astype(np.float64))
    ulp = np.spacing(np.abs(exact).astype(F)).astype(np.float64)
    nz = u != F(1.0)
    assert np.max(np.abs(got[nz].astype(np.float64) - exact[nz]) / ulp[nz]) <= 2.0
    assert got[-1] == F(0.0)
    g = np.random.default_rng(4)
    idx = np.concatenate([[0, 1, 2, (1 << 24) - 1], g.integers(0, 1 << 24, 20000)])
    m = np.float32(1.41421356)
    edge = np.array([m, np.nextafter(m, F(2)), np.nextafter(m, F(0))], F) * F(0.25)
    for v in np.concatenate([u[idx], edge]):
        assert f32_bits(orc.log_unit(float(v))) == f32_bits(RN.log_unit(np.array([v], F))[0]), v


def test_init_scatter_matches_numpy(rps, orc):
    """orc_init_scatter's x and y (Philox + sincos_turns + log_unit Box-Muller, clamped) equal
    the numpy restatement bit for bit, on a shard with a 64-bit id offset."""
    cfg = rps.default_particle_config(50000)
    ext = rps.headline_ext()
    for off, total in ((0, 50000), ((1 << 33) + 7, 1 << 34)):
        soa = orc.init_scatter(cfg, ext, 0xABCDEF0123, 50000, id_offset=off, global_count=total)
        x, y = RN.init_scatter(list(cfg.screen_bounds), 0xABCDEF0123, 50000, id_offset=off, global_count=total)
        assert np.array_equal(soa["x"].view(np.uint32), x.view(np.uint32))
        assert np.array_equal(soa["y"].view(np.uint32), y.view(np.uint32))
        assert (y > cfg.screen_bounds[2]).mean() > 0.99
