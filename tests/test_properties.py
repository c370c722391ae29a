"""Property-based checks of the oracle (hypothesis, CPU only, derandomized
so every run draws the same examples).  Each property ties the C restatement to a second,
independent statement of the reference's arithmetic (tests/ref_numpy.py or plain Python
integers) over inputs the fixed-vector tests do not reach."""
import ctypes

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import ref_numpy as RN
from helpers import assert_bitwise, config_c1, copy_soa, random_soa

SETTINGS = settings(max_examples=200, derandomize=True, deadline=None,
                    suppress_health_check=[HealthCheck.function_scoped_fixture])
I32 = st.integers(min_value=-(1 << 31), max_value=(1 << 31) - 1)


@SETTINGS
@given(cx=I32, cy=I32, n=st.integers(min_value=1, max_value=(1 << 27)))
def test_hash_and_key_wrap_like_u32(orc, cx, cy, n):
    """hash_cell (wgsl:132-137) wraps modulo 2^32 and the key is hash % N (wgsl:139-142)
    for every i32 cell coordinate, negative ones included."""
    L = orc.lib()
    h = RN.hash_cell(cx, cy)
    assert L.orc_hash_cell(cx, cy) == h
    assert L.orc_cell_key(cx, cy, n) == h % n


@SETTINGS
@given(v=st.floats(width=32, allow_nan=True, allow_infinity=True))
def test_f32_to_i32_truncates_and_saturates(orc, v):
    """i32(f32) (particle_position_to_cell_coord, wgsl:121-130): truncation toward zero,
    saturation at the i32 range, NaN -> 0."""
    assert orc.lib().orc_f32_to_i32(ctypes.c_float(v)) == RN.f32_to_i32(np.float32(v))


def _network_sort(entries):
    """The reference's bitonic schedule (src/particle_buffers.rs:108-138, wgsl:480-504) run
    pass by pass over (key, index) pairs, swapping on key only."""
    e = [tuple(x) for x in entries]
    P = len(e)
    for gw, flip in RN.bitonic_passes(P):
        for l, r in RN.bitonic_pairs(P, gw, flip):
            if e[l][0] > e[r][0]:
                e[l], e[r] = e[r], e[l]
    return e


@SETTINGS
@given(log_p=st.integers(min_value=0, max_value=8), data=st.data())
def test_bitonic_sort_permutation_with_ties(orc, log_p, data):
    """The oracle's sort leaves every entry -- ties included, whose order fixes the neighbour
    summation order -- exactly where the pass-by-pass network does, for key sets dense in
    duplicates."""
    P = 1 << log_p
    keys = data.draw(st.lists(st.integers(min_value=0, max_value=max(1, P // 4)), min_size=P, max_size=P))
    lookup = np.zeros(2 * P, np.uint32)
    lookup[0::2] = keys
    lookup[1::2] = np.arange(P, dtype=np.uint32)
    want = _network_sort(zip(keys, range(P)))
    orc.lib().orc_sph_sort(lookup.ctypes.data_as(ctypes.c_void_p), P)
    got = list(zip(lookup[0::2].tolist(), lookup[1::2].tolist()))
    assert got == want


@settings(max_examples=25, derandomize=True, deadline=None,
          suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(n=st.integers(min_value=2, max_value=3000), cut=st.floats(min_value=0.0, max_value=1.0),
       step=st.integers(min_value=0, max_value=1 << 20), seed=st.integers(min_value=0, max_value=1 << 16))
def test_sharding_at_any_cut(rps, orc, n, cut, step, seed):
    """Index-range sharding cut anywhere: two shards with global ids step to the
    same bits as the whole, for the headline extensions at any active step (respawn keyed by
    global id and step)."""
    cfg = config_c1(rps, n)
    ext = rps.headline_ext()
    soa = random_soa(n, list(cfg.screen_bounds), seed=seed, life=(-0.05, 2.0))
    whole = copy_soa(soa)
    orc.stream_step(cfg, ext, whole, step, 0)
    k = int(cut * n)
    parts = []
    for lo, hi in ((0, k), (k, n)):
        s = {key: v[lo:hi].copy() for key, v in soa.items()}
        if hi > lo:
            orc.stream_step(cfg, ext, s, step, lo)
        else:  # an empty shard
            s["exp"] = np.zeros(0, np.uint16)
        parts.append(s)
    for key in ("x", "y", "vx", "vy", "exp"):
        assert_bitwise(np.concatenate([p[key] for p in parts]), whole[key], key)


@SETTINGS
@given(u=st.floats(min_value=float(np.finfo(np.float32).tiny), max_value=1.0, width=32))
def test_log_unit_restatements_agree(orc, u):
    """The fixed-op ln of the Box-Muller scatter (A11): C and numpy restatements agree bit for
    bit and stay within 2 ulp of the exact ln for every normal u in (0, 1] (the scatter draws
    u = k / 2^24, never subnormal; the exponent split assumes a normal input)."""
    c = np.float32(orc.log_unit(u))
    r = np.float32(RN.log_unit(np.float32(u)))
    assert c.view(np.uint32) == r.view(np.uint32)
    exact = np.log(np.float64(np.float32(u)))
    ulp = np.spacing(np.float32(exact)) if exact != 0 else np.float32(1e-45)
    assert abs(np.float64(c) - exact) <= 2 * abs(np.float64(ulp)) + 1e-45
