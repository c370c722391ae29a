"""The static sort schedules of rps_kernels.hip (sph_sort_head_kernel / sph_sort_tail_kernel),
replayed on the host with numpy: every lane's registers, the LDS tile (logical indices), the
DPP partners and the register chunks, exactly as the kernels index them.  They must equal the
reference's pass-per-dispatch bitonic network (compute_shader.wgsl:470-505 with the pass table of
src/particle_compute.rs:117-149) on a tile, including the order of equal keys, which the
network fixes (the payload is the original position).  CPU only: this pins the schedule
arithmetic; the GPU tests pin the kernels (test_gpu_sph.py)."""
import numpy as np
import pytest


def ref_network(keys, stages, first_stage=0, first_step=None):
    """(key, payload) pairs sorted by the reference's passes of stages [first_stage, stages)."""
    a = np.stack([keys, np.arange(len(keys))], 1).astype(np.int64)
    n = len(a)
    for stage in range(first_stage, stages):
        step0 = 0 if first_step is None or stage != first_stage else first_step
        for step in range(step0, stage + 1):
            G = 1 << (stage - step)
            flip = step == 0
            i = np.arange(n // 2)
            h = i % G
            left = h + 2 * G * (i // G)
            right = left + (2 * G - 1 - 2 * h if flip else G)
            sw = a[left, 0] > a[right, 0]
            l, r = a[left[sw]].copy(), a[right[sw]].copy()
            a[left[sw]], a[right[sw]] = r, l
    return a


def cas(v, i, j):
    """v: (threads, 8, 2) lane registers; compare-swap entries i, j of every lane."""
    sw = v[:, i, 0] > v[:, j, 0]
    a, b = v[sw, i].copy(), v[sw, j].copy()
    v[sw, i], v[sw, j] = b, a


def group_passes(v, K):
    M = 1 << K
    for m in range(K - 1, -1, -1):
        for j in range(M):
            if not j & (1 << m):
                cas(v, j, j + (1 << m))


def xlane(v, partner, rev, left):
    p = v[partner][:, ::-1] if rev else v[partner]
    p = p.copy()
    sw = np.where(left[:, None], v[:, :, 0] > p[:, :, 0], p[:, :, 0] > v[:, :, 0])
    v[sw] = p[sw]


def chunk_groups(nt, LNG):
    """chunk_group<LNG>: a wave's 64 * 2^LNG groups, consecutive lanes on consecutive groups."""
    t = np.arange(nt)
    return [((t >> 6) << (6 + LNG)) + (i << 6) + (t & 63) for i in range(1 << LNG)]


def lds_chunk(lds, nt, LG, K, LE=3):
    LGG = LG - K + 1
    g = 1 << LGG
    seen = []
    for q in chunk_groups(nt, LE - K):
        seen.append(q)
        e0 = ((q >> LGG) << (LG + 1)) + (q & (g - 1))
        idx = e0[:, None] + np.arange(1 << K)[None, :] * g
        v = lds[idx].copy()
        group_passes(v, K)
        lds[idx] = v
    q = np.concatenate(seen)
    assert len(q) == len(np.unique(q)) == len(lds) >> K  # every group exactly once


def reg_tail(v, t, S):
    """Strides 32 (xor-2 lanes), 16 (xor-1 lanes) when the stage has them, then 8 .. 1 in-lane."""
    if S >= 8:
        xlane(v, t ^ 2, False, (t & 2) == 0)
    if S >= 7:
        xlane(v, t ^ 1, False, (t & 1) == 0)
    group_passes(v, 4)


def mid_chunks(lds, nt, LG):
    """lds_mid_chunks: non-flip strides 2^LG down to 64, up to four passes per chunk."""
    while LG >= 6:
        K = min(4, LG - 5)
        lds_chunk(lds, nt, LG, K, 4)
        LG -= K


def tail16(tile, TLOG):
    """The sixteen-entries-per-thread tail (measured slower than the eight-entry kernel: DESIGN.md
    Appendix A); kept as a replayed alternative."""
    nt = 1 << (TLOG - 4)
    t = np.arange(nt)
    ia = t[:, None] + np.arange(16)[None, :] * nt
    v = tile[ia].copy()
    group_passes(v, 4)
    lds = np.zeros_like(tile)
    lds[ia] = v
    mid_chunks(lds, nt, TLOG - 5)
    v = lds[16 * t[:, None] + np.arange(16)[None, :]].copy()
    reg_tail(v, t, 8)
    return v.reshape(-1, 2)


def tail(tile, TLOG):
    """sph_sort_tail_kernel<TLOG> (rps_kernels.hip): eight entries per thread."""
    nt = 1 << (TLOG - 3)
    t = np.arange(nt)
    v = tile[t[:, None] + np.arange(8)[None, :] * nt].copy()
    group_passes(v, 3)
    lds = np.zeros_like(tile)
    lds[t[:, None] + np.arange(8)[None, :] * nt] = v
    LO = tail_lds_lo(TLOG)
    LG = TLOG - 4
    while LG >= LO:
        K = min(3, LG - LO + 1)
        lds_chunk(lds, nt, LG, K)
        LG -= K
    v = lds[8 * t[:, None] + np.arange(8)[None, :]].copy()
    if LO > 3:
        xlane(v, t ^ 1, False, (t & 1) == 0)
    group_passes(v, 3)
    return v.reshape(-1, 2)


def tail_lds_lo(TLOG):
    """kTailLdsLo<TLOG>: the last LDS stride's log2 (8192-entry tiles: stride 8 by DPP)."""
    return 4 if TLOG >= 13 else 3


def head_lds_lo(TLOG):
    """kHeadLdsLo<TLOG>: the last LDS stride's log2 (8192-entry tiles: strides 16, 8 by DPP)."""
    return 5 if TLOG >= 13 else 3


def xstrides(v, t, LG):
    """xlane_strides<LG>: strides 2^LG .. 32 as lane exchanges (lane t ^ 2^(LG-3) .. t ^ 4)."""
    while LG >= 5:
        D = 1 << (LG - 3)
        xlane(v, t ^ D, False, (t & D) == 0)
        LG -= 1
    return v


def reg_tail_x(v, t):
    """reg_tail<true>: strides 16 (xor-2 lanes), 8 (xor-1 lanes), then 4, 2, 1 in-lane."""
    xlane(v, t ^ 2, False, (t & 2) == 0)
    xlane(v, t ^ 1, False, (t & 1) == 0)
    group_passes(v, 3)


def mid_chunks_x(lds, nt, LG):
    """lds_mid_chunks_x<LG>: three-pass LDS chunks while the chunk's top stride is >= 512 entries;
    returns the top stride left for the lane exchanges (lds_mid_rem)."""
    while LG >= 9:
        lds_chunk(lds, nt, LG, 3)
        LG -= 3
    return LG


def tail_x(tile, TLOG):
    """The round-5 cross-lane tail (measured slower; the kernels run `tail`):
    strides TILE/2 .. TILE/8 on strided entries, LDS chunks for the strides that cross waves, the
    rest on each lane's eight consecutive entries by lane exchanges."""
    nt = 1 << (TLOG - 3)
    t = np.arange(nt)
    v = tile[t[:, None] + np.arange(8)[None, :] * nt].copy()
    group_passes(v, 3)
    lds = np.zeros_like(tile)
    lds[t[:, None] + np.arange(8)[None, :] * nt] = v
    LG = mid_chunks_x(lds, nt, TLOG - 4)
    v = lds[8 * t[:, None] + np.arange(8)[None, :]].copy()
    xstrides(v, t, LG)
    reg_tail_x(v, t)
    return v.reshape(-1, 2)


def head_x(tile, TLOG):
    """The round-5 cross-lane head (measured slower; the kernels run `head`):
    stages
    5 .. 8 (spans up to 512 = one wave) entirely by lane exchanges (the flip with the mirror lane,
    entries reversed), later stages' flip and cross-wave strides in LDS, the rest by lanes."""
    nt = 1 << (TLOG - 3)
    t = np.arange(nt)
    v = tile.reshape(nt, 8, 2).copy()
    for pairs in ([(0, 1), (2, 3), (4, 5), (6, 7)], [(0, 3), (1, 2), (4, 7), (5, 6)],  # reg_stages012
                  [(0, 1), (2, 3), (4, 5), (6, 7)], [(0, 7), (1, 6), (2, 5), (3, 4)],
                  [(0, 2), (1, 3), (4, 6), (5, 7)], [(0, 1), (2, 3), (4, 5), (6, 7)]):
        for i, j in pairs:
            cas(v, i, j)
    xlane(v, t ^ 1, True, (t & 1) == 0)  # stage 3
    group_passes(v, 3)
    xlane(v, t ^ 3, True, (t & 2) == 0)  # stage 4
    xlane(v, t ^ 1, False, (t & 1) == 0)
    group_passes(v, 3)
    lds = np.zeros_like(tile)
    own = 8 * t[:, None] + np.arange(8)[None, :]
    for S in range(5, TLOG):
        if S <= 8:
            M = 1 << (S - 2)  # lanes per flip block
            xlane(v, t ^ (M - 1), True, (t & (M // 2)) == 0)
            xstrides(v, t, S - 1)
        else:
            lds[own] = v
            g = 1 << (S - 1)
            LP = S - 2
            base = (t >> LP) << (S + 1)
            r = t & ((1 << LP) - 1)
            ia = base[:, None] + r[:, None] + np.arange(4)[None, :] * g
            ib = base[:, None] + (g - 1 - r)[:, None] + np.arange(4)[None, :] * g
            w = np.concatenate([lds[ia], lds[ib]], 1)
            for i, j in ((0, 7), (1, 6), (4, 3), (5, 2), (0, 1), (2, 3), (4, 5), (6, 7)):  # lds_flip_chunk
                cas(w, i, j)
            lds[ia], lds[ib] = w[:, :4], w[:, 4:]
            LG = mid_chunks_x(lds, nt, S - 2)
            v = lds[own].copy()
            xstrides(v, t, LG)
        reg_tail_x(v, t)
    return v.reshape(-1, 2)


def lane_stage(v, S):
    B = 1 << (S + 1)
    for b in range(0, 16, B):
        for r in range(B // 2):
            cas(v, b + r, b + B - 1 - r)
    for m in range(S - 1, -1, -1):
        for j in range(16):
            if not j & (1 << m):
                cas(v, j, j + (1 << m))


def head(tile, TLOG):
    """sph_sort_head_kernel<TLOG> after the bin (rps_kernels.hip): eight entries per thread."""
    nt = 1 << (TLOG - 3)
    t = np.arange(nt)
    v = tile.reshape(nt, 8, 2).copy()
    for pairs in ([(0, 1), (2, 3), (4, 5), (6, 7)], [(0, 3), (1, 2), (4, 7), (5, 6)],  # reg_stages012
                  [(0, 1), (2, 3), (4, 5), (6, 7)], [(0, 7), (1, 6), (2, 5), (3, 4)],
                  [(0, 2), (1, 3), (4, 6), (5, 7)], [(0, 1), (2, 3), (4, 5), (6, 7)]):
        for i, j in pairs:
            cas(v, i, j)
    xlane(v, t ^ 1, True, (t & 1) == 0)  # stage 3
    group_passes(v, 3)
    xlane(v, t ^ 3, True, (t & 2) == 0)  # stage 4
    xlane(v, t ^ 1, False, (t & 1) == 0)
    group_passes(v, 3)
    lds = np.zeros_like(tile)
    own = 8 * t[:, None] + np.arange(8)[None, :]
    for S in range(5, TLOG):
        lds[own] = v
        g = 1 << (S - 1)
        LP = S - 2
        base = (t >> LP) << (S + 1)
        r = t & ((1 << LP) - 1)
        ia = base[:, None] + r[:, None] + np.arange(4)[None, :] * g
        ib = base[:, None] + (g - 1 - r)[:, None] + np.arange(4)[None, :] * g
        w = np.concatenate([lds[ia], lds[ib]], 1)
        for i, j in ((0, 7), (1, 6), (4, 3), (5, 2), (0, 1), (2, 3), (4, 5), (6, 7)):  # lds_flip_chunk
            cas(w, i, j)
        lds[ia], lds[ib] = w[:, :4], w[:, 4:]
        LO = head_lds_lo(TLOG)
        LG = S - 2
        while LG >= LO:
            K = min(3, LG - LO + 1)
            lds_chunk(lds, nt, LG, K)
            LG -= K
        v = lds[own].copy()
        if LO > 3:
            if S >= 6:
                xlane(v, t ^ 2, False, (t & 2) == 0)
            xlane(v, t ^ 1, False, (t & 1) == 0)
        group_passes(v, 3)
    return v.reshape(-1, 2)


def head16(tile, TLOG):
    """The sixteen-entries-per-thread head (measured slower); kept as a replayed alternative."""
    nt = 1 << (TLOG - 4)
    t = np.arange(nt)
    v = tile.reshape(nt, 16, 2).copy()
    for S in range(4):
        lane_stage(v, S)
    xlane(v, t ^ 1, True, (t & 1) == 0)  # stage 4: flip across the lane pair
    group_passes(v, 4)
    xlane(v, t ^ 3, True, (t & 2) == 0)  # stage 5: flip across the lane quad
    xlane(v, t ^ 1, False, (t & 1) == 0)
    group_passes(v, 4)
    lds = np.zeros_like(tile)
    own = 16 * t[:, None] + np.arange(16)[None, :]
    for S in range(6, TLOG):
        lds[own] = v
        g = 1 << (S - 2)
        LP = S - 3
        base = (t >> LP) << (S + 1)
        r = t & ((1 << LP) - 1)
        ia = base[:, None] + r[:, None] + np.arange(8)[None, :] * g
        ib = base[:, None] + (g - 1 - r)[:, None] + np.arange(8)[None, :] * g
        w = np.concatenate([lds[ia], lds[ib]], 1)
        for j in range(4):
            cas(w, j, 15 - j)
            cas(w, 8 + j, 7 - j)
        for c in (0, 8):
            for m in (1, 0):
                for j in range(8):
                    if not j & (1 << m):
                        cas(w, c + j, c + j + (1 << m))
        lds[ia], lds[ib] = w[:, :8], w[:, 8:]
        mid_chunks(lds, nt, S - 3)
        v = lds[own].copy()
        reg_tail(v, t, S)
    return v.reshape(-1, 2)


def store_sixteen(v, t):
    """The quad transposition of store_sixteen: where each lane's sixteen entries land."""
    nt = len(t)
    out = np.full((nt * 16, 2), -1, dtype=v.dtype)
    for h in (0, 1):
        pairs = v[:, 8 * h:8 * h + 8].reshape(nt, 4, 2, 2)  # [lane, pair, entry, (key, payload)]
        # after two quad_swap_bit steps lane l's pair m is lane m's pair l (within the quad)
        q, l = t >> 2, t & 3
        for m in range(4):
            src = pairs[4 * q + m, l]  # lane (4q + m)'s pair l
            dst = 64 * q + 16 * m + 8 * h + 2 * l
            out[dst] = src[:, 0]
            out[dst + 1] = src[:, 1]
    return out


def quad_swap_bit(pairs, B):
    """quad_swap_bit<B> over every lane: lane l trades the pairs whose index bit B differs from
    its own bit B with lane l ^ 2^B's pair j ^ 2^B (pairs: [lane, pair, 2, 2])."""
    out = pairs.copy()
    for ln in range(len(pairs)):
        p = ln ^ (1 << B)
        for j in range(4):
            if ((j >> B) & 1) != ((ln >> B) & 1):
                out[ln, j] = pairs[p, j ^ (1 << B)]
    return out


def store_eight(v):
    """store_eight: the two quad_swap_bit steps, then store m of lane l = 4q + l' at entry
    32q + 8m + 2l' (one whole 64-B segment per quad and store instruction)."""
    nt = len(v)
    pairs = quad_swap_bit(quad_swap_bit(v.reshape(nt, 4, 2, 2), 1), 0)
    out = np.full((nt * 8, 2), -1, dtype=v.dtype)
    for ln in range(nt):
        for m in range(4):
            dst = 32 * (ln >> 2) + 8 * m + 2 * (ln & 3)
            out[dst:dst + 2] = pairs[ln, m]
    return out


def test_store_eight_writes_each_lane_to_its_entries():
    """Lane t's eight entries [8t, 8t + 8) land there after the DPP transposition."""
    v = np.stack([np.arange(512), 1000 + np.arange(512)], 1).reshape(64, 8, 2)
    np.testing.assert_array_equal(store_eight(v), v.reshape(-1, 2))


@pytest.mark.parametrize("TLOG", [11, 12, 13])
@pytest.mark.parametrize("kmax", [7, 1 << 20])
@pytest.mark.parametrize("layout", ["cross-lane", "eight", "sixteen"])
def test_head_schedule_equals_network(TLOG, kmax, layout):
    """eight: the kernels' schedule (every stage from 5 on through LDS); cross-lane (round 5) and
    sixteen (round 3): measured-slower alternatives, kept replayed."""
    g = np.random.default_rng(TLOG * 7 + (kmax & 3))
    keys = g.integers(0, kmax, 1 << TLOG)  # kmax 7: dense ties; 2^20: mostly distinct
    tile = np.stack([keys, np.arange(len(keys))], 1).astype(np.int64)
    run = {"cross-lane": head_x, "eight": head, "sixteen": head16}[layout]
    np.testing.assert_array_equal(run(tile, TLOG), ref_network(keys, TLOG))


@pytest.mark.parametrize("TLOG", [11, 12, 13])
@pytest.mark.parametrize("kmax", [7, 1 << 20])
@pytest.mark.parametrize("layout", ["cross-lane", "eight", "sixteen"])
def test_tail_schedule_equals_network(TLOG, kmax, layout):
    """A later stage s's passes inside one tile: strides 2^(TLOG-1) .. 1, non-flip (the tile
    after the stage's global passes; any input order)."""
    g = np.random.default_rng(TLOG * 11 + (kmax & 5))
    keys = g.integers(0, kmax, 1 << TLOG)
    tile = np.stack([keys, np.arange(len(keys))], 1).astype(np.int64)
    # the reference's stage-(TLOG) passes from step 1 (stride 2^(TLOG-1)) on a tile of 2^TLOG:
    # ref_network over stages [TLOG, TLOG+1) would need 2^(TLOG+1) entries, so run the non-flip
    # passes directly.
    a = tile.copy()
    n = len(a)
    for lg in range(TLOG - 1, -1, -1):
        G = 1 << lg
        i = np.arange(n // 2)
        left = i % G + 2 * G * (i // G)
        right = left + G
        sw = a[left, 0] > a[right, 0]
        l, r = a[left[sw]].copy(), a[right[sw]].copy()
        a[left[sw]], a[right[sw]] = r, l
    np.testing.assert_array_equal({"cross-lane": tail_x, "eight": tail, "sixteen": tail16}[layout](tile, TLOG), a)


def test_store_sixteen_places_each_lane_contiguously():
    """store_sixteen writes lane t's sixteen entries to [16t, 16t + 16), each store instruction
    (fixed m, h) covering one whole 64-B segment per lane quad."""
    nt = 64
    t = np.arange(nt)
    v = np.stack([np.arange(nt * 16), np.arange(nt * 16)], 1).reshape(nt, 16, 2)
    np.testing.assert_array_equal(store_sixteen(v, t), v.reshape(-1, 2))


def ref_passes(a, stage, steps):
    """The reference's passes (stage, step) for step in steps, on (key, payload) rows."""
    a = a.copy()
    n = len(a)
    for step in steps:
        G = 1 << (stage - step)
        flip = step == 0
        i = np.arange(n // 2)
        h = i % G
        left = h + 2 * G * (i // G)
        right = left + (2 * G - 1 - 2 * h if flip else G)
        sw = a[left, 0] > a[right, 0]
        l, r = a[left[sw]].copy(), a[right[sw]].copy()
        a[left[sw]], a[right[sw]] = r, l
    return a


def gather_stage(a, s, lg, T, LW, LE=3):
    """sph_sort_gather_kernel<T, LW, LE> over every workgroup (rps_kernels.hip)."""
    a = a.copy()
    P = len(a)
    TL = T + LW + 1
    TT, W = 1 << TL, 1 << LW
    gp = TT >> (LE - 1)
    M = 1 << (LE - 1)
    nt = TT >> LE
    g = 1 << lg
    rgs = lg - LW - 1
    blocks = (P >> (s + 1)) << rgs
    t = np.arange(nt)
    for blk in range(blocks):
        base = (blk >> rgs) << (s + 1)
        r0 = (blk & ((1 << rgs) - 1)) << LW
        tau = np.arange(TT)
        j, c, k = tau >> (LW + 1), (tau >> LW) & 1, tau & (W - 1)
        pos = base + j * g + np.where(c == 1, g - W - r0 + k, r0 + k)
        lds = a[pos].copy()
        ia = t[:, None] + np.arange(M)[None, :] * gp
        ib = (gp - 1 - t)[:, None] + np.arange(M)[None, :] * gp
        v = np.concatenate([lds[ia], lds[ib]], 1)
        for jj in range(M // 2):
            cas(v, jj, 2 * M - 1 - jj)
            cas(v, M + jj, M - 1 - jj)
        for m in range(LE - 3, -1, -1):
            for cc in (0, M):
                for jj in range(M):
                    if not jj & (1 << m):
                        cas(v, cc + jj, cc + jj + (1 << m))
        lds[ia], lds[ib] = v[:, :M], v[:, M:]
        LG, LO = TL - LE, LW + 1
        while LG - LO + 1 > LE:
            left = LG - LO + 1
            K = LE if (left - LE) % LE == 0 else (left - LE) % LE
            lds_chunk(lds, nt, LG, K, LE)
            LG -= K
        lds_chunk(lds, nt, LG, LG - LO + 1, LE)  # the last chunk (stored to memory by the kernel)
        a[pos] = lds
    return a


@pytest.mark.parametrize("T,LW,LE", [(5, 4, 3), (6, 4, 3), (7, 4, 3), (8, 4, 3), (9, 4, 4), (9, 3, 3)])
@pytest.mark.parametrize("kmax", [5, 1 << 20])
def test_gather_stage_schedule_equals_network(T, LW, LE, kmax):
    """A stage's T global passes (local tiles of 2^lg entries, stage s = lg + T - 1) as the
    gathered-tile launch runs them (2^LE entries per thread), against the reference's passes of
    that stage on the array."""
    lg = LW + 2
    s = lg + T - 1
    P = 1 << (s + 2)
    g = np.random.default_rng(T * 13 + LW + LE + (kmax & 7))
    keys = g.integers(0, kmax, P)
    a = np.stack([keys, np.arange(P)], 1).astype(np.int64)
    np.testing.assert_array_equal(gather_stage(a, s, lg, T, LW, LE), ref_passes(a, s, range(T)))


def cas_at(va, pa, vb, pb):
    """cas_at (rps_kernels.hip): the reference's compare-swap on entries at positions pa, pb
    (row-wise arrays), the lower position being the left one."""
    lo_a = pa < pb
    lk = np.where(lo_a, va[:, 0], vb[:, 0])
    rk = np.where(lo_a, vb[:, 0], va[:, 0])
    sw = lk > rk
    a, b = va[sw].copy(), vb[sw].copy()
    va[sw], vb[sw] = b, a


def folded_tail(a, s, TLOG, TG):
    """sph_sort_tail_kernel<TLOG, TG>: every position's value after stage s's first TG global
    passes, recomputed from its group (folded_global), then the tail's in-tile passes."""
    P = len(a)
    x = np.arange(P)
    m = (2 << s) - 1
    if TG == 1:
        A, MA = a[x].copy(), a[x ^ m].copy()
        cas_at(A, x, MA, x ^ m)
    else:
        h = 1 << (s - 1)
        A, B, MA, MB = a[x].copy(), a[x ^ h].copy(), a[x ^ m].copy(), a[x ^ h ^ m].copy()
        cas_at(A, x, MA, x ^ m)
        cas_at(B, x ^ h, MB, x ^ h ^ m)
        cas_at(A, x, B, x ^ h)
        cas_at(MA, x ^ m, MB, x ^ m ^ h)
    T = 1 << TLOG
    return np.concatenate([tail(A[k:k + T], TLOG) for k in range(0, P, T)])


@pytest.mark.parametrize("TLOG", [11, 13])
@pytest.mark.parametrize("TG", [1, 2])
@pytest.mark.parametrize("kmax", [5, 1 << 20])
def test_folded_tail_equals_network(TLOG, TG, kmax):
    """The folded tails of the first two later stages (s = TLOG, TLOG + 1): every pass of the
    stage, global and in-tile, equal to the reference's, ties included, over the whole array."""
    s = TLOG + TG - 1
    P = 1 << (s + 2)  # two blocks of the stage's span
    g = np.random.default_rng(TLOG * 7 + TG + (kmax & 3))
    keys = g.integers(0, kmax, P)
    a = np.stack([keys, np.arange(P)], 1).astype(np.int64)
    np.testing.assert_array_equal(folded_tail(a, s, TLOG, TG), ref_passes(a, s, range(s + 1)))


def cfold(a, x, lo, TG):
    """cfold<TG> (rps_kernels.hip): the value at each position x after the first TG global passes
    of stage s = lo + TG - 1, computed as the kernel does: the group held at c = u ^ ux (u = bits
    [lo, s] of a position, ux = x's), each pass's direction one bit of ux, x = v[0]."""
    M = 1 << TG
    s = lo + TG - 1
    ux = (x >> lo) & (M - 1)
    lowm = (1 << lo) - 1
    hi = x & ~((2 << s) - 1)
    v = []
    for c in range(M):
        low = np.where(c >> (TG - 1), ~x & lowm, x & lowm)
        v.append(a[hi | ((ux ^ c) << lo) | low].copy())

    def pas(dim, flip):
        d = ((ux >> dim) & 1) == 1  # c's partner is the left entry
        for c in range(M):
            if c & (1 << dim):
                continue
            c1 = c ^ (M - 1) if flip else c | (1 << dim)
            l = np.where(d[:, None], v[c1], v[c])
            r = np.where(d[:, None], v[c], v[c1])
            sw = l[:, 0] > r[:, 0]
            nl = np.where(sw[:, None], r, l)
            nr = np.where(sw[:, None], l, r)
            v[c] = np.where(d[:, None], nr, nl)
            v[c1] = np.where(d[:, None], nl, nr)

    pas(TG - 1, True)
    for b in range(TG - 2, -1, -1):
        pas(b, False)
    return v[0]


@pytest.mark.parametrize("TLOG,TG", [(11, 1), (11, 2), (11, 3), (11, 4), (11, 5), (12, 4), (13, 3)])
@pytest.mark.parametrize("kmax", [5, 1 << 16])
def test_compact_stage_equals_network(TLOG, TG, kmax):
    """sph_csort_stage_kernel<TLOG, TG>: every later stage of the compact sort (P <= 2^16) folds all
    its TG global passes (cfold) in front of the tail's in-tile passes; equal to the reference's
    passes of stage s = TLOG + TG - 1 over the whole array, ties included."""
    s = TLOG + TG - 1
    P = 1 << (s + 1) if TG >= 4 else 1 << (s + 2)  # whole blocks of the stage's span
    g = np.random.default_rng(TLOG * 5 + TG * 3 + (kmax & 7))
    keys = g.integers(0, kmax, P)
    a = np.stack([keys, np.arange(P)], 1).astype(np.int64)
    folded = cfold(a, np.arange(P), TLOG, TG)
    T = 1 << TLOG
    out = np.concatenate([tail(folded[k:k + T], TLOG) for k in range(0, P, T)])
    np.testing.assert_array_equal(out, ref_passes(a, s, range(s + 1)))


def test_compact_entries_fit():
    """The compact sort's packing: key << 16 | payload with key < N <= P <= 2^16 and payload < P;
    comparing the high halves orders by key alone (equal keys compare equal, whatever the
    payloads), as the reference's key compare (wgsl:494-503)."""
    g = np.random.default_rng(3)
    k = g.integers(0, 1 << 16, (1000, 2)).astype(np.uint32)
    p = g.integers(0, 1 << 16, (1000, 2)).astype(np.uint32)
    packed = (k << np.uint32(16)) | p
    np.testing.assert_array_equal((packed[:, 0] >> 16) > (packed[:, 1] >> 16), k[:, 0] > k[:, 1])
