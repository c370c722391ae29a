"""GPU all-pairs N-body (mode NBODY) against the double-precision oracle.

Tolerance: relative 1e-4 on the acceleration vector (v_rsq_f32 + FMA + f32 summation in
tile order vs an f64 direct sum).  The integration that follows is bitwise given
the device accelerations."""
import numpy as np
import pytest

from helpers import F, assert_soa_bitwise, config_c1, copy_soa

pytestmark = pytest.mark.gpu


def _abs_sum(ext, x, y):
    """sum_j |f_ij| per target (f64, chunked): the scale of f32 summation error when the
    net force is a cancelling sum of many large contributions."""
    x64, y64 = x.astype(np.float64), y.astype(np.float64)
    e2 = float(ext.nbody_softening) ** 2
    out = np.zeros(len(x))
    for lo in range(0, len(x), 1024):
        dx = x64[None, :] - x64[lo:lo + 1024, None]
        dy = y64[None, :] - y64[lo:lo + 1024, None]
        r2 = dx * dx + dy * dy + e2
        out[lo:lo + 1024] = (np.sqrt(dx * dx + dy * dy) * r2 ** -1.5).sum(1)
    return out * float(ext.nbody_strength)


def _check_accel(ax, ay, rx, ry, ext, x, y):
    """Relative 1e-4 of |a| where the sum does not cancel; where it does, the bound is the
    f32 summation error of the absolute contributions (1e-5 * sum_j |f_ij|)."""
    mag = np.hypot(rx.astype(np.float64), ry.astype(np.float64))
    err = np.hypot(ax.astype(np.float64) - rx, ay.astype(np.float64) - ry)
    bound = np.maximum(1e-4 * mag, 1e-5 * _abs_sum(ext, x, y))
    worst = np.max(err / bound)
    assert worst <= 1.0, worst
    assert np.median(err / np.maximum(mag, 1e-30)) < 1e-5


@pytest.mark.parametrize("n", [1000, 4096, 20000])
def test_nbody_accel_and_integrate(gpu, orc, n):
    rps = gpu
    cfg = config_c1(rps, n, gravity=3.0)
    ext = rps.make_ext(nbody_strength=50.0, nbody_softening=2.0, shader_delay=0)
    g = np.random.default_rng(n)
    soa = dict(x=g.uniform(-900, 900, n).astype(F), y=g.uniform(-500, 500, n).astype(F),
               vx=g.normal(0, 10, n).astype(F), vy=g.normal(0, 10, n).astype(F))
    with rps.Context(n, rps.MODE_NBODY) as ctx:
        ctx.set_config(cfg, ext)
        ctx.upload_soa(soa)
        ctx.step(1)
        ax = ctx.read_debug(rps.DEBUG_ACCEL_X)
        ay = ctx.read_debug(rps.DEBUG_ACCEL_Y)
        got = ctx.download_soa()
        amt, unit = ctx.step_cost()
        assert unit == "flops" and amt == 20.0 * n * n
    rx, ry = orc.nbody_accel(ext, soa["x"], soa["y"])
    _check_accel(ax, ay, rx, ry, ext, soa["x"], soa["y"])
    ref = copy_soa(soa)
    orc.nbody_integrate(cfg, ext, ax, ay, ref)
    assert_soa_bitwise(got, ref)


@pytest.mark.parametrize("n", [1, 2, 3, 5])
def test_nbody_tiny(gpu, orc, n):
    """Tiny N (one partial tile, mostly far-away pads): a lone particle feels exactly no
    force (its self term has dx = 0 and every pad adds +0); a few particles match the oracle
    within the tolerance; integration bitwise."""
    rps = gpu
    cfg = config_c1(rps, n, gravity=3.0)
    ext = rps.make_ext(nbody_strength=50.0, nbody_softening=2.0, shader_delay=0)
    g = np.random.default_rng(100 + n)
    soa = dict(x=g.uniform(-90, 90, n).astype(F), y=g.uniform(-50, 50, n).astype(F),
               vx=g.normal(0, 10, n).astype(F), vy=g.normal(0, 10, n).astype(F))
    with rps.Context(n, rps.MODE_NBODY) as ctx:
        ctx.set_config(cfg, ext)
        ctx.upload_soa(soa)
        ctx.step(1)
        ax = ctx.read_debug(rps.DEBUG_ACCEL_X)
        ay = ctx.read_debug(rps.DEBUG_ACCEL_Y)
        got = ctx.download_soa()
    if n == 1:
        assert ax[0] == 0.0 and ay[0] == 0.0
    else:
        rx, ry = orc.nbody_accel(ext, soa["x"], soa["y"])
        _check_accel(ax, ay, rx, ry, ext, soa["x"], soa["y"])
    ref = copy_soa(soa)
    orc.nbody_integrate(cfg, ext, ax, ay, ref)
    assert_soa_bitwise(got, ref)


def test_nbody_requires_softening(gpu):
    rps = gpu
    with rps.Context(256, rps.MODE_NBODY) as ctx:
        with pytest.raises(rps.RpsError):
            ctx.set_config(config_c1(rps, 256), rps.make_ext(nbody_strength=1.0, nbody_softening=0.0))


def test_nbody_shard_without_comm_is_rejected(gpu):
    rps = gpu
    with rps.Context(256, rps.MODE_NBODY, id_offset=256, global_count=512) as ctx:
        ctx.set_config(config_c1(rps, 512), rps.make_ext(nbody_strength=1.0, nbody_softening=1.0))
        with pytest.raises(rps.RpsError) as e:
            ctx.step(1)
        assert e.value.status == rps.RPS_ERR_COMM


def test_nbody_kernel_clock(gpu):
    """rps_get_kernel_clock: refused before a profiled force launch; afterwards the median over
    the launch's workgroups of their in-kernel s_memtime / s_memrealtime stamps, a plausible
    shader clock (MI355X: at most 2400 MHz), from every workgroup of the launch."""
    rps = gpu
    n = 1 << 16
    with rps.Context(n, rps.MODE_NBODY) as ctx:
        ctx.set_config(config_c1(rps, n), rps.make_ext(nbody_strength=10.0, nbody_softening=1.0, shader_delay=0))
        ctx.init_scatter(3)
        ctx.step(1)
        with pytest.raises(rps.RpsError):
            ctx.kernel_clock()
        ctx.set_profiling(1)
        ctx.step(2)
        mhz, wgs = ctx.kernel_clock()
        ms, launches = ctx.kernel_time()
    assert launches == 2 and ms > 0
    assert 300.0 < mhz < 2600.0, mhz
    assert wgs == 32 * 64  # 32 target blocks x 64 source splits (kNbodyMaxSplits), every one stamped


def test_nbody_single_rank_comm(gpu, orc):
    """RCCL path with one rank exercises rps_comm_init + the all-gather call."""
    rps = gpu
    n = 2048
    cfg = config_c1(rps, n)
    ext = rps.make_ext(nbody_strength=10.0, nbody_softening=1.0, shader_delay=0)
    g = np.random.default_rng(9)
    soa = dict(x=g.uniform(-900, 900, n).astype(F), y=g.uniform(-500, 500, n).astype(F),
               vx=np.zeros(n, F), vy=np.zeros(n, F))
    with rps.Context(n, rps.MODE_NBODY) as ctx:
        ctx.set_config(cfg, ext)
        ctx.comm_init(0, 1, rps.comm_unique_id())
        ctx.upload_soa(soa)
        ctx.step(1)
        ax = ctx.read_debug(rps.DEBUG_ACCEL_X)
        ay = ctx.read_debug(rps.DEBUG_ACCEL_Y)
    rx, ry = orc.nbody_accel(ext, soa["x"], soa["y"])
    _check_accel(ax, ay, rx, ry, ext, soa["x"], soa["y"])


def test_nbody_sharded_external_exchange(gpu, orc):
    """The sharded all-pairs data path on one GPU: 4 shard contexts (id_offset r*n, global
    4n) whose sources are exchanged by the caller (RPS_EXT_NBODY_EXTERNAL + rps_nbody_sources,
    device-to-device copies standing in for the ncclAllGather of multi-GPU runs).  Each
    shard's accelerations match the unsharded oracle for its targets; the integration given
    them is bitwise; two steps keep the shards consistent."""
    from hip_mem import copy_d2d

    rps = gpu
    R, n = 4, 2048
    N = R * n
    cfg = config_c1(rps, N)
    ext = rps.make_ext(nbody_strength=20.0, nbody_softening=1.5, drag=0.05, shader_delay=0)
    ext.flags |= rps.EXT_NBODY_EXTERNAL
    g = np.random.default_rng(77)
    full = dict(x=g.uniform(-900, 900, N).astype(F), y=g.uniform(-500, 500, N).astype(F),
                vx=g.normal(0, 10, N).astype(F), vy=g.normal(0, 10, N).astype(F))
    ctxs = [rps.Context(n, rps.MODE_NBODY, id_offset=r * n, global_count=N) for r in range(R)]
    try:
        for r, c in enumerate(ctxs):
            c.set_config(cfg, ext)
            c.upload_soa({k: v[r * n:(r + 1) * n] for k, v in full.items()})
        ref = copy_soa(full)
        for step in range(2):
            srcs = [c.nbody_sources(pack=True) for c in ctxs]
            assert all(cnt == N for _, cnt in srcs)
            for r in range(R):
                for q in range(R):
                    if q != r:
                        copy_d2d(srcs[r][0] + q * n * 8, srcs[q][0] + q * n * 8, n * 8)
            for c in ctxs:
                c.step(1)
            rx, ry = orc.nbody_accel(ext, ref["x"], ref["y"])
            got_ax = np.concatenate([c.read_debug(rps.DEBUG_ACCEL_X) for c in ctxs])
            got_ay = np.concatenate([c.read_debug(rps.DEBUG_ACCEL_Y) for c in ctxs])
            _check_accel(got_ax, got_ay, rx, ry, ext, ref["x"], ref["y"])
            orc.nbody_integrate(cfg, ext, got_ax, got_ay, ref)  # bitwise given the device accel
            got = {k: np.concatenate([c.download_soa()[k] for c in ctxs]) for k in ("x", "y", "vx", "vy")}
            assert_soa_bitwise(got, ref, what=f"step{step} ")
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("splits", [1, 2, 7])
def test_nbody_forced_split_variants(gpu, orc, monkeypatch, splits):
    """Both branches of the force launch at a small N: one source split (the kernel writes
    G*a directly, the variant every launch with >= 2048 target blocks runs, e.g. the bench's
    2^22 and the C4 2^24 step) and several splits (partials + the fixed-order reduce),
    forced per context with RPS_NBODY_SPLITS."""
    rps = gpu
    monkeypatch.setenv("RPS_NBODY_SPLITS", str(splits))
    n = 6000
    cfg = config_c1(rps, n)
    ext = rps.make_ext(nbody_strength=30.0, nbody_softening=1.0, shader_delay=0)
    g = np.random.default_rng(100 + splits)
    soa = dict(x=g.uniform(-900, 900, n).astype(F), y=g.uniform(-500, 500, n).astype(F),
               vx=np.zeros(n, F), vy=np.zeros(n, F))
    with rps.Context(n, rps.MODE_NBODY) as ctx:
        ctx.set_config(cfg, ext)
        ctx.upload_soa(soa)
        ctx.step(1)
        ax = ctx.read_debug(rps.DEBUG_ACCEL_X)
        ay = ctx.read_debug(rps.DEBUG_ACCEL_Y)
    rx, ry = orc.nbody_accel(ext, soa["x"], soa["y"])
    _check_accel(ax, ay, rx, ry, ext, soa["x"], soa["y"])


_TARGET_BLOCK = 2048  # targets per workgroup of nbody_accel_kernel (256 lanes x 8)


def _block_sample(n, extra=()):
    """One target in every 2048-target block of a launch over n targets, its place in the
    block varying from block to block (lane t % 256 and pair slot t // 256 % 8 both cycle), plus
    the first and last targets: a block-index, lane or pair-slot bug anywhere shows."""
    blocks = (n + _TARGET_BLOCK - 1) // _TARGET_BLOCK
    b = np.arange(blocks, dtype=np.uint64)
    t = b * _TARGET_BLOCK + (b * np.uint64(769) + np.uint64(13)) % np.uint64(_TARGET_BLOCK)
    t = np.minimum(t, np.uint64(n - 1))
    return np.unique(np.concatenate([t, np.array([0, n - 1] + list(extra), np.uint64)]))


def _check_sampled(orc, ext, idx, gx, gy, sx, sy, what=""):
    """The device accelerations of targets `idx` against the f64 oracle over every source
    (orc_nbody_accel_ref's bits, vectorised over the targets), with the bound of the small
    tests: 1e-4 of |a|, or 1e-5 of G * sum_j |f_ij| where the sum cancels; median 1e-5."""
    rx, ry, ab = orc.nbody_accel_ref_idx(ext, sx, sy, idx)
    mag = np.hypot(rx.astype(np.float64), ry.astype(np.float64))
    err = np.hypot(gx.astype(np.float64) - rx, gy.astype(np.float64) - ry)
    ratio = err / np.maximum(1e-4 * mag, 1e-5 * ab)
    worst = int(np.argmax(ratio))
    assert ratio[worst] <= 1.0, (what, int(idx[worst]), float(ratio[worst]))
    assert np.median(err / mag) < 1e-5, (what, float(np.median(err / mag)))
    return float(ratio[worst])


@pytest.mark.parametrize("n,splits", [(1 << 22, None), (1 << 22, "1"), (1 << 24, None)])
def test_nbody_full_size(gpu, orc, monkeypatch, n, splits):
    """2^22 targets over 2^22 sources -- the all-pairs step at its round-5 bench size: the
    default source splits (12 at this size) and one forced split (the kernel writes G*a
    directly) -- and BASELINE.json's C4 config, 2^24 over 2^24 (bench.py's `allpairs` line;
    8192 target blocks x 3 source splits; one step is ~45 s on one MI355X).  One target in
    every 2048-target block (2 048 / 8 192 targets, each summing every split's sources) is
    checked against the f64 oracle over every source; the integration of every particle given
    the device accelerations is bitwise."""
    if splits:
        monkeypatch.setenv("RPS_NBODY_SPLITS", splits)
    rps = gpu
    cfg = config_c1(rps, n)
    ext = rps.make_ext(nbody_strength=1.0e3, nbody_softening=1.0, shader_delay=0)
    g = np.random.default_rng(2024)
    soa = dict(x=g.uniform(-950, 950, n).astype(F), y=g.uniform(-530, 530, n).astype(F),
               vx=g.normal(0, 10, n).astype(F), vy=g.normal(0, 10, n).astype(F))
    with rps.Context(n, rps.MODE_NBODY) as ctx:
        ctx.set_config(cfg, ext)
        ctx.upload_soa(soa)
        ctx.step(1)
        ax = ctx.read_debug(rps.DEBUG_ACCEL_X)
        ay = ctx.read_debug(rps.DEBUG_ACCEL_Y)
        got = ctx.download_soa()
    idx = _block_sample(n, extra=(2048 * 8 + 5, n // 2 + 123))
    assert len(idx) >= n // _TARGET_BLOCK
    _check_sampled(orc, ext, idx, ax[idx], ay[idx], soa["x"], soa["y"], what=f"n={n}")
    ref = copy_soa(soa)
    orc.nbody_integrate(cfg, ext, ax, ay, ref)
    assert_soa_bitwise(got, ref)


@pytest.mark.parametrize("splits", [None, "3"])
def test_nbody_c5_rank_shard(gpu, orc, monkeypatch, splits):
    """BASELINE.json's C5 (2^27 particles all-pairs over 8 x MI355X) as one rank sees it, on
    one GPU: rank 7's targets start at id_offset 7 * 2^24 and its sources are all 2^27 global
    particles -- the 1-GiB float2 array its ncclAllGather would fill, filled here by the test
    (RPS_EXT_NBODY_EXTERNAL + rps_nbody_sources, host -> device) -- so the source loop, the
    64-bit source and target offsets and the splits run at C5's shape.  2^20 targets (the
    full 2^24-target shard is ~6 min on one GPU; the kernel's work per target is the same):
    the default split count for that launch, and 3 splits, what a full 2^24-target C5 shard
    picks (8192 target blocks x 3 >= 24 576).  One target in every one of the 512 target
    blocks against the f64 oracle over every one of the 2^27 sources (the bound of the other
    full-size tests); integration bitwise.  The full 2^24-target shard: tools/c5_rank_shard.py
    (profiles/r06_c5_rank_shard.txt)."""
    from hip_mem import copy_h2d

    if splits:
        monkeypatch.setenv("RPS_NBODY_SPLITS", splits)
    rps = gpu
    ng, n = 1 << 27, 1 << 20
    off = 7 << 24
    cfg = config_c1(rps, min(ng, 0xFFFFFFFF))
    ext = rps.make_ext(nbody_strength=1.0e3, nbody_softening=1.0, shader_delay=0)
    ext.flags |= rps.EXT_NBODY_EXTERNAL
    g = np.random.default_rng(27)
    pos = np.empty((ng, 2), F)
    pos[:, 0] = g.uniform(-950, 950, ng).astype(F)
    pos[:, 1] = g.uniform(-530, 530, ng).astype(F)
    soa = dict(x=pos[off:off + n, 0].copy(), y=pos[off:off + n, 1].copy(),
               vx=g.normal(0, 10, n).astype(F), vy=g.normal(0, 10, n).astype(F))
    with rps.Context(n, rps.MODE_NBODY, id_offset=off, global_count=ng) as ctx:
        ctx.set_config(cfg, ext)
        ctx.upload_soa(soa)
        src, cnt = ctx.nbody_sources(pack=True)
        assert cnt == ng
        copy_h2d(src, pos[:off])  # the other ranks' shards, as the all-gather would place them
        copy_h2d(src + (off + n) * 8, pos[off + n:])
        ctx.step(1)
        ax = ctx.read_debug(rps.DEBUG_ACCEL_X)
        ay = ctx.read_debug(rps.DEBUG_ACCEL_Y)
        got = ctx.download_soa()
    sx, sy = np.ascontiguousarray(pos[:, 0]), np.ascontiguousarray(pos[:, 1])
    del pos
    rel = _block_sample(n, extra=(2048 * 8 + 5, n // 2 + 123))
    _check_sampled(orc, ext, rel + np.uint64(off), ax[rel], ay[rel], sx, sy, what=f"splits={splits}")
    ref = copy_soa(soa)
    orc.nbody_integrate(cfg, ext, ax, ay, ref)
    assert_soa_bitwise(got, ref)
