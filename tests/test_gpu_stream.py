"""GPU parity of the streaming step (mode STREAM) against the CPU oracle, through the C ABI.

Bar: bitwise for every field (x, y, vx, vy, life and the raw u16 expiry), every step — the kernels and the oracle
both compute IEEE f32 with no contraction and correctly-rounded div/sqrt."""
import numpy as np
import pytest

from helpers import (F, assert_bitwise, assert_soa_bitwise, config_c1, copy_soa, ext_c1_attractor,
                     ext_verlet_1att, random_soa, soa_to_particles)

pytestmark = pytest.mark.gpu

KEYS5 = ("x", "y", "vx", "vy", "life")
KEYS_STEPS = ("x", "y", "vx", "vy", "steps")


def _download_chunk(rps, ctx, start, n):
    """x, y, vx, vy and the exact lifetime steps left of particles [start, start+n)."""
    fields = (rps.FIELD_X, rps.FIELD_Y, rps.FIELD_VX, rps.FIELD_VY, rps.FIELD_LIFE_STEPS)
    return {k: ctx.download_field(f, start, n) for k, f in zip(KEYS_STEPS, fields)}


def _gpu_ctx(rps, n, cfg, ext, soa, id_offset=0, global_count=0):
    ctx = rps.Context(n, rps.MODE_STREAM, id_offset=id_offset, global_count=global_count)
    ctx.set_config(cfg, ext)
    ctx.upload_soa(soa)
    return ctx


def test_c1_reference_subset_with_shader_delay(gpu, orc):
    """C1: 65 536 particles, reference scatter, gravity + Euler + walls, SHADER_DELAY 5."""
    rps = gpu
    n = 65536
    cfg = config_c1(rps, n, gravity=9.8)
    ext = rps.make_ext()  # reference semantics
    parts = rps.setup_particles_scatter(cfg, n, seed=7)
    with rps.Context(n) as ctx:
        ctx.set_config(cfg, ext)
        ctx.upload(parts)
        got0 = ctx.download()
        assert np.array_equal(got0["color"], np.ones((n, 4), F))  # spawn colour before stepping
        assert_bitwise(got0["position"].reshape(-1), parts["position"].reshape(-1), "upload")
        soa = dict(x=parts["position"][:, 0].copy(), y=parts["position"][:, 1].copy(),
                   vx=parts["velocity"][:, 0].copy(), vy=parts["velocity"][:, 1].copy())
        ctx.step(4)
        assert ctx.counters() == (4, 0)
        assert_soa_bitwise(ctx.download_soa(), soa, what="gated ")
        ctx.step(60)
        fc, act = orc.run_steps(0, cfg, ext, soa, 64)
        assert ctx.counters() == (fc, act) == (64, 60)
        got = ctx.download_soa()
        assert_soa_bitwise(got, soa)
        aos = ctx.download()
        want_c = orc.set_color_array(soa["vx"], soa["vy"], cfg.max_energy)
        assert_bitwise(aos["color"].reshape(-1), want_c.reshape(-1), "colour")


def test_c1_single_attractor_euler_baseline_config(gpu, orc):
    """C1 exactly as BASELINE.json configs[0] states it: 65 536 particles of the reference
    scatter, a single point attractor at the origin, semi-implicit Euler, SHADER_DELAY 5
    (4 gated frames, then active steps; compute_shader.wgsl:392-400, :69-99, :426)."""
    rps = gpu
    n = 65536
    cfg = config_c1(rps, n, gravity=9.8)
    ext = ext_c1_attractor(rps)
    ext.shader_delay = 5
    parts = rps.setup_particles_scatter(cfg, n, seed=7)
    soa = dict(x=parts["position"][:, 0].copy(), y=parts["position"][:, 1].copy(),
               vx=parts["velocity"][:, 0].copy(), vy=parts["velocity"][:, 1].copy())
    with rps.Context(n) as ctx:
        ctx.set_config(cfg, ext)
        ctx.upload(parts)
        fc, act = 0, 0
        for chunk in (4, 1, 7, 48):
            ctx.step(chunk)
            fc, act = orc.run_steps(0, cfg, ext, soa, chunk, frame_count=fc, active_steps=act)
            assert ctx.counters() == (fc, act)
            assert_soa_bitwise(ctx.download_soa(), soa, what=f"frame{fc} ")
        assert (fc, act) == (60, 56)
        aos = ctx.download()
    want_c = orc.set_color_array(soa["vx"], soa["vy"], cfg.max_energy)
    assert_bitwise(aos["color"].reshape(-1), want_c.reshape(-1), "colour")


def test_c2_verlet_one_attractor(gpu, orc):
    """C2: 2^20 particles, one attractor, velocity-Verlet fp32; device-side initial scatter."""
    rps = gpu
    n = 1 << 20
    cfg = config_c1(rps, n, gravity=0.0)
    ext = ext_verlet_1att(rps)
    with rps.Context(n) as ctx:
        ctx.set_config(cfg, ext)
        ctx.init_scatter(seed=0x5EED)
        soa = ctx.download_soa()
        for s in range(3):
            ctx.step(1)
            orc.stream_step(cfg, ext, soa, s)
            assert_soa_bitwise(ctx.download_soa(), soa, what=f"step{s} ")


def test_headline_features_bitwise(gpu, orc):
    """C3 features (4 moving attractors, drag, lifetime, Philox respawn) at 2^20, 25 steps."""
    rps = gpu
    n = 1 << 20
    cfg = config_c1(rps, n)
    ext = rps.headline_ext()
    ext.shader_delay = 0
    soa = random_soa(n, list(cfg.screen_bounds), seed=21, life=(-0.05, 0.3))
    with _gpu_ctx(rps, n, cfg, ext, soa) as ctx:
        ref = copy_soa(soa)
        for s in range(25):
            orc.stream_step(cfg, ext, ref, s)
        ctx.step(25)
        assert_soa_bitwise(ctx.download_soa(life=True), ref, keys=KEYS5)
        assert_bitwise(ctx.read_debug(rps.DEBUG_EXPIRY), ref["exp"], "expiry")


_WRAP_N, _WRAP_STEPS = 4099, 70000


@pytest.fixture(scope="module")
def wrap_case(gpu, orc):
    """Inputs and the oracle's state after _WRAP_STEPS C3 steps (shared by both launch modes)."""
    rps = gpu
    cfg = config_c1(rps, _WRAP_N)
    ext = rps.headline_ext()
    ext.shader_delay = 0
    soa = random_soa(_WRAP_N, list(cfg.screen_bounds), seed=77, life=(-0.05, 0.2))
    ref = copy_soa(soa)
    for s in range(_WRAP_STEPS):
        orc.stream_step(cfg, ext, ref, s)
    return cfg, ext, soa, ref


@pytest.mark.parametrize("fuse", [1, 16])
def test_lifetime_clock_wraps(gpu, wrap_case, fuse):
    """The lifetime clock is a u16: expiries and the per-group [next] index
    compare modulo 2^16.  70 000 C3 steps carry it once around (clock 65 535 -> 0) with
    respawns in flight; every field and the raw expiries stay bitwise with the oracle, one
    step per launch and 16 fused per launch, at a ragged N (tail lanes included)."""
    rps = gpu
    cfg, ext, soa, ref = wrap_case
    ext.fuse_steps = fuse
    with _gpu_ctx(rps, _WRAP_N, cfg, ext, soa) as ctx:
        ctx.step(_WRAP_STEPS)
        got = ctx.download_soa(life=True)
        exp = ctx.read_debug(rps.DEBUG_EXPIRY)
    assert_soa_bitwise(got, ref, keys=KEYS5)
    assert_bitwise(exp, ref["exp"], "expiry")


@pytest.mark.parametrize("n", [1, 3, 5, 63, 1023, 4097, 65539])
def test_ragged_sizes(gpu, orc, n):
    rps = gpu
    cfg = config_c1(rps, n)
    ext = rps.headline_ext()
    ext.shader_delay = 0
    soa = random_soa(n, list(cfg.screen_bounds), seed=n, life=(-0.05, 0.2))
    with _gpu_ctx(rps, n, cfg, ext, soa) as ctx:
        ref = copy_soa(soa)
        for s in range(5):
            orc.stream_step(cfg, ext, ref, s)
        ctx.step(5)
        assert_soa_bitwise(ctx.download_soa(life=True), ref, keys=KEYS5)
        assert_bitwise(ctx.read_debug(rps.DEBUG_EXPIRY), ref["exp"], "expiry")


def test_sharded_contexts_use_global_ids(gpu, orc):
    """A rank's shard (id_offset, global_count) equals the matching slice of the whole."""
    rps = gpu
    n, shard = 40000, 10000
    cfg = config_c1(rps, n)
    ext = rps.headline_ext()
    ext.shader_delay = 0
    soa = random_soa(n, list(cfg.screen_bounds), seed=31, life=(-0.1, 0.4))
    whole = copy_soa(soa)
    for s in range(6):
        orc.stream_step(cfg, ext, whole, s)
    for r in range(4):
        lo = r * shard
        part = {k: v[lo:lo + shard].copy() for k, v in soa.items()}
        with _gpu_ctx(rps, shard, cfg, ext, part, id_offset=lo, global_count=n) as ctx:
            ctx.step(6)
            got = ctx.download_soa(life=True)
        for k in KEYS5:
            assert_bitwise(got[k], whole[k][lo:lo + shard], f"rank{r} {k}")


def test_stats_reduction(gpu, orc):
    rps = gpu
    n = 300001
    cfg = config_c1(rps, n)
    ext = rps.headline_ext(stats=True)
    ext.shader_delay = 0
    ext.stats_interval = 1
    soa = random_soa(n, list(cfg.screen_bounds), seed=41, life=(-0.02, 0.5))
    with _gpu_ctx(rps, n, cfg, ext, soa) as ctx:
        ctx.step(1)
        st = ctx.stats()
    ref = copy_soa(soa)
    ost = orc.stream_step(cfg, ext, ref, 0, stats=True)
    assert st.particles == n and st.step == 0
    assert st.respawned == ost.respawned > 0
    assert list(st.bbox) == list(ost.bbox)
    assert abs(st.kinetic_energy - ost.kinetic_energy) <= 1e-9 * abs(ost.kinetic_energy)


def test_init_scatter_matches_oracle(gpu, orc):
    rps = gpu
    n = 100000
    cfg = config_c1(rps, n)
    ext = rps.headline_ext()
    with rps.Context(n, id_offset=5000, global_count=200000) as ctx:
        ctx.set_config(cfg, ext)
        ctx.init_scatter(seed=99)
        got = ctx.download_soa(life=True)
    want = orc.init_scatter(cfg, ext, 99, n, id_offset=5000, global_count=200000)
    # Bitwise, y included: the Box-Muller ln is the fixed-op log_unit on both sides.
    for k in ("x", "y", "vx", "vy", "life"):
        assert_bitwise(got[k], want[k], k)
    assert (got["y"] >= cfg.screen_bounds[2]).all() and (got["y"] <= cfg.screen_bounds[3]).all()


def test_full_size_sampled_parity(gpu, orc):
    """BASELINE C3 size (1e8 particles): every particle is independent, so chunks sampled
    across the whole array checked against the oracle with their global ids pin the full
    launch (grid-stride coverage, 64-bit indexing, Philox counters at large ids)."""
    rps = gpu
    n = 100_000_000
    cfg = config_c1(rps, n)
    ext = rps.headline_ext()
    g = np.random.default_rng(5)
    chunk = 1 << 15
    starts = sorted(set([0, n - chunk] + list(g.integers(0, n - chunk, 10))))
    with rps.Context(n) as ctx:
        ctx.set_config(cfg, ext)
        ctx.init_scatter(seed=0x5EED)
        ctx.step(4)  # gated frames
        ctx.step(30)
        before = [_download_chunk(rps, ctx, s, chunk) for s in starts]
        ctx.step(3)
        _, act = ctx.counters()
        after = [_download_chunk(rps, ctx, s, chunk) for s in starts]
    assert act == 33
    for s, b, a in zip(starts, before, after):
        b["exp"] = orc.exp_from_steps(b.pop("steps"), 30)
        for k in range(30, 33):
            orc.stream_step(cfg, ext, b, k, id_offset=s)
        b["steps"] = orc.steps_from_exp(b["exp"], 33)
        assert_soa_bitwise(a, b, keys=KEYS_STEPS, what=f"chunk@{s} ")


def _assert_full_state(rps, orc, ctx, ref, clock, what, chunk=1 << 24):
    """Every particle of a 10^8 context against the oracle's arrays, bitwise, by chunks of
    2^24 (bounded host memory): x, y, vx, vy, the exact lifetime steps left and the raw u16
    expiries."""
    n = len(ref["x"])
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        got = _download_chunk(rps, ctx, s, m)
        want = {k: ref[k][s:s + m] for k in ("x", "y", "vx", "vy")}
        want["steps"] = orc.steps_from_exp(ref["exp"][s:s + m], clock)
        assert_soa_bitwise(got, want, keys=KEYS_STEPS, what=f"{what} chunk@{s} ")
    assert_bitwise(ctx.read_debug(rps.DEBUG_EXPIRY), ref["exp"], f"{what} expiry")


def test_full_size_every_particle(gpu, orc):
    """BASELINE C3 exactly as bench.py runs it (10^8 particles, 4 moving attractors, drag,
    lifetime U(1, 5) s with Philox respawn on the emitter disc, stats every 100 steps, every
    step active), EVERY particle checked, not a sample: the device scatter against the
    oracle's (orc_init_scatter on the OpenMP build: the serial checker's bits), then 130 steps;
    the two stats steps (0 and 100) run through the serial checker and their stats are compared
    (bbox and counts exact, KE to 1e-9), the other 128 on the oracle's OpenMP build
    (orc_stream_step_omp: the serial checker's operations per particle).  dt = 0.01 s, so the
    1-s lifetimes expire from step 100 on and respawns are part of the compared state.  Every
    field, the exact lifetime steps left and the raw u16 expiries, bitwise, by 2^24-particle
    chunks."""
    rps = gpu
    n, steps, stats_step = 100_000_000, 130, 100
    cfg = rps.default_particle_config(n, gravity=0.0)  # bench.py workload()
    ext = rps.headline_ext(stats=True)
    ext.shader_delay = 0
    assert ext.stats_interval == stats_step

    def check_stats(st, ost, k):
        assert st.step == k and st.particles == n
        assert st.respawned == ost.respawned
        assert list(st.bbox) == list(ost.bbox)
        assert abs(st.kinetic_energy - ost.kinetic_energy) <= 1e-9 * abs(ost.kinetic_energy)

    with rps.Context(n, rps.MODE_STREAM, global_count=n) as ctx:
        ctx.set_config(cfg, ext)
        ctx.init_scatter(0x5EED)
        ref = orc.init_scatter(cfg, ext, 0x5EED, n, global_count=n, omp=True)
        ref["life"] = None  # the u16 expiries are the state; steps are compared exactly
        _assert_full_state(rps, orc, ctx, ref, 0, "init")
        due = int(np.count_nonzero(orc.steps_from_exp(ref["exp"], 0) <= steps))
        assert due > n // 100  # respawns are part of the compared state
        ctx.step(1)
        check_stats(ctx.stats(), orc.stream_step(cfg, ext, ref, 0, stats=True), 0)
        ctx.step(steps - 1)
        ost = None
        for k in range(1, steps):
            if k == stats_step:
                ost = orc.stream_step(cfg, ext, ref, k, stats=True)
                ref["life"] = None
            else:
                orc.stream_step_omp(cfg, ext, ref, k)
        assert ost.respawned > 0
        check_stats(ctx.stats(), ost, stats_step)
        assert ctx.counters() == (steps, steps)
        _assert_full_state(rps, orc, ctx, ref, steps, f"step{steps}")


def test_aos_roundtrip_and_errors(gpu):
    rps = gpu
    n = 5000
    cfg = config_c1(rps, n)
    parts = rps.setup_particles_scatter(cfg, n, seed=3)
    parts["velocity"] = np.random.default_rng(2).normal(0, 50, (n, 2)).astype(F)
    with rps.Context(n) as ctx:
        ctx.set_config(cfg, rps.make_ext())
        ctx.upload(parts)
        got = ctx.download()
        assert_bitwise(got["position"].reshape(-1), parts["position"].reshape(-1))
        assert_bitwise(got["velocity"].reshape(-1), parts["velocity"].reshape(-1))
        sub = ctx.download(offset=100, n=50)
        assert_bitwise(sub["position"].reshape(-1), parts["position"][100:150].reshape(-1))
        with pytest.raises(rps.RpsError) as e:
            ctx.download(offset=n - 1, n=2)
        assert e.value.status == rps.RPS_ERR_INVALID_ARGUMENT
        bad = rps.make_ext()
        bad.num_attractors = 9
        with pytest.raises(rps.RpsError):
            ctx.set_config(cfg, bad)
        with pytest.raises(rps.RpsError) as e:
            ctx.read_debug(rps.DEBUG_DENSITIES)
        assert e.value.status == rps.RPS_ERR_UNSUPPORTED
        with pytest.raises(rps.RpsError) as e:
            ctx.stats()
        assert e.value.status == rps.RPS_ERR_UNSUPPORTED
    with pytest.raises(rps.RpsError):
        rps.Context(0)


def test_profiling_counts_dominant_kernel(gpu):
    rps = gpu
    n = 1 << 20
    cfg = config_c1(rps, n)
    with rps.Context(n) as ctx:
        ctx.set_config(cfg, rps.headline_ext())
        ctx.init_scatter()
        ctx.step(5)
        ctx.set_profiling(True)
        ctx.step(7)
        ms, cnt = ctx.kernel_time()
        assert cnt == 7 and ms > 0
        amt, unit = ctx.step_cost()
        assert unit == "bytes" and amt == (32 + 2 / 64) * n  # x, y, vx, vy r+w + the groups' [next] read
        assert ctx.time_steps(3) > 0
        ctx.set_profiling(2)  # every 2nd launch: 3 of 6 (launch-by-launch view)
        ctx.step(6)
        times = ctx.kernel_times()
        assert len(times) == 3 and all(t > 0 for t in times)
        assert ctx.kernel_times() == []  # a new collection
        with pytest.raises(rps.RpsError):
            ctx.kernel_clock()  # N-body mode only


@pytest.mark.parametrize("fuse,n,steps", [(4, 1 << 20, 13), (16, 65539, 40), (7, 5, 9)])
def test_fused_steps_bitwise(gpu, orc, fuse, n, steps):
    """ext.fuse_steps > 1: several steps per launch in registers == separate steps, bitwise;
    stats steps close a chunk so the reduced state is the stats step's."""
    rps = gpu
    cfg = config_c1(rps, n)
    ext = rps.headline_ext(stats=True)
    ext.shader_delay = 3
    ext.stats_interval = 5
    ext.fuse_steps = fuse
    soa = random_soa(n, list(cfg.screen_bounds), seed=fuse, life=(-0.05, 0.2))
    with _gpu_ctx(rps, n, cfg, ext, soa) as ctx:
        ctx.step(steps)
        got = ctx.download_soa(life=True)
        st = ctx.stats()
        fc, act = ctx.counters()
    ref = copy_soa(soa)
    ofc, oact = orc.run_steps(0, cfg, ext, ref, steps)
    assert (fc, act) == (ofc, oact)
    assert_soa_bitwise(got, ref, keys=KEYS5)
    last_stats = max(k for k in range(act) if k % 5 == 0)
    assert st.step == last_stats


def test_beyond_2pow32_particles(gpu, orc):
    """Maximum-size edge: 2^32 + 12291 particles (86 GB of tiled state in HBM).  Chunks at the
    start, straddling global index 2^32 and at the ragged tail are checked bitwise after a
    step: 64-bit tile addressing, the n % 4 tail and Philox counters with a non-zero high
    word (the reference itself tops out near 4.19 M particles)."""
    rps = gpu
    n = (1 << 32) + 12291  # the straddling chunk [2^32 - 8192, 2^32 + 8192) fits; n % 4 == 3
    cfg = config_c1(rps, 1 << 20)  # particle_count is u32 and informational in STREAM mode
    ext = rps.headline_ext()
    ext.shader_delay = 0
    chunk = 1 << 14
    starts = [0, (1 << 32) - chunk // 2, n - chunk]
    with rps.Context(n) as ctx:
        ctx.set_config(cfg, ext)
        ctx.init_scatter(seed=3)
        ctx.step(1)
        # force respawns inside the checked chunks (0.005 s = 1 step left)
        for s in starts:
            ctx.upload_field(rps.FIELD_LIFE, np.full(chunk, 0.005, F), s)
        before = [_download_chunk(rps, ctx, s, chunk) for s in starts]
        ctx.step(1)
        after = [_download_chunk(rps, ctx, s, chunk) for s in starts]
    for s, b, a in zip(starts, before, after):
        assert (b["steps"] == 1).all()
        b["exp"] = orc.exp_from_steps(b.pop("steps"), 1)
        st = orc.stream_step(cfg, ext, b, 1, id_offset=s, stats=True)
        assert st.respawned == chunk
        b["steps"] = orc.steps_from_exp(b["exp"], 2)
        assert_soa_bitwise(a, b, keys=KEYS_STEPS, what=f"chunk@{s} ")


def test_colour_follows_wgsl_mix(gpu, orc):
    """set_color (wgsl:101-118) colours by mix(a, b, t) = a * (1 - t) + b * t: a NaN speed makes
    all three components NaN (0 * NaN included), as the shader's fixtures show
    (tests/golden/wgsl_sph_n100_sched.npz); finite speeds give exactly t / 1 - t / 0.  Download
    and device export against the oracle, bitwise, over rest, both branches, the 0.5 edge,
    clamping, infinities and NaNs."""
    from hip_mem import DeviceBuffer

    rps = gpu
    cfg = config_c1(rps, 16, gravity=0.0)
    e = float(np.sqrt(2.0 * cfg.max_energy))  # |v| at energy = max_energy
    vel = np.array([[0, 0], [e / 4, 0], [e / 2, 0], [0, e * np.sqrt(0.5)], [e, 0], [2 * e, 0], [np.inf, 0],
                    [-np.inf, 1], [np.nan, 0], [0, np.nan], [np.nan, np.nan], [-e / 3, e / 5], [1e-30, 0],
                    [-0.0, -0.0], [3.0, -4.0], [e * 0.75, 0]], F)
    n = len(vel)
    parts = np.zeros(n, rps.PARTICLE_DTYPE)
    parts["velocity"] = vel
    with rps.Context(n) as ctx, DeviceBuffer(n * 32) as buf:
        ctx.set_config(cfg, rps.make_ext(shader_delay=0))
        ctx.upload(parts)
        ctx.step(1)  # an active step (set_color runs from the first one): no gravity, walls may flip v
        got = ctx.download()
        ctx.export_particles(buf.ptr.value)
        exp = buf.to_host(rps.PARTICLE_DTYPE)
    v = got["velocity"]
    want = orc.set_color_array(v[:, 0], v[:, 1], cfg.max_energy)
    assert np.isnan(want[8:11, :3]).all() and want[0].tolist() == [0.0, 0.0, 1.0, 1.0]
    assert_bitwise(got["color"].reshape(-1), want.reshape(-1), "download colour")
    assert_bitwise(exp["color"].reshape(-1), want.reshape(-1), "export colour")


def test_render_export_matches_download(gpu):
    """rps_export_particles writes the reference's 32-B Particle buffer (position, velocity,
    derived colour) straight into device memory (render interop)."""
    from hip_mem import DeviceBuffer

    rps = gpu
    n = 70001
    cfg = config_c1(rps, n)
    ext = rps.headline_ext()
    ext.shader_delay = 0
    with rps.Context(n) as ctx, DeviceBuffer(n * 32) as buf:
        ctx.set_config(cfg, ext)
        ctx.init_scatter()
        ctx.export_particles(buf.ptr.value)
        first = buf.to_host(rps.PARTICLE_DTYPE)
        assert np.array_equal(first["color"], np.ones((n, 4), F))  # spawn colour before stepping
        ctx.step(7)
        ctx.export_particles(buf.ptr.value)
        got = buf.to_host(rps.PARTICLE_DTYPE)
        want = ctx.download()
        assert_bitwise(got.view(np.uint32), want.view(np.uint32), "export")
        ctx.export_particles(buf.ptr.value, offset=1000, n=500)
        part = buf.to_host(rps.PARTICLE_DTYPE)[:500]
        assert_bitwise(part.view(np.uint32), want[1000:1500].view(np.uint32), "export range")
        with pytest.raises(rps.RpsError):
            host = np.zeros(n, rps.PARTICLE_DTYPE)
            ctx.export_particles(host.ctypes.data)  # host memory is rejected


def test_lifetime_views_clock_and_toggle(gpu, orc):
    """Lifetime kept as a u16 expiry on the lifetime clock: the seconds and
    exact-steps views, and a lifetime clock that stands still while RPS_EXT_LIFETIME is off."""
    rps = gpu
    n = 10007
    cfg = config_c1(rps, n)
    ext = rps.headline_ext()
    ext.shader_delay = 0
    off = rps.headline_ext()
    off.shader_delay = 0
    off.flags = 0
    dt = cfg.fixed_delta_time
    soa = random_soa(n, list(cfg.screen_bounds), seed=51, life=(-0.05, 0.09))
    with _gpu_ctx(rps, n, cfg, ext, soa) as ctx:
        ref = copy_soa(soa)
        ref["exp"] = orc.exp_from_life(ref["life"], 0, dt)
        steps0 = ctx.download_field(rps.FIELD_LIFE_STEPS)
        assert_bitwise(steps0, orc.steps_from_exp(ref["exp"], 0), "steps view")
        assert_bitwise(ctx.download_field(rps.FIELD_LIFE), (steps0 * F(dt)).astype(F), "seconds view")
        ctx.step(3)
        for s in range(3):
            orc.stream_step(cfg, ext, ref, s)
        ctx.set_config(cfg, off)
        frozen = ctx.download_field(rps.FIELD_LIFE_STEPS)
        ctx.step(4)
        for s in range(3, 7):
            orc.stream_step(cfg, off, ref, s)
        assert_bitwise(ctx.download_field(rps.FIELD_LIFE_STEPS), frozen, "clock stopped")
        ctx.set_config(cfg, ext)
        ctx.step(5)
        for s in range(7, 12):
            orc.stream_step(cfg, ext, ref, s, clock=s - 4)
        got = ctx.download_soa()
        assert_soa_bitwise(got, ref)
        assert_bitwise(ctx.read_debug(rps.DEBUG_EXPIRY), ref["exp"], "expiry")
        # exact round trip of the steps view (checkpoint / resume)
        st = ctx.download_field(rps.FIELD_LIFE_STEPS)
        ctx.upload_field(rps.FIELD_LIFE_STEPS, st)
        assert_bitwise(ctx.read_debug(rps.DEBUG_EXPIRY), ref["exp"], "steps round trip")


def test_stats_allreduce_single_rank(gpu, orc):
    """STREAM with a communicator: every stats step all-reduces the shard stats over the ranks
    (RCCL MAX of the bbox terms, SUM of KE / particles / respawns).  With one rank the
    all-rank stats must equal the shard's, through the same RCCL calls; the state is
    untouched by them (bitwise == oracle)."""
    rps = gpu
    n = 300001
    cfg = config_c1(rps, n)
    ext = rps.headline_ext(stats=True)
    ext.shader_delay = 0
    ext.stats_interval = 2
    soa = random_soa(n, list(cfg.screen_bounds), seed=43, life=(-0.02, 0.5))
    ref = copy_soa(soa)
    with _gpu_ctx(rps, n, cfg, ext, soa) as ctx:
        ctx.comm_init(0, 1, rps.comm_unique_id())
        ctx.step(3)  # stats steps 0 and 2
        st = ctx.stats()
        got = ctx.download_soa(life=True)
    for k in range(3):
        ost = orc.stream_step(cfg, ext, ref, k, stats=(k == 2))
    for key in ("x", "y", "vx", "vy", "life"):
        assert_bitwise(got[key], ref[key], key)
    assert st.step == 2 and st.particles == n
    assert st.respawned == ost.respawned
    assert list(st.bbox) == list(ost.bbox)
    assert abs(st.kinetic_energy - ost.kinetic_energy) <= 1e-9 * abs(ost.kinetic_energy)


def test_quad_next_index_after_partial_lifetime_upload(gpu, orc):
    """The per-quad earliest-expiry index ([next], rps_device.hpp) lets a step skip the
    expiries of quads with none due.  It is rebuilt after every expiry write outside the
    kernel: here a LIFE_STEPS upload over a range that starts and ends inside quads, with
    lifetimes of 1-3 steps, then plain and temporally fused steps; every field and the raw
    expiries stay bitwise equal to the oracle (which has no such index)."""
    rps = gpu
    n = 70003
    cfg = config_c1(rps, n)
    ext = rps.headline_ext()
    ext.shader_delay = 0
    soa = random_soa(n, list(cfg.screen_bounds), seed=57, life=(0.5, 3.0))
    g = np.random.default_rng(58)
    lo, m = 1001, 30001  # [1001, 31002): partial quads at both ends
    steps = g.integers(1, 4, m).astype(F)
    with _gpu_ctx(rps, n, cfg, ext, soa) as ctx:
        ctx.step(2)
        ctx.upload_field(rps.FIELD_LIFE_STEPS, steps, offset=lo)
        ref = ctx.download_soa(life=True)
        ref["exp"] = ctx.read_debug(rps.DEBUG_EXPIRY)
        for k in range(2, 6):
            orc.stream_step(cfg, ext, ref, k)
        ctx.step(4)
        assert_bitwise(ctx.read_debug(rps.DEBUG_EXPIRY), ref["exp"], "expiry after plain steps")
        ext.fuse_steps = 3
        ctx.set_config(cfg, ext)
        for k in range(6, 13):
            orc.stream_step(cfg, ext, ref, k)
        ctx.step(7)
        got = ctx.download_soa(life=True)
        assert_soa_bitwise(got, ref, keys=KEYS5, what="fused ")
        assert_bitwise(ctx.read_debug(rps.DEBUG_EXPIRY), ref["exp"], "expiry after fused steps")
