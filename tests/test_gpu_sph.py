"""GPU parity of the reference's SPH pass sequence (mode SPH) against the CPU oracle.

Integer passes (bin, bitonic sort, offsets) must be bitwise equal — including the
bug-compatible next_pow2 pad entries — and the float passes (gravity,
predicted positions, density, pressure, viscosity, Euler, walls) bitwise too: same f32 ops,
same neighbour order, correctly-rounded sqrt/div on both sides."""
import numpy as np
import pytest

from helpers import F, assert_bitwise, assert_soa_bitwise, copy_soa

pytestmark = pytest.mark.gpu


def _blob(n, seed, spread=None):
    g = np.random.default_rng(seed)
    s = spread or max(20.0, np.sqrt(n) * 1.2)
    return dict(x=np.clip(g.normal(0, s, n), -955, 955).astype(F),
                y=np.clip(g.normal(0, s * 0.6, n), -535, 535).astype(F),
                vx=g.normal(0, 30, n).astype(F), vy=g.normal(0, 30, n).astype(F))


@pytest.mark.parametrize("n", [1, 2, 3, 5, 17, 64, 1000, 4096, 50000, 65536])
def test_sph_steps_bitwise(gpu, orc, n):
    rps = gpu
    cfg = rps.default_particle_config(n, gravity=100.0)
    soa = _blob(n, n)
    ext = rps.make_ext()  # SHADER_DELAY 5
    st = orc.SphState(n)
    ref = copy_soa(soa)
    with rps.Context(n, rps.MODE_SPH) as ctx:
        ctx.set_config(cfg, ext)
        ctx.upload_soa(soa)
        for frame in range(1, 9):
            ctx.step(1)
            active = frame >= 5
            st.grid(cfg, ref)
            if active:
                st.pre(cfg, ref)
            assert_bitwise(ctx.read_debug(rps.DEBUG_SPATIAL_LOOKUP), st.lookup, f"lookup f{frame}")
            assert_bitwise(ctx.read_debug(rps.DEBUG_LOOKUP_OFFSETS), st.offsets, f"offsets f{frame}")
            if active:
                assert_bitwise(ctx.read_debug(rps.DEBUG_PREDICTED), st.pred, f"pred f{frame}")
                assert_bitwise(ctx.read_debug(rps.DEBUG_DENSITIES), st.dens, f"dens f{frame}")
                st.sim(cfg, ref)
            assert_soa_bitwise(ctx.download_soa(), ref, what=f"f{frame} ")
        assert ctx.counters() == (8, 4)
        aos = ctx.download()
        assert_bitwise(aos["color"].reshape(-1), orc.set_color_array(ref["vx"], ref["vy"], cfg.max_energy).reshape(-1))


def test_sph_reference_default_scatter(gpu, orc):
    """N = 50 000 reference default (src/main.rs:25), reference scatter, 12 frames."""
    rps = gpu
    n = 50000
    cfg = rps.default_particle_config(n)
    parts = rps.setup_particles_scatter(cfg, n, seed=11)
    soa = dict(x=parts["position"][:, 0].copy(), y=parts["position"][:, 1].copy(),
               vx=parts["velocity"][:, 0].copy(), vy=parts["velocity"][:, 1].copy())
    st = orc.SphState(n)
    with rps.Context(n, rps.MODE_SPH) as ctx:
        ctx.set_config(cfg, rps.make_ext())
        ctx.upload(parts)
        ctx.step(12)
        orc.run_steps(2, cfg, rps.make_ext(), soa, 12, sph=st)
        assert_bitwise(ctx.read_debug(rps.DEBUG_SPATIAL_LOOKUP), st.lookup, "lookup")
        assert_soa_bitwise(ctx.download_soa(), soa)


def test_sph_config_validation(gpu):
    rps = gpu
    cfg = rps.default_particle_config(100)
    with rps.Context(128, rps.MODE_SPH) as ctx:
        with pytest.raises(rps.RpsError):
            ctx.set_config(cfg, None)  # particle_count != 128
        with pytest.raises(rps.RpsError) as e:
            ctx.set_config(rps.default_particle_config(128), rps.headline_ext())
        assert e.value.status == rps.RPS_ERR_UNSUPPORTED


@pytest.mark.parametrize("n", [(1 << 22) + 5, (1 << 20) + 5, 300000])
def test_sph_grid_passes_large(gpu, orc, n):
    """bin + bitonic + offsets at P = 2^23 / 2^21 / 2^19 against the oracle's pass-per-dispatch
    network (OpenMP build, same network): 8192-entry head and tail tiles, register-fused global
    passes, gathered-tile stages of 5-9 global passes, and at P = 2^23 the last stage's ten
    global passes as register-fused launches with non-flip chunks; passes 4-5 gated off
    (shader_delay) so only the integer passes run."""
    rps = gpu
    cfg = rps.default_particle_config(n, gravity=100.0)
    soa = _blob(n, 7, spread=300.0)
    ext = rps.make_ext(shader_delay=100)
    st = orc.SphState(n, omp=True)
    ref = copy_soa(soa)
    with rps.Context(n, rps.MODE_SPH) as ctx:
        ctx.set_config(cfg, ext)
        ctx.upload_soa(soa)
        ctx.step(1)
        st.grid(cfg, ref)
        assert_bitwise(ctx.read_debug(rps.DEBUG_SPATIAL_LOOKUP), st.lookup, "lookup")
        assert_bitwise(ctx.read_debug(rps.DEBUG_LOOKUP_OFFSETS), st.offsets, "offsets")


def _frames_vs_oracle(rps, orc, n, soa, cfg, frames, cfg_at=None, download_at=None):
    """Step `frames` SPH frames (shader_delay 0) and check every frame bitwise: lookup,
    offsets, predicted positions, densities, state.  cfg_at: {frame: new config};
    download_at: the frames after which the state is downloaded (default: every frame; the
    last frame always) -- a download puts slot-resident state back in particle order, so
    frames between downloads carry it over."""
    ext = rps.make_ext(shader_delay=0)
    st = orc.SphState(n)
    ref = copy_soa(soa)
    with rps.Context(n, rps.MODE_SPH) as ctx:
        ctx.set_config(cfg, ext)
        ctx.upload_soa(soa)
        for frame in range(frames):
            if cfg_at and frame in cfg_at:
                cfg = cfg_at[frame]
                ctx.set_config(cfg, ext)
            ctx.step(1)
            st.grid(cfg, ref)
            st.pre(cfg, ref)
            assert_bitwise(ctx.read_debug(rps.DEBUG_SPATIAL_LOOKUP), st.lookup, f"lookup f{frame}")
            assert_bitwise(ctx.read_debug(rps.DEBUG_LOOKUP_OFFSETS), st.offsets, f"offsets f{frame}")
            assert_bitwise(ctx.read_debug(rps.DEBUG_PREDICTED), st.pred, f"pred f{frame}")
            assert_bitwise(ctx.read_debug(rps.DEBUG_DENSITIES), st.dens, f"dens f{frame}")
            st.sim(cfg, ref)
            if download_at is None or frame in download_at or frame == frames - 1:
                assert_soa_bitwise(ctx.download_soa(), ref, what=f"f{frame} ")


@pytest.mark.parametrize("n", [16384, 1 << 21])
def test_sph_resident_state_frames(gpu, orc, monkeypatch, n):
    """Slot-resident state: after a layout frame the state stays in that
    frame's storage order and the sim writes the next frame's bin entries.  Consecutive layout
    frames with no download between them (the debug reads translate the sorted lookup's slot
    payloads back to particle indices), a config change between resident frames (stale bin
    entries rebuilt from the state), downloads at frames 3 and 6: every pass bitwise."""
    rps = gpu
    monkeypatch.setenv("RPS_SPH_LAYOUT", "2")
    if n == 16384:
        cfg = rps.default_particle_config(n, gravity=100.0)
        soa = _blob(n, 41, spread=300.0)
        cfg2 = rps.default_particle_config(n, gravity=60.0, smoothing_radius=7.0)
    else:
        scale = (n / 50000) ** 0.5
        bounds = rps.screen_bounds_for(1920.0 * scale, 1080.0 * scale)
        cfg = rps.default_particle_config(n, screen_bounds=bounds)
        parts = rps.setup_particles_scatter(cfg, n, seed=0x5EED)
        soa = dict(x=parts["position"][:, 0].copy(), y=parts["position"][:, 1].copy(),
                   vx=parts["velocity"][:, 0].copy(), vy=parts["velocity"][:, 1].copy())
        cfg2 = rps.default_particle_config(n, screen_bounds=bounds, gravity=60.0)
    _frames_vs_oracle(rps, orc, n, soa, cfg, 7 if n == 16384 else 4, cfg_at={2: cfg2},
                      download_at={3, 6})


@pytest.mark.parametrize("n", [16384, 16000])
def test_sph_layout_epoch_wrap(gpu, orc, monkeypatch, n):
    """The layout's cell records carry the build's epoch instead of being reset each frame;
    started two builds before the 2^24 wrap, the frames across it (records cleared, epoch 1
    again) stay bitwise.  At 16 000 (P != N) the resident frames' own_s ownership and the pad
    entries' flagged payloads cross the wrap too."""
    rps = gpu
    monkeypatch.setenv("RPS_SPH_LAYOUT", "2")
    monkeypatch.setenv("RPS_SPH_LAYOUT_EPOCH", str((1 << 24) - 3))
    cfg = rps.default_particle_config(n, gravity=100.0)
    _frames_vs_oracle(rps, orc, n, _blob(n, 47, spread=300.0), cfg, 5, download_at={4})


@pytest.mark.parametrize("n", [16384, 16000])
def test_sph_resident_state_api(gpu, orc, monkeypatch, n):
    """Every particle-order API call on slot-resident state: a device export, a partial field
    upload, a download, and gated frames (a config change resetting frame_count, SHADER_DELAY
    3) right after resident frames; the state bitwise after each step, the export bitwise
    against the oracle's particles.  At 16 000 (P != N) the state sits at owner slots and the
    pad entries carry flagged particle indices between frames."""
    from hip_mem import DeviceBuffer

    rps = gpu
    monkeypatch.setenv("RPS_SPH_LAYOUT", "2")
    cfg = rps.default_particle_config(n, gravity=100.0)
    soa = _blob(n, 43, spread=300.0)
    st = orc.SphState(n)
    ref = copy_soa(soa)

    def frames(k, gated=0):
        for f in range(k):
            st.grid(cfg, ref)
            if f >= gated:
                st.pre(cfg, ref)
                st.sim(cfg, ref)

    with rps.Context(n, rps.MODE_SPH) as ctx, DeviceBuffer(n * rps.PARTICLE_DTYPE.itemsize) as buf:
        ctx.set_config(cfg, rps.make_ext(shader_delay=0))
        ctx.upload_soa(soa)
        ctx.step(2)
        frames(2)
        ctx.export_particles(buf.ptr.value)
        got = buf.to_host(rps.PARTICLE_DTYPE)
        assert_bitwise(got["position"][:, 0], ref["x"], "export x")
        assert_bitwise(got["velocity"][:, 1], ref["vy"], "export vy")
        ctx.step(2)
        frames(2)
        assert_soa_bitwise(ctx.download_soa(), ref, what="after export ")
        # the lookup right after the download (which puts the state back in particle order):
        # the reference's spatial_lookup, pads included (particle indices, not slots)
        assert_bitwise(ctx.read_debug(rps.DEBUG_SPATIAL_LOOKUP), st.lookup, "lookup after download")
        ctx.step(2)
        frames(2)
        x_new = (ref["x"][:100] * np.float32(0.5)).astype(F)
        ctx.upload_field(rps.FIELD_X, x_new)
        ref["x"][:100] = x_new
        ctx.step(2)
        frames(2)
        assert_soa_bitwise(ctx.download_soa(), ref, what="after field upload ")
        ctx.step(2)
        frames(2)
        cfg = rps.default_particle_config(n, gravity=80.0)
        ctx.set_config(cfg, rps.make_ext(shader_delay=3))  # frame_count 0: frames 1, 2 gated
        ctx.step(4)
        frames(4, gated=2)
        assert_bitwise(ctx.read_debug(rps.DEBUG_SPATIAL_LOOKUP), st.lookup, "lookup after gated")
        assert_soa_bitwise(ctx.download_soa(), ref, what="after gated ")


@pytest.mark.parametrize("n", [16384, 16000, 5000])
def test_sph_init_scatter_leaves_resident_state(gpu, orc, monkeypatch, n):
    """rps_init_scatter on slot-resident state: resident layout frames, then the
    device scatter, then a gated frame (config change, SHADER_DELAY 3), a lookup readback and
    active frames.  The scatter leaves the resident state like every particle-order write: the
    lookup's pad payloads are particle indices again (P != N at 16 000 and 5 000, where the
    next frames may run the compact sort on 16-bit payloads), so the gated frame's lookup is
    the reference's, and every later frame stays bitwise."""
    rps = gpu
    monkeypatch.setenv("RPS_SPH_LAYOUT", "2")
    cfg = rps.default_particle_config(n, gravity=100.0)
    soa = _blob(n, 53, spread=300.0)
    st = orc.SphState(n)
    ref = copy_soa(soa)

    def frames(k, gated=0):
        for f in range(k):
            st.grid(cfg, ref)
            if f >= gated:
                st.pre(cfg, ref)
                st.sim(cfg, ref)

    with rps.Context(n, rps.MODE_SPH) as ctx:
        ctx.set_config(cfg, rps.make_ext(shader_delay=0))
        ctx.upload_soa(soa)
        ctx.step(3)
        frames(3)
        ctx.init_scatter(0x5EED)
        init = orc.init_scatter(cfg, rps.make_ext(), 0x5EED, n, life=False)
        ref = {k: init[k] for k in ("x", "y", "vx", "vy")}
        cfg = rps.default_particle_config(n, gravity=80.0)
        ctx.set_config(cfg, rps.make_ext(shader_delay=3))  # frame_count 0: frames 1, 2 gated
        ctx.step(1)
        frames(1, gated=1)
        assert_bitwise(ctx.read_debug(rps.DEBUG_SPATIAL_LOOKUP), st.lookup, "lookup after init_scatter + gated")
        ctx.step(3)
        frames(3, gated=1)
        assert_bitwise(ctx.read_debug(rps.DEBUG_SPATIAL_LOOKUP), st.lookup, "lookup after active frames")
        assert_soa_bitwise(ctx.download_soa(), ref, what="after init_scatter ")


@pytest.mark.parametrize("n", [4096, 50000])
def test_sph_every_frame_active(gpu, orc, n):
    """Every frame active from the first (shader_delay 0), every pass checked: at 50 000 the
    non-pow2 pads turn particles NaN within three frames, and NaN neighbours
    then enter the runs of others (NaN payloads excepted from the bitwise bar: helpers)."""
    rps = gpu
    cfg = rps.default_particle_config(n, gravity=100.0)
    _frames_vs_oracle(rps, orc, n, _blob(n, n + 1), cfg, 3)


def test_sph_out_of_bounds_and_config_change(gpu, orc):
    """Particles far outside the walls (cells beyond the grid, hashed like any other), then a
    radius + bounds change mid-run."""
    rps = gpu
    n = 20000
    cfg = rps.default_particle_config(n, gravity=100.0)
    soa = _blob(n, 5, spread=500.0)
    soa["x"][:50] = np.float32(2000.0)
    soa["y"][50:100] = np.float32(-3000.0)
    cfg2 = rps.default_particle_config(n, gravity=100.0, smoothing_radius=14.0,
                                       screen_bounds=rps.screen_bounds_for(2400.0, 1400.0))
    _frames_vs_oracle(rps, orc, n, soa, cfg, 4, cfg_at={2: cfg2})


@pytest.mark.parametrize("n", [300000, 1 << 18])
def test_sph_large_frames_bitwise(gpu, orc, n):
    """Full frames at P = 2^19 / 2^18 (records beyond one XCD's L2) over a dense blob (tens
    of neighbours per particle)."""
    rps = gpu
    cfg = rps.default_particle_config(n, gravity=100.0)
    _frames_vs_oracle(rps, orc, n, _blob(n, 3, spread=260.0), cfg, 2)


@pytest.mark.parametrize("n", [65536, 50000])
@pytest.mark.parametrize("batch", [("RPS_SPH_BATCH_S", "6"), ("RPS_SPH_BATCH_S", "8"), ("RPS_SPH_BATCH_S", "16"),
                                   ("RPS_SPH_BATCH_D", "4"), ("RPS_SPH_BATCH_D", "16")])
def test_sph_forced_scan_batches(gpu, orc, monkeypatch, n, batch):
    """Every scan-batch variant of the density and sim kernels, forced per context at small N
    (the default picks the sim batch 6 only above P = 2^21): P = N (slot self-skip) and
    N = 50 000 (pads, index self-skip), every pass bitwise over 3 frames."""
    rps = gpu
    monkeypatch.setenv(*batch)
    cfg = rps.default_particle_config(n, gravity=100.0)
    _frames_vs_oracle(rps, orc, n, _blob(n, n + 2), cfg, 3)


@pytest.mark.parametrize("n", [1 << 22, 1 << 21, 1 << 20])
def test_sph_bench_workload_full_size(gpu, orc, n):
    """The bench's `sph` workload exactly (2^22): particles of the reference scatter over a
    viewport scaled to the default density, every frame active.  Every size runs the spatial
    record layout (from 2^20) with its 4-entry sim scan; P = 2^22 selects 8192-entry sort
    tiles with 3 passes per register chunk and the five-pass register-fused global stage; at
    P = 2^21 that stage is a gathered-tile launch.  Two frames, every pass bitwise."""
    rps = gpu
    scale = (n / 50000) ** 0.5
    cfg = rps.default_particle_config(n, screen_bounds=rps.screen_bounds_for(1920.0 * scale, 1080.0 * scale))
    parts = rps.setup_particles_scatter(cfg, n, seed=0x5EED)
    soa = dict(x=parts["position"][:, 0].copy(), y=parts["position"][:, 1].copy(),
               vx=parts["velocity"][:, 0].copy(), vy=parts["velocity"][:, 1].copy())
    _frames_vs_oracle(rps, orc, n, soa, cfg, 2)


@pytest.mark.parametrize("n,layout", [(4096, "0"), (3000, "0"), (4096, "2")])
def test_sph_frame_cost_counts(gpu, orc, monkeypatch, n, layout):
    """rps_sph_frame_cost's device counts (the roofline's E) equal the entries of every lookup
    slot's nine runs, walked here on the oracle's lookup, offsets and predicted positions the
    way the reference's scans walk them (wgsl:231-252): keys in the reference cell order, a
    run ends at a key change or at N.  The byte model follows include/rps.h.  Layout "2": the
    spatial record layout forced (the count walks its storage runs, run2, over storage-order
    predictions).  The query is refused before any active frame and after a gated one."""
    import ref_numpy as RN

    rps = gpu
    monkeypatch.setenv("RPS_SPH_LAYOUT", layout)
    cfg = rps.default_particle_config(n, gravity=100.0)
    soa = _blob(n, 40 + n)
    st = orc.SphState(n)
    ref = copy_soa(soa)
    with rps.Context(n, rps.MODE_SPH) as ctx:
        ctx.set_config(cfg, rps.make_ext(shader_delay=2))
        ctx.upload_soa(soa)
        ctx.step(1)  # frame 1 < SHADER_DELAY 2: gated
        with pytest.raises(rps.RpsError):
            ctx.sph_frame_cost()  # no active frame yet
        ctx.step(1)  # frame 2: active
        cost = ctx.sph_frame_cost()
        amt, unit = ctx.step_cost()
        ctx.set_config(cfg, rps.make_ext(shader_delay=2))  # frame_count back to 0
        ctx.step(1)  # gated again: lookup re-sorted, predictions of the older frame
        with pytest.raises(rps.RpsError):
            ctx.sph_frame_cost()
        with pytest.raises(rps.RpsError):
            ctx.step_cost()
    st.grid(cfg, ref)
    st.grid(cfg, ref)
    st.pre(cfg, ref)
    P = st.P
    lk = st.lookup.reshape(P, 2)
    px, py = st.pred[0::2], st.pred[1::2]
    r = F(cfg.smoothing_radius)
    r2 = r * r
    xm, ym = F(cfg.screen_bounds[1]), F(cfg.screen_bounds[3])
    scanned = within = 0
    for t in range(P):
        i = int(lk[t, 1])
        cx = RN.f32_to_i32((px[i] + xm) / r)
        cy = RN.f32_to_i32((py[i] + ym) / r)
        for ox, oy in RN.GRID_OFFSETS:
            key = RN.hash_cell(cx + ox, cy + oy) % n
            j = int(st.offsets[key])
            while j < n and lk[j, 0] == key:
                q = int(lk[j, 1])
                dx, dy = px[i] - px[q], py[i] - py[q]
                scanned += 1
                within += int(not (dx * dx + dy * dy > r2))
                j += 1
    assert (cost["scanned_entries"], cost["within_entries"]) == (scanned, within)
    assert cost["slots"] == P and cost["particles"] == n and cost["sort_launches"] >= 1
    assert cost["density_bytes"] == 8.0 * scanned + 120.0 * P
    assert cost["sim_bytes"] == 32.0 * scanned + 156.0 * P
    assert unit == "bytes" and amt == cost["frame_bytes"]
    assert cost["frame_bytes"] == cost["sort_bytes"] + cost["predict_bytes"] + cost["density_bytes"] + cost["sim_bytes"]


@pytest.mark.parametrize("case", ["blob", "dense", "outside", "batches"])
def test_sph_spatial_layout_forced(gpu, orc, monkeypatch, case):
    """The spatial record layout (rps_kernels.hip; by default only from 2^20 particles) forced
    at small P == N, every pass bitwise: an ordinary blob; a dense one whose runs exceed the
    runs kernel's 32-entry measure (the listed-run path); particles far outside the walls
    (runs owned by cells beyond the grid, lanes whose 3 x 3 block leaves it) with a radius +
    bounds change mid-run (a new grid); other scan batches.  The
    16 384-particle default viewport has ~28 700 cells, within the context's cell capacity
    (at least 2^16), so every frame here runs the layout."""
    rps = gpu
    monkeypatch.setenv("RPS_SPH_LAYOUT", "2")
    n = 16384
    cfg = rps.default_particle_config(n, gravity=100.0)
    cfg_at = None
    if case == "dense":
        soa = _blob(n, 21, spread=12.0)
    else:
        soa = _blob(n, 22, spread=300.0)
    if case == "outside":
        soa["x"][:50] = np.float32(2000.0)
        soa["y"][50:100] = np.float32(-3000.0)
        soa["x"][100:140] = np.float32(961.0)
        cfg_at = {2: rps.default_particle_config(n, gravity=100.0, smoothing_radius=14.0,
                                                 screen_bounds=rps.screen_bounds_for(2400.0, 1400.0))}
    if case == "batches":  # the layout's other scan variants (default: density 8, sim 4)
        monkeypatch.setenv("RPS_SPH_BATCH_S", "6")
        monkeypatch.setenv("RPS_SPH_BATCH_D", "16")
    _frames_vs_oracle(rps, orc, n, soa, cfg, 4, cfg_at=cfg_at)


@pytest.mark.parametrize("n", [3, 17, 100, 3000, 16383, 40000])
def test_sph_spatial_layout_ragged(gpu, orc, monkeypatch, n):
    """The layout forced at non-power-of-two N (P = next_pow2(N) > N): the pad entries sort in
    and only [0, N) is scanned, so the layout's storage covers the N scanned
    slots in cell order and the P - N pad slots after them in lookup order; the lowest slot of
    each particle owns it (its sim), particles pushed past N included.  The state stays at the
    owner slots from frame to frame (downloads only after frames 2 and 5), the pad entries
    carrying flagged particle indices.  Six frames bitwise."""
    rps = gpu
    monkeypatch.setenv("RPS_SPH_LAYOUT", "2")
    cfg = rps.default_particle_config(n, gravity=100.0)
    _frames_vs_oracle(rps, orc, n, _blob(n, 90 + n, spread=max(15.0, (n ** 0.5) * 2.0)), cfg, 6,
                      download_at={2})


@pytest.mark.parametrize("layout,long_min", [("2", None), ("0", None), ("0", "8"), ("2", "128")])
def test_sph_reference_default_long_runs(gpu, orc, monkeypatch, layout, long_min):
    """The reference default (N = 50 000, its scatter and viewport) over 14 active frames:
    the stale pad duplicates grow runs of 150+ entries near key N, and particles turn NaN and
    pile into the key-0 run, so scans exceed 64 / 128 entries; those are walked one slot per
    wave (rps_kernels.hip, SphSlots::long_min; 8 sends most slots there, masked ones included).
    With and without the spatial layout, every frame bitwise."""
    rps = gpu
    monkeypatch.setenv("RPS_SPH_LAYOUT", layout)
    if long_min:
        monkeypatch.setenv("RPS_SPH_LONG_MIN", long_min)
    n = 50000
    cfg = rps.default_particle_config(n)
    parts = rps.setup_particles_scatter(cfg, n, seed=1)
    soa = dict(x=parts["position"][:, 0].copy(), y=parts["position"][:, 1].copy(),
               vx=parts["velocity"][:, 0].copy(), vy=parts["velocity"][:, 1].copy())
    _frames_vs_oracle(rps, orc, n, soa, cfg, 14, download_at={5, 9, 13})


def test_sph_layout_one_million(gpu, orc):
    """BASELINE C2's literal size, N = 10^6 (P = 2^20): the default selects the spatial layout
    (from P = 2^20) with pad slots; the bench's viewport scaled to the default density, three
    frames bitwise."""
    rps = gpu
    n = 1_000_000
    scale = (n / 50000) ** 0.5
    cfg = rps.default_particle_config(n, screen_bounds=rps.screen_bounds_for(1920.0 * scale, 1080.0 * scale))
    parts = rps.setup_particles_scatter(cfg, n, seed=0x5EED)
    soa = dict(x=parts["position"][:, 0].copy(), y=parts["position"][:, 1].copy(),
               vx=parts["velocity"][:, 0].copy(), vy=parts["velocity"][:, 1].copy())
    _frames_vs_oracle(rps, orc, n, soa, cfg, 3, download_at=set())


@pytest.mark.parametrize("layout", ["0", "2"])
@pytest.mark.parametrize("case", ["stacked", "tiny", "huge"])
def test_sph_division_operand_ranges(gpu, orc, monkeypatch, layout, case):
    """Operand ranges of the sim's pressure direction `delta / distance` (wgsl:304-310) and its
    sqrt: stacked: columns and rows of particles with equal coordinates and no velocity along
    them (dx == 0 or dy == 0 exactly: signed-zero quotients); tiny: coordinates 0 < |x| < 2^-60
    at the origin (tiny numerators; the sqrt's scaled path); huge: x beyond 2^36 (quotients and
    squares far from 1).  Without (0) and with (2) the spatial layout, every frame bitwise."""
    rps = gpu
    monkeypatch.setenv("RPS_SPH_LAYOUT", layout)
    n = 4096
    g = np.random.default_rng(43)
    cfg = rps.default_particle_config(n, gravity=100.0)
    soa = _blob(n, 42, spread=40.0)
    if case == "stacked":
        soa["x"][:2048] = np.round(soa["x"][:2048] / 3.0).astype(F) * F(3.0)
        soa["vx"][:2048] = F(0.0)
        soa["y"][1024:3072] = np.round(soa["y"][1024:3072] / 2.0).astype(F) * F(2.0)
        soa["x"][3072:3200] = F(0.0)
        soa["vx"][3072:3200] = F(0.0)
    elif case == "tiny":
        soa["x"][:64] = g.uniform(-1e-20, 1e-20, 64).astype(F)
        soa["x"][64:80] = F(0.0)
        soa["y"][:80] = g.uniform(-2.0, 2.0, 80).astype(F)
        soa["vx"][:80] = F(0.0)
    else:
        soa["x"][:8] = F(1.0e12)
        soa["vx"][:8] = F(0.0)
    _frames_vs_oracle(rps, orc, n, soa, cfg, 3)


# Slider ranges of src/parameter_gui.rs:38-62.
_GUI_RANGES = dict(fixed_delta_time=(0.0015, 0.015), gravity=(0.0, 1000.0), damping_factor=(0.0, 1.0),
                   smoothing_radius=(0.0, 30.0), max_energy=(1000.0, 10000.0), target_density=(0.0, 0.1),
                   pressure_multiplier=(1.0, 100000.0), viscocity_strength=(0.0, 10.0),
                   near_density_multiplier=(1.0, 10000.0))


@pytest.mark.parametrize("layout", ["0", "2"])
@pytest.mark.parametrize("seed", [0, 1, 2, 3, 4, "edges"])
def test_sph_random_gui_configs(gpu, orc, monkeypatch, layout, seed):
    """Configs a user reaches with the reference's sliders (src/parameter_gui.rs:38-62), applied
    as apply_gui_updates does (norms recomputed, :89-91): five seeded draws over the slider
    ranges and one at the ends (radius 0 -- infinite norms --, no gravity, full damping, zero
    target density, maximal pressure); without (0) and with (2) the spatial layout, four frames
    each bitwise against the oracle, NaN/inf spread included."""
    rps = gpu
    monkeypatch.setenv("RPS_SPH_LAYOUT", layout)
    n = 4096
    gui = rps.GUIConfig()
    if seed == "edges":
        vals = dict(fixed_delta_time=0.015, gravity=0.0, damping_factor=1.0, smoothing_radius=0.0,
                    max_energy=1000.0, target_density=0.0, pressure_multiplier=100000.0,
                    viscocity_strength=10.0, near_density_multiplier=10000.0)
    else:
        g = np.random.default_rng(1000 + seed)
        vals = {k: float(np.float32(g.uniform(lo, hi))) for k, (lo, hi) in _GUI_RANGES.items()}
        vals["smoothing_radius"] = float(np.float32(g.uniform(2.0, 30.0)))  # the bench's cells stay bounded
    for k, v in vals.items():
        setattr(gui, k, v)
    gui.applied_changes = True
    cfg = rps.default_particle_config(n)
    rps.apply_gui_updates(cfg, gui)
    soa = _blob(n, 500 + (7 if seed == "edges" else seed), spread=60.0)
    _frames_vs_oracle(rps, orc, n, soa, cfg, 4)


@pytest.mark.parametrize("n", [1, 2, 16, 64, 128, 1024])
def test_sph_spatial_layout_small_n(gpu, orc, monkeypatch, n):
    """The layout forced at power-of-two N below and around one wave (the runs kernel sizes a
    run from the wave's run-start ballot and one look-ahead load past the wave; lanes past N
    take part in the ballots): four frames bitwise."""
    rps = gpu
    monkeypatch.setenv("RPS_SPH_LAYOUT", "2")
    cfg = rps.default_particle_config(n, gravity=100.0)
    _frames_vs_oracle(rps, orc, n, _blob(n, 70 + n, spread=15.0), cfg, 4)


@pytest.mark.parametrize("layout", ["0", "2"])
def test_sph_nan_and_inf_uploads(gpu, orc, monkeypatch, layout):
    """Uploaded non-finite state: NaN positions with finite velocities, infinite positions, NaN
    velocities, amid ordinary particles.  The scans stop a sum once it is NaN in every component
     only where the particle's state ends NaN anyway; a particle whose own
    position is not finite scans everything.  Every frame bitwise (any NaN equals any NaN)."""
    rps = gpu
    monkeypatch.setenv("RPS_SPH_LAYOUT", layout)
    n = 4096
    cfg = rps.default_particle_config(n, gravity=100.0)
    soa = _blob(n, 91, spread=150.0)  # NaN spreads to ~330 particles in 4 frames
    soa["x"][:6] = F(np.nan)
    soa["y"][6:9] = F(np.nan)
    soa["x"][9:12] = F(np.inf)
    soa["y"][12:14] = F(-np.inf)
    soa["vx"][14:20] = F(np.nan)
    _frames_vs_oracle(rps, orc, n, soa, cfg, 4)


def test_sph_spatial_layout_gated_frames(gpu, orc, monkeypatch):
    """Layout frames after gated ones (SHADER_DELAY 5) and a config change that resets
    frame_count (gated again), at P == N with the layout forced: lookup, offsets, state."""
    rps = gpu
    monkeypatch.setenv("RPS_SPH_LAYOUT", "2")
    n = 8192
    cfg = rps.default_particle_config(n, gravity=100.0)
    soa = _blob(n, 31)
    ext = rps.make_ext()
    st = orc.SphState(n)
    ref = copy_soa(soa)
    with rps.Context(n, rps.MODE_SPH) as ctx:
        ctx.set_config(cfg, ext)
        ctx.upload_soa(soa)
        fc = 0
        for frame in range(14):
            if frame == 8:
                cfg = rps.default_particle_config(n, gravity=50.0)
                ctx.set_config(cfg, ext)
                fc = 0
            ctx.step(1)
            fc += 1
            st.grid(cfg, ref)
            if fc >= 5:
                st.pre(cfg, ref)
                st.sim(cfg, ref)
            assert_bitwise(ctx.read_debug(rps.DEBUG_LOOKUP_OFFSETS), st.offsets, f"offsets f{frame}")
            assert_soa_bitwise(ctx.download_soa(), ref, what=f"f{frame} ")


def _clumped_state(rps, n):
    """The reference scatter at 2^21 with 16 clumps of 4096 particles inside one cell each."""
    scale = (n / 50000) ** 0.5
    cfg = rps.default_particle_config(n, screen_bounds=rps.screen_bounds_for(1920.0 * scale, 1080.0 * scale))
    parts = rps.setup_particles_scatter(cfg, n, seed=0x5EED)
    soa = dict(x=parts["position"][:, 0].copy(), y=parts["position"][:, 1].copy(),
               vx=parts["velocity"][:, 0].copy(), vy=parts["velocity"][:, 1].copy())
    g = np.random.default_rng(77)
    r = float(cfg.smoothing_radius)
    b = list(cfg.screen_bounds)
    k = 4096
    for c in range(16):
        cx = np.floor(g.uniform(b[0] + 4 * r, b[1] - 4 * r) / r) * r + 0.5 * r
        cy = np.floor(g.uniform(b[2] + 4 * r, b[3] - 4 * r) / r) * r + 0.5 * r
        sl = slice(c * k, (c + 1) * k)
        soa["x"][sl] = (cx + g.uniform(-0.2 * r, 0.2 * r, k)).astype(F)
        soa["y"][sl] = (cy + g.uniform(-0.2 * r, 0.2 * r, k)).astype(F)
    return cfg, soa


def test_sph_layout_clustered_runs(gpu, orc, monkeypatch):
    """Runs longer than the layout's 32-entry measure (a clump of particles in one cell) are
    'listed' by the runs kernel.  Their lengths come from the per-key run ends and their slots'
    prediction is spread over every thread of the write kernel (round 2 walked and predicted
    each listed run on one lane, O(run length) dependent loads).  At 2^21 (a default layout
    size) with 16 clumps of 4096 particles each inside one cell: the first frame bitwise
    against the oracle, with and without the layout (timing: the next test)."""
    rps = gpu
    n = 1 << 21
    cfg, soa = _clumped_state(rps, n)
    ext = rps.make_ext(shader_delay=0)
    st = orc.SphState(n, omp=True)
    ref = copy_soa(soa)
    st.grid(cfg, ref)
    st.pre(cfg, ref)
    st.sim(cfg, ref)
    for layout in ("1", "0"):
        monkeypatch.setenv("RPS_SPH_LAYOUT", layout)
        with rps.Context(n, rps.MODE_SPH) as ctx:
            ctx.set_config(cfg, ext)
            ctx.upload_soa(soa)
            ctx.step(1)
            assert_bitwise(ctx.read_debug(rps.DEBUG_DENSITIES), st.dens, f"dens layout={layout}")
            assert_soa_bitwise(ctx.download_soa(), ref, what=f"clustered layout={layout} ")


@pytest.mark.parametrize("n,env", [(2000, {}), (8192, {}), (10000, {}), (32768, {}),
                                   (50000, {"RPS_SPH_CSORT_TLOG": "11"}), (50000, {"RPS_SPH_CSORT_TLOG": "13"}),
                                   (65536, {"RPS_SPH_CSORT": "0"}), (65536, {"RPS_SPH_PAIRS": "0"}),
                                   (50000, {"RPS_SPH_SIM_FUSE": "0"}), (50000, {"RPS_SPH_PAIRS": "0"}),
                                   (50000, {"RPS_SPH_GROUP": "2"}), (65536, {"RPS_SPH_GROUP": "4"}),
                                   (100000, {"RPS_SPH_GROUP": "4"}), (65536, {"RPS_SPH_CSORT_WIDE": "0"}), (32768, {"RPS_SPH_CSORT_WIDE": "1"}),
                                   (50000, {"RPS_SPH_CSORT_WIDE": "0", "RPS_SPH_CSORT_TLOG": "11"}),
                                   (50000, {"RPS_SPH_BATCH_S": "1"}), (50000, {"RPS_SPH_GROUP_S": "2"}),
                                   (20000, {"RPS_SPH_GROUP": "2", "RPS_SPH_GROUP_S": "4", "RPS_SPH_SIM_FUSE": "0"})])
def test_sph_compact_sort_shapes(gpu, orc, monkeypatch, n, env):
    """The compact sort (2^11 <= P <= 2^16: 4-byte entries, every later stage's global passes
    folded into its tail launch) at every shape it takes -- one launch (P = 2^11, 2^13), two and
    three later stages (P = 2^14, 2^15), the forced 2048- and 8192-entry tiles at the reference
    default (five / three later stages) --, and the frame with it, the lane-pair scans and the
    sim's fused long-scan blocks switched off: three all-active frames, every pass bitwise (P != N
    included)."""
    rps = gpu
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    cfg = rps.default_particle_config(n, gravity=100.0)
    _frames_vs_oracle(rps, orc, n, _blob(n, n + 7), cfg, 3)


@pytest.mark.parametrize("n", [50000, 8192])
def test_sph_particle_order_bin_entries(gpu, orc, n):
    """Without the layout the sim writes the next frame's bin entries (key, i), which the next
    sort head reads instead of keying the positions: they must be dropped whenever the state or
    the config changes between frames -- a field upload, a whole upload, a config change, a
    gated frame after a config change -- and every frame stays bitwise."""
    rps = gpu
    cfg = rps.default_particle_config(n, gravity=100.0)
    soa = _blob(n, 17)
    st = orc.SphState(n)
    ref = copy_soa(soa)

    def frames(k, gated=0):
        for f in range(k):
            st.grid(cfg, ref)
            if f >= gated:
                st.pre(cfg, ref)
                st.sim(cfg, ref)

    with rps.Context(n, rps.MODE_SPH) as ctx:
        ctx.set_config(cfg, rps.make_ext(shader_delay=0))
        ctx.upload_soa(soa)
        ctx.step(2)
        frames(2)
        x_new = (ref["x"][:500] * np.float32(0.75)).astype(F)
        ctx.upload_field(rps.FIELD_X, x_new)
        ref["x"][:500] = x_new
        ctx.step(2)
        frames(2)
        assert_bitwise(ctx.read_debug(rps.DEBUG_SPATIAL_LOOKUP), st.lookup, "lookup after field upload")
        assert_soa_bitwise(ctx.download_soa(), ref, what="after field upload ")
        soa2 = _blob(n, 19)
        ctx.upload_soa(soa2)
        ref = copy_soa(soa2)
        ctx.step(2)
        frames(2)
        assert_soa_bitwise(ctx.download_soa(), ref, what="after upload ")
        cfg = rps.default_particle_config(n, gravity=70.0, smoothing_radius=9.0)
        ctx.set_config(cfg, rps.make_ext(shader_delay=3))  # frame_count 0: frames 1, 2 gated
        ctx.step(4)
        frames(4, gated=2)
        assert_bitwise(ctx.read_debug(rps.DEBUG_SPATIAL_LOOKUP), st.lookup, "lookup after config change")
        assert_bitwise(ctx.read_debug(rps.DEBUG_LOOKUP_OFFSETS), st.offsets, "offsets after config change")
        assert_soa_bitwise(ctx.download_soa(), ref, what="after config change ")


@pytest.mark.perf
def test_sph_layout_clustered_runs_timing(gpu, monkeypatch):
    """Performance regression bound on the listed-run path: on the clumped 2^21 state a frame
    with the spatial layout costs at most 3x a lookup-order frame (measured ~1x,
    tools/ab_sph.py; round 2's per-lane walk of listed runs was many times slower).  A
    wall-clock bound, so outside the correctness suite (RPS_PERF_TESTS=1 runs it); the
    clumped state's correctness is test_sph_layout_clustered_runs's."""
    rps = gpu
    n = 1 << 21
    cfg, soa = _clumped_state(rps, n)
    ms = {}
    for layout in ("1", "0"):
        monkeypatch.setenv("RPS_SPH_LAYOUT", layout)
        with rps.Context(n, rps.MODE_SPH) as ctx:
            ctx.set_config(cfg, rps.make_ext(shader_delay=0))
            ctx.upload_soa(soa)
            ctx.step(3)
            ctx.sync()
            ms[layout] = ctx.time_steps(10) / 10
    assert ms["1"] <= 3.0 * ms["0"], ms
