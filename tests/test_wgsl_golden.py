"""The oracle against outputs of the reference's own shader (no GPU).

tests/golden/wgsl_*.npz hold every frame's buffers of `assets/compute_shader.wgsl` executed by
tests/wgsl_interp.py under the reference's dispatch sequence (tests/wgsl_harness.py; IEEE f32
per operation, the race schedules of DESIGN.md §3.3).  The oracle (oracle/rps_oracle.c) must
reproduce them bit for bit (NaN payloads excepted, helpers.assert_bitwise), frame by frame:
spatial_lookup, spatial_lookup_offsets, predicted_positions, particle_densities, and the
particles' position, velocity and colour.  This pins the restatement to the reference's code
rather than to itself."""
import numpy as np
import pytest

import wgsl_harness as H
from golden_io import WGSL_SPH, WGSL_SPH_SCHED, WGSL_STREAM, inputs, load, wgsl_config
from helpers import assert_bitwise, copy_soa


def _check_frame(g, f, soa, orc, cfg, st=None):
    for k in ("x", "y", "vx", "vy"):
        assert_bitwise(soa[k], g[f"f{f}_{k}"], f"{k} f{f}")
    colour = orc.set_color_array(soa["vx"], soa["vy"], cfg.max_energy) if f >= 5 else np.ones((len(soa["x"]), 4), np.float32)
    assert_bitwise(colour, g[f"f{f}_color"], f"colour f{f}")
    if st is not None:
        assert_bitwise(st.lookup, g[f"f{f}_lookup"], f"lookup f{f}")
        assert_bitwise(st.offsets, g[f"f{f}_offsets"], f"offsets f{f}")
        if f >= 5:
            assert_bitwise(st.pred, g[f"f{f}_pred"], f"pred f{f}")
            assert_bitwise(st.dens, g[f"f{f}_dens"], f"dens f{f}")


@pytest.mark.parametrize("name", WGSL_SPH)
def test_oracle_sph_matches_reference_shader(rps, orc, name):
    g = load(name)
    cfg, ext = wgsl_config(rps, g)
    soa = inputs(g)
    st = orc.SphState(len(soa["x"]))
    fc = 0
    for f in range(1, int(g["frames"][0]) + 1):
        fc, _ = orc.run_steps(2, cfg, ext, soa, 1, frame_count=fc, sph=st)
        _check_frame(g, f, soa, orc, cfg, st)


@pytest.mark.parametrize("name", WGSL_SPH_SCHED)
def test_oracle_schedule_restatements_match_reference_shader(rps, orc, name):
    """The shader's other legal outcomes of its intra-dispatch races, as the interpreter runs
    them (tests/golden/make_wgsl_golden.py): a frame whose pass 4 is "isolated" (each density
    reads the other particles' predictions of the previous frame, the oracle's
    orc_sph_pre_stale) and / or whose pass 5 is "lockstep" (the viscosity scan sees the
    neighbours' post-pressure velocities: orc_sph_sim_sched with one group of all invocations).
    Bitwise, frame by frame, with the default frames between them: the schedule restatements
    behind tools/wgsl_schedule_envelope.py are the reference's own code's outcomes."""
    g = load(name)
    cfg, _ = wgsl_config(rps, g)
    soa = inputs(g)
    n = len(soa["x"])
    st = orc.SphState(n)
    seen = set()
    for f in range(1, int(g["frames"][0]) + 1):
        cfg.frame_count = f
        st.grid(cfg, soa)
        if f >= 5:  # SHADER_DELAY
            pre, sim = int(g["sched_pre"][f - 1]), int(g["sched_sim"][f - 1])  # 0 lockstep, 1 isolated
            seen.add((pre, sim))
            if pre == 0:
                st.pre(cfg, soa)
            else:
                st.pre_stale(cfg, soa)
            if sim == 1:
                st.sim(cfg, soa)
            else:
                st.sim_sched(cfg, soa, [0], n)
        _check_frame(g, f, soa, orc, cfg, st)
    assert {(1, 1), (0, 0), (1, 0), (0, 1)} <= seen


@pytest.mark.parametrize("name", WGSL_STREAM)
def test_oracle_stream_subset_matches_reference_shader(rps, orc, name):
    """With the pressure, near-pressure and viscosity multipliers at zero, the reference's
    passes 4-5 reduce to gravity -> Euler -> walls -> colour: the oracle's STREAM step with no
    extensions (SHADER_DELAY 5) reproduces the shader's particles frame by frame."""
    g = load(name)
    cfg, ext = wgsl_config(rps, g)
    soa = inputs(g)
    fc = act = 0
    for f in range(1, int(g["frames"][0]) + 1):
        fc, act = orc.run_steps(0, cfg, ext, soa, 1, frame_count=fc, active_steps=act)
        _check_frame(g, f, soa, orc, cfg)


@pytest.mark.skipif(not H.available(), reason="the reference shader is read only in the dev container")
def test_fixture_regenerates_from_reference_shader(rps):
    """The committed fixture is what the reference's shader produces today (the generator and
    the interpreter have not drifted)."""
    g = load("wgsl_sph_n64.npz")
    cfg, _ = wgsl_config(rps, g)
    frames = H.run_reference(cfg, copy_soa(inputs(g)), int(g["frames"][0]))
    for f, buf in enumerate(frames, start=1):
        for k in ("x", "y", "vx", "vy", "color", "lookup", "offsets"):
            assert_bitwise(buf[k], g[f"f{f}_{k}"], f"{k} f{f}")
        if f >= 5:
            assert_bitwise(buf["dens"], g[f"f{f}_dens"], f"dens f{f}")
            assert_bitwise(buf["pred"], g[f"f{f}_pred"], f"pred f{f}")


def test_interpreter_schedule_is_observable(rps):
    """Sanity of the pin: the same shader under a different legal schedule for the sim pass
    (lockstep: neighbours' post-pressure velocities visible to the viscosity scan) gives
    different particles, so the fixtures do discriminate the documented semantics."""
    if not H.available():
        pytest.skip("needs the reference shader")
    import wgsl_interp as W

    g = load("wgsl_sph_n64.npz")
    cfg, _ = wgsl_config(rps, g)
    soa = copy_soa(inputs(g))
    ref = H.ReferenceSPH(H.load_module(), soa, 64)
    orig = W.Dispatch.run

    def run(self, entry, inv, schedule="isolated"):
        return orig(self, entry, inv, "lockstep" if entry == "simulation_step" else schedule)

    W.Dispatch.run = run
    try:
        import copy as _c

        c = _c.copy(cfg)
        for f in range(1, 6):
            c.frame_count = f
            ref.frame(c)
    finally:
        W.Dispatch.run = orig
    got = ref.arrays()
    assert not np.array_equal(got["vx"].view(np.uint32), g["f5_vx"].view(np.uint32))
