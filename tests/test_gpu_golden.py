"""librps against the committed golden fixtures (tests/golden/, oracle outputs frozen by
make_golden.py), through the C ABI: the stored outputs are the expectation, no oracle runs.
Bitwise for STREAM and SPH; the DESIGN.md §3.4 tolerance for the all-pairs accelerations."""
import numpy as np
import pytest

from golden_io import NBODY, SPH, STREAM, WGSL_SPH, WGSL_STREAM, inputs, load, structs, wgsl_config
from helpers import assert_bitwise, assert_soa_bitwise
from test_gpu_nbody import _check_accel

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", STREAM)
def test_stream_golden_gpu(gpu, name):
    rps = gpu
    g = load(name)
    cfg, ext = structs(rps, g)
    ext.flags |= rps.EXT_STATS  # stats of every step; the state is unaffected
    ext.stats_interval = 1
    soa = inputs(g)
    n = len(soa["x"])
    with rps.Context(n) as ctx:
        ctx.set_config(cfg, ext)
        ctx.upload_soa(soa)
        ctx.step(int(g["steps"][0]))
        got = ctx.download_soa(life="out_exp" in g)
        for k in ("x", "y", "vx", "vy") + (("life",) if "out_exp" in g else ()):
            assert_bitwise(got[k], g["out_" + k], k)
        if "out_exp" in g:
            assert_bitwise(ctx.read_debug(rps.DEBUG_EXPIRY), g["out_exp"], "expiry")
        assert_bitwise(ctx.download()["color"].reshape(-1), g["out_colour"].reshape(-1), "colour")
        st = ctx.stats()
    assert list(st.bbox) == list(g["out_stats_bbox"])
    assert st.respawned == g["out_stats_respawned"][0]


@pytest.mark.parametrize("name", SPH)
def test_sph_golden_gpu(gpu, name):
    rps = gpu
    g = load(name)
    cfg, ext = structs(rps, g)
    soa = inputs(g)
    n = len(soa["x"])
    with rps.Context(n, rps.MODE_SPH) as ctx:
        ctx.set_config(cfg, ext)
        ctx.upload_soa(soa)
        for f in range(1, int(g["frames"][0]) + 1):
            ctx.step(1)
            assert_bitwise(ctx.read_debug(rps.DEBUG_SPATIAL_LOOKUP), g[f"f{f}_lookup"], f"lookup f{f}")
            assert_bitwise(ctx.read_debug(rps.DEBUG_LOOKUP_OFFSETS), g[f"f{f}_offsets"], f"offsets f{f}")
            if f >= ext.shader_delay:
                assert_bitwise(ctx.read_debug(rps.DEBUG_PREDICTED), g[f"f{f}_pred"], f"pred f{f}")
                assert_bitwise(ctx.read_debug(rps.DEBUG_DENSITIES), g[f"f{f}_dens"], f"dens f{f}")
        assert_soa_bitwise(ctx.download_soa(), {k: g["out_" + k] for k in ("x", "y", "vx", "vy")})


@pytest.mark.parametrize("name", NBODY)
def test_nbody_golden_gpu(gpu, orc, name):
    rps = gpu
    g = load(name)
    cfg, ext = structs(rps, g)
    soa = inputs(g)
    n = len(soa["x"])
    with rps.Context(n, rps.MODE_NBODY) as ctx:
        ctx.set_config(cfg, ext)
        ctx.upload_soa(soa)
        ctx.step(1)
        ax = ctx.read_debug(rps.DEBUG_ACCEL_X)
        ay = ctx.read_debug(rps.DEBUG_ACCEL_Y)
        got = ctx.download_soa()
    _check_accel(ax, ay, g["out_ax"], g["out_ay"], ext, soa["x"], soa["y"])
    # the integration given the device's accelerations is bitwise (oracle integrate on them)
    ref = {k: v.copy() for k, v in soa.items()}
    orc.nbody_integrate(cfg, ext, ax, ay, ref)
    assert_soa_bitwise(got, ref)
    for k in ("x", "y", "vx", "vy"):
        np.testing.assert_allclose(got[k], g["out_" + k], rtol=1e-4, atol=1e-3)


def _check_gpu_frame(rps, ctx, g, f, n, sph):
    got = ctx.download_soa()
    for k in ("x", "y", "vx", "vy"):
        assert_bitwise(got[k], g[f"f{f}_{k}"], f"{k} f{f}")
    assert_bitwise(ctx.download()["color"].reshape(-1), g[f"f{f}_color"].reshape(-1), f"colour f{f}")
    if sph:
        assert_bitwise(ctx.read_debug(rps.DEBUG_SPATIAL_LOOKUP), g[f"f{f}_lookup"], f"lookup f{f}")
        assert_bitwise(ctx.read_debug(rps.DEBUG_LOOKUP_OFFSETS), g[f"f{f}_offsets"], f"offsets f{f}")
        if f >= 5:
            assert_bitwise(ctx.read_debug(rps.DEBUG_PREDICTED), g[f"f{f}_pred"], f"pred f{f}")
            assert_bitwise(ctx.read_debug(rps.DEBUG_DENSITIES), g[f"f{f}_dens"], f"dens f{f}")


@pytest.mark.parametrize("name", WGSL_SPH)
def test_wgsl_sph_golden_gpu(gpu, name):
    """librps against outputs of the reference's own compute_shader.wgsl (tests/wgsl_interp.py,
    make_wgsl_golden.py): every buffer of every frame, bitwise."""
    rps = gpu
    g = load(name)
    cfg, ext = wgsl_config(rps, g)
    soa = inputs(g)
    n = len(soa["x"])
    with rps.Context(n, rps.MODE_SPH) as ctx:
        ctx.set_config(cfg, ext)
        ctx.upload_soa(soa)
        for f in range(1, int(g["frames"][0]) + 1):
            ctx.step(1)
            _check_gpu_frame(rps, ctx, g, f, n, True)


@pytest.mark.parametrize("name", WGSL_STREAM)
def test_wgsl_stream_golden_gpu(gpu, name):
    """The STREAM mode with no extensions against the reference shader's particles (pressure,
    near-pressure and viscosity multipliers zero), frame by frame."""
    rps = gpu
    g = load(name)
    cfg, ext = wgsl_config(rps, g)
    soa = inputs(g)
    n = len(soa["x"])
    with rps.Context(n, rps.MODE_STREAM) as ctx:
        ctx.set_config(cfg, ext)
        ctx.upload_soa(soa)
        for f in range(1, int(g["frames"][0]) + 1):
            ctx.step(1)
            _check_gpu_frame(rps, ctx, g, f, n, False)
