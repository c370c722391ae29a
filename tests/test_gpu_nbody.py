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
