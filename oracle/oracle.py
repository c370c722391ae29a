"""ctypes wrapper of the CPU oracle (oracle/rps_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg — as the checker or the timed CPU baseline, never as the product path.
PARITY UNPINNED at the WGSL-execution boundary (see rps_oracle.h and DESIGN.md §7).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_BUILD = os.environ.get("RPS_ORACLE_BUILD") or os.path.join(_HERE, "_build")  # override: sanitizer builds
_libs = {}

_P, _U32, _U64, _I, _F = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_float


class OrcStats(ctypes.Structure):
    _fields_ = [("bbox", ctypes.c_float * 4), ("kinetic_energy", ctypes.c_double),
                ("particles", ctypes.c_uint64), ("respawned", ctypes.c_uint64)]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib(omp: bool = False, fma: bool = False) -> ctypes.CDLL:
    """The serial checker; omp: the OpenMP build (same bits); fma: the serial build with a*b+c
    contracted into FMAs (NOT the checker: what a WGSL compiler may emit, for the schedule
    envelope of tools/wgsl_schedule_envelope.py)."""
    name = "librps_oracle_fma.so" if fma else "librps_oracle_omp.so" if omp else "librps_oracle.so"
    if name in _libs:
        return _libs[name]
    path = os.path.join(_BUILD, name)
    if not os.path.exists(path):
        build()
    L = ctypes.CDLL(path)
    sig = {
        "orc_philox4x32_10": (None, [_P, _P, _P]),
        "orc_sincos_turns": (None, [_F, ctypes.POINTER(_F), ctypes.POINTER(_F)]),
        "orc_log_unit": (_F, [_F]),
        "orc_set_threads": (None, [_I]),
        "orc_attractor_pos": (None, [_P, ctypes.c_double, ctypes.POINTER(_F), ctypes.POINTER(_F)]),
        "orc_set_color": (None, [_F, _F, _F, _P]),
        "orc_hash_cell": (_U32, [ctypes.c_int32, ctypes.c_int32]),
        "orc_cell_key": (_U32, [ctypes.c_int32, ctypes.c_int32, _U32]),
        "orc_f32_to_i32": (ctypes.c_int32, [_F]),
        "orc_life_steps": (_U32, [_F, _F]),
        "orc_inv_sqrt": (_F, [_F]),
        "orc_exp_from_life": (None, [_P, _U64, _U32, _F, _P]),
        "orc_life_from_exp": (None, [_P, _U64, _U32, _F, _P]),
        "orc_stream_step": (None, [_P, _P, _U64, _U64, _U32, _P, _P, _P, _P, _P, _U64, _P]),
        "orc_stream_step_omp": (None, [_P, _P, _U64, _U64, _U32, _P, _P, _P, _P, _P, _U64, _I]),
        "orc_init_scatter": (None, [_P, _P, _U64, _U64, _U64, _U32, _P, _P, _P, _P, _P, _U64]),
        "orc_nbody_accel": (None, [_P, _P, _P, _U64, _U64, _U64, _P, _P]),
        "orc_nbody_accel_ref": (None, [_P, _P, _P, _U64, _U64, _U64, _P, _P, _P]),
        "orc_nbody_accel_ref_idx": (None, [_P, _P, _P, _U64, _P, _U64, _P, _P, _P]),
        "orc_nbody_accel_f32_omp": (None, [_P, _P, _P, _U64, _U64, _U64, _P, _P, _I]),
        "orc_nbody_integrate": (None, [_P, _P, _P, _P, _P, _P, _P, _P, _U64]),
        "orc_sph_bin": (None, [_P, _P, _P, _P, _P, _U32]),
        "orc_sph_sort": (_U32, [_P, _U32]),
        "orc_sph_offsets": (None, [_P, _P, _U32]),
        "orc_sph_pre": (None, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _U32]),
        "orc_sph_sim": (None, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _U32]),
        "orc_sph_pre_sched": (None, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _U32, _P, _U32]),
        "orc_sph_sim_sched": (None, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _U32, _P, _U32]),
        "orc_sph_pre_stale": (None, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _U32]),
    }
    for k, (res, args) in sig.items():
        f = getattr(L, k)
        f.restype = res
        f.argtypes = args
    _libs[name] = L
    return L


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _ref(s):
    return ctypes.cast(ctypes.byref(s), ctypes.c_void_p)


def philox(ctr, key):
    C = np.asarray(ctr, dtype=np.uint32)
    K = np.asarray(key, dtype=np.uint32)
    O = np.zeros(4, dtype=np.uint32)
    lib().orc_philox4x32_10(_p(C), _p(K), _p(O))
    return O


def sincos_turns(u):
    c, s = ctypes.c_float(), ctypes.c_float()
    lib().orc_sincos_turns(u, ctypes.byref(c), ctypes.byref(s))
    return c.value, s.value


def log_unit(u):
    return lib().orc_log_unit(u)


def set_color(vx, vy, max_energy):
    out = np.zeros(4, dtype=np.float32)
    lib().orc_set_color(vx, vy, max_energy, _p(out))
    return out


def set_color_array(vx, vy, max_energy):
    """Vectorised set_color restatement (same f32 ops) for whole arrays."""
    vx = np.asarray(vx, np.float32)
    vy = np.asarray(vy, np.float32)
    speed_sq = vx * vx + vy * vy
    energy = np.float32(0.5) * speed_sq
    with np.errstate(divide="ignore", invalid="ignore"):
        nrm = energy / np.float32(max_energy)
    nrm = np.where(nrm < 0, np.float32(0), nrm)
    nrm = np.where(nrm > 1, np.float32(1), nrm).astype(np.float32)
    lo = nrm < np.float32(0.5)
    t = np.where(lo, nrm * np.float32(2.0), (nrm - np.float32(0.5)) * np.float32(2.0)).astype(np.float32)
    u = (np.float32(1) - t).astype(np.float32)
    a = np.where(lo[:, None], np.float32([0, 0, 1]), np.float32([0, 1, 0])).astype(np.float32)  # blue / green
    b = np.where(lo[:, None], np.float32([0, 1, 0]), np.float32([1, 0, 0])).astype(np.float32)  # green / red
    out = np.ones((len(vx), 4), np.float32)
    with np.errstate(invalid="ignore"):  # mix(a, b, t) = a * (1 - t) + b * t: NaN t -> NaN
        out[:, :3] = a * u[:, None] + b * t[:, None]
    return out


def inv_sqrt(r2):
    return lib().orc_inv_sqrt(r2)


def life_steps(life, dt):
    return lib().orc_life_steps(life, dt)


def exp_from_life(life, clock, dt):
    """Lifetime expiries (u16) of `life` seconds written at lifetime clock `clock`."""
    life = np.ascontiguousarray(life, np.float32)
    out = np.zeros(len(life), np.uint16)
    lib().orc_exp_from_life(_p(life), len(life), clock & 0xFFFFFFFF, dt, _p(out))
    return out


def life_from_exp(exp, clock, dt):
    """Life in seconds read at lifetime clock `clock` (the clock of the next step)."""
    exp = np.ascontiguousarray(exp, np.uint16)
    out = np.zeros(len(exp), np.float32)
    lib().orc_life_from_exp(_p(exp), len(exp), clock & 0xFFFFFFFF, dt, _p(out))
    return out


def exp_from_steps(steps, clock):
    """Expiries of particles with `steps` (>= 1) lifetime steps left before clock `clock`."""
    st = np.clip(np.ceil(np.asarray(steps, np.float32)), 1, 65535).astype(np.uint32)
    return ((np.uint32(clock & 0xFFFFFFFF) + st - np.uint32(1)) & np.uint32(0xFFFF)).astype(np.uint16)


def steps_from_exp(exp, clock):
    left = (np.asarray(exp, np.uint32) - np.uint32(clock & 0xFFFF)) & np.uint32(0xFFFF)
    return (left + np.uint32(1)).astype(np.float32)


def _exp_of(soa, cfg, clock):
    """The soa's u16 expiry array, created from its `life` view on first use (at `clock`, the
    lifetime clock at which the GPU side received the same life values)."""
    if soa.get("exp") is None and soa.get("life") is not None:
        soa["exp"] = exp_from_life(soa["life"], clock, cfg.fixed_delta_time)
    return soa.get("exp")


def stream_step(cfg, ext, soa, active_step, id_offset=0, stats=False, clock=None):
    """One active stream step in place on soa = dict(x, y, vx, vy[, life / exp]) arrays.
    clock: this step's lifetime clock (default: active_step, i.e. lifetime on since step 0).
    With lifetime on, soa["exp"] (u16) is the state and soa["life"] its seconds view."""
    clock = active_step if clock is None else clock
    use_life = bool(ext.flags & 1) and (soa.get("life") is not None or soa.get("exp") is not None)
    exp = _exp_of(soa, cfg, clock) if use_life else None
    st = OrcStats() if stats else None
    lib().orc_stream_step(_ref(cfg), _ref(ext), id_offset, active_step, clock & 0xFFFFFFFF, _p(soa["x"]),
                          _p(soa["y"]), _p(soa["vx"]), _p(soa["vy"]), _p(exp), len(soa["x"]),
                          _ref(st) if st is not None else None)
    if use_life:
        soa["life"] = life_from_exp(exp, clock + 1, cfg.fixed_delta_time)
    return st


def stream_step_omp(cfg, ext, soa, active_step, id_offset=0, threads=0, clock=None):
    """Same as stream_step, OpenMP build (bench cpu_baseline); the life view is not refreshed."""
    clock = active_step if clock is None else clock
    use_life = bool(ext.flags & 1) and (soa.get("life") is not None or soa.get("exp") is not None)
    exp = _exp_of(soa, cfg, clock) if use_life else None
    lib(omp=True).orc_stream_step_omp(_ref(cfg), _ref(ext), id_offset, active_step, clock & 0xFFFFFFFF,
                                      _p(soa["x"]), _p(soa["y"]), _p(soa["vx"]), _p(soa["vy"]),
                                      _p(exp), len(soa["x"]), threads)


def init_scatter(cfg, ext, seed, n, id_offset=0, global_count=None, life=True, clock=0, omp=False):
    """omp=True: the OpenMP build (particles independent: the same bits, for 10^8 particles)."""
    global_count = global_count or (id_offset + n)
    soa = {k: np.zeros(n, np.float32) for k in ("x", "y", "vx", "vy")}
    soa["exp"] = np.zeros(n, np.uint16) if life else None
    lib(omp=omp).orc_init_scatter(_ref(cfg), _ref(ext), seed, id_offset, global_count, clock & 0xFFFFFFFF,
                           _p(soa["x"]), _p(soa["y"]), _p(soa["vx"]), _p(soa["vy"]), _p(soa["exp"]), n)
    soa["life"] = life_from_exp(soa["exp"], clock, cfg.fixed_delta_time) if life else None
    return soa


def nbody_accel(ext, sx, sy, t0=0, nt=None):
    sx = np.ascontiguousarray(sx, np.float32)
    sy = np.ascontiguousarray(sy, np.float32)
    nt = len(sx) - t0 if nt is None else nt
    ax = np.zeros(nt, np.float32)
    ay = np.zeros(nt, np.float32)
    lib().orc_nbody_accel(_ref(ext), _p(sx), _p(sy), len(sx), t0, nt, _p(ax), _p(ay))
    return ax, ay


def nbody_accel_ref(ext, sx, sy, t0=0, nt=None, threads=0):
    """orc_nbody_accel's f64 sums for targets [t0, t0 + nt) plus G * sum_j |f_ij| per target
    (f64), on the OpenMP build (targets over threads; each target's sum in source order, so
    the same bits as one thread).  Returns (ax, ay, abs_sum)."""
    sx = np.ascontiguousarray(sx, np.float32)
    sy = np.ascontiguousarray(sy, np.float32)
    nt = len(sx) - t0 if nt is None else nt
    ax = np.zeros(nt, np.float32)
    ay = np.zeros(nt, np.float32)
    ab = np.zeros(nt, np.float64)
    L = lib(omp=True)
    if threads:
        L.orc_set_threads(threads)
    L.orc_nbody_accel_ref(_ref(ext), _p(sx), _p(sy), len(sx), t0, nt, _p(ax), _p(ay), _p(ab))
    return ax, ay, ab


def nbody_accel_ref_idx(ext, sx, sy, idx, threads=0):
    """nbody_accel_ref's bits for the targets `idx` (any spread): eight targets per iteration
    vectorised over the targets, each summing its sources in index order.  Returns (ax, ay,
    abs_sum)."""
    sx = np.ascontiguousarray(sx, np.float32)
    sy = np.ascontiguousarray(sy, np.float32)
    idx = np.ascontiguousarray(idx, np.uint64)
    if len(idx) and int(idx.max()) >= len(sx):
        raise ValueError("target index out of range")
    nt = len(idx)
    ax = np.zeros(nt, np.float32)
    ay = np.zeros(nt, np.float32)
    ab = np.zeros(nt, np.float64)
    L = lib(omp=True)
    if threads:
        L.orc_set_threads(threads)
    if nt:
        L.orc_nbody_accel_ref_idx(_ref(ext), _p(sx), _p(sy), len(sx), _p(idx), nt, _p(ax), _p(ay), _p(ab))
    return ax, ay, ab


def nbody_accel_f32_omp(ext, sx, sy, t0=0, nt=None, threads=0):
    """f32 all-pairs force on every host core (bench cpu_baseline; its own summation order)."""
    sx = np.ascontiguousarray(sx, np.float32)
    sy = np.ascontiguousarray(sy, np.float32)
    nt = len(sx) - t0 if nt is None else nt
    ax = np.zeros(nt, np.float32)
    ay = np.zeros(nt, np.float32)
    lib(omp=True).orc_nbody_accel_f32_omp(_ref(ext), _p(sx), _p(sy), len(sx), t0, nt, _p(ax), _p(ay), threads)
    return ax, ay


def nbody_integrate(cfg, ext, ax, ay, soa):
    lib().orc_nbody_integrate(_ref(cfg), _ref(ext), _p(ax), _p(ay), _p(soa["x"]), _p(soa["y"]),
                              _p(soa["vx"]), _p(soa["vy"]), len(soa["x"]))


class SphState:
    """Host buffers of the reference's SPH path (src/particle_buffers.rs:84-168).
    omp=True runs the passes on the OpenMP build (bench.py's cpu_baseline; same results)."""

    def __init__(self, n, omp=False, threads=0):
        self.n = n
        p = 1
        while p < n:
            p <<= 1
        self.P = p
        self.lookup = np.zeros(2 * p, np.uint32)  # zero-initialised like the wgpu buffer
        self.offsets = np.zeros(n, np.uint32)
        self.dens = np.zeros(2 * n, np.float32)
        self.pred = np.zeros(2 * n, np.float32)
        self.omp = omp
        if omp and threads:
            lib(omp=True).orc_set_threads(threads)

    def grid(self, cfg, soa):
        L = lib(omp=self.omp)
        L.orc_sph_bin(_ref(cfg), _p(soa["x"]), _p(soa["y"]), _p(self.lookup), _p(self.offsets), self.n)
        passes = L.orc_sph_sort(_p(self.lookup), self.n)
        L.orc_sph_offsets(_p(self.lookup), _p(self.offsets), self.n)
        return passes

    def pre(self, cfg, soa, fma=False):
        lib(omp=self.omp and not fma, fma=fma).orc_sph_pre(_ref(cfg), _p(soa["vx"]), _p(soa["vy"]), _p(soa["x"]), _p(soa["y"]),
                                      _p(self.lookup), _p(self.offsets), _p(self.dens), _p(self.pred), self.n)

    def sim(self, cfg, soa, fma=False):
        lib(omp=self.omp and not fma, fma=fma).orc_sph_sim(_ref(cfg), _p(soa["x"]), _p(soa["y"]), _p(soa["vx"]), _p(soa["vy"]),
                                      _p(self.lookup), _p(self.offsets), _p(self.dens), _p(self.pred), self.n)

    def copy(self):
        """An independent copy (to run one frame under several schedules from the same state)."""
        c = SphState.__new__(SphState)
        c.__dict__.update({k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in self.__dict__.items()})
        return c

    # Passes 4-5 under another legal WGSL schedule (orc_sph_pre_sched / orc_sph_sim_sched): groups
    # of `group` invocations in lockstep, one group after another in `order`; fma: the FMA-
    # contracted build.  Test infrastructure for tools/wgsl_schedule_envelope.py, not the checker.
    def pre_sched(self, cfg, soa, order, group, fma=False):
        order = np.ascontiguousarray(order, np.uint32)
        assert len(order) == (self.n + group - 1) // group
        lib(fma=fma).orc_sph_pre_sched(_ref(cfg), _p(soa["vx"]), _p(soa["vy"]), _p(soa["x"]), _p(soa["y"]),
                                       _p(self.lookup), _p(self.offsets), _p(self.dens), _p(self.pred), self.n,
                                       _p(order), group)

    def pre_stale(self, cfg, soa, fma=False):
        prev = self.pred.copy()  # the previous frame's predictions, as the buffer still holds them
        lib(fma=fma).orc_sph_pre_stale(_ref(cfg), _p(soa["vx"]), _p(soa["vy"]), _p(soa["x"]), _p(soa["y"]),
                                       _p(self.lookup), _p(self.offsets), _p(self.dens), _p(self.pred), _p(prev),
                                       self.n)

    def sim_sched(self, cfg, soa, order, group, fma=False):
        order = np.ascontiguousarray(order, np.uint32)
        assert len(order) == (self.n + group - 1) // group
        lib(fma=fma).orc_sph_sim_sched(_ref(cfg), _p(soa["x"]), _p(soa["y"]), _p(soa["vx"]), _p(soa["vy"]),
                                       _p(self.lookup), _p(self.offsets), _p(self.dens), _p(self.pred), self.n,
                                       _p(order), group)


def run_steps(mode, cfg, ext, soa, nsteps, frame_count=0, active_steps=0, id_offset=0, sph=None):
    """rps_step semantics on the CPU: frame_count += 1 per step (particle_buffers.rs:227),
    passes gated by frame_count < shader_delay (wgsl:426/:442).  Returns counters."""
    for _ in range(nsteps):
        frame_count += 1
        active = frame_count >= ext.shader_delay
        if mode == 2:
            cfg.frame_count = frame_count
            sph.grid(cfg, soa)
            if active:
                sph.pre(cfg, soa)
                sph.sim(cfg, soa)
        elif active:
            stream_step(cfg, ext, soa, active_steps, id_offset)
        if active:
            active_steps += 1
    return frame_count, active_steps
