"""rps_amd — Python host mirror of the reference's particle-plugin surface over librps.so.

The reference exposes its hot path as Rust types and Bevy render-graph hooks:

* ``Particle``                      src/particle.rs:20-25       -> :data:`PARTICLE_DTYPE`
* ``ParticleConfig`` + defaults     src/main.rs:25-35, :43-108  -> :class:`ParticleConfig`,
                                                                   :func:`default_particle_config`
* ``prepare_particle_buffers``      src/particle_buffers.rs:38  -> :func:`prepare_particle_buffers`
* ``GPUPipelineBuffers``            src/particle_buffers.rs:17  -> :class:`GPUPipelineBuffers`
* ``ParticleComputeNode::run/update`` src/particle_compute.rs:91-199 -> :class:`ParticleComputeNode`
* ``apply_gui_updates`` norms       src/parameter_gui.rs:78-102 -> :func:`apply_gui_updates`
* ``read_*_from_gpu``               src/debug.rs:121-265        -> :meth:`Context.read_debug`

Everything below calls the C ABI of ``include/rps.h`` through ctypes.  There is no CPU
fallback: if ``librps.so`` (built by ``__graft_entry__.build()``) is missing or cannot load,
importing this module raises.
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(os.path.dirname(_HERE))  # .../rust-particle-system_amd
LIB_PATH = os.path.join(PKG_ROOT, "lib", "librps.so")

# --------------------------------------------------------------------------------------
# ABI structs (must match include/rps.h byte for byte)
# --------------------------------------------------------------------------------------
RPS_OK = 0
RPS_ERR_INVALID_ARGUMENT = 1
RPS_ERR_DEVICE = 2
RPS_ERR_OUT_OF_MEMORY = 3
RPS_ERR_UNSUPPORTED = 4
RPS_ERR_COMM = 5
RPS_ERR_NO_DEVICE = 6

MODE_STREAM, MODE_NBODY, MODE_SPH = 0, 1, 2
EULER, VERLET = 0, 1
EXT_LIFETIME, EXT_STATS, EXT_NBODY_EXTERNAL = 1, 2, 4
MAX_ATTRACTORS = 8
FIELD_X, FIELD_Y, FIELD_VX, FIELD_VY, FIELD_LIFE = 0, 1, 2, 3, 4
FIELD_LIFE_STEPS = 5  # whole lifetime steps left (exact); FIELD_LIFE = that * dt seconds
DEBUG_SPATIAL_LOOKUP, DEBUG_LOOKUP_OFFSETS, DEBUG_DENSITIES, DEBUG_PREDICTED = 16, 17, 18, 19
DEBUG_ACCEL_X, DEBUG_ACCEL_Y = 20, 21
DEBUG_EXPIRY = 22  # u16 lifetime expiry per particle (STREAM)

# Particle, src/particle.rs:20-25 (32 bytes: position @0, velocity @8, color @16)
PARTICLE_DTYPE = np.dtype([("position", "<f4", (2,)), ("velocity", "<f4", (2,)), ("color", "<f4", (4,))])
assert PARTICLE_DTYPE.itemsize == 32


class ParticleConfig(ctypes.Structure):
    """== ParticleConfig, src/main.rs:43-69 / WGSL Config, compute_shader.wgsl:2-25 (144 B)."""

    _fields_ = [
        ("particle_count", ctypes.c_uint32),
        ("particle_size", ctypes.c_float),
        ("smoothing_radius", ctypes.c_float),
        ("max_energy", ctypes.c_float),
        ("damping_factor", ctypes.c_float),
        ("fixed_delta_time", ctypes.c_float),
        ("frame_count", ctypes.c_uint32),
        ("gravity", ctypes.c_float),
        ("density_kernel_norm", ctypes.c_float),
        ("near_density_kernel_norm", ctypes.c_float),
        ("viscocity_kernel_norm", ctypes.c_float),
        ("_padding", ctypes.c_float),
        ("target_density", ctypes.c_float),
        ("pressure_multiplier", ctypes.c_float),
        ("viscocity_strength", ctypes.c_float),
        ("near_density_multiplier", ctypes.c_float),
        ("screen_bounds", ctypes.c_float * 4),
        ("view_proj", ctypes.c_float * 16),
    ]


assert ctypes.sizeof(ParticleConfig) == 144


class Attractor(ctypes.Structure):
    _fields_ = [
        ("center", ctypes.c_float * 2),
        ("orbit_radius", ctypes.c_float),
        ("angular_velocity", ctypes.c_float),
        ("phase", ctypes.c_float),
        ("strength", ctypes.c_float),
        ("softening", ctypes.c_float),
        ("_pad", ctypes.c_float),
    ]


class ExtConfig(ctypes.Structure):
    """Build-defined extensions; all-zero except shader_delay=5 == reference."""

    _fields_ = [
        ("integrator", ctypes.c_uint32),
        ("num_attractors", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
        ("shader_delay", ctypes.c_uint32),
        ("drag", ctypes.c_float),
        ("life_min", ctypes.c_float),
        ("life_max", ctypes.c_float),
        ("emitter_radius", ctypes.c_float),
        ("emitter_center", ctypes.c_float * 2),
        ("spawn_speed_min", ctypes.c_float),
        ("spawn_speed_max", ctypes.c_float),
        ("seed", ctypes.c_uint64),
        ("nbody_strength", ctypes.c_float),
        ("nbody_softening", ctypes.c_float),
        ("stats_interval", ctypes.c_uint32),
        ("fuse_steps", ctypes.c_uint32),
        ("attractors", Attractor * MAX_ATTRACTORS),
    ]


class CreateInfo(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int32),
        ("mode", ctypes.c_uint32),
        ("particle_count", ctypes.c_uint64),
        ("id_offset", ctypes.c_uint64),
        ("global_count", ctypes.c_uint64),
    ]


class Stats(ctypes.Structure):
    _fields_ = [
        ("bbox", ctypes.c_float * 4),
        ("kinetic_energy", ctypes.c_double),
        ("particles", ctypes.c_uint64),
        ("respawned", ctypes.c_uint64),
        ("step", ctypes.c_uint64),
    ]


# --------------------------------------------------------------------------------------
# Library loading (fail loudly; there is no fallback path)
# --------------------------------------------------------------------------------------
class SphCost(ctypes.Structure):
    """rps_sph_cost: algorithmic bytes of one SPH frame (include/rps.h)."""
    _fields_ = [("slots", ctypes.c_uint64), ("particles", ctypes.c_uint64),
                ("scanned_entries", ctypes.c_uint64), ("within_entries", ctypes.c_uint64),
                ("sort_launches", ctypes.c_uint64), ("sort_bytes", ctypes.c_double),
                ("predict_bytes", ctypes.c_double), ("density_bytes", ctypes.c_double),
                ("sim_bytes", ctypes.c_double), ("frame_bytes", ctypes.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class RpsError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"rps status {status}: {message}")
        self.status = status


_lib: Optional[ctypes.CDLL] = None

# (name, restype, argtypes) for every symbol include/rps.h declares.
_P = ctypes.c_void_p
_U32, _U64, _I = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
ABI_SYMBOLS = [
    ("rps_abi_version", _U32, []),
    ("rps_build_id", ctypes.c_char_p, []),
    ("rps_status_string", ctypes.c_char_p, [_I]),
    ("rps_device_count", _I, [ctypes.POINTER(_I)]),
    ("rps_create", _I, [ctypes.POINTER(CreateInfo), ctypes.POINTER(_P)]),
    ("rps_destroy", _I, [_P]),
    ("rps_last_error", ctypes.c_char_p, [_P]),
    ("rps_set_config", _I, [_P, ctypes.POINTER(ParticleConfig), ctypes.POINTER(ExtConfig)]),
    ("rps_get_config", _I, [_P, ctypes.POINTER(ParticleConfig), ctypes.POINTER(ExtConfig)]),
    ("rps_upload_particles", _I, [_P, _P, _U64, _U64]),
    ("rps_download_particles", _I, [_P, _P, _U64, _U64]),
    ("rps_export_particles", _I, [_P, _P, _U64, _U64]),
    ("rps_upload_field", _I, [_P, _I, _P, _U64, _U64]),
    ("rps_download_field", _I, [_P, _I, _P, _U64, _U64]),
    ("rps_read_debug", _I, [_P, _I, _P, _U64]),
    ("rps_init_scatter", _I, [_P, _U64]),
    ("rps_step", _I, [_P, _U32]),
    ("rps_update", _I, [_P]),
    ("rps_sync", _I, [_P]),
    ("rps_get_stats", _I, [_P, ctypes.POINTER(Stats)]),
    ("rps_get_shard_stats", _I, [_P, ctypes.POINTER(Stats)]),
    ("rps_get_counters", _I, [_P, ctypes.POINTER(_U32), ctypes.POINTER(_U64)]),
    ("rps_set_profiling", _I, [_P, _I]),
    ("rps_get_kernel_time", _I, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_U64)]),
    ("rps_get_kernel_times", _I, [_P, ctypes.POINTER(ctypes.c_double), _U64, ctypes.POINTER(_U64)]),
    ("rps_get_kernel_clock", _I, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_U64)]),
    ("rps_time_steps", _I, [_P, _U32, ctypes.POINTER(ctypes.c_double)]),
    ("rps_get_stream", _P, [_P]),
    ("rps_step_cost", _I, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_I)]),
    ("rps_sph_frame_cost", _I, [_P, ctypes.POINTER(SphCost)]),
    ("rps_comm_unique_id", _I, [_P]),
    ("rps_nbody_sources", _I, [_P, _I, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(_U64)]),
    ("rps_comm_init", _I, [_P, _I, _I, _P]),
]


def lib() -> ctypes.CDLL:
    """Load librps.so once.  Raises if the HIP extension was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"librps.so not built at {LIB_PATH}: run __graft_entry__.build() "
                           "(make -C rust-particle-system_amd); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, res, args in ABI_SYMBOLS:
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


# The sources librps.so is built from, in the Makefile's order (SRCS, then HDRS): their sha256
# is the library's rps_build_id() when it was built from this tree.
_BUILD_SOURCES = ("csrc/rps_kernels.hip", "csrc/rps_nbody.hip", "csrc/rps_context.hip",
                  "csrc/rps_device.hpp", "csrc/rps_internal.hpp", "../include/rps.h")


def source_build_id() -> str:
    """sha256 (16 hex digits) of this tree's librps sources, as the Makefile's BUILD_ID."""
    import hashlib

    h = hashlib.sha256()
    for rel in _BUILD_SOURCES:
        with open(os.path.normpath(os.path.join(PKG_ROOT, rel)), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def build_id() -> str:
    """The loaded library's build id (rps_build_id)."""
    return lib().rps_build_id().decode()


def device_count() -> int:
    c = ctypes.c_int(0)
    st = lib().rps_device_count(ctypes.byref(c))
    return c.value if st == RPS_OK else 0


def _check(ctx_ptr, status: int):
    if status != RPS_OK:
        msg = lib().rps_last_error(ctx_ptr)
        raise RpsError(status, msg.decode() if msg else "")


# --------------------------------------------------------------------------------------
# Reference defaults (src/main.rs:25-35, :85-108) and norm recomputation
# --------------------------------------------------------------------------------------
PARTICLE_COUNT = 50000
PARTICLE_SIZE = np.float32(3.0)
SMOOTHING_RADIUS = np.float32(PARTICLE_SIZE * PARTICLE_SIZE)
GRAVITY = np.float32(0.0)
TARGET_DENSITY = np.float32(0.011)
PRESSURE_MULTIPLIER = np.float32(10000.0)
NEAR_DENSITY_MULTIPLIER = np.float32(1000.0)
VISCOCITY_STRENGTH = np.float32(5.0)
DAMPING_FACTOR = np.float32(0.1)
FIXED_DELTA_TIME = np.float32(1.0) / np.float32(100.0)
MAX_ENERGY = np.float32(2000.0)
PI_F32 = np.float32(math.pi)  # std::f32::consts::PI
SHADER_DELAY = 5  # compute_shader.wgsl:66


def kernel_norms(radius) -> tuple:
    """(density, near-density, viscosity) norms, f32 as in src/main.rs:96-98 and
    src/parameter_gui.rs:89-91: 10/(pi r^5), 15/(pi r^6), 4/(pi r^8)."""
    r = np.float32(radius)
    with np.errstate(divide="ignore", over="ignore"):
        d = np.float32(10.0) / (PI_F32 * np.power(r, np.float32(5.0), dtype=np.float32))
        nd = np.float32(15.0) / (PI_F32 * np.power(r, np.float32(6.0), dtype=np.float32))
        v = np.float32(4.0) / (PI_F32 * np.power(r, np.float32(8.0), dtype=np.float32))
    return np.float32(d), np.float32(nd), np.float32(v)


def screen_bounds_for(width: float = 1920.0, height: float = 1080.0, center=(0.0, 0.0)):
    """get_screen_bounds (src/main.rs:136-153) for a camera at `center`."""
    hw, hh = np.float32(width) / np.float32(2.0), np.float32(height) / np.float32(2.0)
    cx, cy = np.float32(center[0]), np.float32(center[1])
    return [float(cx - hw), float(cx + hw), float(cy - hh), float(cy + hh)]


def default_particle_config(particle_count: int = PARTICLE_COUNT, screen_bounds=None,
                            **overrides) -> ParticleConfig:
    """ParticleConfig as inserted by main() (src/main.rs:85-108)."""
    c = ParticleConfig()
    c.particle_count = particle_count
    c.particle_size = PARTICLE_SIZE
    c.smoothing_radius = SMOOTHING_RADIUS
    c.max_energy = MAX_ENERGY
    c.damping_factor = DAMPING_FACTOR
    c.fixed_delta_time = FIXED_DELTA_TIME
    c.frame_count = 0
    c.gravity = GRAVITY
    d, nd, v = kernel_norms(SMOOTHING_RADIUS)
    c.density_kernel_norm, c.near_density_kernel_norm, c.viscocity_kernel_norm = d, nd, v
    c._padding = 0.0
    c.target_density = TARGET_DENSITY
    c.pressure_multiplier = PRESSURE_MULTIPLIER
    c.viscocity_strength = VISCOCITY_STRENGTH
    c.near_density_multiplier = NEAR_DENSITY_MULTIPLIER
    sb = screen_bounds if screen_bounds is not None else screen_bounds_for()
    for k in range(4):
        c.screen_bounds[k] = sb[k]
    for k in range(16):
        c.view_proj[k] = 1.0 if k % 5 == 0 else 0.0  # Mat4::IDENTITY
    for k, val in overrides.items():
        setattr(c, k, val)
    return c


@dataclass
class GUIConfig:
    """GUIConfig, src/parameter_gui.rs:6-22 (slider-editable subset of ParticleConfig)."""

    fixed_delta_time: float = float(FIXED_DELTA_TIME)
    gravity: float = float(GRAVITY)
    damping_factor: float = float(DAMPING_FACTOR)
    smoothing_radius: float = float(SMOOTHING_RADIUS)
    max_energy: float = float(MAX_ENERGY)
    target_density: float = float(TARGET_DENSITY)
    pressure_multiplier: float = float(PRESSURE_MULTIPLIER)
    viscocity_strength: float = float(VISCOCITY_STRENGTH)
    near_density_multiplier: float = float(NEAR_DENSITY_MULTIPLIER)
    applied_changes: bool = False


def apply_gui_updates(sim: ParticleConfig, gui: GUIConfig) -> None:
    """apply_gui_updates, src/parameter_gui.rs:78-102 (copy + norm recomputation)."""
    if not gui.applied_changes:
        return
    sim.fixed_delta_time = gui.fixed_delta_time
    sim.gravity = gui.gravity
    sim.damping_factor = gui.damping_factor
    d, nd, v = kernel_norms(gui.smoothing_radius)
    sim.density_kernel_norm, sim.near_density_kernel_norm, sim.viscocity_kernel_norm = d, nd, v
    sim.smoothing_radius = gui.smoothing_radius
    sim.max_energy = gui.max_energy
    sim.target_density = gui.target_density
    sim.pressure_multiplier = gui.pressure_multiplier
    sim.viscocity_strength = gui.viscocity_strength
    sim.near_density_multiplier = gui.near_density_multiplier
    gui.applied_changes = False


def make_ext(integrator=EULER, attractors: Sequence[dict] = (), drag=0.0, lifetime=None,
             emitter=None, seed=0x5EED, stats=False, stats_interval=1, shader_delay=SHADER_DELAY,
             nbody_strength=0.0, nbody_softening=0.0) -> ExtConfig:
    """Build an ExtConfig.  `lifetime` = (min, max) seconds enables respawn; `emitter` =
    dict(center=(x, y), radius=r, speed=(min, max))."""
    e = ExtConfig()
    e.integrator = integrator
    e.shader_delay = shader_delay
    e.drag = drag
    e.seed = seed
    e.stats_interval = stats_interval
    e.nbody_strength = nbody_strength
    e.nbody_softening = nbody_softening
    flags = 0
    if lifetime is not None:
        flags |= EXT_LIFETIME
        e.life_min, e.life_max = lifetime
    if stats:
        flags |= EXT_STATS
    e.flags = flags
    if emitter:
        e.emitter_center[0], e.emitter_center[1] = emitter.get("center", (0.0, 0.0))
        e.emitter_radius = emitter.get("radius", 0.0)
        e.spawn_speed_min, e.spawn_speed_max = emitter.get("speed", (0.0, 0.0))
    if len(attractors) > MAX_ATTRACTORS:
        raise ValueError("at most 8 attractors")
    e.num_attractors = len(attractors)
    for k, a in enumerate(attractors):
        t = e.attractors[k]
        t.center[0], t.center[1] = a.get("center", (0.0, 0.0))
        t.orbit_radius = a.get("orbit_radius", 0.0)
        t.angular_velocity = a.get("angular_velocity", 0.0)
        t.phase = a.get("phase", 0.0)
        t.strength = a.get("strength", 0.0)
        t.softening = a.get("softening", 1.0)
    return e


def headline_ext(seed=0x5EED, stats=False) -> ExtConfig:
    """4 attractors on circles (r 300, w 0.5 rad/s, phases k*pi/2,
    G 1e5, eps 1), drag 0.1, lifetime U(1, 5) s, emitter disc r 50 at the origin."""
    atts = [dict(center=(0.0, 0.0), orbit_radius=300.0, angular_velocity=0.5,
                 phase=k * math.pi / 2.0, strength=1.0e5, softening=1.0) for k in range(4)]
    return make_ext(EULER, atts, drag=0.1, lifetime=(1.0, 5.0),
                    emitter=dict(center=(0.0, 0.0), radius=50.0, speed=(0.0, 100.0)),
                    seed=seed, stats=stats, stats_interval=100)


# --------------------------------------------------------------------------------------
# Context
# --------------------------------------------------------------------------------------
def _fptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class Context:
    """One device-resident particle system (or one rank's shard of it)."""

    def __init__(self, n: int, mode: int = MODE_STREAM, device: int = 0, id_offset: int = 0,
                 global_count: int = 0):
        L = lib()
        info = CreateInfo(device, mode, n, id_offset, global_count or (id_offset + n))
        ptr = ctypes.c_void_p()
        st = L.rps_create(ctypes.byref(info), ctypes.byref(ptr))
        _check(None, st)
        self._p = ptr
        self.n, self.mode, self.device = n, mode, device
        self.id_offset, self.global_count = id_offset, info.global_count

    # lifetime -------------------------------------------------------------------------
    def close(self):
        if getattr(self, "_p", None):
            lib().rps_destroy(self._p)
            self._p = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _call(self, name, *args):
        _check(self._p, getattr(lib(), name)(self._p, *args))

    # config ---------------------------------------------------------------------------
    def set_config(self, cfg: ParticleConfig, ext: Optional[ExtConfig] = None):
        self._call("rps_set_config", ctypes.byref(cfg), ctypes.byref(ext) if ext is not None else None)

    def get_config(self):
        c, e = ParticleConfig(), ExtConfig()
        self._call("rps_get_config", ctypes.byref(c), ctypes.byref(e))
        return c, e

    # data -----------------------------------------------------------------------------
    def upload(self, particles: np.ndarray, offset: int = 0):
        p = np.ascontiguousarray(particles, dtype=PARTICLE_DTYPE)
        self._call("rps_upload_particles", _fptr(p), offset, len(p))

    def download(self, offset: int = 0, n: Optional[int] = None) -> np.ndarray:
        n = self.n - offset if n is None else n
        out = np.zeros(n, dtype=PARTICLE_DTYPE)
        self._call("rps_download_particles", _fptr(out), offset, n)
        return out

    def export_particles(self, device_ptr: int, offset: int = 0, n: Optional[int] = None):
        """Render interop: AoS Particles (render_shader.wgsl:26-30) into device memory."""
        n = self.n - offset if n is None else n
        self._call("rps_export_particles", ctypes.c_void_p(device_ptr), offset, n)

    def stream_ptr(self) -> int:
        """The context's hipStream_t (rps_get_stream), for callers that order work on it."""
        return int(lib().rps_get_stream(self._p) or 0)

    def upload_field(self, field_id: int, values: np.ndarray, offset: int = 0):
        v = np.ascontiguousarray(values, dtype=np.float32)
        self._call("rps_upload_field", field_id, _fptr(v), offset, len(v))

    def download_field(self, field_id: int, offset: int = 0, n: Optional[int] = None) -> np.ndarray:
        n = self.n - offset if n is None else n
        out = np.zeros(n, dtype=np.float32)
        self._call("rps_download_field", field_id, _fptr(out), offset, n)
        return out

    def upload_soa(self, soa: dict, offset: int = 0):
        for k, fid in (("x", FIELD_X), ("y", FIELD_Y), ("vx", FIELD_VX), ("vy", FIELD_VY), ("life", FIELD_LIFE)):
            if k in soa and soa[k] is not None:
                self.upload_field(fid, soa[k], offset)

    def download_soa(self, life: bool = False) -> dict:
        d = {k: self.download_field(fid) for k, fid in (("x", FIELD_X), ("y", FIELD_Y), ("vx", FIELD_VX), ("vy", FIELD_VY))}
        if life:
            d["life"] = self.download_field(FIELD_LIFE)
        return d

    def read_debug(self, which: int) -> np.ndarray:
        spec = {
            DEBUG_SPATIAL_LOOKUP: (np.uint32, None),
            DEBUG_LOOKUP_OFFSETS: (np.uint32, self.n),
            DEBUG_DENSITIES: (np.float32, 2 * self.n),
            DEBUG_PREDICTED: (np.float32, 2 * self.n),
            DEBUG_ACCEL_X: (np.float32, self.n),
            DEBUG_ACCEL_Y: (np.float32, self.n),
            DEBUG_EXPIRY: (np.uint16, self.n),
        }[which]
        count = spec[1]
        if count is None:
            p = 1
            while p < self.n:
                p <<= 1
            count = 2 * p
        out = np.zeros(count, dtype=spec[0])
        self._call("rps_read_debug", which, _fptr(out), out.nbytes)
        return out

    def init_scatter(self, seed: int = 0x5EED):
        self._call("rps_init_scatter", seed)

    # stepping -------------------------------------------------------------------------
    def step(self, nsteps: int = 1):
        self._call("rps_step", nsteps)

    def update(self):
        self._call("rps_update")

    def sync(self):
        self._call("rps_sync")

    def stats(self) -> Stats:
        s = Stats()
        self._call("rps_get_stats", ctypes.byref(s))
        return s

    def shard_stats(self) -> Stats:
        """This rank's shard only, even with a communicator (rps_get_shard_stats)."""
        s = Stats()
        self._call("rps_get_shard_stats", ctypes.byref(s))
        return s

    def counters(self):
        fc, act = ctypes.c_uint32(), ctypes.c_uint64()
        self._call("rps_get_counters", ctypes.byref(fc), ctypes.byref(act))
        return fc.value, act.value

    def set_profiling(self, period=1):
        """0/False: off; k: HIP-event pair around every k-th dominant-kernel launch."""
        self._call("rps_set_profiling", int(period))

    def kernel_time(self):
        ms, cnt = ctypes.c_double(), ctypes.c_uint64()
        self._call("rps_get_kernel_time", ctypes.byref(ms), ctypes.byref(cnt))
        return ms.value, cnt.value

    def kernel_times(self, cap: int = 1 << 16):
        """Durations (ms, launch order) of the bracketed dominant-kernel launches since
        profiling was enabled (rps_get_kernel_times); starts a new collection."""
        buf = (ctypes.c_double * cap)()
        cnt = ctypes.c_uint64()
        self._call("rps_get_kernel_times", buf, cap, ctypes.byref(cnt))
        return [buf[i] for i in range(min(cap, cnt.value))]

    def kernel_clock(self):
        """(MHz, workgroups): the shader clock sustained by the last profiled N-body force
        launch, the median over its workgroups (rps_get_kernel_clock)."""
        mhz, cnt = ctypes.c_double(), ctypes.c_uint64()
        self._call("rps_get_kernel_clock", ctypes.byref(mhz), ctypes.byref(cnt))
        return mhz.value, cnt.value

    def time_steps(self, nsteps: int) -> float:
        ms = ctypes.c_double()
        self._call("rps_time_steps", nsteps, ctypes.byref(ms))
        return ms.value

    def step_cost(self):
        amt, unit = ctypes.c_double(), ctypes.c_int()
        self._call("rps_step_cost", ctypes.byref(amt), ctypes.byref(unit))
        return amt.value, ("bytes" if unit.value == 0 else "flops")

    def sph_frame_cost(self) -> dict:
        """Algorithmic bytes of one SPH frame of the current state (rps_sph_frame_cost)."""
        c = SphCost()
        self._call("rps_sph_frame_cost", ctypes.byref(c))
        return c.as_dict()

    def nbody_sources(self, pack: bool = True):
        """(device pointer, count) of the global float2 source array (rps_nbody_sources)."""
        ptr, cnt = ctypes.c_void_p(), ctypes.c_uint64()
        self._call("rps_nbody_sources", 1 if pack else 0, ctypes.byref(ptr), ctypes.byref(cnt))
        return ptr.value, cnt.value

    def comm_init(self, rank: int, nranks: int, unique_id: bytes):
        buf = ctypes.create_string_buffer(bytes(unique_id), 128)
        self._call("rps_comm_init", rank, nranks, ctypes.cast(buf, ctypes.c_void_p))


def comm_unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    _check(None, lib().rps_comm_unique_id(ctypes.cast(buf, ctypes.c_void_p)))
    return buf.raw


# --------------------------------------------------------------------------------------
# Reference-shaped host mirror (Bevy plugin surface, minus Bevy)
# --------------------------------------------------------------------------------------
def setup_particles_scatter(config: ParticleConfig, n: Optional[int] = None, seed: int = 0x5EED) -> np.ndarray:
    """Host-side seeded restatement of setup_particles_scatter (src/main.rs:182-216):
    x linear in i, y ~ Normal(centre, 0.125 H) clamped, v = 0, colour white."""
    n = config.particle_count if n is None else n
    x_min, x_max, y_min, y_max = (np.float32(v) for v in config.screen_bounds)
    rng = np.random.default_rng(seed)
    p = np.zeros(n, dtype=PARTICLE_DTYPE)
    t = np.arange(n, dtype=np.float32) / np.float32(n)
    p["position"][:, 0] = x_min + t * (x_max - x_min)
    yc = (y_min + y_max) / np.float32(2.0)
    sd = (y_max - y_min) * np.float32(0.125)
    p["position"][:, 1] = np.clip(rng.normal(yc, sd, n).astype(np.float32), y_min, y_max)
    p["color"] = 1.0
    return p


@dataclass
class ParticleSystem:
    """ParticleSystem component, src/main.rs:37-41."""

    particles: np.ndarray


@dataclass
class GPUPipelineBuffers:
    """GPUPipelineBuffers, src/particle_buffers.rs:17-26: here one rps context owning the
    hipMalloc'd SoA state, the spatial-lookup buffers and the device config."""

    ctx: Context


def prepare_particle_buffers(system: ParticleSystem, config: ParticleConfig,
                             buffers: Optional[GPUPipelineBuffers], mode: int = MODE_SPH,
                             ext: Optional[ExtConfig] = None, device: int = 0) -> GPUPipelineBuffers:
    """prepare_particle_buffers, src/particle_buffers.rs:38-237.

    First call: allocate buffers and upload the particles once (:50-216).  Later calls model
    the render-world config copy: `config` is the main-world resource (frame_count never
    incremented there; the render-world increment of :227 happens in rps_step).  Bevy
    re-extracts it only when it changed (src/particle.rs:35), carrying frame_count = 0, so a
    GUI change resets frame_count and re-arms SHADER_DELAY.
    """
    if buffers is None:
        ctx = Context(len(system.particles), mode=mode, device=device)
        ctx.set_config(config, ext)
        ctx.upload(system.particles)
        return GPUPipelineBuffers(ctx)
    cur, cur_ext = buffers.ctx.get_config()
    probe = ParticleConfig.from_buffer_copy(bytes(config))
    probe.frame_count = cur.frame_count
    changed = bytes(probe) != bytes(cur) or (ext is not None and bytes(ext) != bytes(cur_ext))
    if changed:
        buffers.ctx.set_config(config, ext)
    return buffers


class ParticleComputeNode:
    """ParticleComputeNode, src/particle_compute.rs:84-211."""

    def __init__(self):
        self.entities = []

    def update(self, buffers: GPUPipelineBuffers):  # :197-199
        buffers.ctx.update()
        if buffers not in self.entities:
            self.entities.append(buffers)

    def run(self, buffers: Optional[GPUPipelineBuffers] = None):  # :91-195
        for b in ([buffers] if buffers is not None else self.entities):
            b.ctx.step(1)
