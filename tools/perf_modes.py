"""Throughput of the SPH and N-body modes (run on the GPU box: tools/gpu_run.sh py:tools/perf_modes.py).

SPH: frames/s and particle-steps/s of the full five-pass frame (bin, bitonic, offsets,
pre-sim, sim) at the reference default N = 50 000 and larger; N-body: interactions/s and
TFLOP/s (20 flop/interaction convention) of the force kernel against 157.3 TF FP32."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-particle-system_amd", "python"))

import numpy as np  # noqa: E402

import rps_amd as rps  # noqa: E402

out = {}


def sph(n, frames=50):
    cfg = rps.default_particle_config(n)
    # Spread the reference scatter over a domain that keeps the default density for this N.
    scale = max(1.0, (n / 50000) ** 0.5)
    w, h = 1920.0 * scale, 1080.0 * scale
    cfg = rps.default_particle_config(n, screen_bounds=rps.screen_bounds_for(w, h))
    parts = rps.setup_particles_scatter(cfg, n, seed=1)
    with rps.Context(n, rps.MODE_SPH) as ctx:
        ctx.set_config(cfg, rps.make_ext(shader_delay=0))
        ctx.upload(parts)
        ctx.step(10)
        ctx.sync()
        ctx.set_profiling(1)
        ms = ctx.time_steps(frames) / frames
        sim_ms, cnt = ctx.kernel_time()
    r = dict(n=n, ms_per_frame=ms, frames_per_s=1e3 / ms, particle_steps_per_s=n * 1e3 / ms, sim_kernel_ms=sim_ms)
    print("SPH", json.dumps(r), flush=True)
    out[f"sph_{n}"] = r


def nbody(n, steps=3, warm=1):
    cfg = rps.default_particle_config(n, gravity=0.0)
    ext = rps.make_ext(nbody_strength=1.0, nbody_softening=1.0, shader_delay=0)
    g = np.random.default_rng(0)
    soa = dict(x=g.uniform(-900, 900, n).astype(np.float32), y=g.uniform(-500, 500, n).astype(np.float32),
               vx=np.zeros(n, np.float32), vy=np.zeros(n, np.float32))
    with rps.Context(n, rps.MODE_NBODY) as ctx:
        ctx.set_config(cfg, ext)
        ctx.upload_soa(soa)
        ctx.step(warm)
        ctx.sync()
        ctx.set_profiling(1)
        ctx.step(steps)
        kms, cnt = ctx.kernel_time()
    inter = float(n) * n
    r = dict(n=n, force_kernel_ms=kms, interactions_per_s=inter / (kms * 1e-3),
             tflops_20=20 * inter / (kms * 1e-3) / 1e12, frac_of_157TF=20 * inter / (kms * 1e-3) / 1e12 / 157.3)
    print("NBODY", json.dumps(r), flush=True)
    out[f"nbody_{n}"] = r


def stream(n, fuse, steps=200):
    cfg = rps.default_particle_config(min(n, 0xFFFFFFFF), gravity=0.0)
    ext = rps.headline_ext()
    ext.shader_delay = 0
    ext.fuse_steps = fuse
    with rps.Context(n) as ctx:
        ctx.set_config(cfg, ext)
        ctx.init_scatter()
        ctx.step(steps // 4)
        ctx.sync()
        ms = ctx.time_steps(steps) / steps
    r = dict(n=n, fuse=fuse, ms_per_step=ms, steps_per_s=1e3 / ms, updates_per_s=n * 1e3 / ms,
             hbm_equiv_gbps=40.0 * n / (ms * 1e-3) / 1e9)
    print("STREAM", json.dumps(r), flush=True)
    out[f"stream_{n}_f{fuse}"] = r


def cpu_sph(n, frames=10):
    """Oracle (single-thread C, -O2) SPH frames at the same N: the reference's CPU path."""
    import time
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    scale = max(1.0, (n / 50000) ** 0.5)
    cfg = rps.default_particle_config(n, screen_bounds=rps.screen_bounds_for(1920.0 * scale, 1080.0 * scale))
    parts = rps.setup_particles_scatter(cfg, n, seed=1)
    soa = dict(x=parts["position"][:, 0].copy(), y=parts["position"][:, 1].copy(),
               vx=parts["velocity"][:, 0].copy(), vy=parts["velocity"][:, 1].copy())
    st = orc.SphState(n)
    ext = rps.make_ext(shader_delay=0)
    orc.run_steps(2, cfg, ext, soa, 2, sph=st)
    t0 = time.perf_counter()
    orc.run_steps(2, cfg, ext, soa, frames, sph=st)
    ms = (time.perf_counter() - t0) * 1e3 / frames
    r = dict(n=n, ms_per_frame=ms, frames_per_s=1e3 / ms, cores=1, kind="port (oracle/rps_oracle.c -O2)")
    print("CPU_SPH", json.dumps(r), flush=True)
    out[f"cpu_sph_{n}"] = r


def cpu_nbody(n=8192):
    """Oracle all-pairs (f64 accumulation, single thread) interactions/s."""
    import time
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    ext = rps.make_ext(nbody_strength=1.0, nbody_softening=1.0)
    g = np.random.default_rng(0)
    x = g.uniform(-900, 900, n).astype(np.float32)
    y = g.uniform(-500, 500, n).astype(np.float32)
    t0 = time.perf_counter()
    orc.nbody_accel(ext, x, y)
    el = time.perf_counter() - t0
    r = dict(n=n, interactions_per_s=float(n) * n / el, cores=1, kind="port (oracle, f64 accumulation)")
    print("CPU_NBODY", json.dumps(r), flush=True)
    out[f"cpu_nbody_{n}"] = r


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "cpu":
        cpu_sph(65536)
        cpu_sph(1 << 20, frames=3)
        cpu_nbody()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "sph_small":
        for n in (16384, 65536, 1 << 18):
            sph(n)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "sph":
        for n in (50000, 65536, 1 << 20, 1 << 22):
            sph(n)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "c4":  # BASELINE configs[3]: 2^24 all-pairs, one step
        nbody(1 << 24, steps=1, warm=0)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "nbody":
        for n in (1 << 16, 1 << 17, 1 << 18, 1 << 20):
            nbody(n)
        sys.exit(0)
    for n in (65536, 1 << 20, 1 << 24, 100_000_000):
        for fuse in (1, 4, 16):
            stream(n, fuse)
    for n in (50000, 1 << 20, 1 << 22):
        sph(n)
    for n in (1 << 16, 1 << 18, 1 << 20):
        nbody(n)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "perf_modes.json"), "w") as f:
        json.dump(out, f, indent=1)
