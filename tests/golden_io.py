"""Loading the committed golden fixtures (tests/golden/*.npz, made by make_golden.py)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
STREAM = ("stream_c1_subset.npz", "stream_c1_attractor.npz", "stream_c2_verlet.npz", "stream_c3_features.npz")
SPH = ("sph_n1000.npz", "sph_n2048.npz")
NBODY = ("nbody_n1024.npz",)
# Outputs of the reference's own compute_shader.wgsl (tests/golden/make_wgsl_golden.py):
WGSL_SPH = ("wgsl_sph_n1_tiny.npz", "wgsl_sph_n2_tiny.npz", "wgsl_sph_n3_tiny.npz", "wgsl_sph_n17_tiny.npz",
            "wgsl_sph_n64.npz", "wgsl_sph_n100.npz", "wgsl_sph_n512_default.npz", "wgsl_sph_n200_outside.npz",
            "wgsl_sph_n100_nan.npz")
WGSL_STREAM = ("wgsl_stream_c1_n128.npz",)
# The same shader with frames run under its other legal race outcomes (sched_pre / sched_sim):
WGSL_SPH_SCHED = ("wgsl_sph_n64_sched.npz", "wgsl_sph_n100_sched.npz")


def load(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def structs(rps, g):
    """The fixture's ParticleConfig and ExtConfig, byte for byte."""
    cfg = rps.ParticleConfig.from_buffer_copy(g["cfg"].tobytes())
    ext = rps.ExtConfig.from_buffer_copy(g["ext"].tobytes())
    return cfg, ext


def active_steps(g, ext):
    """(frame, active-step index) of the fixture's active frames: rps_step advances
    frame_count first and runs a step once frame_count >= shader_delay (wgsl:426)."""
    out = []
    for f in range(1, int(g["steps"][0]) + 1):
        if f >= ext.shader_delay:
            out.append((f, len(out)))
    return out


def wgsl_config(rps, g):
    """A WGSL fixture's ParticleConfig (its ext is the reference's: no extensions, SHADER_DELAY 5)."""
    return rps.ParticleConfig.from_buffer_copy(g["cfg"].tobytes()), rps.make_ext()


def inputs(g):
    return {k[3:]: v.copy() for k, v in g.items() if k.startswith("in_")}
