"""Drive the reference's WGSL compute shader (tests/wgsl_interp.py) the way its host code does
(test infrastructure; needs /root/reference, so only tests/golden/make_wgsl_golden.py and a
CPU test that skips without it use this module).

Per frame, as `prepare_particle_buffers` (src/particle_buffers.rs:218-236) and
`ParticleComputeNode::run` (src/particle_compute.rs:91-195) do:
  frame_count += 1, config uploaded;
  pass 1 bin_particles_in_grid      ceil(N/64) workgroups of 64
  pass 2 sort_particles             S(S+1)/2 dispatches of ceil(P/2/64) workgroups, each with
                                    SortingParams {n: P, group_width, group_height, step_index}
                                    (src/particle_buffers.rs:108-138)
  pass 3 calculate_spatial_lookup_offsets
  pass 4 pre_simulation_step        lockstep schedule (every prediction written before any
                                    density reads one: DESIGN.md §3.3)
  pass 5 simulation_step            isolated schedule (neighbour velocities from the pass's
                                    start, the particle's own post-pressure: DESIGN.md §3.3)
  (other schedules per frame on request: the shader's other legal outcomes)
Buffers start zero-filled, as wgpu's do; the lookup holds next_pow2(N) entries.
"""
import os

import numpy as np

import wgsl_interp as W

REF_SHADER = "/root/reference/assets/compute_shader.wgsl"
WG = 64
F32, U32 = np.float32, np.uint32

CONFIG_FIELDS = ["particle_count", "particle_size", "smoothing_radius", "max_energy", "damping_factor",
                 "fixed_delta_time", "frame_count", "gravity", "density_kernel_norm", "near_density_kernel_norm",
                 "viscocity_kernel_norm", "_padding", "target_density", "pressure_multiplier", "viscocity_strength",
                 "near_density_multiplier"]


def available():
    return os.path.exists(REF_SHADER)


def load_module():
    with open(REF_SHADER) as f:
        return W.Module(f.read())


def config_uniform(cfg):
    """rps_config (ParticleConfig, 144 B) -> the WGSL Config uniform's field values."""
    out = {}
    for name in CONFIG_FIELDS:
        v = getattr(cfg, name)
        out[name] = U32(v) if name in ("particle_count", "frame_count") else F32(v)
    out["screen_bounds"] = np.array(list(cfg.screen_bounds), dtype=F32)
    out["view_proj"] = np.array(list(cfg.view_proj), dtype=F32).reshape(4, 4)
    return out


class ReferenceSPH:
    """The reference's buffers and per-frame dispatch sequence over the WGSL interpreter."""

    def __init__(self, mod, soa, n):
        self.m, self.n = mod, n
        self.P = 1
        while self.P < n:
            self.P <<= 1
        self.buffers = {
            "particles": W.Buffer([{"position": np.array([soa["x"][i], soa["y"][i]], F32),
                                    "velocity": np.array([soa["vx"][i], soa["vy"][i]], F32),
                                    "color": np.ones(4, F32)} for i in range(n)]),
            "spatial_lookup": W.Buffer([np.zeros(2, U32) for _ in range(self.P)]),
            "spatial_lookup_offsets": W.Buffer([U32(0) for _ in range(n)]),
            "particle_densities": W.Buffer([np.zeros(2, F32) for _ in range(n)]),
            "predicted_positions": W.Buffer([np.zeros(2, F32) for _ in range(n)]),
        }

    def frame(self, cfg, pre_schedule="lockstep", sim_schedule="isolated"):
        """One frame.  The default schedules are the oracle's; the others give
        the other legal outcomes of the shader's intra-dispatch races (tools/wgsl_schedule_envelope.py)."""
        n, P = self.n, self.P
        groups = lambda k: (k + WG - 1) // WG * WG
        uni = {"config": config_uniform(cfg), "sorting_params": None}
        d = W.Dispatch(self.m, self.buffers, uni)
        d.run("bin_particles_in_grid", groups(n))
        stages = P.bit_length() - 1
        for stage in range(stages):
            for step in range(stage + 1):
                gw = 1 << (stage - step)
                uni["sorting_params"] = {"n": U32(P), "group_width": U32(gw), "group_height": U32(2 * gw - 1),
                                         "step_index": U32(step)}
                d.run("sort_particles", groups(P // 2))
        d.run("calculate_spatial_lookup_offsets", groups(n))
        d.run("pre_simulation_step", groups(n), schedule=pre_schedule)
        d.run("simulation_step", groups(n), schedule=sim_schedule)

    def arrays(self):
        b = self.buffers
        p = b["particles"].e
        return {
            "x": np.array([q["position"][0] for q in p], F32), "y": np.array([q["position"][1] for q in p], F32),
            "vx": np.array([q["velocity"][0] for q in p], F32), "vy": np.array([q["velocity"][1] for q in p], F32),
            "color": np.array([q["color"] for q in p], F32),
            "lookup": np.array(b["spatial_lookup"].e, U32).reshape(-1),
            "offsets": np.array(b["spatial_lookup_offsets"].e, U32),
            "dens": np.array(b["particle_densities"].e, F32).reshape(-1),
            "pred": np.array(b["predicted_positions"].e, F32).reshape(-1),
        }


def run_reference(cfg, soa, frames, frame_count=0, schedules=None):
    """`frames` frames of the reference over a copy of `soa`; per-frame buffer snapshots.
    schedules: {frame index (1-based): (pre_schedule, sim_schedule)} for frames run under
    other schedules than the oracle's."""
    import copy

    mod = load_module()
    n = len(soa["x"])
    ref = ReferenceSPH(mod, soa, n)
    out = []
    c = copy.copy(cfg)
    for _ in range(frames):
        frame_count += 1
        c.frame_count = frame_count
        ref.frame(c, *((schedules or {}).get(frame_count, ("lockstep", "isolated"))))
        out.append(ref.arrays())
    return out
