"""CPU test double of rps_amd for tests/test_bench_launcher.py ONLY.

bench.py loads it when RPS_BENCH_TEST_STUB=bench_stub, so its launcher (`--gpus N` starting N
ranks), the max-over-ranks timing, the stats cross-check and the side-run watchdog can be
exercised on a CPU box over gloo.  It computes nothing; no product path imports it.

Knobs (environment): RPS_STUB_HANG=nbody  -> the all-pairs side run never returns;
                     RPS_STUB_BAD_STATS=1 -> the "library" all-rank stats are off by one.
"""
import os
import time
import types

MODE_STREAM, MODE_NBODY, MODE_SPH = 0, 1, 2


def default_particle_config(n, gravity=0.0, screen_bounds=None):
    return types.SimpleNamespace(particle_count=n, gravity=gravity, screen_bounds=screen_bounds)


def headline_ext(seed=0x5EED, stats=False):
    return types.SimpleNamespace(shader_delay=5, stats=stats)


def make_ext(**kw):
    return types.SimpleNamespace(**kw)


def comm_unique_id() -> bytes:
    return b"stub-unique-id".ljust(128, b"\0")


def _shard(rank, n):
    r = float(rank)
    return types.SimpleNamespace(bbox=[-(r + 1.0), r + 1.0, -(2.0 * r + 1.0), 2.0 * r + 1.0],
                                 kinetic_energy=0.5 * (r + 1.0), particles=n, respawned=rank, step=400)


class Context:
    def __init__(self, n, mode=MODE_STREAM, device=0, id_offset=0, global_count=None):
        self.n, self.mode, self.n_global = n, mode, global_count
        self.rank = id_offset // n if n else 0
        self.world = 1

    def set_config(self, cfg, ext=None):
        pass

    def comm_init(self, rank, nranks, unique_id):
        assert len(unique_id) == 128
        self.rank, self.world = rank, nranks

    def init_scatter(self, seed=0):
        pass

    def upload(self, parts):
        pass

    def step(self, nsteps=1):
        if self.mode == MODE_NBODY and os.environ.get("RPS_STUB_HANG") == "nbody":
            time.sleep(3600)
        time.sleep(1e-5 * nsteps)

    def sync(self):
        pass

    def time_steps(self, nsteps):
        self.step(nsteps)
        return 0.5 * nsteps

    def set_profiling(self, period=1):
        pass

    def kernel_time(self):
        return 0.5, 10

    def kernel_times(self, cap=1 << 16):
        return [0.5] * 10

    def kernel_clock(self):
        return 2100.0, 64

    def step_cost(self):
        return 32.03 * self.n, "bytes"

    def shard_stats(self):
        return _shard(self.rank, self.n)

    def stats(self):
        if self.world == 1:
            return _shard(self.rank, self.n_global or self.n)
        w = self.world
        s = types.SimpleNamespace(bbox=[-float(w), float(w), -(2.0 * w - 1.0), 2.0 * w - 1.0],
                                  kinetic_energy=sum(0.5 * (r + 1.0) for r in range(w)),
                                  particles=self.n_global or self.n * w, respawned=sum(range(w)), step=400)
        if os.environ.get("RPS_STUB_BAD_STATS") == "1":
            s.particles += 1
        return s

    def close(self):
        pass
