#!/usr/bin/env python3
"""bench.py — particle-updates/s of the per-particle step on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2]): 1e8 particles in all, 4 attractors moving
on circles, drag, lifetime decay + Philox respawn, semi-implicit Euler, walls.  One "step" = one
fused stream-kernel launch over every particle of the rank's shard (in place, tiled SoA).  The
kernel moves 32.03 B per particle-step (x, y, vx, vy read+written and a u16 per group of 64
particles naming its earliest lifetime expiry); SURVEY §8(d)'s 40 B counted an f32 lifetime that
this representation never moves, so `roofline` divides the moved bytes.
Multi-GPU: one process per GPU, the 1e8 particles split into contiguous index shards with
global particle ids, no data-path collective: the metric's configuration at every N (strong
scaling; `--particles P` instead runs P particles per GPU, weak scaling).  Side lines: "sph",
the reference's five-pass SPH frame at 2^22 particles (replicas); "allpairs", the all-pairs
N-body step with its RCCL all-gather, strong-scaled over the ranks.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

A plain `python bench.py --gpus N` (N > 1, no WORLD_SIZE in the environment) starts the N ranks
itself through torch.distributed.run as a child process, before any GPU call, and exits with
its status.  Under a launcher, `--gpus` must equal WORLD_SIZE (exit 2 otherwise).

Prints ONE JSON line on rank 0 (fields: see the contract in DESIGN.md §6).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rust-particle-system_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

METRIC = "particle-updates/sec + achieved HBM GB/s, 10^8 particles, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector peak at the 2400-MHz max clock
FP32_PEAK_CLOCK_MHZ = 2400.0
L2_PEAK_GBPS = 34500.0  # MI355X_MICROARCH.md §L2: aggregate over the 8 XCDs, ~34.5 TB/s
# SURVEY.md §8(d) / BASELINE.md, C3 counted 40 B per particle-step (read and write x, y, vx, vy
# and an f32 lifetime).  The kernel keeps the lifetime as a u16 expiry read and written only in the
# group-steps where one is due, found from a u16 per group of 64 particles:
# it moves 32.03 B, the figure `roofline.achieved` / `frac` use (rps_step_cost); the 40-B rate is
# reported beside it as `algorithmic_equiv_gbps`, and `traffic` is what the PMC counters measured.
ALGO_BYTES_PER_PARTICLE = 40.0
GLOBAL_PARTICLES = 100_000_000  # BASELINE.json metric: 10^8 particles at 1/2/4/8 GPUs
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--global-particles", type=int, default=GLOBAL_PARTICLES,
                    help="particles over all ranks, split into contiguous shards (strong scaling; the metric's 1e8)")
    ap.add_argument("--particles", type=int, default=0,
                    help="particles per GPU instead (weak scaling: the global count grows with N); 0: strong")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline time budget")
    ap.add_argument("--cpu-sample", type=int, default=1 << 22, help="CPU-baseline particles")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--allpairs-n", type=int, default=1 << 24,
                    help="global particles of the all-pairs N-body side measurement (BASELINE.json "
                         "configs[3], C4: 2^24; 0: skip)")
    ap.add_argument("--allpairs-steps", type=int, default=1,
                    help="timed all-pairs steps (one C4 step is ~45 s on one MI355X)")
    ap.add_argument("--allpairs-warmup", type=int, default=1,
                    help="untimed all-pairs steps first (RCCL channels, code objects, clocks)")
    ap.add_argument("--allpairs-cpu-n", type=int, default=65536,
                    help="all-pairs CPU baseline size (SURVEY 8d: 65 536, every target x every source; 0: skip)")
    ap.add_argument("--sph-n", type=int, default=1 << 22,
                    help="particles of the SPH-frame side measurement per rank (0: skip)")
    ap.add_argument("--sph-frames", type=int, default=200,
                    help="timed SPH frames after --sph-warm untimed ones (the window every SPH timing here uses: "
                         "the frame cost drifts with the frame index, DESIGN.md App. B)")
    ap.add_argument("--sph-warm", type=int, default=20)
    ap.add_argument("--sph-cpu-n", type=int, default=1 << 22,
                    help="particles of the SPH CPU-baseline sample (oracle, OpenMP)")
    ap.add_argument("--sph-cpu-frames", type=int, default=3)
    ap.add_argument("--no-configs", action="store_true", help="skip the C1/C2 side measurement")
    ap.add_argument("--sides-first", default="configs",
                    help="comma list of side runs (configs, sph, allpairs) measured before the headline "
                         "(default configs: the chip leaves its idle clock state before the timed region; "
                         "DESIGN.md §6)")
    ap.add_argument("--export-reps", type=int, default=20,
                    help="render-interop export (rps_export_particles) repetitions timed on the headline state; 0: skip")
    ap.add_argument("--fuse-k", type=int, default=16,
                    help="temporal fusion side measure on the headline context after its timed region: "
                         "ext.fuse_steps = K steps per launch (0/1: skip)")
    ap.add_argument("--fuse-steps", type=int, default=64, help="steps timed with --fuse-k (a multiple of K)")
    ap.add_argument("--export-after", action="store_true",
                    help="measure the export after the headline's timed region instead of before its warmup")
    ap.add_argument("--allpairs-timeout", type=float, default=300.0,
                    help="watchdog: print the headline line and exit non-zero if a side run hangs")
    ap.add_argument("--master-port", type=int, default=0,
                    help="rendezvous port when bench.py starts its own ranks (0: a free port)")
    return ap.parse_args()


_T_START = time.perf_counter()


def progress(d, msg):
    """A progress line on rank 0's stderr (the JSON line stays the only stdout line): the C4
    all-pairs side run alone is ~1.5 min without output otherwise."""
    if d.rank == 0:
        print(f"bench.py [{time.perf_counter() - _T_START:6.1f} s] {msg}", file=sys.stderr, flush=True)


WATCHDOG_RC = 3  # a side run hung: the headline line is printed, the process still fails
STATS_MISMATCH_RC = 4  # librps's RCCL stats all-reduce disagrees with torch.distributed's


def launch_ranks(args) -> int:
    """`--gpus N` without a launcher: run N ranks of this script under torch.distributed.run
    (one process per GPU, rendezvous on 127.0.0.1) as a child process.  Nothing here touches
    the GPU, so the ranks own their devices."""
    import socket
    import subprocess

    port = args.master_port
    if not port:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


class Dist:
    """torch.distributed when launched by torchrun; a no-op single process otherwise."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
            import torch  # imported before librps so both share torch's HIP runtime
            import torch.distributed as dist

            backend = "nccl" if torch.cuda.is_available() else "gloo"
            if backend == "nccl":
                torch.cuda.set_device(self.local)
            dist.init_process_group(backend=backend)
            self.torch, self.dist, self.backend = torch, dist, backend

    def barrier(self):
        if self.dist:
            if self.backend == "nccl":
                self.dist.barrier(device_ids=[self.local])
            else:
                self.dist.barrier()

    def sync_device(self):
        if self.dist and self.backend == "nccl":
            self.torch.cuda.synchronize()

    def broadcast_bytes(self, b: bytes) -> bytes:
        if not self.dist:
            return b
        obj = [b if self.rank == 0 else None]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def max(self, v: float) -> float:
        if not self.dist:
            return v
        dev = f"cuda:{self.local}" if self.backend == "nccl" else "cpu"
        t = self.torch.tensor([v], dtype=self.torch.float64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def reduce(self, vals, op: str):
        """Element-wise MAX or SUM of a list of floats over the ranks (f64)."""
        if not self.dist:
            return list(vals)
        dev = f"cuda:{self.local}" if self.backend == "nccl" else "cpu"
        t = self.torch.tensor(list(vals), dtype=self.torch.float64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max" else self.dist.ReduceOp.SUM)
        return [float(x) for x in t.cpu()]

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def load_impl():
    """The library binding.  RPS_BENCH_TEST_STUB names a CPU test double of rps_amd, and only
    tests/test_bench_launcher.py sets it (launcher, aggregation and watchdog checks without a
    GPU); every real run loads the HIP library, which fails loudly when it is missing."""
    import importlib

    stub = os.environ.get("RPS_BENCH_TEST_STUB")
    return importlib.import_module(stub) if stub else importlib.import_module("rps_amd")


def shard(args, d):
    """(particles of this rank, its first global id, global particles).  Strong scaling (the
    default): the global count split into contiguous index ranges, rank r owning
    [r·G/W, (r+1)·G/W).  Weak (`--particles P`): P per rank, G = P·W."""
    if args.particles:
        return args.particles, d.rank * args.particles, args.particles * d.world
    g = args.global_particles
    lo, hi = g * d.rank // d.world, g * (d.rank + 1) // d.world
    return hi - lo, lo, g


def workload(rps, n_global):
    cfg = rps.default_particle_config(min(n_global, 0xFFFFFFFF), gravity=0.0)
    ext = rps.headline_ext(stats=True)  # stats reduced every 100 steps (amortised)
    ext.shader_delay = 0  # every timed step is an active step
    return cfg, ext


def global_stats(d, st):
    """The last stats step over every rank's shard, combined after the timed region in the
    form librps's own all-reduce uses (rps_get_stats with a communicator): MAX of the negated
    minima and the maxima, SUM of KE, particles and respawns."""
    mm = d.reduce([-st.bbox[0], st.bbox[1], -st.bbox[2], st.bbox[3]], "max")
    ke, parts, resp = d.reduce([st.kinetic_energy, float(st.particles), float(st.respawned)], "sum")
    return {"step": st.step, "bbox": [-mm[0], mm[1], -mm[2], mm[3]], "kinetic_energy": ke,
            "respawned_last": int(resp), "particles": int(parts), "ranks": d.world}


def pmc_traffic(workload_name, n_rank):
    """The dominant kernel's HBM bytes per launch from the committed PMC run of this workload
    (profiles/pmc_traffic.json, tools/pmc_table.py, keyed by the workload name, which carries the
    global particle count), when that run processed the same number of particles per launch as
    this rank; None otherwise (another workload, or shards of another size)."""
    try:
        with open(PMC_FILE) as f:
            rec = json.load(f).get(workload_name, {})
    except (OSError, ValueError):
        return None
    if not rec or rec.get("particles_per_launch", 100_000_000) != n_rank:
        return None
    return rec.get("hbm_bytes_per_launch")


def pmc_sph():
    """The SPH frame's measured per-kernel traffic (tools/collect_sph_traffic.py), or None."""
    try:
        with open(PMC_FILE) as f:
            return json.load(f).get("SPH-2^22-frame")
    except (OSError, ValueError):
        return None


def cpu_baseline(rps, args, cfg, ext):
    """The oracle's OpenMP build (same f32 semantics as the kernel) on the host cores, on a
    bounded sample of the workload: the same per-particle step over `cpu_sample` particles
    with the C3 configuration, repeated for about `cpu_seconds`."""
    import oracle as orc

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    n = args.cpu_sample
    soa = orc.init_scatter(cfg, ext, args.seed, n, global_count=args.global_particles)
    orc.stream_step_omp(cfg, ext, soa, 0, threads=threads)  # warm (page-in, thread pool)
    t0 = time.perf_counter()
    steps = 0
    while True:
        orc.stream_step_omp(cfg, ext, soa, 1 + steps, threads=threads)
        steps += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds or steps >= 10000:
            break
    return {"value": n * steps / el, "unit": "particle-updates/s", "cores": threads, "kind": "port",
            "sample": f"{n} particles x {steps} steps of the C3 step (oracle/rps_oracle.c, -O3 -fopenmp, "
                      f"{threads} threads), {el:.1f} s"}


def allpairs(rps, args, d):
    """Side measurement (north_star C4/C5 shape, strong scaling): all-pairs softened gravity
    over `allpairs_n` global particles (A11 scatter), targets index-sharded over the ranks,
    sources = every particle via the library's in-place ncclAllGather of float2 positions
    over xGMI each step.  Not the headline `value`; reported under "allpairs"."""
    ng = args.allpairs_n
    if ng % d.world:
        raise ValueError("allpairs_n must divide by the world size")
    n = ng // d.world
    cfg = rps.default_particle_config(min(ng, 0xFFFFFFFF), gravity=0.0)
    ext = rps.make_ext(nbody_strength=1.0e5, nbody_softening=1.0, shader_delay=0)
    ctx = rps.Context(n, rps.MODE_NBODY, device=d.local if d.dist else 0, id_offset=d.rank * n,
                      global_count=ng)
    try:
        ctx.set_config(cfg, ext)
        if d.dist:  # under a launcher, even with one rank: the library's own RCCL all-gather
            ctx.comm_init(d.rank, d.world, d.broadcast_bytes(rps.comm_unique_id() if d.rank == 0 else b""))
        ctx.init_scatter(args.seed)
        if args.allpairs_warmup > 0:
            ctx.step(args.allpairs_warmup)  # warm: RCCL channels, LDS kernels
        ctx.sync()
        d.sync_device()
        d.barrier()
        ctx.set_profiling(1)
        progress(d, f"allpairs: {args.allpairs_steps} timed step(s) of {n} targets x {ng} sources")
        t0 = time.perf_counter()
        ctx.step(args.allpairs_steps)
        ctx.sync()
        d.sync_device()
        t1 = time.perf_counter()
        d.barrier()
        el = d.max(t1 - t0)
        kms, _ = ctx.kernel_time()
        kms = d.max(kms)
        # The shader clock the chip held under the force kernel (median over its workgroups of
        # in-kernel s_memtime / s_memrealtime stamps, last timed launch; rps_get_kernel_clock).
        clk_mhz, clk_wgs = ctx.kernel_clock()
        clk_mhz = -d.max(-clk_mhz)  # the slowest rank's clock
    finally:
        ctx.close()
    inter = float(ng) * ng * args.allpairs_steps
    flop = 20.0 * float(n) * ng  # per rank per step (GPU Gems 3 convention, rsqrt = 4)
    tf = flop / (kms * 1e-3) / 1e12
    peak_at_clk = FP32_PEAK_TFLOPS * clk_mhz / FP32_PEAK_CLOCK_MHZ
    cfg_name = {1 << 24: "C4 (BASELINE.json configs[3])", 1 << 27: "C5 (BASELINE.json configs[4])"}.get(ng, "")
    return {"workload": f"all-pairs softened gravity, {ng} global particles, index-sharded x{d.world}"
                        + (f" -- {cfg_name}" if cfg_name else ""),
            "particles": ng, "particles_per_rank": n, "interactions_per_step": float(ng) * ng,
            "scaling": "strong", "steps": args.allpairs_steps, "warmup": args.allpairs_warmup, "ms_per_step": el * 1e3 / args.allpairs_steps,
            "interactions_per_s": inter / el, "force_kernel_ms": kms,
            "roofline": {"bound": "valu", "achieved": tf, "peak": FP32_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": tf / FP32_PEAK_TFLOPS,
                         "sustained_clock_mhz": clk_mhz, "clock_samples": clk_wgs,
                         "peak_at_sustained_clock": peak_at_clk, "frac_at_sustained_clock": tf / peak_at_clk,
                         "issue_floor_frac": 0.822,
                         "note": "peak 157.3 TF assumes 2400 MHz; frac_at_sustained_clock divides by the peak "
                                 "at the clock the chip held (in-kernel stamps), i.e. the clock-independent share; "
                                 "the loop's issue floor is 0.822 of either (DESIGN.md §5)"},
            "collective": f"ncclAllGather {8 * ng} B per step" if d.dist else "none (no launcher)",
            **({"cpu_baseline": allpairs_cpu_baseline(rps, args, ext)}
               if d.rank == 0 and d.world == 1 and not args.no_cpu_baseline and args.allpairs_cpu_n > 0 else {})}


def allpairs_cpu_baseline(rps, args, ext):
    """SURVEY 8(d)'s all-pairs CPU baseline: the same softened-gravity force at N = 65 536
    (every target against every source), f32, vectorised with OpenMP on the host cores
    (oracle/rps_oracle.c orc_nbody_accel_f32_omp), repeated for about 3 s.  Interactions/s; the
    rate at 2^22 or 2^24 is this one extrapolated (the work per interaction does not depend on N)."""
    import numpy as np
    import oracle as orc

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    n = args.allpairs_cpu_n
    g = np.random.default_rng(args.seed)
    sx = g.uniform(-960.0, 960.0, n).astype(np.float32)
    sy = g.uniform(-540.0, 540.0, n).astype(np.float32)
    orc.nbody_accel_f32_omp(ext, sx, sy, nt=min(n, 1024), threads=threads)  # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        orc.nbody_accel_f32_omp(ext, sx, sy, threads=threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= 3.0 or reps >= 100:
            break
    return {"value": float(n) * n * reps / el, "unit": "interactions/s", "cores": threads, "kind": "port",
            "sample": f"{n} x {n} interactions x {reps} (f32, oracle/rps_oracle.c orc_nbody_accel_f32_omp, "
                      f"-O3 -fopenmp omp simd, {threads} threads), {el:.1f} s; extrapolated to {args.allpairs_n}"}


def configs_side(rps, args, d):
    """BASELINE.json's other single-GPU streaming configs, measured beside the headline (each
    rank its own replica; they are parity-test configs, and SURVEY 8(d) does not grade their
    roofline: their state is a few MB to 32 MiB, cache-resident or launch-bound).  C1: 65 536
    particles, one point attractor, Euler; C2: 2^20 particles, one attractor, velocity-Verlet.
    Both with the reference's scatter and walls, every step active, 32 B/particle-step moved."""
    out = {}
    att = [dict(center=(0.0, 0.0), strength=1.0e5, softening=1.0)]
    for key, n, integ, steps in (("c1", 65536, rps.EULER, 2000), ("c2", 1 << 20, rps.VERLET, 1000)):
        cfg = rps.default_particle_config(n, gravity=9.8)
        ext = rps.make_ext(integ, att, shader_delay=0)
        ctx = rps.Context(n, rps.MODE_STREAM, device=d.local if d.dist else 0)
        try:
            ctx.set_config(cfg, ext)
            ctx.upload(rps.setup_particles_scatter(cfg, n, seed=args.seed))
            ctx.step(100)
            ctx.sync()
            t0 = time.perf_counter()
            gpu_ms = ctx.time_steps(steps)
            wall = time.perf_counter() - t0
        finally:
            ctx.close()
        out[key] = {"particles": n, "integrator": "euler" if integ == rps.EULER else "verlet", "attractors": 1,
                    "steps": steps, "us_per_step": gpu_ms * 1e3 / steps, "wall_us_per_step": wall * 1e6 / steps,
                    "updates_per_s": n * steps / (gpu_ms * 1e-3),
                    "moved_gbps": 32.0 * n * steps / (gpu_ms * 1e-3) / 1e9}
    return out


def sph_roofline(cost, sim_ms, frame_ms, pmc):
    """The SPH line's `roofline` and `frame_cost` objects.  Measured traffic (PMC, the bench
    workload at 2^22; profiles/pmc_traffic.json): the sim kernel's L1 -> L2 request bytes and
    memory-side bytes per launch, and every SPH kernel's memory-side bytes per frame.  `frac` is a
    utilisation: the measured L1 -> L2 bytes' rate against the aggregate L2 peak (the scans'
    gathers are mostly L1 hits, so the algorithmic bytes -- every neighbour gather charged -- only
    give an equivalence rate, `algorithmic_equiv_*`).  Without a PMC record the rates are null."""
    pmc_src = f"profiles/pmc_traffic.json 'SPH-2^22-frame' (round {pmc.get('round')}; not this run)" if pmc else None
    sim_name, sim_pmc = next(((k, v) for k, v in (pmc or {}).get("per_dispatch", {}).items()
                              if k.startswith("sph_sim")), (None, None))
    sim_l2 = sim_pmc["l2_read_bytes"] + sim_pmc["l2_write_bytes"] if sim_pmc else None
    sim_hbm = sim_pmc.get("hbm_bytes") if sim_pmc else None

    def rate(b, ms):
        return b / (ms * 1e-3) / 1e9 if b else None

    def frac(b, ms, peak):
        return rate(b, ms) / peak if b else None

    # The sim's utilisation of the units that bound it (PMC counter pass of the same workload,
    # tools/sph_counter_table.py): the texture addressers and the VALU, not bytes.
    cnt = ((pmc or {}).get("counters", {}).get("per_kernel", {}) or {}).get(sim_name or "", {})
    hbm_frame = (pmc or {}).get("frame_sum_of_kernels", {}).get("hbm_bytes")
    l2_frame = (pmc or {}).get("frame_sum_of_kernels", {}).get("l2_bytes")
    sim_algo_gbps = cost["sim_bytes"] / (sim_ms * 1e-3) / 1e9
    roofline = {"bound": "l2", "kernel": sim_name or "sph_sim_kernel",
                "achieved": rate(sim_l2, sim_ms), "peak": L2_PEAK_GBPS, "unit": "GB/s",
                "frac": frac(sim_l2, sim_ms, L2_PEAK_GBPS), "traffic": sim_l2,
                "hbm_bytes_per_launch": sim_hbm, "hbm_gbps": rate(sim_hbm, sim_ms),
                "hbm_frac": frac(sim_hbm, sim_ms, HBM_PEAK_GBPS),
                "traffic_source": pmc_src,
                "algorithmic_bytes_per_launch": cost["sim_bytes"],
                "algorithmic_equiv_gbps": sim_algo_gbps,
                "algorithmic_equiv_frac": sim_algo_gbps / L2_PEAK_GBPS,
                "ta_busy": cnt.get("ta_busy"), "valu_busy": cnt.get("valu_busy"), "l1_hit": cnt.get("l1_hit"),
                "lines_per_load": cnt.get("lines_per_load"),
                "scanned_entries_per_particle": cost["scanned_entries"] / cost["slots"],
                "within_radius_per_particle": cost["within_entries"] / cost["slots"],
                "note": "achieved/frac: the sim kernel's L1 -> L2 request bytes measured by the PMC counters "
                        "(traffic, per launch) / this run's kernel time, against the aggregate L2 peak; "
                        "hbm_frac: its memory-side bytes against HBM; algorithmic_equiv_*: every neighbour "
                        "gather charged (mostly L1 hits) -- an equivalence, not a utilisation; ta_busy / valu_busy: "
                        "the units that bound the scan (texture addressers at ~29 cache lines per gather "
                        "instruction, and the VALU), from the committed counter pass (DESIGN.md App. B)"}
    frame_cost = {"hbm_bytes_measured": hbm_frame, "hbm_bytes_source": pmc_src,
                  "hbm_gbps": rate(hbm_frame, frame_ms), "frac": frac(hbm_frame, frame_ms, HBM_PEAK_GBPS),
                  "bound": "hbm", "peak": HBM_PEAK_GBPS,
                  "l2_bytes_measured": l2_frame, "l2_frac": frac(l2_frame, frame_ms, L2_PEAK_GBPS),
                  "algorithmic_bytes": cost["frame_bytes"],
                  "algorithmic_equiv_frac_of_l2": cost["frame_bytes"] / (frame_ms * 1e-3) / 1e9 / L2_PEAK_GBPS,
                  "sort_launches": cost["sort_launches"],
                  "note": "frac: the frame's memory-side bytes (sum over its kernels, PMC) per frame time against HBM"}
    return roofline, frame_cost


def sph_side(rps, args, d):
    """Side measurement: the reference's full five-pass SPH frame (bin,
    bitonic sort, offsets, pre-simulation, simulation) at `sph_n` particles, the reference
    scatter spread over a viewport scaled to keep the default density.  SPH does not shard in
    this tier, so every rank runs its own replica; the aggregate is
    replicas x particles x frames / max-over-ranks time."""
    n = args.sph_n
    scale = max(1.0, (n / 50000) ** 0.5)
    cfg = rps.default_particle_config(n, screen_bounds=rps.screen_bounds_for(1920.0 * scale, 1080.0 * scale))
    parts = rps.setup_particles_scatter(cfg, n, seed=args.seed)
    ctx = rps.Context(n, rps.MODE_SPH, device=d.local if d.dist else 0)
    try:
        ctx.set_config(cfg, rps.make_ext(shader_delay=0))
        ctx.upload(parts)
        ctx.step(args.sph_warm)
        ctx.sync()
        d.sync_device()
        d.barrier()
        ctx.set_profiling(1)
        t0 = time.perf_counter()
        ctx.step(args.sph_frames)
        ctx.sync()
        d.sync_device()
        t1 = time.perf_counter()
        d.barrier()
        el = d.max(t1 - t0)
        sim_ms, _ = ctx.kernel_time()
        cost = ctx.sph_frame_cost()  # algorithmic bytes of the last frame (include/rps.h)
    finally:
        ctx.close()
    sim_ms = d.max(sim_ms)
    frame_ms = el * 1e3 / args.sph_frames
    pmc = pmc_sph() if n == 1 << 22 else None
    rl, fc = sph_roofline(cost, sim_ms, frame_ms, pmc)
    slots = 1 << max(0, (n - 1).bit_length())  # P = next_pow2(N) (particle_buffers.rs:86)
    layout = os.environ.get("RPS_SPH_LAYOUT", "1")
    spatial = layout == "2" or (layout == "1" and slots >= (1 << 20))  # rps_context.hip
    out = {"workload": f"SPH frame (5 passes, bitwise == oracle), {n} particles per rank, reference scatter",
           "record_layout": "cell tiles (spatial)" if spatial else "lookup order",
           "scaling": "replicas", "warm_frames": args.sph_warm, "frames": args.sph_frames, "ms_per_frame": frame_ms,
           "particle_steps_per_s": float(n) * d.world * args.sph_frames / el,
           "sim_kernel_ms": sim_ms, "roofline": rl, "frame_cost": fc}
    out["reference_sizes"] = [sph_small(rps, args, d, m) for m in (50000, 65536)]
    if d.rank == 0 and d.world == 1 and not args.no_cpu_baseline and args.sph_cpu_n > 0:
        out["cpu_baseline"] = sph_cpu_baseline(rps, args)
    return out


def sph_small(rps, args, d, n):
    """The SPH frame at the reference's own scale: its default N = 50 000 (src/main.rs:25; P =
    2^16 with the pad entries of src/particle_buffers.rs:86) and 65 536, where launches and
    latency, not bytes, set the frame time.  The reference dispatches 4 + S(S+1)/2 passes per
    frame (S = log2 P; src/particle_compute.rs:105-191); `sort_launches` is this build's launch
    count for the same network (the frame's other kernels: DESIGN.md §5.2)."""
    cfg = rps.default_particle_config(n)
    parts = rps.setup_particles_scatter(cfg, n, seed=args.seed)
    frames = args.sph_frames
    ctx = rps.Context(n, rps.MODE_SPH, device=d.local if d.dist else 0)
    try:
        ctx.set_config(cfg, rps.make_ext(shader_delay=0))
        ctx.upload(parts)
        ctx.step(args.sph_warm)
        ctx.sync()
        ms = ctx.time_steps(frames) / frames
        cost = ctx.sph_frame_cost()
    finally:
        ctx.close()
    s = max(0, (n - 1).bit_length())
    return {"particles": n, "warm_frames": args.sph_warm, "frames": frames, "ms_per_frame": d.max(ms),
            "sort_launches": cost["sort_launches"],
            "reference_dispatches_per_frame": 4 + s * (s + 1) // 2,
            "timing": "one HIP event pair around the frames on the context stream (rps_time_steps), every frame active"}


def sph_cpu_baseline(rps, args):
    """The reference's SPH frame on the host: the oracle's restatement of the five WGSL passes
    (oracle/rps_oracle.c, the OpenMP build at the stream baseline's thread count; results
    identical to the serial checker) over a bounded sample of the same workload (the reference
    scatter at the default density), timed after one warm frame."""
    import oracle as orc

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    n = args.sph_cpu_n
    scale = max(1.0, (n / 50000) ** 0.5)
    cfg = rps.default_particle_config(n, screen_bounds=rps.screen_bounds_for(1920.0 * scale, 1080.0 * scale))
    parts = rps.setup_particles_scatter(cfg, n, seed=args.seed)
    soa = dict(x=parts["position"][:, 0].copy(), y=parts["position"][:, 1].copy(),
               vx=parts["velocity"][:, 0].copy(), vy=parts["velocity"][:, 1].copy())
    st = orc.SphState(n, omp=True, threads=threads)
    ext = rps.make_ext(shader_delay=0)
    fc, _ = orc.run_steps(2, cfg, ext, soa, 1, sph=st)  # warm frame
    t0 = time.perf_counter()
    orc.run_steps(2, cfg, ext, soa, args.sph_cpu_frames, frame_count=fc, sph=st)
    el = time.perf_counter() - t0
    return {"value": float(n) * args.sph_cpu_frames / el, "unit": "particle-steps/s", "cores": threads,
            "kind": "port",
            "sample": f"{n} particles x {args.sph_cpu_frames} frames of the five passes (oracle/rps_oracle.c, "
                      f"-O3 -fopenmp, {threads} threads), {el:.1f} s; {el * 1e3 / args.sph_cpu_frames:.0f} ms/frame"}


def fused_side(ctx, d, cfg, ext, n_global, k, steps):
    """ext.fuse_steps = k (include/rps.h) on the headline's context once its timed region, stats and
    export are done: k steps per launch with the state in registers, bitwise == k separate steps
    (tests/test_gpu_stream.py).  Reported beside the headline, not as it: the reference renders
    between frames (one dispatch per frame), so the headline keeps one launch per step."""
    import copy

    fext = copy.copy(ext)
    fext.fuse_steps = k
    ctx.set_config(cfg, fext)
    steps = max(k, steps - steps % k)
    ctx.step(k)  # warm: one fused launch
    ctx.sync()
    d.sync_device()
    d.barrier()
    ms = d.max(ctx.time_steps(steps))
    moved, _ = ctx.step_cost()
    return {"fuse_steps": k, "steps": steps, "launches": steps // k, "ms_per_step": ms / steps,
            "updates_per_s": float(n_global) * steps / (ms * 1e-3),
            "moved_bytes_per_step": d.max(moved) / k if moved else None,
            "timing": "one HIP event pair on the context stream around the fused launches; max over ranks",
            "note": "opt-in temporal fusion (ext.fuse_steps): each particle read and written once per k steps, "
                    "so the step is VALU-bound (attractor force), not HBM-bound; headless use only"}


def export_side(ctx, n, reps):
    """SURVEY 8(f)3, render interop: rps_export_particles writes the headline state as the
    reference's 32-B Particle buffer (render_shader.wgsl:26-30; colour derived, set_color)
    into device memory, on the context stream.  Timed with HIP events on that stream over
    `reps` exports of all n particles; algorithmic bytes 48 per particle (16 read, 32 written)."""
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime librps already loaded
    vp = ctypes.c_void_p
    hip.hipMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t]
    hip.hipFree.argtypes = [vp]
    hip.hipEventCreate.argtypes = [ctypes.POINTER(vp)]
    hip.hipEventRecord.argtypes = [vp, vp]
    hip.hipEventSynchronize.argtypes = [vp]
    hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), vp, vp]
    hip.hipEventDestroy.argtypes = [vp]
    buf, e0, e1 = vp(), vp(), vp()
    if hip.hipMalloc(ctypes.byref(buf), n * 32) != 0:
        return {"error": "hipMalloc of the export buffer failed"}
    try:
        if hip.hipEventCreate(ctypes.byref(e0)) != 0 or hip.hipEventCreate(ctypes.byref(e1)) != 0:
            raise RuntimeError("hipEventCreate failed")
        stream = vp(ctx.stream_ptr())
        ctx.export_particles(buf.value)  # warm
        if hip.hipEventRecord(e0, stream) != 0:
            raise RuntimeError("hipEventRecord failed")
        for _ in range(reps):
            ctx.export_particles(buf.value)
        if hip.hipEventRecord(e1, stream) != 0 or hip.hipEventSynchronize(e1) != 0:
            raise RuntimeError("hipEventRecord/Synchronize failed")
        ms = ctypes.c_float()
        if hip.hipEventElapsedTime(ctypes.byref(ms), e0, e1) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        per = ms.value / reps
        gbps = 48.0 * n / (per * 1e-3) / 1e9
        return {"what": "rps_export_particles: SoA state -> 32-B AoS Particle (render_shader.wgsl:26-30) in device memory",
                "particles": n, "reps": reps, "ms_per_export": per, "particles_per_s": n / (per * 1e-3),
                "roofline": {"bound": "hbm", "achieved": gbps, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                             "frac": gbps / HBM_PEAK_GBPS, "algorithmic_bytes": 48.0 * n}}
    finally:
        ctx.sync()  # no export still writing into the buffer
        for ev in (e0, e1):
            if ev.value:
                hip.hipEventDestroy(ev)
        hip.hipFree(buf)


def stats_check(d, st_all, st_shard):
    """With more than one rank the stream context holds an RCCL communicator, and librps
    all-reduces every stats step itself (rps_get_stats).  Its result must equal the same
    combination of the shard stats (rps_get_shard_stats) done by torch.distributed."""
    ref = global_stats(d, st_shard)
    lib = {"bbox": list(st_all.bbox), "kinetic_energy": st_all.kinetic_energy,
           "respawned_last": int(st_all.respawned), "particles": int(st_all.particles)}
    ok = (lib["bbox"] == ref["bbox"] and lib["particles"] == ref["particles"]
          and lib["respawned_last"] == ref["respawned_last"]
          and abs(lib["kinetic_energy"] - ref["kinetic_energy"]) <= 1e-12 * abs(ref["kinetic_energy"]))
    ref["librps_rccl_allreduce"] = "matches torch.distributed" if ok else {"mismatch": lib}
    return ref, ok


SIDES = ("configs", "sph", "allpairs")


def run_sides(rps, args, d, line, keys):
    """The side measurements `keys`, each under a watchdog: a hung side run must not cost the
    headline line (when it was measured already), but fails the run."""
    import threading

    fns = {"configs": (configs_side, not args.no_configs), "sph": (sph_side, args.sph_n > 0),
           "allpairs": (allpairs, args.allpairs_n > 0)}
    for key in keys:
        fn, on = fns[key]
        if not on:
            continue

        def _watchdog(key=key):
            if d.rank == 0:
                line[key] = {"error": f"watchdog: no result within {args.allpairs_timeout} s"}
                if "value" in line:
                    print(json.dumps(line), flush=True)
            print(f"bench.py: side run '{key}' hung; exiting {WATCHDOG_RC}", file=sys.stderr, flush=True)
            os._exit(WATCHDOG_RC)

        progress(d, f"side run '{key}'")
        timer = threading.Timer(args.allpairs_timeout, _watchdog)
        timer.daemon = True
        timer.start()
        try:
            line[key] = fn(rps, args, d)
        except Exception as ex:  # report, keep the headline
            line[key] = {"error": f"{type(ex).__name__}: {ex}"}
        timer.cancel()


def main():
    args = parse()
    launched = "WORLD_SIZE" in os.environ
    if args.gpus > 1 and not launched:
        sys.exit(launch_ranks(args))
    d = Dist()
    if d.world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {d.world} rank(s)", file=sys.stderr)
        sys.exit(2)
    rps = load_impl()
    # Side runs asked for before the headline (their own contexts; the headline's timed work is
    # the same either way).
    first = [k for k in args.sides_first.split(",") if k in SIDES]
    early = {}
    run_sides(rps, args, d, early, first)

    n, id_offset, n_global = shard(args, d)
    progress(d, f"headline: {n} particles on this rank, {args.warmup} warm-up + {args.steps} timed steps")
    cfg, ext = workload(rps, n_global)
    wl = f"C3-{n_global:.0e}-4att-drag-respawn-euler".replace("e+0", "e").replace("e+", "e")
    ctx = rps.Context(n, rps.MODE_STREAM, device=d.local if d.dist else 0,
                      id_offset=id_offset, global_count=n_global)
    ctx.set_config(cfg, ext)
    if d.dist:  # under a launcher the stats steps all-reduce over the ranks inside librps (RCCL)
        ctx.comm_init(d.rank, d.world, d.broadcast_bytes(rps.comm_unique_id() if d.rank == 0 else b""))
    ctx.init_scatter(args.seed)
    do_export = args.export_reps > 0 and hasattr(ctx, "stream_ptr")
    export = None
    if do_export and not args.export_after:  # reads the state only: the headline's work is unchanged
        export = export_side(ctx, n, args.export_reps)
    ctx.step(args.warmup)
    ctx.sync()

    d.sync_device()
    d.barrier()
    t0 = time.perf_counter()
    # The K steps between one pair of HIP events on the context stream (rps_time_steps): the
    # average launch is their span / K.  Launches run back to back (no event between them:
    # round 2 bracketed launches one by one, and each event pair left a ~12-us idle gap on the
    # GPU); the span includes the stats steps that fall in the region (one
    # two-kernel fold every 100th step, ~10 us).
    gpu_ms = ctx.time_steps(args.steps)
    ctx.sync()
    d.sync_device()
    t1 = time.perf_counter()
    d.barrier()
    elapsed = d.max(t1 - t0)
    kern_ms = d.max(gpu_ms / args.steps)
    moved_per_launch, _ = ctx.step_cost()  # bytes the kernel moves: 32.03 B per particle
    moved_per_launch = d.max(moved_per_launch)  # the largest shard (ragged splits)
    n_max = int(d.max(float(n)))
    algo_per_launch = ALGO_BYTES_PER_PARTICLE * n_max
    if do_export and args.export_after:
        export = export_side(ctx, n, args.export_reps)
    if d.dist:
        stats, stats_ok = stats_check(d, ctx.stats(), ctx.shard_stats())
    else:
        stats, stats_ok = global_stats(d, ctx.stats()), True
    # The last stats step (every stats_interval-th active step) is the one reported: a step of the
    # timed region when one fell in it, else a warm-up step (the driver's --warmup 5 --steps 20).
    first_timed = args.warmup
    stats["when"] = ("timed region" if stats["step"] >= first_timed else
                     f"warm-up step {stats['step']} (no stats step among the timed steps "
                     f"{first_timed}..{first_timed + args.steps - 1})")
    fused = None
    if args.fuse_k > 1:
        progress(d, f"fused: ext.fuse_steps = {args.fuse_k}")
        fused = fused_side(ctx, d, cfg, ext, n_global, args.fuse_k, args.fuse_steps)
    ctx.close()

    updates = float(n_global) * args.steps
    value = updates / elapsed
    achieved = moved_per_launch / (kern_ms * 1e-3) / 1e9  # the slowest rank's kernel, its bytes
    algo_gbps = algo_per_launch / (kern_ms * 1e-3) / 1e9
    hbm_wall = moved_per_launch * args.steps / elapsed / 1e9  # per GPU, wall clock incl. gaps
    traffic = pmc_traffic(wl, n_max)
    strong = not args.particles
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "particle-updates/s",
        "n_gpus": d.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded device scatter of src/main.rs:182-216; Philox respawn)",
        "config": {"workload": wl, "global_particles": n_global, "particles_per_gpu": n_max,
                   "attractors": 4, "drag": 0.1, "lifetime_s": [1.0, 5.0], "integrator": "euler",
                   "bytes_per_particle_step": moved_per_launch / n_max,
                   "parallelism": f"index-shard x{d.world} ({'strong: the global count split' if strong else 'weak: per-GPU count fixed'})"},
        "hbm_gbps_per_gpu": hbm_wall,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS,
                     "traffic": traffic, "kernel": "stream_step_kernel<euler,lifetime>",
                     "avg_kernel_ms": kern_ms, "launches": args.steps,
                     "avg_step_gpu_ms": kern_ms,
                     "stats_steps_in_region": sum(1 for k in range(args.warmup, args.warmup + args.steps)
                                                  if k % max(1, getattr(ext, "stats_interval", 100)) == 0),
                     "timing": "one HIP event pair on the context stream around the K timed launches "
                               "(includes the stats fold of any 100th step in the region, counted in "
                               "stats_steps_in_region; avg_kernel_ms = avg_step_gpu_ms = span / K); max over ranks",
                     "bytes_per_launch": moved_per_launch,
                     "bytes_basis": "bytes the kernel moves (rps_step_cost: 32.03 B per particle; PMC agrees "
                                    "within 0.3 %, profiles/pmc_traffic.json)",
                     "algorithmic_bytes_per_launch_survey": algo_per_launch,
                     "algorithmic_equiv_gbps": algo_gbps,
                     "note": "SURVEY 8(d)'s 40 B per particle-step counts an f32 lifetime read and written every "
                             "step; the kernel keeps a u16 expiry behind a per-group index and moves 32.03 B, "
                             "so the utilisation is the moved bytes' rate (DESIGN.md §5.1); "
                             "algorithmic_equiv_gbps is the 40-B rate, an equivalence, not traffic"},
        "stats": stats,
    }
    # The per-rank state (16 B per particle + the expiry arrays) against the 256-MB Infinity Cache
    # (MI355X_MICROARCH.md): when it fits, FETCH_SIZE counts cache hits and the "HBM" rate is
    # not DRAM traffic alone (the strong-scaled 8-GPU shard: 200 MB).
    state_bytes = 16.0 * n_max + 2.0 * n_max + 2.0 * n_max / 64.0
    line["roofline"]["state_bytes_per_rank"] = state_bytes
    line["roofline"]["infinity_cache_resident"] = state_bytes <= 256 * 1024 * 1024
    if export is not None:
        line["export"] = export
    if fused is not None:
        line["fused"] = fused
    if d.rank == 0 and d.world == 1 and not args.no_cpu_baseline:
        progress(d, "cpu_baseline")
        line["cpu_baseline"] = cpu_baseline(rps, args, cfg, ext)
    line.update(early)
    run_sides(rps, args, d, line, [k for k in SIDES if k not in first])
    if d.rank == 0:
        print(json.dumps(line), flush=True)
    d.close()
    if not stats_ok:
        print("bench.py: librps stats all-reduce != torch.distributed", file=sys.stderr)
        sys.exit(STATS_MISMATCH_RC)


if __name__ == "__main__":
    main()
