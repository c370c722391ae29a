"""BASELINE.json configs[4] (C5: 2^27 particles all-pairs, index-sharded over 8 x MI355X) as
one rank runs it, at full size, on one GPU (run on the GPU box; ~6 min of force kernel).

    python tools/c5_rank_shard.py [--rank 7] [--out gpurun_out/r06_c5_rank_shard.txt]

Rank r of 8 owns targets [r * 2^24, (r + 1) * 2^24) and needs all 2^27 sources: the 1-GiB
float2 array its ncclAllGather fills over xGMI.  One GPU cannot hold the other seven ranks, so
the array is filled from the host (RPS_EXT_NBODY_EXTERNAL + rps_nbody_sources), exactly as
tests/test_gpu_nbody.py::test_nbody_c5_rank_shard does at 2^20 targets.  One profiled step
(the split count the library picks for this launch: 8192 target blocks x 3); its force-kernel
time (HIP events), the held shader clock (in-kernel stamps) and the FP32 roofline fraction
(20 flop per interaction); then one target in every 8th 2048-target block (1 024 targets,
their place in the block varying) against the f64 oracle over all 2^27 sources, with the
bound of the test suite, and the integration of every particle bitwise.

A heartbeat line every 30 s while the kernel runs (gpurun treats 3 silent minutes as a hang).
"""
import argparse
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-particle-system_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

FP32_PEAK_TFLOPS, PEAK_CLOCK_MHZ = 157.3, 2400.0
BLOCK = 2048


def heartbeat(stop, t0, what):
    while not stop.wait(30.0):
        print(f"  ... {what}: {time.perf_counter() - t0:.0f} s", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, default=7)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--log2-global", type=int, default=27)
    ap.add_argument("--sample-stride", type=int, default=8, help="check one target per this many blocks")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "r06_c5_rank_shard.txt"))
    args = ap.parse_args()

    import oracle as orc
    import rps_amd as rps
    from helpers import F, assert_soa_bitwise, config_c1, copy_soa
    from hip_mem import copy_h2d

    ng = 1 << args.log2_global
    n = ng // args.ranks
    off = args.rank * n
    lines = []

    def log(s):
        print(s, flush=True)
        lines.append(s)

    log(f"C5 rank shard: rank {args.rank} of {args.ranks}, targets [{off}, {off + n}) = {n}, sources {ng}")
    log(f"librps build {rps.build_id()}")
    cfg = config_c1(rps, min(ng, 0xFFFFFFFF))
    ext = rps.make_ext(nbody_strength=1.0e3, nbody_softening=1.0, shader_delay=0)
    ext.flags |= rps.EXT_NBODY_EXTERNAL
    t = time.perf_counter()
    g = np.random.default_rng(27)
    pos = np.empty((ng, 2), F)
    pos[:, 0] = g.uniform(-950, 950, ng).astype(F)
    pos[:, 1] = g.uniform(-530, 530, ng).astype(F)
    soa = dict(x=pos[off:off + n, 0].copy(), y=pos[off:off + n, 1].copy(),
               vx=g.normal(0, 10, n).astype(F), vy=g.normal(0, 10, n).astype(F))
    log(f"host inputs: {time.perf_counter() - t:.1f} s (uniform positions in the 1900 x 1060 viewport, seed 27)")
    with rps.Context(n, rps.MODE_NBODY, id_offset=off, global_count=ng) as ctx:
        ctx.set_config(cfg, ext)
        ctx.upload_soa(soa)
        src, cnt = ctx.nbody_sources(pack=True)
        assert cnt == ng
        copy_h2d(src, pos[:off])  # the other ranks' shards where the all-gather would put them
        copy_h2d(src + (off + n) * 8, pos[off + n:])
        ctx.sync()
        ctx.set_profiling(1)
        stop = threading.Event()
        t0 = time.perf_counter()
        hb = threading.Thread(target=heartbeat, args=(stop, t0, "force step"), daemon=True)
        hb.start()
        try:
            ctx.step(1)
            ctx.sync()
        finally:
            stop.set()
        wall = time.perf_counter() - t0
        kms, launches = ctx.kernel_time()
        mhz, wgs = ctx.kernel_clock()
        ax = ctx.read_debug(rps.DEBUG_ACCEL_X)
        ay = ctx.read_debug(rps.DEBUG_ACCEL_Y)
        got = ctx.download_soa()
    inter = float(n) * ng
    tf = 20.0 * inter / (kms * 1e-3) / 1e12
    log(f"step wall {wall:.2f} s; force kernel {kms:.1f} ms (HIP events, {launches} launch); "
        f"{inter:.4e} interactions = {inter / (kms * 1e-3):.4e} interactions/s")
    log(f"FP32 roofline: {tf:.2f} TFLOP/s of {FP32_PEAK_TFLOPS} = {tf / FP32_PEAK_TFLOPS:.4f}; held clock "
        f"{mhz:.0f} MHz (median of {wgs} workgroups' stamps) -> {tf / (FP32_PEAK_TFLOPS * mhz / PEAK_CLOCK_MHZ):.4f} "
        f"at that clock; issue floor 0.822")
    log(f"8-rank C5 step estimate: max over ranks of this shard's time (equal shards) + the 1-GiB all-gather "
        f"(~1 ms over xGMI) = {wall:.1f} s per step, {8 * inter / wall:.4e} interactions/s over 8 GPUs")

    sx, sy = np.ascontiguousarray(pos[:, 0]), np.ascontiguousarray(pos[:, 1])
    del pos
    blocks = (n + BLOCK - 1) // BLOCK
    b = np.arange(0, blocks, args.sample_stride, dtype=np.uint64)
    rel = b * BLOCK + (b * np.uint64(769) + np.uint64(13)) % np.uint64(BLOCK)
    rel = np.unique(np.concatenate([rel, np.array([0, n - 1], np.uint64)]))
    t = time.perf_counter()
    stop = threading.Event()
    hb = threading.Thread(target=heartbeat, args=(stop, t, "f64 oracle"), daemon=True)
    hb.start()
    try:
        rx, ry, ab = orc.nbody_accel_ref_idx(ext, sx, sy, rel + np.uint64(off))
    finally:
        stop.set()
    mag = np.hypot(rx.astype(np.float64), ry.astype(np.float64))
    err = np.hypot(ax[rel].astype(np.float64) - rx, ay[rel].astype(np.float64) - ry)
    ratio = err / np.maximum(1e-4 * mag, 1e-5 * ab)
    ok = bool(ratio.max() <= 1.0 and np.median(err / mag) < 1e-5)
    log(f"parity: {len(rel)} targets (one per {args.sample_stride} blocks of {BLOCK}, place in block varying, "
        f"+ first/last) vs the f64 oracle over all {ng} sources ({time.perf_counter() - t:.0f} s on the host): "
        f"max err/bound {ratio.max():.4f} (<= 1), median |err|/|a| {np.median(err / mag):.3e} (< 1e-5), "
        f"max |err|/|a| {np.max(err / mag):.3e} -> {'PASS' if ok else 'FAIL'}")
    ref = copy_soa(soa)
    orc.nbody_integrate(cfg, ext, ax, ay, ref)
    try:
        assert_soa_bitwise(got, ref)
        log(f"integration of all {n} particles given the device accelerations: bitwise == oracle")
    except AssertionError as e:
        ok = False
        log(f"integration: FAIL {e}")
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        f.write("\n".join(lines) + "\n")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
