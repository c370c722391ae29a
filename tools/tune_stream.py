"""Stream-kernel tuning sweep (run on the GPU box via tools/gpu_run.sh py:tools/tune_stream.py).

Interleaved rounds in ONE process (cdna_hip_programming.md §5.4 rule 24): variants of the
launch grid (RPS_STREAM_GRID; 0 = one-shot) and nontemporal loads/stores (RPS_STREAM_NT),
each timed by per-launch HIP events.  A torch device-to-device copy of the same byte count
is the known-good bandwidth reference on the same GPU (rule 10)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-particle-system_amd", "python"))

import torch  # noqa: E402  (first: one HIP runtime in the process)

import rps_amd as rps  # noqa: E402

N = int(os.environ.get("TUNE_N", 100_000_000))
STEPS = 50
ROUNDS = int(os.environ.get("TUNE_ROUNDS", 4))


def copy_ref(nbytes):
    a = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
    b = torch.empty_like(a)
    a.uniform_()
    for _ in range(3):
        b.copy_(a)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        b.copy_(a)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 20
    del a, b
    torch.cuda.empty_cache()
    return 2 * nbytes / (ms * 1e-3) / 1e9, ms


def main():
    variants = []
    if os.environ.get("TUNE_SET") == "xcd":
        for xcd in (1, 0):
            variants.append(dict(grid=0, nt=3, lifetime=True, xcd=xcd))
            variants.append(dict(grid=0, nt=3, lifetime=False, xcd=xcd))
    else:
        for nt in (3, 1, 2, 0):  # bit 0 nontemporal loads, bit 1 nontemporal stores
            variants.append(dict(grid=0, nt=nt, lifetime=True))
        variants.append(dict(grid=16384, nt=3, lifetime=True))
        variants.append(dict(grid=0, nt=3, lifetime=False))
        variants.append(dict(grid=0, nt=1, lifetime=False))
    results = {json.dumps(v, sort_keys=True): [] for v in variants}
    cfg = rps.default_particle_config(N, gravity=0.0)
    for r in range(ROUNDS):
        for v in variants:
            os.environ["RPS_STREAM_GRID"] = str(v["grid"])
            os.environ["RPS_STREAM_NT"] = str(v["nt"])
            os.environ["RPS_STREAM_XCD"] = str(v.get("xcd", 1))
            ext = rps.headline_ext()
            ext.shader_delay = 0
            if not v["lifetime"]:
                ext.flags = 0
            with rps.Context(N) as ctx:
                ctx.set_config(cfg, ext)
                ctx.init_scatter()
                ctx.step(5)
                ctx.set_profiling(True)
                ctx.step(STEPS)
                ms, cnt = ctx.kernel_time()
                nbytes, _ = ctx.step_cost()
            gbps = nbytes / (ms * 1e-3) / 1e9
            results[json.dumps(v, sort_keys=True)].append((ms, gbps))
            print(f"round {r} {v}: {ms:.4f} ms  {gbps:.0f} GB/s", flush=True)
    ref_gbps, ref_ms = copy_ref(40 * N // 2)
    print(f"torch D2D copy of {40 * N // 2} B: {ref_ms:.4f} ms = {ref_gbps:.0f} GB/s (read+write)")
    summary = {k: {"median_ms": sorted(x[0] for x in v)[len(v) // 2], "best_gbps": max(x[1] for x in v)}
               for k, v in results.items()}
    summary["torch_copy_gbps"] = ref_gbps
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "tune_stream.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
