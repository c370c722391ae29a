"""bench.py's multi-rank contract on the CPU (gloo), with the library replaced by the test
double tests/bench_stub.py: `--gpus N` starts N ranks itself, a launcher world that differs
from `--gpus` fails, the librps all-rank stats are cross-checked against torch.distributed,
and a hung side run exits non-zero after printing the headline line."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
ARGS = ["--steps", "20", "--warmup", "2", "--no-cpu-baseline", "--sph-n", "0", "--no-configs"]
WEAK = ["--particles", "4096"]


def _run(extra, env_extra=None, timeout=240):
    env = dict(os.environ, RPS_BENCH_TEST_STUB="bench_stub", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(ROOT, "tests"), env.get("PYTHONPATH", "")])
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, BENCH] + ARGS + extra, env=env, cwd=ROOT, capture_output=True,
                       text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, [json.loads(ln) for ln in lines]


def test_gpus2_starts_two_ranks():
    p, lines = _run(WEAK + ["--gpus", "2", "--allpairs-n", "8192"])
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1, p.stdout  # rank 0 prints the one line
    line = lines[0]
    assert line["n_gpus"] == 2
    assert line["config"]["global_particles"] == 2 * 4096
    assert line["scaling"] == "weak"
    assert line["value"] > 0 and line["steps"] == 20
    st = line["stats"]
    assert st["ranks"] == 2 and st["particles"] == 2 * 4096
    assert st["bbox"] == [-2.0, 2.0, -3.0, 3.0]
    assert st["librps_rccl_allreduce"] == "matches torch.distributed"
    assert line["allpairs"]["collective"].startswith("ncclAllGather")


@pytest.mark.parametrize("gpus", [1, 8])
def test_allpairs_default_is_c4(gpus):
    """Without --allpairs-n the all-pairs side line is BASELINE.json configs[3] (C4): 2^24
    particles, one timed step after one warm step, targets strong-sharded 2^24 / N per rank
    with the library's all-gather under a launcher (8 gloo ranks here, as the driver's 8-GPU
    node runs it)."""
    p, lines = _run(WEAK + ["--gpus", str(gpus)], timeout=400)
    assert p.returncode == 0, p.stderr[-3000:]
    ap = lines[0]["allpairs"]
    assert ap["particles"] == 1 << 24 and ap["particles_per_rank"] == (1 << 24) // gpus
    assert "16777216 global particles" in ap["workload"] and "C4" in ap["workload"]
    assert ap["steps"] == 1 and ap["warmup"] == 1 and ap["scaling"] == "strong"
    assert ap["collective"].startswith("ncclAllGather") == (gpus > 1)
    assert ap["roofline"]["peak"] == 157.3 and ap["roofline"]["unit"] == "TFLOP/s"


def test_single_process_defaults_to_one_gpu():
    p, lines = _run(WEAK + ["--allpairs-n", "0"])
    assert p.returncode == 0, p.stderr[-3000:]
    assert lines[0]["n_gpus"] == 1


@pytest.mark.parametrize("gpus", [1, 2])
def test_fused_side_beside_the_headline(gpus):
    """The temporally fused measure (ext.fuse_steps = 16) rides on the headline context after its
    timed region: its steps round to whole launches and its rate counts every rank's particles
    (the stub times 0.5 ms per step); --fuse-k 0 drops it."""
    p, lines = _run(WEAK + ["--gpus", str(gpus), "--allpairs-n", "0", "--fuse-steps", "70"])
    assert p.returncode == 0, p.stderr[-3000:]
    f = lines[0]["fused"]
    assert f["fuse_steps"] == 16 and f["steps"] == 64 and f["launches"] == 4
    assert f["ms_per_step"] == pytest.approx(0.5)
    assert f["updates_per_s"] == pytest.approx(gpus * 4096 * 64 / (0.5 * 64 * 1e-3))
    assert lines[0]["value"] > 0 and "fused" not in lines[0]["config"]
    p, lines = _run(WEAK + ["--allpairs-n", "0", "--fuse-k", "0"])
    assert p.returncode == 0, p.stderr[-3000:]
    assert "fused" not in lines[0]


@pytest.mark.parametrize("gpus", [1, 2])
def test_strong_default_is_the_metric_config(gpus):
    """Without --particles the headline is BASELINE's metric configuration at every N: 1e8
    particles in all, split into contiguous shards; value counts the global particles."""
    p, lines = _run(["--gpus", str(gpus), "--allpairs-n", "0", "--export-reps", "0"])
    assert p.returncode == 0, p.stderr[-3000:]
    line = lines[0]
    assert line["scaling"] == "strong" and line["n_gpus"] == gpus
    assert line["config"]["global_particles"] == 10 ** 8
    assert line["config"]["particles_per_gpu"] == 10 ** 8 // gpus
    assert line["config"]["workload"].startswith("C3-1e8-")
    assert line["stats"]["particles"] == 10 ** 8
    assert abs(line["value"] - 1e8 * 20 / (line["ms_per_step"] * 20e-3)) <= 1e-6 * line["value"]
    rf = line["roofline"]
    assert rf["frac"] <= 1.0 and rf["bytes_per_launch"] == pytest.approx(32.03 * 10 ** 8 / gpus)
    assert rf["achieved"] == pytest.approx(rf["bytes_per_launch"] / (rf["avg_kernel_ms"] * 1e-3) / 1e9)


def test_strong_ragged_split():
    """A global count that does not divide: shards [r*G/W, (r+1)*G/W), the line reports the
    largest shard and all G particles."""
    p, lines = _run(["--gpus", "2", "--global-particles", "8193", "--allpairs-n", "0", "--export-reps", "0"])
    assert p.returncode == 0, p.stderr[-3000:]
    line = lines[0]
    assert line["config"]["global_particles"] == 8193 and line["config"]["particles_per_gpu"] == 4097


def test_launcher_world_must_match_gpus():
    env = {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0", "MASTER_PORT": "29631"}
    p, lines = _run(WEAK + ["--gpus", "2", "--allpairs-n", "0"], env)
    assert p.returncode == 2 and not lines
    assert "--gpus 2" in p.stderr


def test_stats_mismatch_fails():
    p, lines = _run(WEAK + ["--gpus", "2", "--allpairs-n", "0"], {"RPS_STUB_BAD_STATS": "1"})
    assert p.returncode != 0
    assert lines and "mismatch" in json.dumps(lines[0]["stats"]["librps_rccl_allreduce"])


@pytest.mark.parametrize("gpus", [1, 2])
def test_side_run_watchdog_exits_nonzero(gpus):
    p, lines = _run(WEAK + ["--gpus", str(gpus), "--allpairs-n", "8192", "--allpairs-timeout", "3"],
                    {"RPS_STUB_HANG": "nbody"})
    assert p.returncode != 0
    assert len(lines) == 1 and "watchdog" in lines[0]["allpairs"]["error"]
    assert lines[0]["n_gpus"] == gpus and lines[0]["value"] > 0
