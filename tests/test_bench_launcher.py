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
ARGS = ["--steps", "20", "--warmup", "2", "--particles", "4096", "--no-cpu-baseline", "--sph-n", "0", "--no-configs"]


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
    p, lines = _run(["--gpus", "2", "--allpairs-n", "8192"])
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1, p.stdout  # rank 0 prints the one line
    line = lines[0]
    assert line["n_gpus"] == 2
    assert line["config"]["global_particles"] == 2 * 4096
    assert line["value"] > 0 and line["steps"] == 20
    st = line["stats"]
    assert st["ranks"] == 2 and st["particles"] == 2 * 4096
    assert st["bbox"] == [-2.0, 2.0, -3.0, 3.0]
    assert st["librps_rccl_allreduce"] == "matches torch.distributed"
    assert line["allpairs"]["collective"].startswith("ncclAllGather")


def test_single_process_defaults_to_one_gpu():
    p, lines = _run(["--allpairs-n", "0"])
    assert p.returncode == 0, p.stderr[-3000:]
    assert lines[0]["n_gpus"] == 1


def test_launcher_world_must_match_gpus():
    env = {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0", "MASTER_PORT": "29631"}
    p, lines = _run(["--gpus", "2", "--allpairs-n", "0"], env)
    assert p.returncode == 2 and not lines
    assert "--gpus 2" in p.stderr


def test_stats_mismatch_fails():
    p, lines = _run(["--gpus", "2", "--allpairs-n", "0"], {"RPS_STUB_BAD_STATS": "1"})
    assert p.returncode != 0
    assert lines and "mismatch" in json.dumps(lines[0]["stats"]["librps_rccl_allreduce"])


@pytest.mark.parametrize("gpus", [1, 2])
def test_side_run_watchdog_exits_nonzero(gpus):
    p, lines = _run(["--gpus", str(gpus), "--allpairs-n", "8192", "--allpairs-timeout", "3"],
                    {"RPS_STUB_HANG": "nbody"})
    assert p.returncode != 0
    assert len(lines) == 1 and "watchdog" in lines[0]["allpairs"]["error"]
    assert lines[0]["n_gpus"] == gpus and lines[0]["value"] > 0
