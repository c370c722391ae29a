"""bench.py's roofline objects on the CPU: the SPH line's `frac` is the PMC-measured L1 -> L2
bytes of the sim kernel per kernel time against the aggregate L2 peak (a utilisation, not the
algorithmic-bytes rate), the frame's `frac` its measured memory-side bytes against HBM, and the
headline's PMC traffic is looked up by workload name and shard size."""
import importlib.util
import os

import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


COST = {"sim_bytes": 6.04e9, "frame_bytes": 9.49e9, "scanned_entries": 40.15 * (1 << 22),
        "within_entries": 14.42 * (1 << 22), "slots": 1 << 22, "sort_launches": 19}


def test_sph_frac_is_measured_l2_utilisation(bench):
    pmc = bench.pmc_sph()
    assert pmc, "profiles/pmc_traffic.json holds the SPH frame's PMC record"
    sim = next(v for k, v in pmc["per_dispatch"].items() if k.startswith("sph_sim"))
    sim_ms, frame_ms = 0.306, 0.931
    rl, fc = bench.sph_roofline(COST, sim_ms, frame_ms, pmc)
    l2 = sim["l2_read_bytes"] + sim["l2_write_bytes"]
    assert rl["traffic"] == l2
    assert rl["frac"] == pytest.approx(l2 / (sim_ms * 1e-3) / 1e9 / bench.L2_PEAK_GBPS, rel=1e-12)
    assert rl["hbm_frac"] == pytest.approx(sim["hbm_bytes"] / (sim_ms * 1e-3) / 1e9 / bench.HBM_PEAK_GBPS)
    assert 0 < rl["frac"] < 1 and 0 < rl["hbm_frac"] < 1 and 0 < fc["frac"] < 1
    # the algorithmic rate is reported beside it, not as the utilisation
    assert rl["algorithmic_equiv_frac"] > rl["frac"]
    hbm = pmc["frame_sum_of_kernels"]["hbm_bytes"]
    assert fc["frac"] == pytest.approx(hbm / (frame_ms * 1e-3) / 1e9 / bench.HBM_PEAK_GBPS)


def test_sph_roofline_without_pmc_reports_no_rates(bench):
    rl, fc = bench.sph_roofline(COST, 0.1, 0.3, None)
    assert rl["frac"] is None and rl["achieved"] is None and fc["frac"] is None
    assert rl["algorithmic_equiv_frac"] > 0


def test_headline_traffic_keyed_by_workload(bench):
    wl = "C3-1e8-4att-drag-respawn-euler"
    assert bench.pmc_traffic(wl, 10 ** 8) > 0
    assert bench.pmc_traffic(wl, 5 * 10 ** 7) is None  # another shard size
    assert bench.pmc_traffic("C3-2e8-4att-drag-respawn-euler", 10 ** 8) is None  # another workload
