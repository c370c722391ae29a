"""Turn rocprofv3 output under gpurun_out/ into the committed evidence under profiles/.

  python tools/collect_profiles.py <round-tag> [gpurun_out subdirectory]

reads  gpurun_out/prof_trace/run_kernel_{stats,trace}.csv   (--kernel-trace --stats run of
       the bench command) and gpurun_out/pmc_{fetch,write}/run_counter_collection.csv (two
       separate --pmc passes, MI355X_MICROARCH.md §HBM / §rocprofv3 PMC slots)
writes profiles/<tag>_kernel_stats.csv, profiles/<tag>_kernel_summary.json and
       profiles/pmc_traffic.json (what bench.py reports as roofline.traffic).

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE/WRITE_SIZE are KiB
and gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced stream (16 B/lane
global loads), WRITE_SIZE is exact for 16-B/lane stores (MI355X_MICROARCH.md §HBM).
"""
import csv
import json
import os
import shutil
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")
WORKLOAD = "C3-1e8-4att-drag-respawn-euler"
DOMINANT = "stream_step_kernel<false, true, false, 3>"


def main(tag, sub=""):
    os.makedirs(PROF, exist_ok=True)
    base = os.path.join(OUT, sub)
    trace_dir = "prof_bench" if sub else "prof_trace"
    stats = os.path.join(base, trace_dir, "run_kernel_stats.csv")
    trace = os.path.join(base, trace_dir, "run_kernel_trace.csv")
    summary = {}
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    if os.path.exists(trace):
        per = defaultdict(list)
        for r in csv.DictReader(open(trace)):
            per[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for k, v in per.items():
            summary[k] = {"calls": len(v), "avg_us": statistics.mean(v), "median_us": statistics.median(v),
                          "min_us": min(v), "max_us": max(v)}
    pmc = defaultdict(dict)
    for name, counter in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
        f = os.path.join(base, name, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        vals = defaultdict(list)
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
        for k, v in vals.items():
            pmc[k][counter] = statistics.mean(v)
            pmc[k][counter + "_launches"] = len(v)
    traffic = {}
    for k, d in pmc.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch"] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
            if DOMINANT in k:
                traffic[WORKLOAD] = {"kernel": k, "FETCH_SIZE_KiB": d["FETCH_SIZE"], "WRITE_SIZE_KiB": d["WRITE_SIZE"],
                                     "hbm_bytes_per_launch": d["hbm_bytes_per_launch"],
                                     "algorithmic_bytes_per_launch": 40.0 * 1e8,
                                     "moved_bytes_per_launch": (32.0 + 2.0 / 64) * 1e8,
                                     "correction": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE = 1/2 of wide-stream bytes)",
                                     "round": tag}
    with open(os.path.join(PROF, f"{tag}_kernel_summary.json"), "w") as f:
        json.dump({"trace": summary, "pmc": pmc}, f, indent=1, sort_keys=True)
    if traffic:  # merged into the file (it also holds the SPH entry, tools/collect_sph_traffic.py)
        path = os.path.join(PROF, "pmc_traffic.json")
        old = json.load(open(path)) if os.path.exists(path) else {}
        old.update(traffic)
        with open(path, "w") as f:
            json.dump(old, f, indent=1, sort_keys=True)
    print(json.dumps({"trace": {k[:90]: v for k, v in summary.items()}, "traffic": traffic}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01", sys.argv[2] if len(sys.argv) > 2 else "")
