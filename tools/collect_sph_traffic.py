"""Measured traffic behind the SPH roofline, from the three rocprofv3 --pmc passes of
tools/pmc_sph_traffic.sh (workload: tools/sph_traffic_frames.py).

  python tools/collect_sph_traffic.py <round-tag>

Per SPH kernel, per dispatch (averaged over the frames):
  l2_read_bytes / l2_write_bytes  TCP_TCC_READ_REQ / _WRITE_REQ (the L1s' requests to the L2s)
                                  x bytes per request, calibrated on the workload's stream
                                  launches (2^24 particles, 16 B read and 16 B written each);
  hbm_bytes                       (FETCH_SIZE * f + WRITE_SIZE) * 1024, f calibrated on the same
                                  stream launches (gfx950: 2 for wide streaming reads,
                                  MI355X_MICROARCH.md §HBM; uncalibrated for gathers, so an
                                  estimate for the scans).
Writes profiles/<tag>_sph_traffic.json and merges "SPH-2^22-frame" into profiles/pmc_traffic.json
(bench.py's sph.roofline.traffic reads it)."""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")
CAL_KERNEL = "stream_step_kernel<false, false, false, 2>"
CAL_PARTICLES = 1 << 24


def per_kernel(pass_dir):
    f = None
    for dp, _, fs in os.walk(os.path.join(OUT, pass_dir)):
        for n in fs:
            if n.endswith("counter_collection.csv"):
                f = os.path.join(dp, n)
    vals = defaultdict(lambda: defaultdict(list))
    if f is None:
        return {}
    for r in csv.DictReader(open(f)):
        vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: statistics.mean(v) for c, v in d.items()} for k, d in vals.items()}


def short(name):
    return name.replace("void ", "").replace("rps::(anonymous namespace)::", "").split("(")[0]


def main(tag):
    fetch, write, req = per_kernel("pmc_sph_fetch"), per_kernel("pmc_sph_write"), per_kernel("pmc_sph_l2req")
    cal = [k for k in req if CAL_KERNEL in k]
    if not cal:
        sys.exit("calibration stream kernel missing from the l2req pass")
    stream_bytes = 16.0 * CAL_PARTICLES
    rb = stream_bytes / req[cal[0]]["TCP_TCC_READ_REQ_sum"]
    wb = stream_bytes / req[cal[0]]["TCP_TCC_WRITE_REQ_sum"]
    ff = stream_bytes / (1024.0 * fetch[[k for k in fetch if CAL_KERNEL in k][0]]["FETCH_SIZE"])
    table = {}
    for k in req:
        if "sph_" not in k:
            continue
        e = {"l2_read_bytes": req[k]["TCP_TCC_READ_REQ_sum"] * rb,
             "l2_write_bytes": req[k].get("TCP_TCC_WRITE_REQ_sum", 0.0) * wb,
             "l1_accesses": req[k].get("TCP_TOTAL_CACHE_ACCESSES_sum")}
        if k in fetch and k in write:
            e["hbm_bytes"] = (fetch[k]["FETCH_SIZE"] * ff + write[k]["WRITE_SIZE"]) * 1024.0
        table[short(k)] = e
    frame = {"l2_bytes": sum(v["l2_read_bytes"] + v["l2_write_bytes"] for v in table.values()),
             "hbm_bytes": sum(v.get("hbm_bytes", 0.0) for v in table.values())}
    doc = {"workload": "bench sph: 2^22 particles, reference scatter, every frame active (tools/sph_traffic_frames.py)",
           "calibration": {"kernel": CAL_KERNEL, "bytes_per_read_req": rb, "bytes_per_write_req": wb,
                           "fetch_size_factor": ff},
           "per_dispatch": table, "frame_sum_of_kernels": frame, "round": tag}
    with open(os.path.join(PROF, f"{tag}_sph_traffic.json"), "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    path = os.path.join(PROF, "pmc_traffic.json")
    old = json.load(open(path)) if os.path.exists(path) else {}
    if "counters" in old.get("SPH-2^22-frame", {}):  # tools/sph_counter_table.py --merge keeps its rows here
        doc["counters"] = old["SPH-2^22-frame"]["counters"]
    old["SPH-2^22-frame"] = doc
    with open(path, "w") as f:
        json.dump(old, f, indent=1, sort_keys=True)
    print(json.dumps(doc, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r03")
