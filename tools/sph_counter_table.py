"""DESIGN.md §5.2's per-kernel counter table of the SPH frame, from tools/pmc_sph_counters.sh.

    python tools/sph_counter_table.py [N] [--merge TAG] > profiles/<tag>_sph_counters_2p22.txt

--merge TAG also stores each kernel's row under "counters" in profiles/pmc_traffic.json's
"SPH-2^22-frame" entry (bench.py's sph.roofline reports the sim's), tagged with the round.

Kernel times: the kernel trace of the same box (no counters collected in that run).  Per kernel
(counters averaged over the dispatches):
  lines/ld   TCP_TOTAL_CACHE_ACCESSES / SQ_INSTS_VMEM_RD (cache lines per vector load instruction)
  L1 hit     1 - TCP_TCC_READ_REQ / TCP_TOTAL_CACHE_ACCESSES
  L2 hit     TCC_HIT / (TCC_HIT + TCC_MISS)
  TA busy    TA_TA_BUSY_sum / 256 CUs / kernel cycles (2400 MHz)
  VALU busy  SQ_INSTS_VALU x 2 cycles / 1024 SIMDs / kernel cycles (a wave64 VALU op issues over 2)
  wait / instwait / valu   SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_VALU over SQ_WAVE_CYCLES"""
import csv
import os
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
CLK_MHZ, CUS, SIMDS = 2400.0, 256, 1024


def find(d, suffix):
    for dp, _, fs in os.walk(os.path.join(OUT, d)):
        for f in fs:
            if f.endswith(suffix):
                return os.path.join(dp, f)
    sys.exit(f"{d}: no *{suffix}")


def short(name):
    return name.replace("void ", "").replace("rps::(anonymous namespace)::", "").split("(")[0]


def counters(d):
    vals = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(find(d, "counter_collection.csv"))):
        vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: statistics.mean(v) for c, v in cs.items()} for k, cs in vals.items()}


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    merge = sys.argv[sys.argv.index("--merge") + 1] if "--merge" in sys.argv else None
    if merge in args:
        args.remove(merge)
    n = args[0] if args else "4194304"
    rows = {}
    times = {}
    for r in csv.DictReader(open(find(f"cnt_trace_{n}", "kernel_stats.csv"))):
        times[short(r["Name"])] = float(r["AverageNs"]) / 1e3
    m1, m2 = counters(f"cnt_m1_{n}"), counters(f"cnt_m2_{n}")
    log = [ln for ln in open(os.path.join(OUT, f"cnt_trace_{n}.log")) if "ms/frame" in ln]
    print(f"# SPH frame kernels at N = {n} (tools/pmc_sph_counters.sh; trace run: {log[-1].strip() if log else '?'})")
    print("# times: that kernel trace; counters: two --pmc passes of 8 frames each, averaged per dispatch")
    print(f"{'kernel':44} {'us':>7} {'lines/ld':>8} {'L1hit':>6} {'L2hit':>6} {'TAbusy':>6} {'VALUbusy':>8} "
          f"{'wait':>5} {'instw':>5} {'valu':>5}")
    for k, us in sorted(times.items(), key=lambda kv: -kv[1]):
        if not k.startswith("sph_") or k not in m1 or k not in m2:
            continue
        a, b = m1[k], m2[k]
        cyc = us * CLK_MHZ
        vm = a.get("SQ_INSTS_VMEM_RD", 0.0)
        acc = a.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0.0)
        hit, miss = b.get("TCC_HIT_sum", 0.0), b.get("TCC_MISS_sum", 0.0)
        wc = b.get("SQ_WAVE_CYCLES", 0.0) or float("nan")
        rows[k] = {"us": us, "lines_per_load": acc / vm if vm else None,
                   "l1_hit": 1.0 - a.get("TCP_TCC_READ_REQ_sum", 0.0) / acc if acc else None,
                   "l2_hit": hit / (hit + miss) if hit + miss else None,
                   "ta_busy": a.get("TA_TA_BUSY_sum", 0.0) / CUS / cyc,
                   "valu_busy": a.get("SQ_INSTS_VALU", 0.0) * 2.0 / SIMDS / cyc,
                   "sq_wait": b.get("SQ_WAIT_ANY", 0.0) / wc, "sq_instwait": b.get("SQ_WAIT_INST_ANY", 0.0) / wc}
        print(f"{k[:44]:44} {us:7.1f} {acc / vm if vm else float('nan'):8.1f} "
              f"{1.0 - a.get('TCP_TCC_READ_REQ_sum', 0.0) / acc if acc else float('nan'):6.3f} "
              f"{hit / (hit + miss) if hit + miss else float('nan'):6.3f} "
              f"{a.get('TA_TA_BUSY_sum', 0.0) / CUS / cyc:6.2f} {a.get('SQ_INSTS_VALU', 0.0) * 2.0 / SIMDS / cyc:8.2f} "
              f"{b.get('SQ_WAIT_ANY', 0.0) / wc:5.2f} {b.get('SQ_WAIT_INST_ANY', 0.0) / wc:5.2f} "
              f"{b.get('SQ_ACTIVE_INST_VALU', 0.0) / wc:5.2f}")
    if merge:
        import json

        path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        doc = json.load(open(path))
        doc.setdefault("SPH-2^22-frame", {})["counters"] = {"round": merge, "per_kernel": rows,
                                                            "source": "tools/pmc_sph_counters.sh + tools/sph_counter_table.py"}
        with open(path, "w") as f:
            json.dump(doc, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
