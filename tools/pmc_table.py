"""Aggregate a rocprofv3 --pmc counter_collection.csv: mean counter value per kernel."""
import csv
import re
import sys
from collections import defaultdict

for path in sys.argv[1:]:
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("rps::(anonymous namespace)::", "").replace("void ", "")
        name = re.sub(r"\(.*", "", name)
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("==", path)
    for k, d in acc.items():
        vals = {c: sum(v) / len(v) for c, v in d.items()}
        s = " ".join(f"{c.replace('SQ_', '')}={v:.4g}" for c, v in sorted(vals.items()))
        wc = vals.get("SQ_WAVE_CYCLES")
        extra = ""
        if wc:
            extra = " | wait%={:.0f} instwait%={:.0f} active%={:.0f} valu%={:.0f}".format(
                100 * vals.get("SQ_WAIT_ANY", 0) / wc, 100 * vals.get("SQ_WAIT_INST_ANY", 0) / wc,
                100 * vals.get("SQ_ACTIVE_INST_ANY", 0) / wc, 100 * vals.get("SQ_ACTIVE_INST_VALU", 0) / wc)
        print(f"{k[:40]:40s} {s}{extra}")
