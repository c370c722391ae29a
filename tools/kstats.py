"""Print a rocprofv3 kernel_stats.csv compactly: short name, calls, avg us, total us, %."""
import csv
import re
import sys

for path in sys.argv[1:]:
    print("==", path)
    for r in csv.DictReader(open(path)):
        name = re.sub(r"\(.*", "", r["Name"].replace("rps::(anonymous namespace)::", "")).replace("void ", "")
        if "<" in r["Name"] and "<" not in name:
            name = name
        m = re.search(r"(\w+)(<[^>(]*>)?", r["Name"].replace("rps::(anonymous namespace)::", "").replace("void ", ""))
        print(f"{m.group(0):45s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:10.2f} us {float(r['TotalDurationNs'])/1e3:12.1f} us {float(r['Percentage']):6.2f}%")
