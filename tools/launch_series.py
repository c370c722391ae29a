"""Per-launch durations of one kernel, in launch order, from a rocprofv3 kernel trace.

  python tools/launch_series.py <run_kernel_trace.csv> [kernel-substring] [--first K]

Prints every launch's duration and the gap since the previous launch of any kernel on the
device, then summaries over the first K launches and over all of them.  Used to compare the
driver's short bench (`--steps 20 --warmup 5`: 25 stream launches) with a long one.
"""
import csv
import statistics
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    first = 25
    if "--first" in sys.argv:
        first = int(sys.argv[sys.argv.index("--first") + 1])
        args = [a for a in args if a != str(first)]
    path = args[0]
    sub = args[1] if len(args) > 1 else "stream_step_kernel<false, true, false, 3>"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    prev_end = None
    series = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if sub in r["Kernel_Name"]:
            gap = (s - prev_end) / 1e3 if prev_end is not None else float("nan")
            series.append(((e - s) / 1e3, gap))
        prev_end = e
    for i, (d, g) in enumerate(series):
        print(f"{i:5d} {d:10.2f} us   gap {g:8.2f} us")

    def summ(tag, v):
        if not v:
            return
        d = [x[0] for x in v]
        print(f"{tag}: n={len(d)} mean={statistics.mean(d):.2f} median={statistics.median(d):.2f} "
              f"min={min(d):.2f} max={max(d):.2f} us")

    summ(f"first {first}", series[:first])
    summ(f"launches {first}..", series[first:])
    summ("all", series)


if __name__ == "__main__":
    main()
