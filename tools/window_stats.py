"""Kernel statistics over the timed region only.

bench.py launches a one-wave spin kernel (torch.cuda._sleep) on each side of
every timed region (bench._window_marker). Given a rocprofv3 kernel trace of
a bench run, this keeps the dispatches between the markers of one region
(``--window``: 0 = the headline's, 1 = the next timed leg, ...) and writes
the table rocprofv3 --stats writes (Name, Calls, TotalDurationNs, AverageNs,
Percentage, MinNs, MaxNs, StdDev) over them alone, so the setup's sorts,
copies and generators do not enter the Percentage column.

  python tools/window_stats.py gpurun_out/prof/run_kernel_trace.csv \
      --window 0 --out profiles/r06/bench_kernel_stats_timed.csv
"""
import argparse
import collections
import csv
import math
import sys


def windows(rows):
    marks = [r for r in rows if "spin_kernel" in r["Kernel_Name"]]
    marks.sort(key=lambda r: int(r["Start_Timestamp"]))
    return [(int(a["End_Timestamp"]), int(b["Start_Timestamp"]))
            for a, b in zip(marks[0::2], marks[1::2])]


def stats(rows, lo, hi):
    per = collections.defaultdict(list)
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s >= lo and e <= hi and "spin_kernel" not in r["Kernel_Name"]:
            per[r["Kernel_Name"]].append(e - s)
    total = sum(sum(v) for v in per.values()) or 1
    out = []
    for name, d in per.items():
        n = len(d)
        mean = sum(d) / n
        sd = math.sqrt(sum((x - mean) ** 2 for x in d) / n)
        out.append((name, n, sum(d), mean, 100.0 * sum(d) / total, min(d), max(d), sd))
    out.sort(key=lambda t: -t[2])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window", type=int, default=0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    with open(a.trace) as f:
        rows = list(csv.DictReader(f))
    ws = windows(rows)
    if a.window >= len(ws):
        sys.exit("%d timed windows in the trace, asked for #%d" % (len(ws), a.window))
    lo, hi = ws[a.window]
    table = stats(rows, lo, hi)
    f = open(a.out, "w", newline="") if a.out else sys.stdout
    w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs",
                "StdDev"])
    for t in table:
        w.writerow(list(t))
    if a.out:
        f.close()
        print("window %d: %.3f ms wide, %d kernels" % (a.window, (hi - lo) / 1e6, len(table)))


if __name__ == "__main__":
    main()
