"""Per-call g-SpMM kernel time from a rocprofv3 kernel trace (csv): every
dispatch whose name contains the substring, summed and divided by the number
of API calls (a blocked or chunked call launches several kernels), to set
beside bench.py's in-process roofline.kernel_ms.

  python tools/kernel_per_call.py <kernel_trace.csv> <calls> [substring] [bench_json]
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    path, calls = sys.argv[1], int(sys.argv[2])
    sub = sys.argv[3] if len(sys.argv) > 3 else "gspmm"
    by_name = defaultdict(lambda: [0, 0.0])
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if sub in name:
                e = by_name[name.split("(")[0][:120]]
                e[0] += 1
                e[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    total = sum(v[1] for v in by_name.values())
    res = {"trace": path, "calls": calls, "substring": sub,
           "dispatches": sum(v[0] for v in by_name.values()),
           "kernel_ms_per_call": total / calls,
           "by_kernel": {k: {"dispatches": v[0], "ms_total": v[1]} for k, v in by_name.items()}}
    if len(sys.argv) > 4:
        lines = open(sys.argv[4]).read().strip().splitlines()
        bench = json.loads(lines[-1])
        res["bench_kernel_ms"] = bench["roofline"]["kernel_ms"]
        res["ratio_trace_over_bench"] = res["kernel_ms_per_call"] / bench["roofline"]["kernel_ms"]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
