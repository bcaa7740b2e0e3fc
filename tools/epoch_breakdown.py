"""Per-epoch kernel breakdown from a rocprofv3 kernel trace.

One epoch = the kernels between two consecutive launches of a marker kernel
(default: the F = 128 mean g-SpMM, launched once per GraphSAGE epoch); the
last full window is summarised: wall time, busy time, and the kernels by total
duration.

  python tools/epoch_breakdown.py gpurun_out/sageprof/run_kernel_trace.csv \\
      [--marker 'gspmm_sum_kernel<2, 64, 16, 0, 1, true, false'] [--top 25]
"""
import argparse
import collections
import csv
import json


def breakdown(path, marker, top):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(idx) < 2:
        raise SystemExit("fewer than two launches of the marker kernel")
    a, b = idx[-2], idx[-1]
    win = rows[a:b]
    agg = collections.defaultdict(lambda: [0, 0])
    for r in win:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[r["Kernel_Name"]][0] += d
        agg[r["Kernel_Name"]][1] += 1
    kernels = sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]
    return {"wall_ms": (int(rows[b]["Start_Timestamp"]) - int(win[0]["Start_Timestamp"])) / 1e6,
            "busy_ms": sum(v[0] for v in agg.values()) / 1e6, "launches": len(win),
            "kernels": [{"name": k[:160], "ms": v[0] / 1e6, "calls": v[1]} for k, v in kernels]}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="gspmm_sum_kernel<2, 64, 16, 0, 1, true, false")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    print(json.dumps(breakdown(a.trace, a.marker, a.top), indent=1))
