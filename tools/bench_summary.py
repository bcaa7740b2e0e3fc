"""One line per leg of a bench.py JSON line: ms per step / epoch, kernel ms and
roofline fraction (what the one-off GPU scripts used to print by hand).

  python tools/bench_summary.py gpurun_out/benchlegs.json
"""
import json
import sys


def main(path):
    line = open(path).read().strip().splitlines()[-1]
    d = json.loads(line)
    r = d.get("roofline") or {}
    print("headline %.3f ms/step, kernel %.3f ms, frac %s" % (
        d["ms_per_step"], r.get("kernel_ms") or 0.0, r.get("frac")))
    for k, v in d.items():
        if not isinstance(v, dict) or k in ("roofline", "config", "cpu_baseline"):
            continue
        ms = v.get("ms_per_step", v.get("ms_per_epoch"))
        if ms is None:
            continue
        rr = v.get("roofline") or {}
        extra = ""
        for key in ("ms_per_epoch_hip_graph", "ms_per_step_hip_graph"):
            if key in v:
                extra = ", HIP graph %.3f ms" % v[key]
        print("%-14s %.3f ms%s, kernel %s ms, frac %s" % (
            k, ms, extra, v.get("kernel_ms", v.get("kernel_ms_rank0")), rr.get("frac")))


if __name__ == "__main__":
    main(sys.argv[1])
