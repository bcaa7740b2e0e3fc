"""Group a rocprofv3 kernel trace by what the kernels do (r04 verdict, Weak 5:
where the model legs' non-engine time goes).

Reads ``<dir>/<run>_kernel_trace.csv`` (rocprofv3 --kernel-trace
--output-format csv) and, when present, the memory-copy trace. Over the
trace's last ``--tail`` fraction of time (past the first steps' one-time
builds), per step: each group's kernel time and launches, the GPU busy time
(the union of kernel intervals), the idle gaps between kernels, and the
device-to-host copies (each one a host sync inside the step).

  python tools/trace_groups.py <dir> --steps 20 [--tail 0.8] [--out groups.json]
"""
import argparse
import collections
import csv
import glob
import json
import os
import re

GROUPS = [
    ("engine: typed-block g-SpMM", r"typed_block"),
    ("engine: GAT fused", r"gat_aggregate|gat_backward|rowsum_heads|gsddmm|gat_"),
    ("engine: g-SpMM", r"gspmm|short_rows"),
    ("engine: other", r"dglhip|node_linear|xent|div_rows|plan_|block_walk|block_scatter"),
    ("GEMM (Linear, bmm)", r"Cijk_|gemm|Gemm|MT\d+x\d+"),
    ("optimizer (Adam, clip)", r"multi_tensor_apply|[Aa]dam|Lerp|Foreach|foreach"),
    ("sort / scan (CSR builds)", r"rocprim|radix|merge_sort|scan|searchsorted|sort"),
    ("reductions (norms, means, min/max)", r"reduce_kernel|Reduce|norm"),
    ("gather / scatter / index", r"gather|scatter|index|Index|embedding|Embedding"),
    ("loss / activations", r"binary_cross|cross_entropy|nll|softmax|sigmoid|elu|relu|Relu|"
                           r"threshold|log_"),
    ("dropout / random", r"dropout|Dropout|philox|random|Random|bernoulli"),
    ("fill / copy", r"fill|Fill|copyBuffer|copy_kernel|CopyKernel|direct_copy"),
    ("elementwise", r"elementwise|Functor|Binary|Unary"),
]


def group_of(name):
    for g, pat in GROUPS:
        if re.search(pat, name):
            return g
    return "other"


def load(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, required=True, help="steps in the trace's tail window")
    ap.add_argument("--tail", type=float, default=0.8)
    ap.add_argument("--wall-ms", type=float, default=None, help="measured wall ms per step")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    kt = glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True)
    if not kt:
        raise SystemExit("no kernel trace under %s" % args.dir)
    rows = load(kt[0])
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in rows)
    t_first, t_last = ev[0][0], max(e[1] for e in ev)
    t0 = t_last - args.tail * (t_last - t_first)
    ev = [e for e in ev if e[0] >= t0]
    span = (ev[-1][1] - ev[0][0]) / 1e6 if ev else 0.0
    per = collections.defaultdict(lambda: [0.0, 0])
    busy, cur_s, cur_e = 0.0, None, None
    for s, e, name in ev:
        g = per[group_of(name)]
        g[0] += (e - s) / 1e6
        g[1] += 1
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += (cur_e - cur_s) / 1e6
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += (cur_e - cur_s) / 1e6
    # the window holds about args.tail of the steps
    steps = max(args.steps * args.tail, 1e-9)
    res = {"window_ms": span, "steps_in_window": steps,
           "gpu_busy_ms_per_step": busy / steps,
           "gpu_idle_ms_per_step": (span - busy) / steps,
           "groups": {g: {"ms_per_step": v[0] / steps, "launches_per_step": v[1] / steps}
                      for g, v in sorted(per.items(), key=lambda kv: -kv[1][0])}}
    mc = glob.glob(os.path.join(args.dir, "**", "*memory_copy_trace.csv"), recursive=True)
    if mc:
        cp = [r for r in load(mc[0]) if int(r["Start_Timestamp"]) >= t0]
        d2h = [r for r in cp if "DEVICE_TO_HOST" in r.get("Direction", "") or
               "DeviceToHost" in r.get("Direction", "")]
        res["copies_per_step"] = len(cp) / steps
        res["device_to_host_copies_per_step"] = len(d2h) / steps
    if args.wall_ms:
        res["wall_ms_per_step"] = args.wall_ms
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
