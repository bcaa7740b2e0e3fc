"""Where the headline's L2-miss traffic goes (r03 verdict, "Next" 5).

The source-blocked copy_u + sum over the Reddit-shaped graph (bench.py's N = 1
step) runs one launch per source block. Each launch gathers its block's
source rows (L2-resident by design) and passes once over the output rows of
its items (read + write; the first block's launch only writes). This tool

  run    builds the bench graph, prints the plan (items and slots per block)
         as JSON, then runs ``--calls`` g-SpMM calls — run it under
         ``rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum`` (and a second pass with
         ``TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum``);
  parse  splits each launch's counters into the running-row part (each item
         reads and writes its 512-B row: 4 + 4 128-B lines; the first block
         only writes) and the rest (the gathered H rows and the slot stream).

  python tools/l2_split.py run --out gpurun_out/l2_plan.json
  python tools/l2_split.py parse gpurun_out/l2_plan.json <counter csv> [<csv> ...]
"""
import argparse
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]


def run(args):
    import torch
    from dgl import data, kernel
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(scale=1, seed=0, device=dev)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    h = torch.rand(n, 128, device=dev) * 2 - 1
    plan = kernel._block_plan(adj.fwd, h, 128)
    info = {"nodes": n, "edges": adj.fwd.nnz, "calls": args.calls,
            "blocks": [{"items": int(it.rows.numel()), "slots": int(it.nnz),
                        "suffix": bool(it.suffix)} for it in plan]}
    with open(args.out, "w") as f:
        json.dump(info, f)
    for _ in range(args.calls):
        kernel.gspmm(adj, "copy_u", "sum", h)
    torch.cuda.synchronize()
    print(json.dumps({"launches_per_call": len(plan), "calls": args.calls}))


def parse(args):
    info = json.load(open(args.plan))
    blocks = info["blocks"]
    B = len(blocks)
    per = collections.defaultdict(dict)  # dispatch -> counter -> value
    names = {}
    for path in args.csvs:
        with open(path) as f:
            for r in csv.DictReader(f):
                if "gspmm_items" not in r["Kernel_Name"] and "gspmm_sum" not in r["Kernel_Name"]:
                    continue
                d = int(r["Dispatch_Id"])
                per[(path, d)][r["Counter_Name"]] = float(r["Counter_Value"])
                names[(path, d)] = r["Kernel_Name"]
    out = {}
    for path in args.csvs:
        ds = sorted(d for (p, d) in per if p == path)
        if len(ds) % B:
            raise SystemExit("%s: %d g-SpMM dispatches, not a multiple of %d launches"
                             % (path, len(ds), B))
        calls = len(ds) // B
        for b in range(B):
            for c in range(calls):
                for k, v in per[(path, ds[c * B + b])].items():
                    out.setdefault(b, collections.defaultdict(float))[k] += v / calls
    rows = []
    tot = collections.defaultdict(float)
    for b in range(B):
        it = blocks[b]["items"]
        row_lines = it * 4 * (1 if b == 0 else 2)  # 512-B rows: 4 lines each way
        entry = {"block": b, "items": it, "slots": blocks[b]["slots"],
                 "row_pass_lines": row_lines, "gather_lines": blocks[b]["slots"] * 4}
        for k, v in out[b].items():
            entry[k] = v
            tot[k] += v
        rows.append(entry)
        tot["row_pass_lines"] += row_lines
        tot["gather_lines"] += blocks[b]["slots"] * 4
    res = {"per_launch": rows, "per_call": dict(tot),
           "note": "TCC counts are 128-B requests summed over the 8 XCDs' L2 channels; "
                   "row_pass_lines = items x 4 lines read (not the first block) + 4 written; "
                   "gather_lines = slots x 4 lines of 512-B source rows"}
    if "TCC_MISS_sum" in tot and "TCC_HIT_sum" in tot:
        res["per_call"]["miss_rate"] = tot["TCC_MISS_sum"] / (tot["TCC_MISS_sum"] +
                                                              tot["TCC_HIT_sum"])
        # if every row-pass line misses, the rest of the misses are the gathers'
        res["per_call"]["gather_misses_if_row_pass_all_miss"] = (tot["TCC_MISS_sum"] -
                                                                 tot["row_pass_lines"])
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd")
    r = sub.add_parser("run")
    r.add_argument("--calls", type=int, default=3)
    r.add_argument("--out", default="gpurun_out/l2_plan.json")
    p = sub.add_parser("parse")
    p.add_argument("plan")
    p.add_argument("csvs", nargs="+")
    p.add_argument("--out", default=None)
    args = ap.parse_args()
    run(args) if args.cmd == "run" else parse(args)


if __name__ == "__main__":
    main()
