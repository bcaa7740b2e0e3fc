"""Where the GAT backward's traffic goes (r04 verdict, "Next" 2).

The fused GAT layer's backward over the transpose (gat_backward_t_kernel, one
launch per source block of the transposed CSR's plan) gathers one 512-B dout
row per slot from its block's slice, reads per slot the pair operands (the
column id, the forward slot, er and dz of the destination) and stores the
attention gradient g (32 B) at the edge's forward slot; rowsum_heads8_kernel
then sums g per destination row (d_er). This tool

  run    builds the Reddit-shaped graph, runs ``--calls`` GAT 8 x 16 forward +
         backward steps (run it under ``rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum``
         and again with ``TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum``), and writes the
         transposed plan (items and slots per block) as JSON;
  parse  averages each kernel's counters per call and sets them beside the
         algorithmic line counts of each stream:
           gather    slots x 4 lines (the dout rows)
           operands  slots x (4 + 8 B of column id and forward slot, sequential)
                     + pairs' er / dz reads (2 x 32 B of one line each, per slot)
           g_store   slots x 32 B scattered (one partial line per slot)
           row_pass  items x (4 lines of d_ft read, not the first block, + 4 written)

  python tools/gat_bwd_split.py run --out gpurun_out/gat_plan.json
  python tools/gat_bwd_split.py parse gpurun_out/gat_plan.json <counter csv> [...]
"""
import argparse
import collections
import csv
import json
import os
import re
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
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    ft = (torch.rand(n, 8, 16, generator=gen, device=dev) * 2 - 1).requires_grad_(True)
    el = (torch.rand(n, 8, generator=gen, device=dev) - 0.5).requires_grad_(True)
    er = (torch.rand(n, 8, generator=gen, device=dev) - 0.5).requires_grad_(True)
    gout = torch.rand(n, 8, 16, generator=gen, device=dev)
    gz = torch.rand(n, 8, 1, generator=gen, device=dev)

    def fb():
        fs, z = kernel.gat_aggregate(adj, ft, el, er)
        torch.autograd.backward([fs, z], [gout, gz])
        ft.grad = el.grad = er.grad = None

    fb()  # builds the transposed CSR and its plan
    torch.cuda.synchronize()
    # marker: parse counts only the dispatches after the last spin kernel
    # (the timed calls; not the graph build, the sort or the plan's call)
    torch.cuda._sleep(1000)
    plan = kernel._block_plan(adj.bwd, torch.empty(2, 128, device=dev), 128,
                              kernel._GAT_BWD_BLOCK_BYTES)
    info = {"nodes": n, "edges": adj.fwd.nnz, "calls": args.calls,
            "blocks": [] if plan is None else
            [{"items": int(it.rows.numel()), "slots": int(it.nnz), "suffix": bool(it.suffix)}
             for it in plan]}
    with open(args.out, "w") as f:
        json.dump(info, f)
    for _ in range(args.calls):
        fb()
    torch.cuda.synchronize()
    print(json.dumps({"launches_per_call": len(info["blocks"]), "calls": args.calls + 1}))


def kernel_key(full):
    """The kernel's own name from a demangled signature: namespaces (the
    anonymous one included), template arguments and parameters dropped."""
    s = full.replace("(anonymous namespace)", "anon").replace("void ", "").strip()
    s = re.split(r"[(<]", s, maxsplit=1)[0]
    return s.split("::")[-1]


def parse(args):
    info = json.load(open(args.plan))
    blocks = info["blocks"]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    marked = True
    for path in args.csvs:
        with open(path) as f:
            rows = list(csv.DictReader(f))
        marks = [int(r["Dispatch_Id"]) for r in rows if "spin_kernel" in r["Kernel_Name"]]
        start = max(marks) if marks else -1
        marked = marked and bool(marks)
        for r in rows:
            if int(r["Dispatch_Id"]) <= start:
                continue
            name = kernel_key(r["Kernel_Name"])
            per[name][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[name].add((path, r["Dispatch_Id"]))
    # with the marker only the timed calls are counted; an old capture
    # without one also holds the plan-building call
    calls = info["calls"] if marked else info["calls"] + 1
    slots = sum(b["slots"] for b in blocks)
    items = sum(b["items"] for b in blocks)
    first = blocks[0]["items"] if blocks else 0
    model = {"gather_lines": slots * 4,
             "operand_seq_bytes": slots * 12,
             "pair_operand_lines": slots * 2,
             "g_store_partial_lines": slots,
             "row_pass_lines": (items - first) * 4 + items * 4}
    res = {"model_per_call": model, "calls_counted": calls,
           "window": "dispatches after the spin-kernel marker (the timed calls only)"
           if marked else "every dispatch (no marker in the capture)", "kernels": {}}
    for name, cs in per.items():
        # each capture (one per counter pass) holds every dispatch once
        res["kernels"][name] = {"dispatches_per_call":
                                len(disp[name]) / float(calls * len(args.csvs)),
                                "per_call": {k: v / calls for k, v in cs.items()}}
    bt = res["kernels"].get("gat_backward_t_kernel", {}).get("per_call", {})
    if "TCC_HIT_sum" in bt and "TCC_MISS_sum" in bt:
        bt["miss_rate"] = bt["TCC_MISS_sum"] / (bt["TCC_HIT_sum"] + bt["TCC_MISS_sum"])
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd")
    r = sub.add_parser("run")
    r.add_argument("--calls", type=int, default=3)
    r.add_argument("--out", default="gpurun_out/gat_plan.json")
    p = sub.add_parser("parse")
    p.add_argument("plan")
    p.add_argument("csvs", nargs="+")
    p.add_argument("--out", default=None)
    args = ap.parse_args()
    run(args) if args.cmd == "run" else parse(args)


if __name__ == "__main__":
    main()
