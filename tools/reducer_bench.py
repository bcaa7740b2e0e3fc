"""Kernel time of each g-SpMM reducer / message on the Reddit-shaped bench
graph (hipEvent pairs on the launch stream, dglhip_timing_*), with the
algorithmic bandwidth of each: every slot gathers one source row (4F B) plus
its 4-B column id (+ 8-B eid and the edge values when the message reads edge
features), every row writes 4F B (+ 8F B of argmax ids for max).

  python tools/reducer_bench.py [--feat 128] [--iters 10]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import data, kernel  # noqa: E402

# frac against the gather's regime ceiling (bench.py gather_peak): the
# guide's L2 indexed-row rate when the call ran source-blocked (several
# launches), its Infinity-Cache random-row rate otherwise (the 119 MB table
# fits the 256 MiB cache)
L2_PEAK_GBS = 18800.0
IC_PEAK_GBS = 8600.0


def peak_of(launches_per_call):
    return L2_PEAK_GBS if launches_per_call > 1 else IC_PEAK_GBS


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--feat", type=int, default=128)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(device=dev)
    E = int(src.numel())
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    F = args.feat
    h = torch.rand(n, F, device=dev) * 2 - 1
    w = torch.rand(E, device=dev)
    cases = [("copy_u", "sum", None, "eid"), ("copy_u", "mean", None, "eid"),
             ("copy_u", "max", None, "eid"), ("u_mul_e", "sum", w, "eid"),
             ("u_mul_e", "max", w, "eid"),
             # the weights laid out in forward-CSR slot order (GATConv's
             # attention): no per-slot eid gather
             ("u_mul_e", "sum", w, "slot")]
    res = []
    for msg, red, e, order in cases:
        kernel.gspmm(adj, msg, red, h, e, edge_order=order)
        torch.cuda.synchronize()
        kernel.timing_enable(True)
        for _ in range(args.iters):
            kernel.gspmm(adj, msg, red, h, e, edge_order=order)
        ms, cnt = kernel.timing_read()
        kernel.timing_enable(False)
        t = ms / args.iters  # per call (a blocked call launches several kernels)
        per_edge = 4 * F + 4 + ((12 if order == "eid" else 4) if e is not None else 0)
        per_row = 4 * F + 8
        byts = E * per_edge + n * per_row
        res.append({"msg": msg, "reduce": red, "edge_order": order, "kernel_ms": round(t, 3),
                    "edges_per_s": E / (t * 1e-3),
                    "algorithmic_GBs": round(byts / (t * 1e-3) / 1e9, 1),
                    "launches": cnt // args.iters, "peak_GBs": peak_of(cnt // args.iters),
                    "frac": round(byts / (t * 1e-3) / 1e9 / peak_of(cnt // args.iters), 3)})
    # g-SDDMM dot (u_mul_e weight gradient; GAT per-head dots): per slot one
    # lhs row (the destination's, reused along the row) and one gathered rhs row
    for heads in (1, 2, 4, 8, 16, 32):
        for alt in (0, 1):
            for order in ("eid", "slot"):
                if order == "slot" and alt:
                    continue
                kernel.set_sddmm_variant(alt)
                kernel.gsddmm_dot(adj, h, h, E, heads, edge_order=order)
                torch.cuda.synchronize()
                kernel.timing_enable(True)
                for _ in range(args.iters):
                    kernel.gsddmm_dot(adj, h, h, E, heads, edge_order=order)
                ms, cnt = kernel.timing_read()
                kernel.timing_enable(False)
                kernel.set_sddmm_variant(0)
                t = ms / args.iters  # per call (a blocked call launches several kernels)
                byts = E * (4 * F + 4 + (8 if order == "eid" else 0) + 4 * heads) + \
                    n * (4 * F + 8)
                res.append({"msg": "sddmm_dot", "reduce": "heads=%d" % heads,
                            "variant": "alternate depth" if alt else "default",
                            "edge_order": order, "kernel_ms": round(t, 3),
                            "edges_per_s": E / (t * 1e-3),
                            "algorithmic_GBs": round(byts / (t * 1e-3) / 1e9, 1),
                            "launches": cnt // args.iters, "peak_GBs": peak_of(cnt // args.iters),
                    "frac": round(byts / (t * 1e-3) / 1e9 / peak_of(cnt // args.iters), 3)})
    # GAT edge attention (fused u_add_v -> leaky_relu -> exp), 8 heads
    a1 = torch.rand(n, 8, device=dev)
    a2 = torch.rand(n, 8, device=dev)
    for order in ("eid", "slot"):
        kernel.edge_attention(adj, a1, a2, E, edge_order=order)
        torch.cuda.synchronize()
        kernel.timing_enable(True)
        for _ in range(args.iters):
            kernel.edge_attention(adj, a1, a2, E, edge_order=order)
        ms, cnt = kernel.timing_read()
        kernel.timing_enable(False)
        t = ms / args.iters  # per call (a blocked call launches several kernels)
        byts = E * (4 + 32 + 32 + (8 if order == "eid" else 0)) + n * (32 + 8)
        res.append({"msg": "edge_attention", "reduce": "heads=8", "edge_order": order,
                    "kernel_ms": round(t, 3), "edges_per_s": E / (t * 1e-3),
                    "algorithmic_GBs": round(byts / (t * 1e-3) / 1e9, 1),
                    "launches": cnt // args.iters, "peak_GBs": peak_of(cnt // args.iters),
                    "frac": round(byts / (t * 1e-3) / 1e9 / peak_of(cnt // args.iters), 3)})
    print(json.dumps({"graph": "reddit_like", "nodes": n, "edges": E, "feat": F,
                      "note": "max also writes the (N, F) int64 argmax only under autograd; "
                              "timed here without it", "cases": res}, indent=1))


if __name__ == "__main__":
    main()
