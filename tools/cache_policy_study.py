"""Cache-policy study of copy_u + sum on an HBM-bound graph (RMAT).

RMAT's sources are heavily skewed (scale 24: the 0.8 % of nodes with the most
out-edges are the sources of 57 % of the edges), yet the caches save only
~4 % of the gathered bytes under the default policy, because once-read rows
and the output stream evict the rows that are read again. This interleaves
(variants x rounds in one process) the kernel's cache policies:
  default, all-nt, nt-output, and hot-marked (column-id bit 31 set on the
  sources with the most out-edges, up to a byte budget of their rows; hot rows
  load with the default policy, the rest and the output non-temporal).
Every variant's output must equal the default's bit for bit.

  python tools/cache_policy_study.py [--rmat-scale 26] [--rounds 3]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import _ffi, data, kernel  # noqa: E402


def log(msg):
    print("[policy] " + msg, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--rmat-scale", type=int, default=26)
    ap.add_argument("--budgets-mb", default="32,96,192,320")
    ap.add_argument("--no-row-split", action="store_true")
    ap.add_argument("--workload", default="rmat", choices=["rmat", "reddit"])
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    t0 = time.time()
    if args.workload == "rmat":
        src, dst, n = data.rmat(args.rmat_scale, 16, device=dev)
    else:
        src, dst, n = data.reddit_like(device=dev)
    if not args.no_row_split and args.workload == "rmat":
        kernel.set_row_split("auto")
    outdeg = torch.bincount(src, minlength=n)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    E = int(src.numel())
    del src, dst
    order = torch.argsort(outdeg, descending=True)
    cum = torch.cumsum(outdeg[order].double(), 0) / E
    log("graph %d nodes %d edges built in %.1fs" % (n, E, time.time() - t0))
    h = torch.rand(n, 128, device=dev) * 2 - 1
    plain = adj.fwd.indices
    variants = [("auto", -1, None), ("default", 0, None), ("nt_all", 1, None),
                ("nt_out", 3, None)]
    marked = {}
    for mb in [float(x) for x in args.budgets_mb.split(",") if x]:
        k = max(1, min(n, int(mb * 2**20) // (128 * 4)))
        hot = torch.zeros(n, dtype=torch.bool, device=dev)
        hot[order[:k]] = True
        flag = torch.tensor(-2**31, dtype=torch.int32, device=dev)
        ind = torch.where(hot[plain.long()], plain | flag, plain)
        marked[mb] = (ind, float(cum[k - 1]))
        variants.append(("hot_%gMB" % mb, 2, mb))
        del hot
    log("hot coverage: " + ", ".join("%gMB: %.3f of edges" % (mb, c)
                                     for mb, (_, c) in marked.items()))
    _ffi.check_call(_ffi.LIB.dglhip_set_cache_policy(0))
    ref = kernel.gspmm(adj, "copy_u", "sum", h)
    times = {v[0]: [] for v in variants}
    for r in range(args.rounds):
        for name, pol, mb in variants:
            adj.fwd.indices = marked[mb][0] if mb is not None else plain
            _ffi.check_call(_ffi.LIB.dglhip_set_cache_policy(pol))
            out = kernel.gspmm(adj, "copy_u", "sum", h)
            assert torch.equal(out, ref), name
            del out
            kernel.timing_enable(True)
            for _ in range(args.iters):
                kernel.gspmm(adj, "copy_u", "sum", h)
            ms, _ = kernel.timing_read()
            kernel.timing_enable(False)
            times[name].append(ms / args.iters)
        log("round %d: %s" % (r, ", ".join("%s %.1f" % (k, v[-1]) for k, v in times.items())))
    adj.fwd.indices = plain
    _ffi.check_call(_ffi.LIB.dglhip_set_cache_policy(-1))
    res = {k: {"median_ms": sorted(v)[len(v) // 2], "min_ms": min(v)} for k, v in times.items()}
    for mb, (_, c) in marked.items():
        res["hot_%gMB" % mb]["hot_edge_fraction"] = c
    wl = "rmat-%d" % args.rmat_scale if args.workload == "rmat" else "reddit-shaped"
    print(json.dumps({"workload": wl, "edges": E,
                      "row_split": not args.no_row_split, "variants": res}, indent=1))


if __name__ == "__main__":
    main()
