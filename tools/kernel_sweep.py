"""Interleaved A/B sweep of g-SpMM copy_u+sum kernel variants on the bench graph
(cdna_hip_programming.md §5.4 rule 24: variants x rounds in one process).

  python tools/kernel_sweep.py [--rounds 5] [--workload reddit|rmat] [--rmat-scale 26]

RMAT runs with the heavy-row split on (kernel.set_row_split("auto")), as
bench.py's RMAT line does.
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import _ffi, data, kernel  # noqa: E402

VARIANTS = [(0, 0, 0, 0), (2, 64, 8, 0), (2, 64, 16, 0), (2, 64, 32, 0), (4, 32, 16, 0),
            (4, 32, 32, 0), (2, 64, 8, 1), (2, 64, 16, 1), (4, 32, 8, 1), (4, 32, 16, 1)]
# (vec, lanes per row, gathers per batch, software-pipelined batches); (0,0,0,0) = default


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--workload", default="reddit")
    ap.add_argument("--rmat-scale", type=int, default=24)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    if args.workload == "rmat":
        src, dst, n = data.rmat(args.rmat_scale, 16, device=dev)
        kernel.set_row_split("auto")  # as bench.py's RMAT line
    else:
        src, dst, n = data.reddit_like(device=dev)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    h = torch.rand(n, 128, device=dev) * 2 - 1
    ref = kernel.gspmm(adj, "copy_u", "sum", h)
    times = {v: [] for v in VARIANTS}
    for _ in range(args.rounds):
        for v in VARIANTS:
            _ffi.check_call(_ffi.LIB.dglhip_set_spmm_variant(*v))
            out = kernel.gspmm(adj, "copy_u", "sum", h)
            assert torch.equal(out, ref), v
            kernel.timing_enable(True)
            for _ in range(args.iters):
                kernel.gspmm(adj, "copy_u", "sum", h)
            ms, _ = kernel.timing_read()
            kernel.timing_enable(False)
            times[v].append(ms / args.iters)  # per g-SpMM call (all its launches)
    _ffi.check_call(_ffi.LIB.dglhip_set_spmm_variant(0, 0, 0, 0))
    res = {"%d,%d,%d,%d" % v: {"median_ms": sorted(t)[len(t) // 2], "min_ms": min(t)}
           for v, t in times.items()}
    print(json.dumps({"workload": args.workload, "variants": res}, indent=1))


if __name__ == "__main__":
    main()
