"""Where the RMAT g-SpMM's time goes by row length: the light-row launch
(heavy rows excluded, as under the heavy-row split) timed over growing
prefixes of its degree-descending schedule — rows with more than 64, 16, 8, 4
slots, every non-empty row, every row (empty rows only store zeros). The
increments show what the short and empty rows of an R-MAT graph cost per
edge / per row, against their bytes.

  python tools/rmat_tail_study.py [--rmat-scale 26] [--iters 3]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import _ffi, data, kernel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rmat-scale", type=int, default=26)
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    F = 128
    src, dst, n = data.rmat(args.rmat_scale, 16, seed=0, device=dev)
    E = int(src.numel())
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    csr = adj.fwd
    kernel.set_row_split("auto")
    t = kernel._split_threshold(csr)
    plan = csr.split_plan(t) if t else None
    light = plan["light"] if plan is not None else csr.row_order
    ip = csr.host_indptr.numpy()
    deg = (ip[1:] - ip[:-1])[light.cpu().numpy()]
    h = torch.rand(n, F, device=dev) * 2 - 1
    out = torch.empty(n, F, device=dev)
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    res = []
    for cut in (64, 16, 8, 4, 0, -1):
        rows = int((deg > cut).sum())
        for _ in range(2):
            kernel.timing_enable(True)
            for _ in range(args.iters):
                _ffi.check_call(_ffi.LIB.dglhip_gspmm_device(
                    0, 0, rows, F, _ffi.ptr(csr.indptr), _ffi.ptr(csr.indices), None,
                    _ffi.ptr(h), None, 0, _ffi.ptr(out), None, _ffi.ptr(light), stream))
            ms, cnt = kernel.timing_read()
            kernel.timing_enable(False)
        edges = int(deg[:rows].sum())
        res.append({"rows_with_deg_gt": cut, "rows": rows, "edges": edges,
                    "ms": round(ms / cnt, 3)})
        print(res[-1], file=sys.stderr, flush=True)
    # the same tail through the batched short-row kernel, tier by tier
    tiers = []
    n_long, tail = csr.tiers(threshold=t)  # the plan's tiers of the same list
    lo = n_long
    for maxd, (rows_t, sp, cols), cnt_rows in tail:
        hi = lo + cnt_rows
        for _ in range(2):
            kernel.timing_enable(True)
            for _ in range(args.iters):
                _ffi.check_call(_ffi.LIB.dglhip_gspmm_short_rows_device(
                    0, 0, cnt_rows, F, maxd, n, _ffi.ptr(rows_t), _ffi.ptr(sp),
                    _ffi.ptr(cols), _ffi.ptr(h), _ffi.ptr(out), 0, stream))
            ms, cnt = kernel.timing_read()
            kernel.timing_enable(False)
        edges = int(deg[lo:hi].sum())
        byts = edges * (4 * F + 4) + (hi - lo) * (4 * F + 8)
        tiers.append({"max_deg": maxd, "rows": hi - lo, "edges": edges, "ms": round(ms / cnt, 3),
                      "GBs": round(byts / (ms / cnt * 1e-3) / 1e9, 1)})
        print(tiers[-1], file=sys.stderr, flush=True)
        lo = hi
    print(json.dumps({"graph": "rmat-%d" % args.rmat_scale, "nodes": n, "edges": E,
                      "heavy_split_threshold": t, "light_rows": int(light.numel()),
                      "prefixes": res, "long_rows": n_long, "short_row_tiers": tiers},
                     indent=1))


if __name__ == "__main__":
    main()
