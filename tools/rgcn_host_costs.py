"""Host (enqueue) microseconds of the R-GCN step's building blocks on the
device at configs[4]'s sizes (a 30,000-edge sampled graph, 11,8xx rows, 474
relations, 500 features), no synchronisation inside the timed loops.

  python tools/rgcn_host_costs.py --out gpurun_out/rgcn_host_costs.json
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import kernel  # noqa: E402
from dgl._ffi import LIB, ptr  # noqa: E402


def host_us(fn, n=200):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    host = (time.perf_counter() - t) / n * 1e6
    torch.cuda.synchronize()
    return round(host, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    E, N, R, F = 30000, 11800, 474, 500
    row = torch.randint(0, N, (E,), generator=g, device=dev)
    col = torch.randint(0, N, (E,), generator=g, device=dev)
    rel = torch.randint(0, R, (E,), generator=g, device=dev)
    res = {}
    res["ctypes call, no launch (typed_block_msg_ok)"] = host_us(
        lambda: LIB.dglhip_typed_block_msg_ok(100, 5, 5))
    x = torch.empty(1 << 20, device=dev)
    res["torch fill_ (one launch)"] = host_us(lambda: x.fill_(1.0))
    res["torch empty"] = host_us(lambda: torch.empty(1000, device=dev))
    res["torch mul"] = host_us(lambda: x * 2.0)
    res["build_csr device (validate=False)"] = host_us(
        lambda: kernel.build_csr(N, N, row, col, kernel.ORDER_EID, dev, schedule=False,
                                 validate=False))
    c = kernel.build_csr(N, N, row, col, kernel.ORDER_EID, dev, schedule=False, validate=False)
    res["_typed_items"] = host_us(lambda: kernel._typed_items(c.indptr, E))
    res["row_ids"] = host_us(lambda: torch.repeat_interleave(
        torch.arange(c.num_rows, device=dev), c.indptr[1:] - c.indptr[:-1], output_size=E))
    res["_RelationGroups"] = host_us(lambda: kernel._RelationGroups(c, rel, R))
    res["_position_groups (2n = 60k)"] = host_us(
        lambda: kernel._position_groups(torch.cat([row, col]), N))
    grp = kernel._RelationGroups(c, rel, R)
    h = torch.randn(N, F, device=dev)
    w = torch.randn(R, 100, 5, 5, device=dev)
    res["_run_typed_msg (msg + sum)"] = host_us(
        lambda: kernel._run_typed_msg(c, None, grp, grp.src, h, w, None, 100, 5, 5))
    res["typed_block_spmm forward (autograd off)"] = host_us(
        lambda: kernel.typed_block_spmm(kernel.SparseAdj(c, None, (N, N)), h, w, rel))
    for k, v in res.items():
        print("%-50s %s" % (k, v), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
