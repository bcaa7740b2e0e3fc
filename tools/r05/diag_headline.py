"""r05 diagnostic: the headline update_all call against the direct
kernel.gspmm_into call on the same Reddit-shaped graph (per-call GPU span,
launches, the plan's choice)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
import dgl  # noqa: E402
import dgl.function as fn  # noqa: E402
from dgl import data, kernel  # noqa: E402


def timed(fn_, iters=10):
    fn_()
    torch.cuda.synchronize()
    kernel.timing_enable(True, per_call=True)
    t0 = time.perf_counter()
    for _ in range(iters):
        fn_()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / iters * 1e3
    ms, calls = kernel.timing_read()
    kernel.timing_enable(False)
    return {"gpu_ms_per_call": ms / max(calls, 1), "calls": calls / iters, "wall_ms": wall}


def main():
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(device=dev)
    gen = torch.Generator(device=dev).manual_seed(0)
    h = torch.rand(n, 128, generator=gen, device=dev) * 2 - 1
    res = {}
    g = dgl.DGLGraph((src.cpu(), dst.cpu()))
    g.ndata["h"] = h
    adj_g = g.sparse_adjacency(dev)
    res["graph_adj_blocks"] = kernel.blocked_schedule(adj_g, h)
    res["graph_adj_stats"] = adj_g.fwd.plan.stats() if hasattr(adj_g.fwd.plan, "stats") else None
    res["update_all"] = timed(lambda: g.update_all(fn.copy_src("h", "m"), fn.sum("m", "h_out")))
    print(json.dumps(res), flush=True)
    out = torch.empty(n, 128, device=dev)
    res["gspmm_into_graph_adj"] = timed(lambda: kernel.gspmm_into(adj_g.fwd, out, h))
    res["gspmm_graph_adj"] = timed(lambda: kernel.gspmm(adj_g, "copy_u", "sum", h))
    print(json.dumps(res), flush=True)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    res["coo_adj_blocks"] = kernel.blocked_schedule(adj, h)
    res["gspmm_into_coo_adj"] = timed(lambda: kernel.gspmm_into(adj.fwd, out, h))
    ref = out.clone()
    kernel.gspmm_into(adj_g.fwd, out, h)
    res["same_bits"] = bool(torch.equal(out, ref))
    f1, f2 = adj.fwd, adj_g.fwd
    res["indptr_equal"] = bool(torch.equal(f1.indptr, f2.indptr))
    res["indices_equal"] = bool(torch.equal(f1.indices, f2.indices))
    res["row_order_equal"] = bool(torch.equal(f1.row_order, f2.row_order)) \
        if f1.row_order is not None and f2.row_order is not None else None
    res["policy"] = kernel.schedule_policy()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
