"""A/B of the blocked schedule's launches on the Reddit-shaped graph (copy_u +
sum, F = 128): default cache policy vs non-temporal running rows
(dglhip_set_cache_policy(3): each item's partial row loaded and stored
non-temporally), and eager launches vs one replayed HIP graph of the call.
Times are wall time per call between events on the stream (launch gaps
included) and kernel time per call (dglhip timing); outputs compared bit for
bit.

  python tools/items_policy_ab.py [--rounds 3] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import _ffi, data, kernel  # noqa: E402


def wall(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def kern(fn, iters):
    fn()
    torch.cuda.synchronize()
    kernel.timing_enable(True)
    for _ in range(iters):
        fn()
    ms, cnt = kernel.timing_read()
    kernel.timing_enable(False)
    return ms / iters, cnt // iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(device=dev)
    h = torch.rand(n, 128, device=dev) * 2 - 1
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    csr = adj.fwd
    out = torch.empty(n, 128, device=dev)

    def call():
        kernel.gspmm_into(csr, out, h)

    call()
    ref = out.clone()
    res = {"graph": "reddit_like", "nodes": n, "edges": csr.nnz, "rounds": []}
    # one replayed graph of the whole call (plan cached above)
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(stream):
        call()
    torch.cuda.current_stream().wait_stream(stream)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        call()
    torch.cuda.synchronize()
    for r in range(args.rounds):
        row = {}
        for name, pol in (("default", -1), ("nt_rows", 3)):
            _ffi.check_call(_ffi.LIB.dglhip_set_cache_policy(pol))
            row[name + "_wall_ms"] = wall(call, args.iters)
            row[name + "_kernel_ms"], row["launches"] = kern(call, args.iters)
            row[name + "_bits_equal"] = bool(torch.equal(out, ref))
        _ffi.check_call(_ffi.LIB.dglhip_set_cache_policy(-1))
        row["hip_graph_wall_ms"] = wall(g.replay, args.iters)
        row["hip_graph_bits_equal"] = bool(torch.equal(out, ref))
        res["rounds"].append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
