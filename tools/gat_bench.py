"""GAT layer aggregation, fused vs three kernels.

Per graph and head shape: the kernel ms per forward call (every kernel of the
call, hipEvent pairs on the launch stream) of
* fused      kernel.gat_aggregate under no_grad (nothing per edge stored)
* fused+a    the same with autograd on (the E x H attention stored, slot order)
* fused+drop the same with attention dropout 0.6 (the dropped copy stored too)
* *_one_launch  the same with the source-blocked schedule off
* unfused    edge_attention(slot) + u_mul_e sum + copy_e sum (the r02 path)
and the forward + backward ms of the fused and unfused paths.
Algorithmic bytes of the fused forward: per edge the gathered feature row
(4F), its column id (4) and the source's H attention logits (4H), plus the
stored attention (4H, +4H with dropout) when kept; per row the output row,
its H normalisers and H logits, and its indptr entry (4F + 8H + 8).

  python tools/gat_bench.py [--iters 10]
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
# launches), its Infinity-Cache random-row rate otherwise (every table here
# fits the 256 MiB cache)
L2_PEAK_GBS = 18800.0
IC_PEAK_GBS = 8600.0


def timed(fn, iters):
    """(kernel ms per call, launches per call)."""
    fn()
    torch.cuda.synchronize()
    kernel.timing_enable(True)
    for _ in range(iters):
        fn()
    ms, cnt = kernel.timing_read()
    kernel.timing_enable(False)
    return ms / iters, cnt // iters


def wall(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def bench_graph(name, adj, n, E, H, D, iters):
    dev = torch.device("cuda", 0)
    F = H * D
    ft = (torch.rand(n, H, D, device=dev) * 2 - 1).requires_grad_(True)
    el = (torch.rand(n, H, device=dev) - 0.5).requires_grad_(True)
    er = (torch.rand(n, H, device=dev) - 0.5).requires_grad_(True)
    res = {"graph": name, "nodes": n, "edges": E, "heads": H, "head_dim": D}

    def fused_ng():
        with torch.no_grad():
            kernel.gat_aggregate(adj, ft, el, er)

    def fused_g():
        kernel.gat_aggregate(adj, ft, el, er)

    def fused_drop():
        kernel.gat_aggregate(adj, ft, el, er, attn_drop=0.6)

    def unfused():
        a = kernel.edge_attention(adj, el, er, E, edge_order="slot").unsqueeze(-1)
        kernel.gspmm(adj, "u_mul_e", "sum", ft, a, edge_order="slot")
        kernel.gspmm(adj, "copy_e", "sum", None, a, edge_order="slot")

    def one_launch(fn):
        def run():
            old = kernel.set_blocked("off")
            try:
                fn()
            finally:
                kernel.set_blocked(old)
        return run

    def variant(v, fn):
        def run():
            kernel.set_gat_variant(v)
            try:
                fn()
            finally:
                kernel.set_gat_variant(0)
        return run

    for key, fn, stored in (("fused", fused_ng, 0), ("fused+a", fused_g, 4 * H),
                            ("fused+drop", fused_drop, 8 * H),
                            ("fused_one_launch", one_launch(fused_ng), 0),
                            ("fused+drop_one_launch", one_launch(fused_drop), 8 * H),
                            ("per_lane_kernel", variant(1, fused_ng), 0),
                            ("lds_kernel", variant(2, fused_ng), 0),
                            ("per_lane_kernel+drop", variant(1, fused_drop), 8 * H),
                            ("lds_kernel+drop", variant(2, fused_drop), 8 * H),
                            ("unfused", unfused, None)):
        t, launches = timed(fn, iters)
        entry = {"kernel_ms": round(t, 3), "launches": launches}
        if stored is not None:
            b = E * (4 * F + 4 + 4 * H + stored) + n * (4 * F + 8 * H + 8)
            peak = L2_PEAK_GBS if launches > 1 else IC_PEAK_GBS
            entry.update({"algorithmic_GBs": round(b / (t * 1e-3) / 1e9, 1), "peak_GBs": peak,
                          "frac": round(b / (t * 1e-3) / 1e9 / peak, 3)})
        res[key] = entry

    gout = torch.rand(n, H, D, device=dev)
    gz = torch.rand(n, H, 1, device=dev)

    def fb_fused():
        fs, z = kernel.gat_aggregate(adj, ft, el, er)
        torch.autograd.backward([fs, z], [gout, gz])

    def fb_unfused():
        a = kernel.edge_attention(adj, el, er, E, edge_order="slot").unsqueeze(-1)
        fs = kernel.gspmm(adj, "u_mul_e", "sum", ft, a, edge_order="slot")
        z = kernel.gspmm(adj, "copy_e", "sum", None, a, edge_order="slot")
        torch.autograd.backward([fs, z], [gout, gz])

    res["fwd_bwd_wall_ms"] = {"fused": round(wall(fb_fused, iters), 3),
                              "fused_one_launch": round(wall(one_launch(fb_fused), iters), 3),
                              "unfused": round(wall(fb_unfused, iters), 3)}
    return res


def fwd_bwd_only(iters):
    """Reddit-shaped 8 x 16 forward + backward of the fused path only (for a
    rocprofv3 kernel breakdown)."""
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(device=dev)
    E = int(src.numel())
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    ft = (torch.rand(n, 8, 16, device=dev) * 2 - 1).requires_grad_(True)
    el = (torch.rand(n, 8, device=dev) - 0.5).requires_grad_(True)
    er = (torch.rand(n, 8, device=dev) - 0.5).requires_grad_(True)
    gout = torch.rand(n, 8, 16, device=dev)
    gz = torch.rand(n, 8, 1, device=dev)

    def fb():
        fs, z = kernel.gat_aggregate(adj, ft, el, er)
        torch.autograd.backward([fs, z], [gout, gz])
    print(json.dumps({"edges": E, "fwd_bwd_wall_ms": round(wall(fb, iters), 3)}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--fwd-bwd-only", action="store_true")
    args = ap.parse_args()
    if args.fwd_bwd_only:
        return fwd_bwd_only(args.iters)
    dev = torch.device("cuda", 0)
    out = []
    src, dst, n = data.reddit_like(device=dev)
    E = int(src.numel())
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    out.append(bench_graph("reddit_like", adj, n, E, 8, 16, args.iters))
    del adj
    torch.cuda.empty_cache()
    src, dst, n = data.chung_lu(19717, 88651, 10.0, seed=0, device=dev)
    E = int(src.numel())
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    out.append(bench_graph("pubmed_shape", adj, n, E, 8, 8, args.iters))
    out.append(bench_graph("pubmed_shape", adj, n, E, 8, 3, args.iters))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
