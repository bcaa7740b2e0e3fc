"""Variants of the one-pass GAT backward over the transpose
(dglhip_set_gat_bwd_variant), Reddit-shaped graph, 8 heads x 16: forward +
backward wall ms per variant, interleaved over rounds, gradients vs the
default. Variants: the attention gradient's store at its forward slot
(0 plain, 1 non-temporal, 2 skipped: how much the scattered 32-B stores cost;
d_er is then not valid and is left out of the comparison). The first runs
(profiles/r04/gat_bwd/) also had bit 2, since removed: the kernel built for 8
waves per SIMD, then the first form of the kernel.

  python tools/gat_bwd_variants.py [--rounds 3] [--out file.json]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import _ffi, data, kernel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--variants", type=int, nargs="+", default=[0, 1, 2])
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
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
        r = (ft.grad, el.grad, er.grad)
        ft.grad = el.grad = er.grad = None
        return r

    def wall():
        fb()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(args.iters):
            fb()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / args.iters

    def bwd_kernel_ms():
        fb()
        torch.cuda.synchronize()
        kernel.timing_enable(True)
        fb()
        ms, cnt = kernel.timing_read()
        kernel.timing_enable(False)
        return ms, cnt

    ref = fb()
    res, same, kms = {}, {}, {}
    try:
        for _ in range(args.rounds):
            for v in args.variants:
                _ffi.check_call(_ffi.LIB.dglhip_set_gat_bwd_variant(v))
                got = fb()
                pairs = list(zip(got, ref))
                if v == 2:
                    pairs = pairs[:2]  # d_er reads the unwritten gradient buffer
                same[v] = all(bool(torch.equal(a, b)) for a, b in pairs)
                res.setdefault(v, []).append(wall())
                kms.setdefault(v, []).append(bwd_kernel_ms()[0])
    finally:
        _ffi.check_call(_ffi.LIB.dglhip_set_gat_bwd_variant(0))
    line = json.dumps({"fwd_bwd_ms": res, "min": {k: min(x) for k, x in res.items()},
                       "library_kernel_ms_fwd_bwd": {k: min(x) for k, x in kms.items()},
                       "bit_identical": same,
                       "variants": {"0": "plain g store", "1": "non-temporal g store",
                                    "2": "no g store (timing only)"}})
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
