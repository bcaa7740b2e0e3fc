"""The fused GAT forward (8 heads x 16, Reddit-shaped, source-blocked) with
its waves per SIMD forced (dglhip_set_gat_fwd_waves): 81 VGPRs give 5 waves,
one register over 6; forcing 6 spills one register, forcing 5 on the dropout
kernel (109 VGPRs, 4 waves) spills 15. Kernel ms per call interleaved over
rounds, outputs compared bit for bit.

  python tools/r05/gat_fwd_waves_ab.py [--rounds 3] [--iters 10]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import data, kernel  # noqa: E402
from dgl._ffi import LIB, check_call  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    kernel.timing_enable(True)
    for _ in range(iters):
        fn()
    ms, _ = kernel.timing_read()
    kernel.timing_enable(False)
    return ms / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(device=dev)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    H, D = 8, 16
    g = torch.Generator(device=dev).manual_seed(3)
    ft = torch.rand(n, H, D, device=dev, generator=g) * 2 - 1
    el = torch.rand(n, H, device=dev, generator=g) - 0.5
    er = torch.rand(n, H, device=dev, generator=g) - 0.5
    cases = {
        "plain": ((0, 6), lambda: kernel.gat_aggregate(adj, ft, el, er)),
        "drop": ((0, 5, 6), lambda: kernel.gat_aggregate(adj, ft, el, er, attn_drop=0.6,
                                                         seed=1234)),
    }
    res = {"graph": "reddit_like", "heads": H, "head_dim": D, "bits_equal": {}, "rounds": []}
    with torch.no_grad():
        for cname, (waves, fn) in cases.items():
            outs = []
            for w in waves:
                check_call(LIB.dglhip_set_gat_fwd_waves(w))
                outs.append([t.detach().clone() for t in fn()])
            check_call(LIB.dglhip_set_gat_fwd_waves(0))
            res["bits_equal"][cname] = all(
                all(torch.equal(a, b) for a, b in zip(outs[0], o)) for o in outs[1:])
        for _ in range(args.rounds):
            row = {}
            for cname, (waves, fn) in cases.items():
                for w in waves:
                    check_call(LIB.dglhip_set_gat_fwd_waves(w))
                    row["%s_w%d_ms" % (cname, w)] = timed(fn, args.iters)
                check_call(LIB.dglhip_set_gat_fwd_waves(0))
            res["rounds"].append(row)
            print(json.dumps(row), flush=True)
    print(json.dumps(res["bits_equal"]))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
