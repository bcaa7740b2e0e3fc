"""Node-Linear kernels (csrc/node_linear.hip) against torch's GEMMs at the
shapes of GraphSAGE's layers on RMAT-26 (67.1M rows), per launch shape.

  python tools/node_linear_bench.py [--rows 67108864] > profiles/.../node_linear.json
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dgl-1_amd"))
from dgl import _ffi  # noqa: E402
from dgl.nn.pytorch import linear as L  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 26)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, k = args.rows, 128
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    x = torch.randn(n, k, device=dev, generator=g)
    agg = torch.randn(n, k, device=dev, generator=g)
    ws, wn = torch.randn(128, k, device=dev) * 0.1, torch.randn(128, k, device=dev) * 0.1
    b = torch.randn(128, device=dev)
    w41s, w41n = torch.randn(41, k, device=dev) * 0.1, torch.randn(41, k, device=dev) * 0.1
    dy = torch.randn(n, 41, device=dev, generator=g)
    dpre = torch.randn(n, 41, device=dev, generator=g)
    res = {"rows": n}

    def torch_cat():
        o = torch.addmm(b, x, ws.t())
        o.addmm_(agg, wn.t())

    def torch_pre():
        torch.mm(x, w41n.t())
        torch.addmm(b[:41], x, w41s.t())

    def torch_dgrad():
        d = dy.mm(w41s)
        d.addmm_(dpre, w41n)

    res["torch"] = {"cat_128x(128+128)": timed(torch_cat), "pre_2x41": timed(torch_pre),
                    "dgrad_41+41": timed(torch_dgrad)}
    for threads, per_cu in ((0, 0), (256, 0), (512, 1), (512, 2), (256, 2), (256, 3), (256, 4)):
        _ffi.check_call(_ffi.LIB.dglhip_set_node_linear_variant(threads, per_cu))
        res["mfma_%d_%d" % (threads, per_cu)] = {
            "cat_128x(128+128)": timed(lambda: L._node_linear_cat(x, ws, agg, wn, b)),
            "pre_2x41": timed(lambda: L._node_linear2(x, w41n, 48, w41s, b[:41])),
            "dgrad_41+41": timed(lambda: L._node_dgrad2(k, dy, w41s, dpre, w41n))}
        print(json.dumps(res), file=sys.stderr, flush=True)
    _ffi.check_call(_ffi.LIB.dglhip_set_node_linear_variant(0, 0))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
