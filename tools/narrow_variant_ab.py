"""GCN's output-layer aggregation (copy_u + sum, F = 41 at its 48-float padded
stride, the headline graph) per kernel variant of the blocked schedule
(dglhip_set_spmm_variant: vec, lanes per row, gathers per batch), interleaved
rounds, each checked bit-identical to the automatic choice; kernel ms from
the library's launch events.

  python tools/narrow_variant_ab.py [--feats 41 64] [--rounds 3]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import _ffi, data, kernel  # noqa: E402

VARIANTS = [(0, 0, 0, 0), (2, 32, 8, 0), (2, 32, 16, 0), (2, 32, 32, 0), (2, 64, 8, 0),
            (2, 64, 32, 0), (1, 64, 16, 0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--feats", type=int, nargs="+", default=[41])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(device=dev)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    res = {}
    for F in a.feats:
        h = torch.rand(n, F, device=dev) * 2 - 1
        ref = kernel.gspmm(adj, "copy_u", "sum", h)
        times = {v: [] for v in VARIANTS}
        bad = set()
        for _ in range(a.rounds):
            for v in VARIANTS:
                if v in bad:
                    continue
                try:
                    _ffi.check_call(_ffi.LIB.dglhip_set_spmm_variant(*v))
                    o = kernel.gspmm(adj, "copy_u", "sum", h)
                except Exception as err:  # noqa: BLE001 - a variant the path rejects
                    bad.add(v)
                    times[v] = str(err)[:120]
                    continue
                assert torch.equal(o, ref), (F, v)
                torch.cuda.synchronize()
                kernel.timing_enable(True)
                for _ in range(a.iters):
                    kernel.gspmm(adj, "copy_u", "sum", h)
                ms, _ = kernel.timing_read()
                kernel.timing_enable(False)
                times[v].append(ms / a.iters)
        _ffi.check_call(_ffi.LIB.dglhip_set_spmm_variant(0, 0, 0, 0))
        res[F] = {",".join(map(str, v)): (min(t) if isinstance(t, list) and t else t)
                  for v, t in times.items()}
        print(F, json.dumps(res[F]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
