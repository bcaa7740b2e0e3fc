"""A/B of the headline's row gathers under the blocked schedule
(dglhip_set_gather_mode): 0 = global loads with a 64-bit address per gather
(70 VGPRs, 7 waves per SIMD), 2 = per-row buffer descriptors (the row base in
SGPRs, one shared 32-bit lane offset: 42 VGPRs, 8 waves). Per mode the mean
GPU span of a copy_u + sum call on the Reddit-shaped graph (events around the
calls on the launch stream), interleaved over rounds, output bits vs mode 0;
also at 5 and 8 MiB blocks (more waves may move the slice optimum).

  python tools/gather_mode_ab.py [--calls 20 --rounds 3] [--out file.json]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import data, kernel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--mib", type=float, nargs="+", default=[5, 6, 8])
    ap.add_argument("--modes", type=int, nargs="+", default=[0, 2])
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(scale=1, seed=0, device=dev)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    h = torch.rand(n, 128, device=dev) * 2 - 1
    ref = kernel.gspmm(adj, "copy_u", "sum", h)
    old_bytes = kernel.schedule_policy()["block_bytes"]
    res, same = {}, {}
    try:
        for _ in range(args.rounds):
            for mib in args.mib:
                kernel.set_schedule_policy(block_bytes=int(mib * (1 << 20)))
                for mode in args.modes:
                    kernel.check_call(kernel.LIB.dglhip_set_gather_mode(mode))
                    key = "%g MiB / mode %d" % (mib, mode)
                    out = kernel.gspmm(adj, "copy_u", "sum", h)
                    same[key] = bool(torch.equal(out, ref))
                    torch.cuda.synchronize()
                    s = torch.cuda.Event(enable_timing=True)
                    e = torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(args.calls):
                        kernel.gspmm(adj, "copy_u", "sum", h)
                    e.record()
                    e.synchronize()
                    res.setdefault(key, []).append(s.elapsed_time(e) / args.calls)
    finally:
        kernel.set_schedule_policy(block_bytes=old_bytes)
        kernel.check_call(kernel.LIB.dglhip_set_gather_mode(2))  # the default
    line = json.dumps({"ms_per_call": res, "min": {k: min(v) for k, v in res.items()},
                       "bit_identical": same})
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
