"""Wall time of the source-blocked plan's build on the bench graph: the
first update_all-style call (plan built inside) against the next ones, for
the forward CSR and the transposed one.

  python tools/plan_build_time.py
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import data, kernel  # noqa: E402


def wall(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3


def main():
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(device=dev)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    h = torch.rand(n, 128, device=dev)
    res = {}
    for name, csr in (("forward", adj.fwd), ("transposed", adj.bwd)):
        first = wall(lambda: kernel._run_gspmm(csr, kernel.MSG_COPY_U, kernel.RED_SUM, h, None,
                                               0, 128, False))
        rest = [wall(lambda: kernel._run_gspmm(csr, kernel.MSG_COPY_U, kernel.RED_SUM, h,
                                               None, 0, 128, False)) for _ in range(5)]
        res[name] = {"first_call_ms": round(first, 2), "next_calls_ms": round(min(rest), 2),
                     "plan_build_ms": round(first - min(rest), 2)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
