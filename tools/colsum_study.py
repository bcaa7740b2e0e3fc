"""Column sums of a tall (n, F) fp32 matrix (the bias gradient of a
per-node Linear) and its split-K weight gradient: which formulation runs
fastest on the MI355X. One process, interleaved rounds, hipEvent timing.

  python tools/colsum_study.py [--rows 16777216] [--feat 128]
"""
import argparse
import json

import torch


def timeit(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 24)
    ap.add_argument("--feat", type=int, default=128)
    args = ap.parse_args()
    n, F = args.rows, args.feat
    dy = torch.randn(n, F, device="cuda")
    x = torch.randn(n, F, device="cuda")
    ones = torch.ones(n, device="cuda")
    C = 256
    k = n // C
    cases = {
        "sum0": lambda: dy.sum(0),
        "mv_t": lambda: torch.mv(dy.t(), ones),
        "ones_mm": lambda: ones.unsqueeze(0).matmul(dy),
        "view_sum1_sum0": lambda: dy.view(C, k, F).sum(1).sum(0),
        "bmm_ones": lambda: torch.bmm(dy.view(C, k, F).transpose(1, 2),
                                      ones.view(C, k, 1)).sum(0),
        "wgrad_mm": lambda: dy.t().matmul(x),
        "wgrad_splitk_bmm": lambda: torch.bmm(dy.view(C, k, F).transpose(1, 2),
                                              x.view(C, k, F)).sum(0),
    }
    ref = dy.double().sum(0)
    res = {}
    for name, fn in cases.items():
        out = fn().reshape(-1)
        if out.numel() == F:
            err = float((out.double() - ref).abs().max())
        else:
            err = None
        res[name] = {"ms": round(timeit(fn), 3), "max_abs_err_vs_f64": err}
    print(json.dumps({"rows": n, "feat": F, "chunks": C, "cases": res}, indent=1))


if __name__ == "__main__":
    main()
