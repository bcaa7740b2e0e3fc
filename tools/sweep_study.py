"""Study: the source-swept g-SpMM schedule (kernel.set_sweep,
dglhip_gspmm_sweep_device) against the one-launch and source-blocked
schedules on the Reddit-shaped graph (copy_u + sum, F = 128): kernel time per
call over slice sizes, rows per wave and the heavy-row threshold; every
variant's output compared with the one-launch kernel's bits.

  python tools/sweep_study.py [--slices-mib 1 2 3 4 6] [--rows 4 8 16] [--iters 10]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import data, kernel  # noqa: E402


def timed(fn, iters):
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
    ap.add_argument("--slices-mib", type=float, nargs="+", default=[1, 2, 3, 4, 6])
    ap.add_argument("--rows", type=int, nargs="+", default=[4, 8, 16])
    ap.add_argument("--heavy", type=int, nargs="+", default=[1024])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--feat", type=int, default=128)
    ap.add_argument("--scale", type=float, default=1.0, help="source table scale (1 = Reddit)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(device=dev)
    E = int(src.numel())
    F = args.feat
    h = torch.rand(n, F, device=dev) * 2 - 1
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    csr = adj.fwd
    del src, dst
    byts = E * (4 * F + 4) + n * (4 * F + 8)
    res = {"graph": "reddit_like", "nodes": n, "edges": E, "feat": F, "variants": []}

    def run():
        return kernel.gspmm(adj, "copy_u", "sum", h)

    old_b = kernel.set_blocked("off")
    ref = run().clone()
    ref_mean = kernel.gspmm(adj, "copy_u", "mean", h).clone()
    ms, launches = timed(run, args.iters)
    res["one_launch_ms"] = ms
    print(json.dumps({"one_launch_ms": ms}), flush=True)
    kernel.set_blocked(old_b)
    ms, launches = timed(run, args.iters)
    res["blocked_ms"], res["blocked_launches"] = ms, launches
    print(json.dumps({"blocked_ms": ms, "launches": launches}), flush=True)
    for heavy in args.heavy:
        for rows in args.rows:
            for mib in args.slices_mib:
                old = kernel.set_sweep("on", slice_bytes=int(mib * (1 << 20)), rows=rows,
                                       heavy=heavy)
                out = run()
                same = bool(torch.equal(out, ref))
                mean_same = bool(torch.equal(kernel.gspmm(adj, "copy_u", "mean", h), ref_mean))
                acc = ref.clone()
                kernel.gspmm_into(csr, acc, h, accumulate=True)
                acc_ref = ref.clone()
                kernel.set_sweep("off")
                old_b = kernel.set_blocked("off")
                kernel.gspmm_into(csr, acc_ref, h, accumulate=True)
                kernel.set_blocked(old_b)
                kernel.set_sweep("on", slice_bytes=int(mib * (1 << 20)), rows=rows, heavy=heavy)
                acc_same = bool(torch.equal(acc, acc_ref))
                ms, launches = timed(run, args.iters)
                entry = {"slice_MiB": mib, "rows_per_wave": rows, "heavy": heavy,
                         "kernel_ms": ms, "launches": launches,
                         "algorithmic_TBs": byts / (ms * 1e-3) / 1e12,
                         "bits_equal_one_launch": same, "mean_bits_equal": mean_same,
                         "accum_bits_equal": acc_same}
                res["variants"].append(entry)
                print(json.dumps(entry), flush=True)
                kernel.set_sweep(*old)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
