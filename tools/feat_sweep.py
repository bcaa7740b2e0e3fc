"""g-SpMM copy_u+sum across feature widths on the Reddit-shaped bench graph:
kernel time of the automatic choice and of each applicable (vec, lanes, unroll)
variant, interleaved in rounds in one process (cdna_hip_programming.md §5.4
rule 24), every variant checked bit-identical to the automatic one.

Two byte counts per width:
  algorithmic : E * (4F + 4) + N * (4F + 8)   
  line bytes  : the 128-B cache lines a row gather really touches -- a row of
                4F bytes at offset 4F*u straddles ceil-or-one-more lines when
                4F is not a multiple of 128 (F = 41: 164 B -> 2.3 lines on average)

  python tools/feat_sweep.py [--feats 16,32,41,64,100,128,256,602] [--rounds 3]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import _ffi, data, kernel  # noqa: E402

PEAK_GBS = 8000.0
VARIANTS = [(0, 0, 0, 0), (1, 64, 8, 0), (1, 64, 16, 0), (1, 64, 32, 0), (2, 64, 16, 0),
            (2, 64, 32, 0), (2, 32, 16, 0), (2, 32, 32, 0), (1, 32, 32, 0), (4, 32, 16, 0)]


def applicable(v, F):
    vec, grp = v[0], v[1]
    if vec == 0:
        return True
    if F % vec:
        return False
    w = vec * grp
    if w < F and F % w:
        return False
    # no more than one idle half-wave: a variant spanning 2x the row is waste
    return w < 2 * F or (w == 64 and F >= 16)


def mean_lines(F):
    """Average 128-B lines touched by a 4F-byte row at byte offset 4F*u."""
    rb = 4 * F
    tot = 0
    for u in range(128):  # offsets repeat with period 128 / gcd
        off = (rb * u) % 128
        tot += (off + rb + 127) // 128
    return tot / 128.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--feats", default="16,24,32,41,50,64,100,128,256,602")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(device=dev)
    E = int(src.numel())
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    out = []
    for F in [int(x) for x in args.feats.split(",")]:
        h = torch.rand(n, F, device=dev) * 2 - 1
        ref = kernel.gspmm(adj, "copy_u", "sum", h)
        vs = [v for v in VARIANTS if applicable(v, F)]
        times = {v: [] for v in vs}
        for _ in range(args.rounds):
            for v in vs:
                _ffi.check_call(_ffi.LIB.dglhip_set_spmm_variant(*v))
                o = kernel.gspmm(adj, "copy_u", "sum", h)
                assert torch.equal(o, ref), (F, v)
                torch.cuda.synchronize()
                kernel.timing_enable(True)
                for _ in range(args.iters):
                    kernel.gspmm(adj, "copy_u", "sum", h)
                ms, _ = kernel.timing_read()
                kernel.timing_enable(False)
                times[v].append(ms / args.iters)
        _ffi.check_call(_ffi.LIB.dglhip_set_spmm_variant(0, 0, 0, 0))
        # padded-stride gathers (kernel.padded_width): the automatic choice with
        # the source rows gathered from a padded copy vs in place; kernel time
        # from the hooks, call time (copy included) from events around the call
        pad = {}
        for _ in range(args.rounds):
            for pol in ("auto", "off"):
                old = kernel.set_pad_rows(pol)
                o = kernel.gspmm(adj, "copy_u", "sum", h)
                assert torch.equal(o, ref), (F, pol)
                torch.cuda.synchronize()
                kernel.timing_enable(True)
                t0 = torch.cuda.Event(enable_timing=True)
                t1 = torch.cuda.Event(enable_timing=True)
                t0.record()
                for _ in range(args.iters):
                    kernel.gspmm(adj, "copy_u", "sum", h)
                t1.record()
                torch.cuda.synchronize()
                ms, _ = kernel.timing_read()
                kernel.timing_enable(False)
                kernel.set_pad_rows(old)
                pad.setdefault(pol, []).append((ms / args.iters, t0.elapsed_time(t1) / args.iters))
        alg = E * (4 * F + 4) + n * (4 * F + 8)
        lines = E * (128 * mean_lines(F) + 4) + n * (4 * F + 8)
        row = {"feat": F, "algorithmic_GB": round(alg / 1e9, 2),
               "line_GB": round(lines / 1e9, 2), "variants": {}}
        for v, t in times.items():
            med = sorted(t)[len(t) // 2]
            row["variants"]["%d,%d,%d,%d" % v] = {
                "ms": round(med, 3),
                "alg_GBs": round(alg / (med * 1e-3) / 1e9, 1),
                "frac": round(alg / (med * 1e-3) / 1e9 / PEAK_GBS, 3),
                "line_GBs": round(lines / (med * 1e-3) / 1e9, 1)}
        ld = kernel.padded_width(F)
        for pol, t in pad.items():
            t.sort()
            km, cm = t[len(t) // 2]
            row["padded" if pol == "auto" else "unpadded"] = {
                "stride": ld if pol == "auto" else F, "kernel_ms": round(km, 3),
                "call_ms": round(cm, 3), "lines_per_row": round(
                    kernel._lines_per_row(F, ld if pol == "auto" else F), 3),
                "alg_GBs": round(alg / (km * 1e-3) / 1e9, 1)}
        out.append(row)
        print("F=%d" % F, {k: x["ms"] for k, x in row["variants"].items()},
              file=sys.stderr, flush=True)
        del h, ref
    print(json.dumps({"graph": "reddit_like", "nodes": n, "edges": E, "widths": out},
                     indent=1))


if __name__ == "__main__":
    main()
