"""Per-segment study of the source-blocked schedule on an emulated rank of
the weak-scaled graph (bench.py --emulate-world): each pipelined segment
(own rows, then each halo chunk) timed alone, one launch vs blocked, with its
span, slots per row and block count.

  python tools/segment_block_study.py [--worlds 2 4 8] [--chunks 4]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import data, kernel  # noqa: E402
from dgl.distributed import PartitionedGraph, balanced_bounds  # noqa: E402


def timed(fn, iters=10):
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
    ap.add_argument("--worlds", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--chunks", type=int, default=4)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = []
    for W in args.worlds:
        src, dst, n = data.reddit_like(scale=W, seed=0, device=dev)
        bounds = balanced_bounds(torch.bincount(dst, minlength=n), W)
        lo, hi = int(bounds[0]), int(bounds[1])
        sel = (dst >= lo) & (dst < hi)
        pg = PartitionedGraph(n, src[sel], dst[sel], bounds, dev, pipeline_chunks=args.chunks,
                              rank=0, world=W)
        del src, dst, sel
        h_local = torch.rand(hi - lo, 128, device=dev) * 2 - 1
        pg.update_all(h_local)
        halo = pg.halo if not isinstance(pg.halo, list) else None
        for i, csr in enumerate(pg.seg_csrs):
            feat = h_local if i == 0 else halo
            o = torch.empty(csr.num_rows, 128, device=dev)
            lo_c, hi_c = kernel._column_span(csr)
            res = {"world": W, "segment": "own" if i == 0 else "chunk %d" % (i - 1),
                   "span_MB": (hi_c - lo_c) * 512 / 1e6, "nnz": csr.nnz,
                   "slots_per_row": csr.nnz / max(csr.num_nonempty, 1)}
            for pol in ("off", "auto"):
                old = kernel.set_blocked(pol)
                ms, cnt = timed(lambda: kernel.gspmm_into(csr, o, feat, accumulate=i > 0))
                kernel.set_blocked(old)
                res[pol] = {"ms": round(ms, 3), "launches": cnt}
            out.append(res)
            print(json.dumps(res), flush=True)
        del pg, h_local, halo
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
