"""How many slots a "carry" of small (row, block) items would move on the
headline graph (r03 verdict, "Next" 5): the source-blocked plan of the
Reddit-shaped graph (bench.py's N = 1 step, the plan's row ranges at the
plan's block count), its items' slot counts, and what carrying a row's items
of fewer than T slots into its next block's item would merge. Host only.

  python tools/carry_study.py [--out profiles/r04/carry_study.json]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import data, kernel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    src, dst, n = data.reddit_like(scale=1, seed=0, device="cpu")
    csr = kernel.build_csr(n, n, dst, src, kernel.ORDER_EID, "cpu")
    del src, dst
    # the plan's row ranges per block: counts = cuts[b + 1] - cuts[b]
    cuts = kernel._block_cuts(csr, 512, kernel.schedule_policy()["block_bytes"])
    B = len(cuts) - 1
    sfx = None
    if cuts[-1].equal(csr.indptr[1:]) and B > 1 and not cuts[-2].equal(csr.indptr[1:]):
        sfx = cuts[-1] - cuts[-2]  # a suffix range (rows whose blocks decrease)
        B -= 1
    c = torch.stack([cuts[b + 1] - cuts[b] for b in range(B)], 1).numpy()
    nz = c[c > 0]
    res = {"rows": n, "edges": csr.nnz, "blocks": B, "items": int(nz.size),
           "slots_per_item_mean": float(nz.mean()), "slots_per_item_min": int(nz.min()),
           "suffix_slots": 0 if sfx is None else int(sfx.sum()), "below": {}, "carry": {}}
    for T in (2, 4, 8, 12, 16, 24, 32):
        small = nz[nz < T]
        res["below"][T] = {"items": int(small.size), "slots": int(small.sum())}
    for T in (4, 8, 16):
        items = carried = 0
        for row in c:
            acc = 0
            nzb = np.nonzero(row)[0]
            for i, b in enumerate(nzb):
                carried += acc
                acc += row[b]
                if acc >= T or i == len(nzb) - 1:
                    items += 1
                    acc = 0
        res["carry"][T] = {"items": items, "items_removed": int(nz.size) - items,
                           "carried_slots": int(carried)}
    line = json.dumps(res, indent=1)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
