"""Time the fused node-row cross-entropy (csrc/node_loss.hip) at configs[3]'s
shape: 67M rows x 41 classes (RMAT-26 GraphSAGE output layer), forward and
backward, with hipEvents around each pass on the current stream.

  python tools/loss_bench.py [--rows N] [--classes C] [--reps R]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dgl-1_amd"))

import torch  # noqa: E402

from dgl.nn.pytorch import weighted_cross_entropy  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 26)
    ap.add_argument("--classes", type=int, default=41)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    n, C = a.rows, a.classes
    gen = torch.Generator(device=dev).manual_seed(0)
    z = (torch.randn(n, C, device=dev, generator=gen) * 3.0).requires_grad_(True)
    y = torch.randint(0, C, (n,), device=dev, generator=gen)
    w = (torch.rand(n, device=dev, generator=gen) < 0.6).float()
    fwd, bwd = [], []
    for i in range(a.reps + 2):
        z.grad = None
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        loss = weighted_cross_entropy(z, y, w)
        e1.record()
        loss.backward()
        e2.record()
        torch.cuda.synchronize()
        if i >= 2:
            fwd.append(e0.elapsed_time(e1))
            bwd.append(e1.elapsed_time(e2))
    fb = n * (4 * C + 12)
    bb = n * (8 * C + 12)
    fm, bm = sorted(fwd)[len(fwd) // 2], sorted(bwd)[len(bwd) // 2]
    print(json.dumps({"rows": n, "classes": C, "fwd_ms": fm, "bwd_ms": bm,
                      "fwd_TBps": fb / fm / 1e9, "bwd_TBps": bb / bm / 1e9,
                      "loss": loss.item()}))


if __name__ == "__main__":
    main()
