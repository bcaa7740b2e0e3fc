"""Generate golden vectors for the g-SpMM path with the reference's own arithmetic.

The reference computes builtin message passing as torch.sparse.mm on an
uncoalesced COO built from its edge list (python/dgl/graph_index.py:574-583,
src/graph/graph.cc:509-524, python/dgl/backend/pytorch/tensor.py:45-51,145-146;
src_mul_edge: python/dgl/runtime/ir/executor.py:535-566; send_and_recv /
pull: python/dgl/runtime/spmv.py:154-227). Running the reference package
itself is denied in this environment, so this script rebuilds
exactly those COO inputs and calls the third-party product (torch 2.10.0,
importable here) directly. max / mean are the reference's degree-bucketing
UDF reduce (torch.max / torch.mean over each node's mailbox in edge order,
degree_bucketing.py:13-190), reproduced with torch ops per node.

Run:  python tests/golden/make_golden.py   (writes tests/golden/*.npz)
"""
from __future__ import absolute_import

import os

import numpy as np
import torch

OUT = os.path.dirname(os.path.abspath(__file__))


def coo_spmm(n_rows, n_cols, row, col, H, val=None, grad=None):
    """torch.sparse.mm on the reference's uncoalesced COO (+ optional backward)."""
    idx = torch.stack([torch.as_tensor(row), torch.as_tensor(col)])
    H = torch.as_tensor(H).clone().requires_grad_(grad is not None)
    if val is None:
        vals = torch.ones(len(row))
    else:
        vals = torch.as_tensor(val).clone().requires_grad_(grad is not None)
    A = torch.sparse_coo_tensor(idx, vals, (n_rows, n_cols))
    out = torch.sparse.mm(A, H)
    res = {"out": out.detach().numpy()}
    if grad is not None:
        out.backward(torch.as_tensor(grad))
        res["grad_h"] = H.grad.numpy()
        if val is not None:
            res["grad_w"] = vals.grad.to_dense().numpy() if vals.grad.is_sparse \
                else vals.grad.numpy()
    return res


def mailbox_reduce(n_rows, dst, msgs, op):
    """Degree-bucketing style reduce with torch ops, zero for empty mailboxes."""
    msgs = torch.as_tensor(msgs)
    out = torch.zeros((n_rows,) + tuple(msgs.shape[1:]))
    dst = torch.as_tensor(dst)
    for v in range(n_rows):
        ids = (dst == v).nonzero(as_tuple=True)[0]
        if len(ids) == 0:
            continue
        box = msgs[ids].unsqueeze(0)
        out[v] = torch.max(box, 1)[0][0] if op == "max" else torch.mean(box, 1)[0]
    return out.numpy()


def spec10():
    """tests/compute/test_specialization.py:9-21 fixture: 0->1..8, 1..8->9, 9->0."""
    src = [0] * 8 + list(range(1, 9)) + [9]
    dst = list(range(1, 9)) + [9] * 8 + [0]
    return np.array(src, np.int64), np.array(dst, np.int64), 10


def random_graph(rng, n, m, self_loops=False, allow_dup=False):
    if allow_dup:
        src = rng.integers(0, n, m)
        dst = rng.integers(0, n, m)
    else:
        keys = rng.choice(n * n, size=m, replace=False)
        src, dst = keys // n, keys % n
    if self_loops:
        src = np.concatenate([src, np.arange(n)])
        dst = np.concatenate([dst, np.arange(n)])
    return src.astype(np.int64), dst.astype(np.int64)


def reddit_rows_case():
    import portable as P
    src, dst, H, W, G = P.reddit_rows()
    n = P.N
    r_copy = coo_spmm(n, n, dst, src, H, None, G)
    r_mul = coo_spmm(n, n, dst, src, H, W, G)
    deg = np.bincount(dst, minlength=n)
    rng = np.random.default_rng(5)
    top = np.argsort(-deg, kind="stable")[:16]
    rows = np.unique(np.concatenate([top, rng.choice(n, 112, replace=False),
                                     np.nonzero(deg == 0)[0][:2]])).astype(np.int64)
    case = dict(n=n, e=len(src), f=H.shape[1], rows=rows, max_in_degree=int(deg.max()),
                torch_version=np.array(torch.__version__))
    for k, a in (("src", src), ("dst", dst), ("h", H), ("w", W), ("g", G)):
        case["sha_" + k] = np.array(P.digest(a))
    for k, a in (("copy_out", r_copy["out"]), ("copy_grad_h", r_copy["grad_h"]),
                 ("mul_out", r_mul["out"]), ("mul_grad_h", r_mul["grad_h"])):
        case["sha_" + k] = np.array(P.digest(a))
        case[k + "_rows"] = a[rows]
    return case


def main():
    rng = np.random.default_rng(20181205)
    cases = {}

    # 1. specialization fixture graph, D=5 features, scalar edge weights
    src, dst, n = spec10()
    h = rng.standard_normal((n, 5)).astype(np.float32)
    w = rng.standard_normal(len(src)).astype(np.float32)
    g = rng.standard_normal((n, 5)).astype(np.float32)
    r_copy = coo_spmm(n, n, dst, src, h, None, g)
    r_mul = coo_spmm(n, n, dst, src, h, w, g)
    cases["spec10"] = dict(src=src, dst=dst, n=n, h=h, w=w, g=g, copy_out=r_copy["out"],
                           copy_grad_h=r_copy["grad_h"], mul_out=r_mul["out"],
                           mul_grad_h=r_mul["grad_h"], mul_grad_w=r_mul["grad_w"])

    # 2. Cora-shaped: 2708 nodes, 10556 edges + self loops, F=16
    n = 2708
    src, dst = random_graph(rng, n, 10556, self_loops=True)
    h = rng.uniform(-1, 1, (n, 16)).astype(np.float32)
    g = rng.standard_normal((n, 16)).astype(np.float32)
    r = coo_spmm(n, n, dst, src, h, None, g)
    cases["cora"] = dict(src=src, dst=dst, n=n, h=h, g=g, copy_out=r["out"],
                         copy_grad_h=r["grad_h"])

    # 3. multigraph with duplicate edges and scalar weights, F=7
    n = 50
    src, dst = random_graph(rng, n, 2000, allow_dup=True)
    h = rng.standard_normal((n, 7)).astype(np.float32)
    w = rng.standard_normal(len(src)).astype(np.float32)
    g = rng.standard_normal((n, 7)).astype(np.float32)
    r_copy = coo_spmm(n, n, dst, src, h, None, g)
    r_mul = coo_spmm(n, n, dst, src, h, w, g)
    msgs = h[src]
    cases["multi"] = dict(src=src, dst=dst, n=n, h=h, w=w, g=g, copy_out=r_copy["out"],
                          copy_grad_h=r_copy["grad_h"], mul_out=r_mul["out"],
                          mul_grad_h=r_mul["grad_h"], mul_grad_w=r_mul["grad_w"],
                          max_out=mailbox_reduce(n, dst, msgs, "max"),
                          mean_out=mailbox_reduce(n, dst, msgs, "mean"))

    # 4. zero-in-degree nodes (test_basics.py:442-477 semantics), F=3
    n = 20
    src = np.array([0, 1, 2, 3, 0, 5, 7, 7], np.int64)
    dst = np.array([4, 4, 4, 6, 6, 8, 9, 9], np.int64)
    h = rng.standard_normal((n, 3)).astype(np.float32)
    r = coo_spmm(n, n, dst, src, h)
    cases["zerodeg"] = dict(src=src, dst=dst, n=n, h=h, copy_out=r["out"],
                            max_out=mailbox_reduce(n, dst, h[src], "max"))

    # 5. send_and_recv on a subset: rectangular (|recv|, N) COO in given edge order
    c = cases["cora"]
    n = int(c["n"])
    sel = rng.choice(len(c["src"]), size=3000, replace=False)
    u, v = c["src"][sel], c["dst"][sel]
    recv = np.unique(v)
    rows = np.searchsorted(recv, v)
    r = coo_spmm(len(recv), n, rows, u, c["h"])
    cases["snr"] = dict(sel=sel.astype(np.int64), recv=recv.astype(np.int64), out=r["out"])

    # 6. 3-D node features (test_specialization.py:517-569): 100 nodes, density 0.1
    n = 100
    src, dst = random_graph(rng, n, 1000)
    h = rng.standard_normal((n, 5, 5)).astype(np.float32)
    r = coo_spmm(n, n, dst, src, h.reshape(n, 25))
    cases["feat3d"] = dict(src=src, dst=dst, n=n, h=h, copy_out=r["out"].reshape(n, 5, 5))

    # 7. Reddit row lengths (tests/golden/portable.py): 1.5M edges, F = 128,
    #    rows of 13k-54k in-edges, heavy duplicates. The inputs are regenerated
    #    from a portable integer hash; the fixture keeps their digests, the
    #    digests of the whole outputs and the outputs of a row sample.
    cases["reddit_rows"] = reddit_rows_case()

    for name, arrays in cases.items():
        np.savez_compressed(os.path.join(OUT, name + ".npz"),
                            **{k: np.asarray(val) for k, val in arrays.items()})
        print("wrote", name)


if __name__ == "__main__":
    main()
