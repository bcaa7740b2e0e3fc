"""Synthetic graph generators (offline stand-ins for the reference's datasets).

The reference downloads Cora / Pubmed / Reddit / FB15k from S3
(python/dgl/data/utils.py:18-27, data/__init__.py:15-25); nothing can be
fetched here, so benchmarks use seeded synthetic graphs of the same shape
(SURVEY.md §8d):

* ``reddit_like``: Chung-Lu power-law graph with Reddit's node count,
  directed edge count (114,615,892, both directions of each undirected pair),
  mean degree ~492 and max/mean degree ratio ~44 (Reddit's max degree is
  21,657), symmetric, no duplicates, node ids permuted; GCN self-loops added
  (examples/pytorch/gcn/gcn_spmv.py:136).
* ``rmat``: Graph500 R-MAT edges (a, b, c, d) = (0.57, 0.19, 0.19, 0.05),
  directed, duplicates kept (multigraph), ids permuted.

Generation runs on whatever device is given (torch RNG seeded per call), so a
1-GPU box builds the 115M-edge graph in seconds. Edge ids are assigned in
(src, dst) order.

On-disk formats, read with loaders that execute nothing
from the file (numpy / scipy with pickling disabled, plain text):

* ``CoraTextDataset``: the pygcn text release (``cora/cora.content``,
  ``cora/cora.cites``) as the reference's CoraDataset._load parses it
  (python/dgl/data/citation_graph.py:349-380).
* ``RedditDataset``: DGL's Reddit release (``reddit/reddit_graph.npz``, a
  scipy sparse matrix, and ``reddit/reddit_data.npz`` with feature / label /
  node_types).
* ``load_edge_list``: a plain edge list (text "src dst" lines, an (E, 2)
  ``.npy`` or an ``.npz`` with src / dst arrays).

``load_data(name, root=...)`` (or ``$DGL_DATA_DIR``) uses these files when
they are present and falls back to the synthetic stand-ins otherwise.
"""
from __future__ import absolute_import

import torch

import os

import numpy as np

__all__ = ["reddit_like", "chung_lu", "rmat", "REDDIT_NODES", "REDDIT_EDGES", "load_data",
           "load_edge_list", "CoraTextDataset", "RedditDataset", "SyntheticNodeDataset"]

REDDIT_NODES = 232965
REDDIT_EDGES = 114615892
REDDIT_MAX_OVER_MEAN = 21657.0 / (REDDIT_EDGES / REDDIT_NODES)


def _powerlaw_alpha(n, ratio):
    """alpha with w_i = (i+1)^-alpha and max(w)/mean(w) == ratio (bisection)."""
    lo, hi = 0.0, 1.5
    idx = torch.arange(1, n + 1, dtype=torch.float64)
    for _ in range(60):
        a = 0.5 * (lo + hi)
        r = 1.0 / (idx.pow(-a).mean().item())
        if r < ratio:
            lo = a
        else:
            hi = a
    return 0.5 * (lo + hi)


def reddit_like(scale=1, seed=0, device="cpu", self_loops=True):
    """(src, dst, num_nodes) int64 tensors on ``device``.

    ``scale`` multiplies nodes and edges (weak-scaling family: scale = number
    of GPUs); scale=1 is the Reddit-shaped graph of BASELINE.json configs[1].
    """
    return chung_lu(int(REDDIT_NODES * scale), int(REDDIT_EDGES * scale), REDDIT_MAX_OVER_MEAN,
                    seed, device, self_loops)


def chung_lu(n, num_edges, max_over_mean, seed=0, device="cpu", self_loops=True):
    """Symmetric power-law graph with ``num_edges`` directed edges (pairs in
    both directions, no duplicates or self-loops) plus optional self-loops."""
    device = torch.device(device)
    target_pairs = num_edges // 2
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    alpha = _powerlaw_alpha(n, max_over_mean)
    w = torch.arange(1, n + 1, device=device, dtype=torch.float64).pow(-alpha)
    perm = torch.randperm(n, generator=gen, device=device)
    weights = torch.empty_like(w)
    weights[perm] = w
    cdf = torch.cumsum(weights, 0)
    cdf = (cdf / cdf[-1]).to(torch.float64)
    keys = torch.empty(0, dtype=torch.int64, device=device)
    need = target_pairs
    for _ in range(8):
        m = int(need * 1.08) + 1024
        a = torch.searchsorted(cdf, torch.rand(m, generator=gen, device=device,
                                               dtype=torch.float64)).clamp_(max=n - 1)
        b = torch.searchsorted(cdf, torch.rand(m, generator=gen, device=device,
                                               dtype=torch.float64)).clamp_(max=n - 1)
        keep = a != b
        lo_, hi_ = torch.minimum(a[keep], b[keep]), torch.maximum(a[keep], b[keep])
        keys = torch.unique(torch.cat([keys, lo_ * n + hi_]))
        del a, b, keep, lo_, hi_
        if keys.numel() >= target_pairs:
            break
        need = target_pairs - keys.numel()
    if keys.numel() > target_pairs:
        pick = torch.randperm(keys.numel(), generator=gen, device=device)[:target_pairs]
        keys = torch.sort(keys[pick])[0]
    u, v = keys // n, keys % n
    del keys
    src = torch.cat([u, v])
    dst = torch.cat([v, u])
    del u, v
    if self_loops:
        ar = torch.arange(n, device=device)
        src = torch.cat([src, ar])
        dst = torch.cat([dst, ar])
    order = torch.argsort(src * n + dst)
    return src[order].contiguous(), dst[order].contiguous(), n


def rmat(scale, edge_factor=16, seed=0, device="cpu", abcd=(0.57, 0.19, 0.19, 0.05),
         chunk=1 << 26):
    """Graph500 R-MAT: (src, dst, num_nodes); 2^scale nodes, edge_factor*2^scale edges."""
    device = torch.device(device)
    n = 1 << scale
    m = edge_factor * n
    a, b, c, _ = abcd
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    srcs, dsts = [], []
    for start in range(0, m, chunk):
        k = min(chunk, m - start)
        s = torch.zeros(k, dtype=torch.int64, device=device)
        d = torch.zeros(k, dtype=torch.int64, device=device)
        for bit in range(scale):
            r = torch.rand(k, generator=gen, device=device)
            sbit = (r >= a + b).to(torch.int64)           # quadrants c, d
            dbit = (((r >= a) & (r < a + b)) | (r >= a + b + c)).to(torch.int64)  # b, d
            s |= sbit << bit
            d |= dbit << bit
        srcs.append(s)
        dsts.append(d)
    src, dst = torch.cat(srcs), torch.cat(dsts)
    perm = torch.randperm(n, generator=gen, device=device)
    src, dst = perm[src], perm[dst]
    order = torch.argsort(src * n + dst)
    return src[order].contiguous(), dst[order].contiguous(), n


def expected_reddit_edges(scale=1, self_loops=True):
    """Edge count reddit_like produces (exact by construction)."""
    return (REDDIT_EDGES * scale) // 2 * 2 + (REDDIT_NODES * scale if self_loops else 0)



# -- synthetic node-classification datasets (BASELINE.json configs) -----------
_SHAPES = {
    # name: (nodes, directed edges without self-loops, features, classes, max/mean degree)
    "cora": (2708, 10556, 1433, 7, 42.0),
    "citeseer": (3327, 9228, 3703, 6, 36.0),
    "pubmed": (19717, 88651, 500, 3, 38.0),
    "reddit": (REDDIT_NODES, REDDIT_EDGES, 602, 41, REDDIT_MAX_OVER_MEAN),
}


class SyntheticNodeDataset(object):
    """Shape-matched stand-in for the reference's citation / Reddit datasets
    (python/dgl/data/citation_graph.py, the Reddit numbers of SURVEY.md §8a):
    a symmetric Chung-Lu graph with the dataset's node and edge counts and
    degree skew, row-normalised sparse binary features (dense Gaussian for
    Reddit), random labels and 140/500/1000-style
    train/val/test masks. ``graph`` is (src, dst) without self-loops."""

    def __init__(self, name, seed=0, device="cpu"):
        if name not in _SHAPES:
            raise ValueError("unknown dataset %s (have %s)" % (name, sorted(_SHAPES)))
        n, m, nfeat, ncls, ratio = _SHAPES[name]
        self.name = name
        src, dst, n = chung_lu(n, m, ratio, seed=seed, device=device, self_loops=False)
        self.graph = (src, dst)
        gen = torch.Generator(device=device)
        gen.manual_seed(seed + 1)
        if name == "reddit":  # dense embeddings
            self.features = 0.1 * torch.randn(n, nfeat, generator=gen, device=device)
        else:  # row-normalised sparse bag-of-words, as the citation loaders produce
            bow = (torch.rand(n, nfeat, generator=gen, device=device) < 0.0127).float()
            bow[:, 0] += (bow.sum(1) == 0).float()
            self.features = bow / bow.sum(1, keepdim=True)
        self.labels = torch.randint(0, ncls, (n,), generator=gen, device=device)
        self.num_labels = ncls
        self.num_nodes = n
        ntrain = min(20 * ncls, n // 10) if name != "reddit" else int(0.66 * n)
        perm = torch.randperm(n, generator=gen, device=device)
        self.train_mask = torch.zeros(n, dtype=torch.bool, device=device)
        self.val_mask = torch.zeros(n, dtype=torch.bool, device=device)
        self.test_mask = torch.zeros(n, dtype=torch.bool, device=device)
        self.train_mask[perm[:ntrain]] = True
        self.val_mask[perm[ntrain:ntrain + min(500, n // 10)]] = True
        self.test_mask[perm[-min(1000, n // 5):]] = True


def load_edge_list(path, num_nodes=None):
    """(src, dst, num_nodes) int64 tensors from an edge-list file: text lines
    "src dst" (whitespace or comma separated, '#' comments), an (E, 2) integer
    ``.npy``, or an ``.npz`` holding ``src`` and ``dst``. Edge ids follow the
    file order; num_nodes defaults to max id + 1."""
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            src, dst = np.asarray(z["src"]), np.asarray(z["dst"])
    elif path.endswith(".npy"):
        e = np.load(path, allow_pickle=False)
        if e.ndim != 2 or e.shape[1] != 2:
            raise ValueError("%s: expected an (E, 2) array, got %s" % (path, e.shape))
        src, dst = e[:, 0], e[:, 1]
    else:
        e = np.loadtxt(path, dtype=np.int64, comments="#",
                       delimiter="," if path.endswith(".csv") else None, ndmin=2)
        if e.size and e.shape[1] != 2:
            raise ValueError("%s: expected 2 columns, got %d" % (path, e.shape[1]))
        src, dst = (e[:, 0], e[:, 1]) if e.size else (np.zeros(0), np.zeros(0))
    src = torch.from_numpy(np.ascontiguousarray(src, dtype=np.int64))
    dst = torch.from_numpy(np.ascontiguousarray(dst, dtype=np.int64))
    if src.numel() and min(int(src.min()), int(dst.min())) < 0:
        raise ValueError("%s: negative node id" % path)
    top = int(max(int(src.max()), int(dst.max()))) + 1 if src.numel() else 0
    n = top if num_nodes is None else int(num_nodes)
    if n < top:
        raise ValueError("%s: node id %d >= num_nodes %d" % (path, top - 1, n))
    return src, dst, n


def _masks(n, train, val, test, device):
    out = []
    for idx in (train, val, test):
        m = torch.zeros(n, dtype=torch.bool)
        m[torch.as_tensor(np.asarray(idx, dtype=np.int64))] = True
        out.append(m.to(device))
    return out


class CoraTextDataset(object):
    """The pygcn text release of Cora, parsed as the reference's
    CoraDataset._load does (citation_graph.py:349-380): one line per paper
    "id word_0 .. word_k label" in cora.content, "cited citing" pairs in
    cora.cites; the adjacency is symmetrised (max of A and A^T); features are
    row-normalised; train / val / test = ids 0-139 / 200-499 / 500-1499.
    Deterministic where the reference is not: class ids follow the sorted
    label names (the reference's set() order varies with the hash seed), and
    the edges of the symmetric adjacency come in (src, dst) order, as
    networkx yields them from the CSR matrix. ``graph`` = (src, dst)."""

    def __init__(self, root, device="cpu"):
        base = os.path.join(root, "cora")
        rows = np.genfromtxt(os.path.join(base, "cora.content"), dtype=np.dtype(str), ndmin=2)
        ids = rows[:, 0].astype(np.int64)
        feats = rows[:, 1:-1].astype(np.float32)
        names = rows[:, -1]
        classes = sorted(set(names.tolist()))
        self.labels = torch.as_tensor(np.searchsorted(np.asarray(classes), names),
                                      dtype=torch.int64, device=device)
        self.num_labels = len(classes)
        n = len(ids)
        pos = {int(j): i for i, j in enumerate(ids)}
        cites = np.genfromtxt(os.path.join(base, "cora.cites"), dtype=np.int64, ndmin=2)
        u = np.array([pos[int(a)] for a in cites[:, 0]], dtype=np.int64)
        v = np.array([pos[int(b)] for b in cites[:, 1]], dtype=np.int64)
        # symmetric pattern of max(A, A^T): every (u, v) and (v, u), once each
        key = np.unique(np.concatenate([u * n + v, v * n + u]))
        self.graph = (torch.from_numpy(key // n), torch.from_numpy(key % n))
        rowsum = feats.sum(1, keepdims=True)
        with np.errstate(divide="ignore", invalid="ignore"):
            feats = feats * np.power(rowsum, -1)  # inf rows stay inf, as _normalize
        self.features = torch.from_numpy(feats).to(device)
        self.num_nodes = n
        self.train_mask, self.val_mask, self.test_mask = _masks(
            n, range(min(140, n)), range(min(200, n), min(500, n)),
            range(min(500, n), min(1500, n)), device)


class RedditDataset(object):
    """DGL's Reddit release: ``reddit_graph.npz`` (scipy sparse adjacency,
    read with pickling disabled) and ``reddit_data.npz`` (feature, label,
    node_types with 1 / 2 / 3 = train / val / test). Edges in the stored
    COO order. ``graph`` = (src, dst)."""

    def __init__(self, root, device="cpu"):
        import scipy.sparse as sp
        base = os.path.join(root, "reddit")
        adj = sp.load_npz(os.path.join(base, "reddit_graph.npz")).tocoo()
        with np.load(os.path.join(base, "reddit_data.npz"), allow_pickle=False) as z:
            feat, label, types = z["feature"], z["label"], z["node_types"]
        n = adj.shape[0]
        self.graph = (torch.from_numpy(adj.row.astype(np.int64)),
                      torch.from_numpy(adj.col.astype(np.int64)))
        self.features = torch.from_numpy(np.asarray(feat, dtype=np.float32)).to(device)
        self.labels = torch.from_numpy(np.asarray(label, dtype=np.int64)).to(device)
        self.num_labels = int(self.labels.max()) + 1 if n else 0
        self.num_nodes = n
        t = torch.from_numpy(np.asarray(types))
        self.train_mask, self.val_mask, self.test_mask = (
            (t == k).to(device) for k in (1, 2, 3))


def _on_disk(name, root):
    if not root:
        return None
    if name == "cora" and os.path.exists(os.path.join(root, "cora", "cora.content")):
        return CoraTextDataset
    if name == "reddit" and os.path.exists(os.path.join(root, "reddit", "reddit_graph.npz")):
        return RedditDataset
    return None


def load_data(name, seed=0, device="cpu", root=None):
    """dgl.data.load_data counterpart (python/dgl/data/__init__.py:15-25):
    the on-disk release under ``root`` (default ``$DGL_DATA_DIR``) when its
    files are there, else the seeded synthetic stand-in (nothing is ever
    downloaded)."""
    root = root if root is not None else os.environ.get("DGL_DATA_DIR")
    cls = _on_disk(name, root)
    if cls is not None:
        ds = cls(root, device)
        ds.name, ds.source = name, "files under %s" % root
        return ds
    ds = SyntheticNodeDataset(name, seed, device)
    ds.source = "synthetic (seed %d)" % seed
    return ds
