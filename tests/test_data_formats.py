"""On-disk graph formats: the pygcn Cora text release as the
reference's CoraDataset._load reads it (python/dgl/data/citation_graph.py:
349-380), DGL's Reddit npz release, plain edge lists, and load_data's choice
between files and the synthetic stand-ins. Fixture files are written here."""
import os

import numpy as np
import pytest
import torch

from dgl import DGLGraph, data


def _write_cora(root):
    d = os.path.join(root, "cora")
    os.makedirs(d)
    # paper id, 4 binary words, label (ids are sparse, as in the release)
    papers = [(31336, [0, 1, 0, 1], "Neural_Networks"),
              (1061127, [1, 0, 0, 0], "Rule_Learning"),
              (1106406, [0, 0, 1, 1], "Neural_Networks"),
              (13195, [1, 1, 1, 1], "Theory"),
              (37879, [0, 0, 0, 1], "Theory")]
    with open(os.path.join(d, "cora.content"), "w") as f:
        for pid, words, lab in papers:
            f.write("%d\t%s\t%s\n" % (pid, "\t".join(map(str, words)), lab))
    # cited -> citing; a duplicate, a reciprocal pair and a self-citation
    cites = [(31336, 1061127), (31336, 1061127), (1061127, 31336), (13195, 37879),
             (1106406, 1106406), (37879, 31336)]
    with open(os.path.join(d, "cora.cites"), "w") as f:
        for a, b in cites:
            f.write("%d\t%d\n" % (a, b))
    return papers, cites


def test_cora_text_release(tmp_path):
    papers, cites = _write_cora(str(tmp_path))
    ds = data.CoraTextDataset(str(tmp_path))
    assert ds.num_nodes == 5 and ds.num_labels == 3
    # class ids = sorted label names
    assert ds.labels.tolist() == [0, 1, 0, 2, 2]
    pos = {p[0]: i for i, p in enumerate(papers)}
    pairs = set()
    for a, b in cites:
        pairs.add((pos[a], pos[b]))
        pairs.add((pos[b], pos[a]))
    src, dst = ds.graph
    got = list(zip(src.tolist(), dst.tolist()))
    assert got == sorted(pairs)  # union of A and A^T, each pair once, (src, dst) order
    words = np.array([p[1] for p in papers], np.float32)
    np.testing.assert_allclose(ds.features.numpy(), words / words.sum(1, keepdims=True))
    assert ds.train_mask.all() and not ds.val_mask.any() and not ds.test_mask.any()
    g = DGLGraph(ds.graph)
    assert g.number_of_nodes() == 5 and g.number_of_edges() == len(pairs)


def test_edge_list_formats(tmp_path):
    src = np.array([0, 3, 1, 1, 4])
    dst = np.array([1, 0, 2, 2, 4])
    txt = tmp_path / "g.txt"
    txt.write_text("# comment\n" + "".join("%d %d\n" % e for e in zip(src, dst)))
    csv = tmp_path / "g.csv"
    csv.write_text("".join("%d,%d\n" % e for e in zip(src, dst)))
    npy = tmp_path / "g.npy"
    np.save(str(npy), np.stack([src, dst], 1))
    npz = tmp_path / "g.npz"
    np.savez(str(npz), src=src, dst=dst)
    for p in (txt, csv, npy, npz):
        s, d, n = data.load_edge_list(str(p))
        assert s.tolist() == src.tolist() and d.tolist() == dst.tolist() and n == 5
    assert data.load_edge_list(str(txt), num_nodes=9)[2] == 9
    with pytest.raises(ValueError):
        data.load_edge_list(str(txt), num_nodes=3)
    bad = tmp_path / "bad.txt"
    bad.write_text("0 -1\n")
    with pytest.raises(ValueError):
        data.load_edge_list(str(bad))
    empty = tmp_path / "empty.txt"
    empty.write_text("# nothing\n")
    s, d, n = data.load_edge_list(str(empty))
    assert s.numel() == 0 and n == 0


def test_reddit_release_and_load_data(tmp_path, monkeypatch):
    import scipy.sparse as sp
    d = tmp_path / "reddit"
    d.mkdir()
    row = np.array([0, 1, 2, 2, 3])
    col = np.array([1, 0, 3, 0, 2])
    sp.save_npz(str(d / "reddit_graph.npz"), sp.coo_matrix((np.ones(5), (row, col)),
                                                           shape=(4, 4)))
    feat = np.arange(8, dtype=np.float32).reshape(4, 2)
    np.savez(str(d / "reddit_data.npz"), feature=feat, label=np.array([3, 0, 1, 3]),
             node_types=np.array([1, 2, 3, 1]))
    ds = data.load_data("reddit", root=str(tmp_path))
    assert ds.source.startswith("files")
    s, t = ds.graph
    assert sorted(zip(s.tolist(), t.tolist())) == sorted(zip(row.tolist(), col.tolist()))
    assert ds.num_nodes == 4 and ds.num_labels == 4
    assert ds.train_mask.tolist() == [True, False, False, True]
    assert ds.val_mask.tolist() == [False, True, False, False]
    assert torch.equal(ds.features, torch.from_numpy(feat))
    # $DGL_DATA_DIR is the default root; without files the synthetic stand-in is used
    monkeypatch.setenv("DGL_DATA_DIR", str(tmp_path))
    assert data.load_data("reddit").source.startswith("files")
    assert data.load_data("pubmed").source.startswith("synthetic")
