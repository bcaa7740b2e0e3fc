"""DGLGraph message passing through the engine, checked against the golden
vectors (the reference's arithmetic) and the oracle, on the host device and —
under the `gpu` marker — on the MI355X HIP kernels.

Style follows the reference's tests/compute/test_specialization.py (builtin
SPMV path vs UDF path) and test_basics.py (0-degree semantics), with exact
comparisons where the reference's arithmetic is reproduced bit for bit.
"""
import numpy as np
import pytest
import torch

import dgl
import dgl.function as fn
from dgl.runtime import ir
from oracle import oracle as O

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _dev(device):
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device(device)


def build(c, device, readonly=False):
    g = dgl.DGLGraph(multigraph=True)
    g.add_nodes(int(c["n"]))
    g.add_edges(c["src"], c["dst"])
    if readonly:
        g = dgl.DGLGraph((torch.as_tensor(c["src"]), torch.as_tensor(c["dst"])),
                         readonly=True)
    return g


def t(x, device):
    return torch.as_tensor(np.asarray(x)).to(device)


def exact(a, b):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    assert a.shape == np.asarray(b).shape
    assert np.array_equal(a, np.asarray(b)), np.abs(a - b).max()


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("case", ["spec10", "cora", "multi", "zerodeg"])
def test_update_all_copy_sum_bit_exact(golden, device, case):
    dev = _dev(device)
    c = golden(case)
    g = build(c, dev)
    g.ndata["h"] = t(c["h"], dev)
    with ir.prog() as p:
        g.update_all(fn.copy_src("h", "m"), fn.sum("m", "h"))
    assert "SPMV" in p.opcodes()
    exact(g.ndata["h"], c["copy_out"])


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("case", ["spec10", "multi"])
def test_update_all_src_mul_edge_bit_exact(golden, device, case):
    dev = _dev(device)
    c = golden(case)
    g = build(c, dev)
    g.ndata["h"] = t(c["h"], dev)
    for w in (t(c["w"], dev), t(c["w"], dev).unsqueeze(1)):  # (E,) and (E,1)
        g.edata["w"] = w
        g.update_all(fn.src_mul_edge("h", "w", "m"), fn.sum("m", "o"))
        exact(g.ndata["o"], c["mul_out"])


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("case", ["spec10", "cora", "multi"])
def test_backward_bit_exact(golden, device, case):
    dev = _dev(device)
    c = golden(case)
    g = build(c, dev)
    h = t(c["h"], dev).requires_grad_(True)
    g.ndata["h"] = h
    g.update_all(fn.copy_src("h", "m"), fn.sum("m", "o"))
    g.ndata["o"].backward(t(c["g"], dev))
    exact(h.grad, c["copy_grad_h"])
    if "w" in c:
        h = t(c["h"], dev).requires_grad_(True)
        w = t(c["w"], dev).requires_grad_(True)
        g.ndata["h"] = h
        g.edata["w"] = w
        g.update_all(fn.src_mul_edge("h", "w", "m"), fn.sum("m", "o"))
        g.ndata["o"].backward(t(c["g"], dev))
        exact(h.grad, c["mul_grad_h"])
        np.testing.assert_allclose(w.grad.cpu().numpy(), c["mul_grad_w"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("device", DEVICES)
def test_send_and_recv_and_pull_push(golden, device):
    dev = _dev(device)
    c, s = golden("cora"), golden("snr")
    g = build(c, dev)
    h = t(c["h"], dev)
    g.ndata["h"] = h
    g.ndata["o"] = torch.full_like(h, 7.0)
    sel = torch.as_tensor(s["sel"])
    g.send_and_recv(sel, fn.copy_src("h", "m"), fn.sum("m", "o"))  # edges by id
    recv = torch.as_tensor(s["recv"])
    exact(g.ndata["o"][recv.to(dev)], s["out"])
    mask = torch.ones(g.number_of_nodes(), dtype=torch.bool)
    mask[recv] = False
    assert bool((g.ndata["o"][mask.to(dev)] == 7.0).all())
    # pull on every node == update_all; push from every node == update_all
    g.pull(torch.arange(g.number_of_nodes()), fn.copy_src("h", "m"), fn.sum("m", "p"))
    exact(g.ndata["p"], c["copy_out"])
    # push sends along out_edges(u): the reference's COO is in that (src-major)
    # order, so each row accumulates in it (spmv.py:154-227 keeps edge order)
    g.push(torch.arange(g.number_of_nodes()), fn.copy_src("h", "m"), fn.sum("m", "q"))
    pu, pv = g.out_edges(torch.arange(g.number_of_nodes()))
    exact(g.ndata["q"], O.spmm_coo(int(c["n"]), pv.numpy(), pu.numpy(), c["h"]))


@pytest.mark.parametrize("device", DEVICES)
def test_pull_zero_degree_nodes(golden, device):
    """pull on nodes with no in-edges: rows reduced to 0 on the SPMV path."""
    dev = _dev(device)
    c = golden("zerodeg")
    g = build(c, dev)
    g.ndata["h"] = t(c["h"], dev)
    g.pull([4, 5, 6, 9], fn.copy_src("h", "m"), fn.sum("m", "h"))
    ref = c["h"].copy()
    ref[[4, 5, 6, 9]] = c["copy_out"][[4, 5, 6, 9]]
    exact(g.ndata["h"], ref)


@pytest.mark.parametrize("device", DEVICES)
def test_builtin_vs_udf(golden, device):
    """test_specialization.py style: builtin kernel path == UDF path."""
    dev = _dev(device)
    c = golden("multi")
    g = build(c, dev)
    g.ndata["h"] = t(c["h"], dev)
    g.edata["w"] = t(c["w"], dev).unsqueeze(1)

    def msg(edges):
        return {"m": edges.src["h"] * edges.data["w"]}

    def red_sum(nodes):
        return {"o": nodes.mailbox["m"].sum(1)}

    def red_max(nodes):
        return {"o": nodes.mailbox["m"].max(1)[0]}

    def red_mean(nodes):
        return {"o": nodes.mailbox["m"].mean(1)}

    for builtin, udf, tol in ((fn.sum, red_sum, 1e-5), (fn.max, red_max, 0.0),
                              (fn.mean, red_mean, 1e-5)):
        g.update_all(fn.src_mul_edge("h", "w", "m"), builtin("m", "o"))
        a = g.ndata["o"].clone()
        with ir.prog() as p:
            g.update_all(msg, udf)
        assert "DEGREE_BUCKETING" in p.opcodes()
        b = g.ndata["o"]
        if tol == 0.0:
            exact(a, b.cpu().numpy())
        else:
            np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=tol, atol=tol)


@pytest.mark.parametrize("device", DEVICES)
def test_max_mean_golden(golden, device):
    dev = _dev(device)
    for case in ("multi", "zerodeg"):
        c = golden(case)
        g = build(c, dev)
        g.ndata["h"] = t(c["h"], dev)
        g.update_all(fn.copy_src("h", "m"), fn.max("m", "mx"))
        exact(g.ndata["mx"], c["max_out"])
        if "mean_out" in c:
            g.update_all(fn.copy_src("h", "m"), fn.mean("m", "mn"))
            np.testing.assert_allclose(g.ndata["mn"].cpu().numpy(), c["mean_out"],
                                       rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("device", DEVICES)
def test_copy_edge_e2v_and_multi_fn(golden, device):
    """GAT-style: [src_mul_edge, copy_edge] x [sum, sum] (gat/train.py:77-78)."""
    dev = _dev(device)
    c = golden("multi")
    g = build(c, dev)
    g.ndata["h"] = t(c["h"], dev)
    g.edata["a"] = t(c["w"], dev).unsqueeze(1)
    g.update_all([fn.src_mul_edge("h", "a", "m"), fn.copy_edge("a", "am")],
                 [fn.sum("m", "ft"), fn.sum("am", "z")])
    exact(g.ndata["ft"], c["mul_out"])
    z = O.spmm_coo(int(c["n"]), c["dst"], np.arange(len(c["src"])), c["w"][:, None])
    exact(g.ndata["z"], z)


@pytest.mark.parametrize("device", DEVICES)
def test_feat_shapes(golden, device):
    dev = _dev(device)
    c = golden("feat3d")
    g = build(c, dev)
    g.ndata["h"] = t(c["h"], dev)
    g.update_all(fn.copy_src("h", "m"), fn.sum("m", "o"))
    exact(g.ndata["o"], c["copy_out"])
    s = golden("spec10")  # 1-D node features
    g = build(s, dev)
    g.ndata["x"] = t(s["h"][:, 0], dev)
    g.update_all(fn.copy_src("x", "m"), fn.sum("m", "x"))
    exact(g.ndata["x"], s["copy_out"][:, 0])


@pytest.mark.parametrize("device", DEVICES)
def test_vector_edge_weights(device):
    """u_mul_e with a per-feature edge weight (not specialised by the reference)."""
    dev = _dev(device)
    rng = np.random.default_rng(3)
    n, m, F = 40, 300, 6
    src, dst = rng.integers(0, n, m), rng.integers(0, n, m)
    h = rng.standard_normal((n, F)).astype(np.float32)
    w = rng.standard_normal((m, F)).astype(np.float32)
    g = dgl.DGLGraph(multigraph=True)
    g.add_nodes(n)
    g.add_edges(src, dst)
    g.ndata["h"] = t(h, dev)
    g.edata["w"] = t(w, dev)
    g.update_all(fn.src_mul_edge("h", "w", "m"), fn.sum("m", "o"))
    ref = np.zeros((n, F), np.float64)
    for e in range(m):
        ref[dst[e]] += h[src[e]].astype(np.float64) * w[e]
    np.testing.assert_allclose(g.ndata["o"].cpu().numpy(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("device", DEVICES)
def test_readonly_graph_slot_order(golden, device):
    """Immutable graphs accumulate in (dst, src) order (immutable_graph.cc:206-237)."""
    dev = _dev(device)
    c = golden("multi")
    g = build(c, dev, readonly=True)
    g.ndata["h"] = t(c["h"], dev)
    g.update_all(fn.copy_src("h", "m"), fn.sum("m", "o"))
    order = np.lexsort((np.arange(len(c["src"])), c["src"], c["dst"]))
    ref = O.spmm_coo(int(c["n"]), c["dst"][order], c["src"][order], c["h"])
    exact(g.ndata["o"], ref)


@pytest.mark.parametrize("device", DEVICES)
def test_send_recv_and_apply(golden, device):
    dev = _dev(device)
    c = golden("spec10")
    g = build(c, dev)
    g.ndata["h"] = t(c["h"], dev)
    g.send(g.edges(), fn.copy_src("h", "m"))
    g.recv(g.nodes(), fn.sum("m", "o"))
    exact(g.ndata["o"], c["copy_out"])
    g.update_all(fn.copy_src("h", "m"), fn.sum("m", "o2"),
                 lambda nodes: {"o2": nodes.data["o2"] * 2})
    exact(g.ndata["o2"], c["copy_out"] * 2)
    g.apply_edges(lambda edges: {"e": edges.src["h"] + edges.dst["h"]})
    ref = c["h"][c["src"]] + c["h"][c["dst"]]
    exact(g.edata["e"], ref)


@pytest.mark.parametrize("device", DEVICES)
def test_backend_spmm_boundary(golden, device):
    """F.sparse_matrix + F.spmm (backend.py:77-148,558-572) on the engine."""
    dev = _dev(device)
    from dgl import backend as F
    c = golden("multi")
    idx = torch.stack([torch.as_tensor(c["dst"]), torch.as_tensor(c["src"])])
    A, shuffle = F.sparse_matrix(torch.ones(idx.shape[1]), ("coo", idx), (50, 50))
    assert shuffle is None and F.get_preferred_sparse_format() == "csr"
    exact(F.spmm(A, t(c["h"], dev)), c["copy_out"])
    Aw, _ = F.sparse_matrix(t(c["w"], dev), ("coo", idx), (50, 50))
    exact(F.spmm(Aw, t(c["h"], dev)), c["mul_out"])


def test_gcn_layer_and_training_step(golden):
    """nn.GraphConvolutionLayer drives update_all(copy_src, sum) + Linear."""
    c = golden("cora")
    g = build(c, "cpu")
    torch.manual_seed(0)
    layer = dgl.nn.GraphConvolutionLayer("h", 16, 4, torch.relu)
    g.ndata["h"] = t(c["h"], "cpu")
    layer(g)
    lin = layer.update_func.linear
    ref = torch.relu(lin(torch.as_tensor(c["copy_out"])))
    torch.testing.assert_close(g.ndata["h"], ref)
    g.ndata["h"].sum().backward()
    assert lin.weight.grad is not None and torch.isfinite(lin.weight.grad).all()


def test_graph_queries():
    g = dgl.DGLGraph()
    g.add_nodes(4)
    g.add_edges([0, 0, 1, 2], [1, 2, 2, 3])
    assert g.number_of_edges() == 4
    assert g.in_degrees().tolist() == [0, 1, 2, 1]
    assert g.out_degrees().tolist() == [2, 1, 1, 0]
    u, v = g.in_edges(2)
    assert u.tolist() == [0, 1] and v.tolist() == [2, 2]
    assert g.edge_id(1, 2) == 2
    assert g.has_edge_between(2, 3) and not g.has_edge_between(3, 2)
    assert g.successors(0).tolist() == [1, 2]
    assert g.all_edges("eid").tolist() == [0, 1, 2, 3]
    g.ndata["x"] = torch.ones(4, 2)
    g.nodes[[0, 3]].data["x"] = torch.zeros(2, 2)
    assert g.ndata["x"][:, 0].tolist() == [0, 1, 1, 0]
    g.add_nodes(1)
    assert g.ndata["x"].shape == (5, 2)


@pytest.mark.parametrize("device", DEVICES)
def test_gat_head_broadcast(device):
    """GAT: update_all(src_mul_edge(ft (N,H,D), a (E,H,1)), sum) fused in the kernel
    (gat/train.py:77-78) == the materialised UDF path, forward and gradients."""
    dev = _dev(device)
    rng = np.random.default_rng(21)
    n, m, H, D = 300, 4000, 8, 8
    src, dst = rng.integers(0, n, m), rng.integers(0, n, m)
    ft = torch.from_numpy(rng.standard_normal((n, H, D)).astype(np.float32)).to(dev)
    a = torch.from_numpy(rng.uniform(0, 1, (m, H, 1)).astype(np.float32)).to(dev)
    G = torch.from_numpy(rng.standard_normal((n, H, D)).astype(np.float32)).to(dev)
    outs = []
    for fused in (True, False):
        g = dgl.DGLGraph(multigraph=True)
        g.add_nodes(n)
        g.add_edges(src, dst)
        f1, a1 = ft.clone().requires_grad_(True), a.clone().requires_grad_(True)
        g.ndata["ft"] = f1
        g.edata["a"] = a1
        with ir.prog() as p:
            if fused:
                g.update_all(fn.src_mul_edge("ft", "a", "m"), fn.sum("m", "o"))
            else:
                g.update_all(lambda e: {"m": e.src["ft"] * e.data["a"]},
                             lambda nd: {"o": nd.mailbox["m"].sum(1)})
        assert ("SPMV_WITH_DATA" in p.opcodes()) == fused
        g.ndata["o"].backward(G)
        outs.append((g.ndata["o"].detach().cpu(), f1.grad.cpu(), a1.grad.cpu()))
    for x, y in zip(outs[0], outs[1]):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("device", DEVICES)
def test_gat_edge_attention_fused(device):
    """kernel.edge_attention == the reference's edge UDF (gat/train.py:90-96):
    exp(leaky_relu(a1[src] + a2[dst])).clamp(-10, 10), forward and gradients."""
    dev = _dev(device)
    from dgl import kernel
    rng = np.random.default_rng(8)
    n, m, H = 200, 3000, 8
    src, dst = rng.integers(0, n, m), rng.integers(0, n, m)
    g = dgl.DGLGraph(multigraph=True)
    g.add_nodes(n)
    g.add_edges(src, dst)
    a1 = torch.from_numpy(rng.standard_normal((n, H, 1)).astype(np.float32)).to(dev)
    a2 = torch.from_numpy(rng.standard_normal((n, H, 1)).astype(np.float32)).to(dev) * 2
    G = torch.from_numpy(rng.standard_normal((m, H)).astype(np.float32)).to(dev)
    x1, x2 = a1.clone().requires_grad_(True), a2.clone().requires_grad_(True)
    att = kernel.edge_attention(g.sparse_adjacency(dev), x1, x2, m, alpha=0.2)
    att.backward(G)
    y1, y2 = a1.clone().requires_grad_(True), a2.clone().requires_grad_(True)
    s, d = torch.as_tensor(src).to(dev), torch.as_tensor(dst).to(dev)
    ref = torch.exp(torch.nn.functional.leaky_relu(y1[s] + y2[d], 0.2)).clamp(-10, 10)
    ref = ref.reshape(m, H)
    ref.backward(G)
    torch.testing.assert_close(att, ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(x1.grad, y1.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(x2.grad, y2.grad, rtol=1e-5, atol=1e-5)


def test_degree_bucketing_schedule_native():
    """Native bucket schedule (scheduler.cc:13-93 semantics): buckets by ascending
    degree, nodes ascending, messages in message order; 0-degree nodes omitted."""
    import ctypes
    from dgl._ffi import LIB, check_call, ptr
    recv = torch.tensor([3, 1, 3, 0, 3, 1, 4], dtype=torch.int64)  # message -> receiver
    n = 6
    nb = ctypes.c_int64()
    bdeg, bptr = torch.empty(n, dtype=torch.int64), torch.empty(n + 1, dtype=torch.int64)
    nodes, mids = torch.empty(n, dtype=torch.int64), torch.empty(7, dtype=torch.int64)
    check_call(LIB.dglhip_degree_bucketing_host(7, ptr(recv), n, ctypes.byref(nb), ptr(bdeg),
                                                ptr(bptr), ptr(nodes), ptr(mids)))
    assert nb.value == 3
    assert bdeg[:3].tolist() == [1, 2, 3]
    assert bptr[:4].tolist() == [0, 2, 3, 4]
    assert nodes[:4].tolist() == [0, 4, 1, 3]
    assert mids.tolist() == [3, 6, 1, 5, 0, 2, 4]


def test_pickle_roundtrip(golden):
    """Graph structure + features survive pickling (graph_index.py:35-59)."""
    import pickle
    c = golden("spec10")
    g = build(c, "cpu")
    g.ndata["h"] = t(c["h"], "cpu")
    g2 = pickle.loads(pickle.dumps(g))
    assert g2.number_of_edges() == g.number_of_edges()
    g2.update_all(fn.copy_src("h", "m"), fn.sum("m", "o"))
    exact(g2.ndata["o"], c["copy_out"])
