"""send / recv / in-place semantics around the kernels, restating the
scenarios of the reference's tests/compute/test_inplace_update.py and
tests/compute/test_multi_send_recv.py:

* every trigger (recv, send_and_recv, push, pull, apply_nodes) with
  inplace=True gives the out-of-place result and writes it into the column
  tensor that was set, for the degree-bucketing (UDF), v2v SPMV (builtin pair:
  the g-SpMM kernel) and e2v (UDF message + builtin sum) paths;
* pending-message bookkeeping over repeated sends and partial receives, 0-deg
  receivers with a custom initializer, a second send overwriting a message,
  two fields sent separately, graphs growing between rounds, recv without a
  send, and message passing after from_networkx / from_scipy_sparse_matrix.

The reference checks the pending set through its private _msg_index; this
engine keeps it in DGLGraph._msg_pending (a bool per edge).
"""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

import dgl
import dgl.function as fn
from dgl import DGLGraph

D = 5
DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _dev(device):
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device(device)


def _star_graph(dev, back_edge=True, seed=0):
    """0 -> 1..8 -> 9 (16 edges), plus 9 -> 0 (edge 16) when back_edge."""
    g = DGLGraph()
    g.add_nodes(10)
    for i in range(1, 9):
        g.add_edge(0, i)
        g.add_edge(i, 9)
    if back_edge:
        g.add_edge(9, 0)
    gen = torch.Generator().manual_seed(seed)
    g.set_n_initializer(dgl.init.zero_initializer)
    g.set_e_initializer(dgl.init.zero_initializer)
    g.ndata["f"] = torch.randn(10, D, generator=gen).to(dev)
    g.edata["e"] = torch.randn(g.number_of_edges(), D, generator=gen).to(dev)
    return g


def _msg_src(edges):
    return {"m": edges.src["f"]}


def _sum_udf(nodes):
    return {"f": nodes.mailbox["m"].sum(1)}


def _double(nodes):
    return {"f": 2 * nodes.data["f"]}


def _check_inplace(g, f0, run_ref, run_inplace):
    g.ndata["f"] = f0
    run_ref()
    result = g.ndata["f"]
    v1 = f0.clone()
    g.ndata["f"] = v1
    run_inplace()
    torch.testing.assert_close(g.ndata["f"], result)
    torch.testing.assert_close(v1, result)  # written into the tensor that was set


U = [0, 0, 0, 3, 4, 9]
V = [1, 2, 3, 9, 9, 0]


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("apply", [_double, None])
@pytest.mark.parametrize("path", ["bucket", "v2v", "e2v"])
def test_inplace_send_and_recv(device, apply, path):
    dev = _dev(device)
    g = _star_graph(dev)
    mfn, rfn = {"bucket": (_msg_src, _sum_udf),
                "v2v": (fn.copy_src("f", "m"), fn.sum("m", "f")),
                "e2v": (_msg_src, fn.sum("m", "f"))}[path]
    f0 = g.ndata["f"]

    def ref():
        g.ndata["f"] = f0
        g.send_and_recv((U, V), fn.copy_src("f", "m"), fn.sum("m", "f"), apply)
    _check_inplace(g, f0, ref,
                   lambda: g.send_and_recv((U, V), mfn, rfn, apply, inplace=True))


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("trigger", ["push", "pull", "recv"])
def test_inplace_push_pull_recv(device, trigger):
    dev = _dev(device)
    g = _star_graph(dev)
    f0 = g.ndata["f"]
    for mfn, rfn in ((_msg_src, _sum_udf), (fn.copy_src("f", "m"), fn.sum("m", "f")),
                     (_msg_src, fn.sum("m", "f"))):
        for apply in (_double, None):
            if trigger == "push":
                nodes = [0, 3, 4, 9]
                run = lambda inplace: g.push(nodes, mfn, rfn, apply,  # noqa: E731
                                             inplace=inplace)
            elif trigger == "pull":
                nodes = [1, 2, 3, 9]
                run = lambda inplace: g.pull(nodes, mfn, rfn, apply,  # noqa: E731
                                             inplace=inplace)
            else:
                def run(inplace):
                    g.send((U, V), mfn if callable(mfn) else _msg_src)
                    g.recv([0, 1, 2, 3, 9], rfn, apply, inplace=inplace)

            def ref():
                g.ndata["f"] = f0
                run(False)
            _check_inplace(g, f0, ref, lambda: run(True))


@pytest.mark.parametrize("device", DEVICES)
def test_inplace_apply(device):
    dev = _dev(device)
    g = _star_graph(dev)
    nodes = [1, 2, 3, 9]
    f0 = g.ndata["f"]

    def ref():
        g.ndata["f"] = f0
        g.apply_nodes(_double, nodes)
    _check_inplace(g, f0, ref, lambda: g.apply_nodes(_double, nodes, inplace=True))
    e0 = g.edata["e"].clone()
    g.apply_edges(lambda edges: {"e": edges.data["e"] * 3}, [0, 4], inplace=True)
    torch.testing.assert_close(g.edata["e"][[0, 4]], e0[[0, 4]] * 3)


def _pending(g):
    return g._msg_pending.to(torch.int64)


def test_multi_send_pending():
    g = _star_graph("cpu", back_edge=False)
    g.register_message_func(_msg_src)
    g.send(([0] * 5, [1, 2, 3, 4, 5]))
    g.send(([0], [1, 2, 3, 4, 5]))          # the same edges again
    g.send(([1, 2, 3, 4, 5], [9]))
    expected = torch.zeros(g.number_of_edges(), dtype=torch.int64)
    expected[g.edge_ids([0, 0, 0, 0, 0, 1, 2, 3, 4, 5], [1, 2, 3, 4, 5, 9, 9, 9, 9, 9])] = 1
    assert torch.equal(_pending(g), expected)


def test_multi_recv_pending_and_results():
    g = _star_graph("cpu", back_edge=False)
    h = g.ndata["f"]
    g.register_message_func(_msg_src)
    g.register_reduce_func(lambda nodes: {"acc": nodes.mailbox["m"].sum(1)})
    g.register_apply_node_func(lambda nodes: {"f": nodes.data["f"] + nodes.data["acc"]})
    expected = torch.zeros(g.number_of_edges(), dtype=torch.int64)
    for u, v in (([4, 5, 6], [9]), ([0], [1, 2, 3])):  # two separate rounds
        g.send((u, v))
        expected[g.edge_ids(u, v)] = 1
        assert torch.equal(_pending(g), expected)
        g.recv(v)
        expected[g.edge_ids(u, v)] = 0
        assert torch.equal(_pending(g), expected)
    h1 = g.ndata["f"]
    g.ndata["f"] = h  # one send, two receives
    g.send(([0, 0, 0, 4, 5, 6], [1, 2, 3, 9, 9, 9]))
    g.recv([9])
    assert int(_pending(g).sum()) == 3
    g.recv([1, 2, 3])
    assert int(_pending(g).sum()) == 0
    torch.testing.assert_close(g.ndata["f"], h1)


def test_recv_zero_degree_with_initializer():
    g = DGLGraph()
    g.register_message_func(lambda edges: {"m": edges.src["h"]})
    g.register_reduce_func(lambda nodes: {"h": nodes.data["h"] + nodes.mailbox["m"].sum(1)})
    g.register_apply_node_func(lambda nodes: {"h": nodes.data["h"] * 2})
    g.set_n_initializer(lambda shape, dtype, ctx, ids: 2 + torch.zeros(shape, dtype=dtype))
    g.add_nodes(2)
    g.add_edge(0, 1)
    old = torch.randn(2, 5)
    g.ndata["h"] = old
    g.send((0, 1))
    g.recv([0, 1])
    new = g.ndata["h"]
    torch.testing.assert_close(new[0], torch.full((5,), 4.0))   # initializer, then apply
    torch.testing.assert_close(new[1], old.sum(0) * 2)
    g.recv([0])
    torch.testing.assert_close(g.nodes[0].data["h"][0], torch.full((5,), 8.0))
    g.recv([1])  # nothing pending for node 1: only the apply runs
    torch.testing.assert_close(g.nodes[1].data["h"][0], old.sum(0) * 4)


def test_send_twice_overwrites_message():
    g = DGLGraph()
    g.set_n_initializer(dgl.init.zero_initializer)
    g.add_nodes(3)
    g.add_edges([0, 2], [1, 1])
    old = torch.randn(3, 5)
    reduce_max = lambda nodes: {"a": nodes.mailbox["a"].max(1)[0]}  # noqa: E731
    g.ndata["a"] = old
    g.send((0, 1), lambda edges: {"a": edges.src["a"]})
    g.send((0, 1), lambda edges: {"a": edges.src["a"] * 3})
    g.recv(1, reduce_max)
    torch.testing.assert_close(g.ndata["a"][1], old[0] * 3)
    g.ndata["a"] = old
    g.send((0, 1), lambda edges: {"a": edges.src["a"]})
    g.send((2, 1), lambda edges: {"a": edges.src["a"] * 3})
    g.recv(1, reduce_max)
    torch.testing.assert_close(g.ndata["a"][1], torch.max(old[0], old[2] * 3))


def test_send_twice_different_fields():
    g = DGLGraph()
    g.set_n_initializer(dgl.init.zero_initializer)
    g.add_nodes(2)
    g.add_edge(0, 1)
    a, b = torch.randn(2, 5), torch.randn(2, 5)
    g.set_n_repr({"a": a, "b": b})
    g.send((0, 1), lambda edges: {"a": edges.src["a"]})
    g.send((0, 1), lambda edges: {"b": edges.src["b"]})
    g.recv([1], lambda nodes: {"a": nodes.mailbox["a"].sum(1), "b": nodes.mailbox["b"].sum(1)})
    torch.testing.assert_close(g.get_n_repr()["a"][1], a[0])
    torch.testing.assert_close(g.get_n_repr()["b"][1], b[0])


def test_graph_growing_between_rounds():
    g = DGLGraph()
    g.set_n_initializer(dgl.init.zero_initializer)
    g.set_e_initializer(dgl.init.zero_initializer)
    g.register_message_func(lambda edges: {"m": edges.src["h1"] + edges.dst["h2"] +
                                           edges.data["h1"] + edges.data["h2"]})
    g.register_reduce_func(lambda nodes: {"h": nodes.mailbox["m"].sum(1)})
    g.register_apply_node_func(lambda nodes: {"h": nodes.data["h"]})
    g.add_nodes(3)
    g.ndata.update({"h1": torch.randn(3, 1), "h2": torch.randn(3, 1)})
    g.add_nodes(3)
    g.add_edges([0, 1], [1, 0])
    g.edata.update({"h1": torch.randn(2, 1), "h2": torch.randn(2, 1)})
    g.send()
    assert torch.equal(_pending(g), torch.ones(2, dtype=torch.int64))
    g.add_edges([0, 2], [2, 0], {"h1": torch.randn(2, 1)})
    g.send(([0, 2], [2, 0]))
    g.recv(0)
    g.add_edge(1, 2)
    g.edges[4].data["h1"] = torch.randn(1, 1)
    g.send((1, 2))
    g.recv([1, 2])
    h = g.ndata.pop("h")
    g.send()   # one full round on the final graph gives the same values
    g.recv()
    torch.testing.assert_close(h, g.ndata["h"])


def test_recv_without_send_and_after_clear():
    g = _star_graph("cpu", back_edge=False)
    g.recv(1, _sum_udf)  # nothing pending: no error
    g.clear()
    g.add_nodes(3)
    g.add_edges([0, 1], [1, 2])
    g.set_n_initializer(dgl.init.zero_initializer)
    g.ndata["f"] = torch.randn(3, D)
    g.send((1, 2), _msg_src)
    assert _pending(g).tolist() == [0, 1]
    g.recv(2, _sum_udf)
    assert _pending(g).tolist() == [0, 0]


@pytest.mark.parametrize("device", DEVICES)
def test_message_passing_after_conversion(device):
    dev = _dev(device)
    g = _star_graph("cpu", back_edge=False)
    row, col = g.all_edges()
    n = g.number_of_nodes()
    a = sp.coo_matrix((np.arange(len(row)), (row.numpy(), col.numpy())), shape=(n, n))
    g2 = DGLGraph()
    g2.add_nodes(5)
    g2.add_edges([1, 2, 4], [2, 3, 0])   # replaced by the conversion
    g2.from_scipy_sparse_matrix(a)
    g3 = DGLGraph()
    g3.add_nodes(4)
    g3.add_edges([1, 2], [2, 3])
    g3.from_networkx(g.to_networkx())
    outs = []
    for gg in (g, g2, g3):
        gg.ndata["f"] = g.ndata["f"].to(dev)
        gg.update_all(fn.copy_src("f", "m"), fn.sum("m", "o"))
        outs.append(gg.ndata["o"].cpu())
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


def test_to_networkx_attributes():
    g = DGLGraph(multigraph=True)
    g.add_nodes(5, {"n1": torch.randn(5, 3)})
    g.add_edges([0, 1, 3, 4, 0], [2, 4, 0, 3, 2], {"e1": torch.randn(5, 2)})
    nxg = g.to_networkx(node_attrs=["n1"], edge_attrs=["e1"])
    assert nxg.number_of_nodes() == 5 and nxg.number_of_edges() == 5
    for u, v, d in nxg.edges(data=True):
        e = d["id"]
        assert (int(g._graph.src()[e]), int(g._graph.dst()[e])) == (u, v)
        assert torch.equal(d["e1"], g.edata["e1"][e])
    assert torch.equal(nxg.nodes[3]["n1"], g.ndata["n1"][3])
    back = DGLGraph(multigraph=True)
    back.from_networkx(nxg, node_attrs=["n1"], edge_attrs=["e1"])
    assert torch.equal(back.edata["e1"], g.edata["e1"])   # edge order kept through 'id'
    assert torch.equal(back.ndata["n1"], g.ndata["n1"])
