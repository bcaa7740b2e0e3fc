"""The reference's known-answer incidence matrices of the e2v path, exactly.

/root/reference/python/dgl/runtime/spmv.py:263-277 (build_inc_matrix_eid:
seven edges, eid=[1,2,3,5,6], dst=[1,1,3,4,4], reduce_nodes=0..4 with the
0-degree nodes 0 and 2) and :324-334 (build_inc_matrix_dst, five edges). The
engine's builders are runtime/spmv.build_inc_eid / build_inc_dst; each matrix
is read back through the g-SpMM itself (A = A @ I, copy_u and copy_e), so the
integer entries are what the kernels see. The same matrices then come out of
recv (the reference's scheduler.py:451-456 route: incidence by edge id over
the whole message frame) and send_and_recv (incidence by message position),
both lowered to SPMV_E2V.
"""
import pytest
import torch

import dgl
from dgl import kernel
from dgl.runtime import ir, spmv

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]

INC_EID = [[0, 0, 0, 0, 0, 0, 0],
           [0, 1, 1, 0, 0, 0, 0],
           [0, 0, 0, 0, 0, 0, 0],
           [0, 0, 0, 1, 0, 0, 0],
           [0, 0, 0, 0, 0, 1, 1]]
INC_DST = [[0, 0, 0, 0, 0],
           [1, 1, 0, 0, 0],
           [0, 0, 0, 0, 0],
           [0, 0, 1, 0, 0],
           [0, 0, 0, 1, 1]]


def _dense(adj, m, device):
    """The (n, m) matrix through both kernel routes: copy_u over I (columns)
    and copy_e over I (slot eids); they must agree."""
    eye = torch.eye(m, dtype=torch.float32, device=device)
    a = kernel.gspmm(adj, "copy_u", "sum", eye)
    b = kernel.gspmm(adj, "copy_e", "sum", None, eye)
    assert torch.equal(a, b)
    return a.cpu()


@pytest.mark.parametrize("device", DEVICES)
def test_build_inc_eid_known_answer(device):
    eid = torch.tensor([1, 2, 3, 5, 6])
    dst = torch.tensor([1, 1, 3, 4, 4])
    adj = spmv.build_inc_eid(7, eid, dst, torch.arange(5), torch.device(device))
    assert tuple(adj.shape) == (5, 7)
    assert torch.equal(_dense(adj, 7, device), torch.tensor(INC_EID, dtype=torch.float32))


@pytest.mark.parametrize("device", DEVICES)
def test_build_inc_dst_known_answer(device):
    dst = torch.tensor([1, 1, 3, 4, 4])
    adj = spmv.build_inc_dst(dst, torch.arange(5), torch.device(device))
    assert tuple(adj.shape) == (5, 5)
    assert torch.equal(_dense(adj, 5, device), torch.tensor(INC_DST, dtype=torch.float32))


def _seven_edge_graph(device):
    """Three edges into node 1 (eid 0-2), two into 3 (eid 3-4), two into 4
    (eid 5-6); nodes 0 and 2 have none. Edge feature x = one-hot of the eid."""
    g = dgl.DGLGraph()
    g.add_nodes(5)
    g.add_edges([0, 2, 3, 1, 4, 0, 3], [1, 1, 1, 3, 3, 4, 4])
    g.edata["x"] = torch.eye(7, dtype=torch.float32, device=device)
    g.ndata["o"] = torch.full((5, 7), -1.0, device=device)
    return g


def _msg(edges):
    return {"m": edges.data["x"]}


def _sum(name, out):
    return dgl.function.sum(name, out)


@pytest.mark.parametrize("device", DEVICES)
def test_recv_reduces_through_inc_eid(device):
    g = _seven_edge_graph(device)
    g.send([1, 2, 3, 5, 6], _msg)
    with ir.prog() as p:
        g.recv([0, 1, 2, 3, 4], _sum("m", "o"))
    ops = p.opcodes()
    assert "SPMV_E2V" in ops and "READ_ROW" not in ops[:ops.index("SPMV_E2V")]
    # every receiver is written: 0-degree rows get the sum's 0
    assert torch.equal(g.ndata["o"].cpu(), torch.tensor(INC_EID, dtype=torch.float32))


@pytest.mark.parametrize("device", DEVICES)
def test_send_and_recv_reduces_through_inc_dst(device):
    g = _seven_edge_graph(device)
    with ir.prog() as p:
        g.send_and_recv([1, 2, 3, 5, 6], _msg, _sum("m", "o"))
    assert "SPMV_E2V" in p.opcodes()
    o = g.ndata["o"].cpu()
    want = torch.tensor(INC_EID, dtype=torch.float32)
    # receivers are the unique destinations 1, 3, 4; rows 0 and 2 untouched
    assert torch.equal(o[[1, 3, 4]], want[[1, 3, 4]])
    assert torch.equal(o[[0, 2]], torch.full((2, 7), -1.0))
