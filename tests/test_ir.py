"""The message-passing mini-IR (runtime/ir, runtime/runtime.py; the
reference's python/dgl/runtime/ir/{executor,program,var}.py and
runtime/runtime.py): each API call lowers to a program of executors that
the runtime runs in order. Checks the programs the scheduler emits for the
reference's lowering cases, the variables' types, pprint, nesting, and a
program built and run by hand."""
import pytest
import torch

import dgl
import dgl.function as fn
from dgl.runtime import ir
from dgl.runtime.ir import var
from dgl.runtime.runtime import Runtime


def _graph():
    g = dgl.DGLGraph()
    g.add_nodes(5)
    g.add_edges([0, 1, 2, 3, 4, 0], [1, 2, 3, 4, 0, 2])
    g.ndata["h"] = torch.arange(10, dtype=torch.float32).reshape(5, 2)
    g.edata["w"] = torch.arange(6, dtype=torch.float32).reshape(6, 1)
    return g


def test_update_all_builtin_program():
    g = _graph()
    with ir.prog() as p:
        g.update_all(fn.copy_src("h", "m"), fn.sum("m", "o"))
    assert p.opcodes() == ["NEW_DICT", "READ_COL", "SPMV", "WRITE_COL_", "WRITE_DICT_"]
    spmv = [e for e in p.trace if e.opcode() == ir.OpCode.SPMV][0]
    spmat, feat, red = spmv.arg_vars()
    assert spmat.typecode == var.VarType.SPMAT and feat.typecode == var.VarType.FEAT
    assert red.data == "sum" and spmv.ret_var().typestr() == "Feat"
    text = p.pprint()
    assert "Feat _z" in text and "SPMV(" in text and 'WRITE_DICT_(nf' in text
    assert torch.equal(g.ndata["o"][2], g.ndata["h"][1] + g.ndata["h"][0])


def test_src_mul_edge_and_copy_edge_programs():
    g = _graph()
    with ir.prog() as p:
        g.update_all([fn.src_mul_edge("h", "w", "m"), fn.copy_edge("w", "z")],
                      [fn.sum("m", "o"), fn.max("z", "zz")])
    ops = p.opcodes()
    assert "SPMV_WITH_DATA" in ops and "SPMV_E2V" in ops and "EDGE_UDF" not in ops


def test_udf_programs():
    g = _graph()
    with ir.prog() as p:
        g.update_all(lambda e: {"m": e.src["h"] * 2}, fn.sum("m", "o"))
    assert p.opcodes()[-4:-1] == ["READ_COL", "SPMV_E2V", "WRITE_COL_"]
    assert "EDGE_UDF" in p.opcodes() and p.opcodes()[-1] == "WRITE_DICT_"
    with ir.prog() as p:
        g.update_all(fn.copy_src("h", "m"), lambda nodes: {"o": nodes.mailbox["m"].sum(1)},
                     lambda nodes: {"o": nodes.data["o"] + 1})
    assert "DEGREE_BUCKETING" in p.opcodes() and "NODE_UDF" in p.opcodes()
    assert p.opcodes()[-1] == "WRITE_DICT_"


def test_send_recv_and_row_writes():
    g = _graph()
    with ir.prog() as p:
        g.send_and_recv(([0, 1], [1, 2]), fn.copy_src("h", "m"), fn.sum("m", "o"))
    assert p.opcodes()[-1] == "WRITE_ROW_"
    with ir.prog() as p:
        g.send(([0, 1], [1, 2]), lambda e: {"m": e.src["h"]})
        g.recv([1, 2], fn.sum("m", "o"))
    ops = p.opcodes()
    assert ops[:3] == ["EDGE_UDF", "WRITE_ROW_", "CALL_"]
    assert ops[-1] == "CALL_" and "SPMV_E2V" in ops
    with ir.prog() as p:
        g.apply_nodes(lambda nodes: {"h": nodes.data["h"] * 1}, inplace=True)
    assert p.opcodes() == ["READ_ROW", "NODE_UDF", "WRITE_ROW_INPLACE_"]


def test_hand_built_program():
    """Issue executors directly and run them: READ_COL -> SPMV -> WRITE_COL_."""
    from dgl import kernel
    adj = kernel.from_coo(3, 3, [1, 2, 2], [0, 0, 1], kernel.ORDER_EID, "cpu")
    fd = {"h": torch.tensor([[1.0], [2.0], [4.0]])}
    with ir.prog() as p:
        fdv = var.FEAT_DICT(fd, "fd")
        h = ir.READ_COL(fdv, var.STR("h"))
        out = ir.SPMV(var.SPMAT(adj, "A"), h, var.STR("sum"))
        ir.WRITE_COL_(fdv, var.STR("o"), out)
        assert [e.opcode() for e in p.execs] == [ir.OpCode.READ_COL, ir.OpCode.SPMV,
                                                ir.OpCode.WRITE_COL_]
        assert out.data is None  # symbolic until the program runs
        Runtime.run(p)
    assert fd["o"].flatten().tolist() == [0.0, 1.0, 3.0]
    assert ir.IR_REGISTRY[ir.OpCode.SPMV]["name"] == "SPMV"


def test_issue_outside_program_fails():
    with pytest.raises(RuntimeError):
        ir.NEW_DICT()
