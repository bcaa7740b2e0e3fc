"""The product path at Reddit row lengths against the reddit_rows golden
fixture (torch.sparse.mm on the reference's uncoalesced COO; see
tests/golden/portable.py and make_golden.py): 1.5M edges, F = 128, rows of
13k-54k in-edges, heavy parallel duplicates.

update_all(copy_src, sum) and update_all(src_mul_edge, sum), forward and
dH, through the DGLGraph API (scheduler -> cached CSR -> libdgl_hip: HIP
kernels on the MI355X, the library's host kernels on CPU), bit for bit over
the whole output (digest) and the stored rows. Heavy-row chunking is switched
off, the documented bit-exact setting (dgl.kernel.set_row_split("off")).
"""
import numpy as np
import pytest
import torch

import dgl
import dgl.function as fn
from dgl import kernel

from test_oracle import _reddit_rows_inputs

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


@pytest.mark.parametrize("device", DEVICES)
def test_update_all_reddit_rows_bit_exact(golden, device):
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    dev = torch.device(device)
    c, P, src, dst, H, W, G = _reddit_rows_inputs(golden)
    rows = torch.from_numpy(c["rows"])
    g = dgl.DGLGraph(multigraph=True)
    g.add_nodes(int(c["n"]))
    g.add_edges(torch.from_numpy(src), torch.from_numpy(dst))
    old = kernel.set_row_split("off")
    try:
        for msg, key in ((fn.copy_src("h", "m"), "copy"), (fn.src_mul_edge("h", "w", "m"), "mul")):
            h = torch.from_numpy(H).to(dev).requires_grad_(True)
            g.ndata["h"] = h
            g.edata["w"] = torch.from_numpy(W).to(dev)
            g.update_all(msg, fn.sum("m", "o"))
            out = g.ndata["o"]
            out.backward(torch.from_numpy(G).to(dev))
            o = out.detach().cpu().numpy()
            gh = h.grad.cpu().numpy()
            assert np.array_equal(o[rows], c[key + "_out_rows"]), key
            assert P.digest(o) == str(c["sha_%s_out" % key]), key
            assert np.array_equal(gh[rows], c[key + "_grad_h_rows"]), key
            assert P.digest(gh) == str(c["sha_%s_grad_h" % key]), key
    finally:
        kernel.set_row_split(old)
