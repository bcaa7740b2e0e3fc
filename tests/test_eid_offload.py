"""SparseAdj.offload_edge_ids (kernel.CSR.offload_eid): the CSRs' edge-id
arrays move to host memory for graphs whose messages read node features
only (17 GB of HBM at RMAT-26's 1.07B edges, the configs[3] model step), and
come back on the first operation that reads them, with the same results."""
import pytest
import torch

from dgl import kernel


@pytest.mark.gpu
def test_offload_and_restore_edge_ids():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    dev = torch.device("cuda", 0)
    gen = torch.Generator().manual_seed(0)
    n, m = 5000, 200_000
    src = torch.randint(0, n, (m,), generator=gen)
    dst = torch.randint(0, n, (m,), generator=gen)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    h = torch.randn(n, 64, generator=gen).to(dev).requires_grad_(True)
    w = torch.randn(m, generator=gen).to(dev)
    ref_sum = kernel.gspmm(adj, "copy_u", "mean", h)
    (ref_grad,) = torch.autograd.grad(ref_sum.sum(), h)
    ref_mul = kernel.gspmm(adj, "u_mul_e", "sum", h.detach(), w)
    adj.offload_edge_ids()
    assert adj.fwd._eid is None and adj.fwd._eid_host.device.type == "cpu"
    # node-feature messages and their transposed backward never read eid
    out = kernel.gspmm(adj, "copy_u", "mean", h)
    (grad,) = torch.autograd.grad(out.sum(), h)
    assert torch.equal(out, ref_sum) and torch.equal(grad, ref_grad)
    assert adj.fwd._eid is None and adj.bwd._eid is None
    # an edge-feature message brings it back, same bits
    assert torch.equal(kernel.gspmm(adj, "u_mul_e", "sum", h.detach(), w), ref_mul)
    assert adj.fwd._eid is not None and adj.fwd._eid.device == dev
