"""The reference-side binding of the tensor-backend route
(dgl/backend/hip_tensor.py): sparse_matrix / spmm as the
reference's python/dgl/backend/pytorch/tensor.py:45-51,145-146 would call
them, bound to libdgl_hip.so with ctypes alone. The products (forward and the
autograd backward) equal torch.sparse.mm on the reference's uncoalesced COO
(graph.cc:509-524: row 0 = destinations, row 1 = sources, edge-id order)
bit for bit; the adjacency's CSR and plan are built once per matrix and
device, not per call."""
import numpy as np
import pytest
import torch

from dgl.backend import hip_tensor as B
from oracle import oracle as O


def _coo(n, m, seed, sorted_src=True):
    rng = np.random.default_rng(seed)
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n, m)
    if sorted_src:
        o = np.lexsort((dst, src))
        src, dst = src[o], dst[o]
    return src.astype(np.int64), dst.astype(np.int64)


@pytest.mark.parametrize("weighted", [False, True])
def test_binding_matches_torch_sparse_mm_host(weighted):
    n, m, F = 700, 20_000, 24
    src, dst = _coo(n, m, 1)
    idx = torch.from_numpy(np.stack([dst, src]))
    gen = torch.Generator().manual_seed(2)
    data = torch.rand(m, generator=gen) if weighted else torch.ones(m)
    y = torch.randn(n, F, generator=gen, requires_grad=True)
    y_ref = y.detach().clone().requires_grad_(True)
    mat, shuffle = B.sparse_matrix(data, ("coo", idx), (n, n))
    assert shuffle is None and B.sparse_matrix_indices(mat)[1] is idx
    out = B.spmm(mat, y)
    ref = torch.sparse.mm(torch.sparse_coo_tensor(idx, data, (n, n)), y_ref)
    assert torch.equal(out, ref)
    dc = torch.randn(n, F, generator=gen)
    out.backward(dc)
    ref.backward(dc)
    assert torch.equal(y.grad, y_ref.grad)
    # the matrix's CSR and plan are made once (per orientation and device)
    assert set(mat._st.dev) == {("cpu", False), ("cpu", True)}
    B.spmm(mat, y.detach())
    assert len(mat._st.dev) == 2
    if not weighted:
        assert np.array_equal(out.detach().numpy(), O.spmm_coo(n, dst, src, y.detach().numpy()))


def test_binding_rejects_csr_format():
    with pytest.raises(TypeError):
        B.sparse_matrix(torch.ones(3), ("csr", None, None), (3, 3))


@pytest.mark.gpu
def test_binding_on_device_blocked_and_bit_exact():
    """A Reddit-shaped graph (quarter scale: 58k nodes, 28.7M edges) through
    the binding on the MI355X: the plan's source-blocked schedule, the
    oracle's bits forward and backward with every row one chain
    (row_split 0), with no upload per call. Under the default policy this
    graph's hub rows (in-degree up to 17,086 against a mean of 493) are the
    launch's critical path and are chunked: within 1e-5 of each row's Σ|x|
    (DESIGN.md §2)."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from dgl import data, kernel
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(scale=0.25, seed=0, device=dev)
    idx = torch.stack([dst, src])
    m = src.numel()
    mat, _ = B.sparse_matrix(torch.ones(m, device=dev), ("coo", idx), (n, n))
    gen = torch.Generator(device=dev).manual_seed(3)
    y0 = torch.rand(n, 128, generator=gen, device=dev) * 2 - 1
    dc = torch.rand(n, 128, generator=gen, device=dev) * 2 - 1
    s_np, d_np = src.cpu().numpy(), dst.cpu().numpy()
    fwd = O.coo_to_csr(n, d_np, s_np)
    bwd = O.coo_to_csr(n, s_np, d_np)
    ref_out = O.spmm_csr(*fwd, y0.cpu().numpy(), num_threads=16)
    ref_dy = O.spmm_csr(*bwd, dc.cpu().numpy(), num_threads=16)
    with kernel.scheduled(row_split=0):
        y = y0.clone().requires_grad_(True)
        out = B.spmm(mat, y)
        out.backward(dc)
        assert np.array_equal(out.detach().cpu().numpy(), ref_out)
        assert np.array_equal(y.grad.cpu().numpy(), ref_dy)
    y = y0.clone().requires_grad_(True)
    out = B.spmm(mat, y)
    out.backward(dc)
    for got, csr, x, ref in ((out.detach(), fwd, y0, ref_out), (y.grad, bwd, dc, ref_dy)):
        mag = O.spmm_csr(*csr, np.abs(x.cpu().numpy()), num_threads=16)
        assert np.all(np.abs(got.cpu().numpy() - ref) <= 1e-5 * mag + 1e-30)
    # blocked launches per product, none of them a sort or a copy
    kernel.timing_enable(True)
    B.spmm(mat, y.detach())
    _, launches = kernel.timing_read()
    kernel.timing_enable(False)
    assert launches >= 2


def _executor_spmv_with_data(adj, a_data, h):
    """SPMVWithDataExecutor.run's sequence
    (/root/reference/python/dgl/runtime/ir/executor.py:535-566) on a cached
    adjacency ``adj``: its index, a matrix rebuilt on it with the edge data,
    then spmm."""
    if a_data.dim() > 1:
        a_data = a_data.squeeze(1)
    spidx = B.sparse_matrix_indices(adj)
    spa, _ = B.sparse_matrix(a_data, spidx, adj.shape)
    return B.spmm(spa, h)


def _dot_bound(row, col, dc, h):
    """float64 per-edge dot and its Σ|dc·h| (the fp32 dot's condition bound)."""
    return O.sddmm_dot(row, col, dc, h), O.sddmm_dot(row, col, np.abs(dc), np.abs(h))


@pytest.mark.parametrize("dup,sorted_src", [(False, True), (True, True), (False, False)])
def test_spmv_with_data_sequence_host(dup, sorted_src):
    """The executor's src_mul_edge sequence, twice, on the host, with a
    learnable (E, 1) edge weight: output and dH equal torch.sparse.mm on the
    same COO bit for bit, d(weights) is torch's value gradient (every
    duplicate gets the full dot) within 1e-5 of the float64 dot, and the
    second call builds nothing. Source-sorted edges take the transposed
    walk for the weight gradient, unsorted ones the forward walk."""
    n, m, F = 600, 15_000, 20
    src, dst = _coo(n, m, 5, sorted_src)
    if dup:  # multigraph: repeated (dst, src) pairs stay separate COO positions
        src[1::7], dst[1::7] = src[0::7][:len(src[1::7])], dst[0::7][:len(dst[1::7])]
    idx = torch.from_numpy(np.stack([dst, src]))
    adj, _ = B.sparse_matrix(torch.ones(m), ("coo", idx), (n, n))
    assert adj.ones
    gen = torch.Generator().manual_seed(6)
    for call in range(2):
        before = B.builds
        w = torch.rand(m, 1, generator=gen).requires_grad_(True)
        h = torch.randn(n, F, generator=gen).requires_grad_(True)
        dc = torch.randn(n, F, generator=gen)
        out = _executor_spmv_with_data(adj, w, h)
        out.backward(dc)
        w_ref = w.detach().clone().requires_grad_(True)
        h_ref = h.detach().clone().requires_grad_(True)
        ref = torch.sparse.mm(torch.sparse_coo_tensor(idx, w_ref.squeeze(1), (n, n)), h_ref)
        ref.backward(dc)
        assert torch.equal(out, ref)
        assert torch.equal(h.grad, h_ref.grad)
        assert w.grad.shape == (m, 1)
        want, mag = _dot_bound(dst, src, dc.numpy(), h.detach().numpy())
        got = w.grad.squeeze(1).numpy()
        assert np.all(np.abs(got - want) <= 1e-5 * mag + 1e-30)
        assert np.allclose(got, w_ref.grad.squeeze(1).numpy(), rtol=1e-5, atol=1e-5 * np.abs(want).max())
        if call == 1:
            assert B.builds == before  # the cached adjacency's CSRs and plans
    # a weight that asks for no gradient gets none; the dense operand still does
    h = torch.randn(n, F, generator=gen).requires_grad_(True)
    _executor_spmv_with_data(adj, torch.rand(m, generator=gen), h).sum().backward()
    assert h.grad is not None


def test_binding_rejects_non_float32_dense():
    """torch.sparse.mm raises on a dense operand of another dtype; so does
    the binding (it never reads float64 bytes as float32)."""
    idx = torch.tensor([[0, 1], [1, 0]])
    mat, _ = B.sparse_matrix(torch.ones(2), ("coo", idx), (2, 2))
    with pytest.raises(RuntimeError):
        B.spmm(mat, torch.ones(2, 3, dtype=torch.float64))


def test_structure_cache_follows_the_index_tensor():
    """The CSR cache is keyed by the index tensor itself: a new index (or
    one written in place) builds anew, and the entry leaves with its tensor."""
    import gc
    idx = torch.tensor([[0, 1, 1], [1, 0, 1]])
    y = torch.ones(2, 4)
    mat, _ = B.sparse_matrix(torch.ones(3), ("coo", idx), (2, 2))
    B.spmm(mat, y)
    b0 = B.builds
    B.spmm(B.sparse_matrix(torch.rand(3), B.sparse_matrix_indices(mat), (2, 2))[0], y)
    assert B.builds == b0
    idx[1, 2] = 0  # in-place write: the cached CSR no longer describes it
    out = B.spmm(B.sparse_matrix(torch.ones(3), ("coo", idx), (2, 2))[0], y)
    assert B.builds == b0 + 1 and torch.equal(out, torch.tensor([[1.] * 4, [2.] * 4]))
    key = id(idx)
    del mat, idx
    gc.collect()
    assert key not in B._structures


@pytest.mark.gpu
def test_spmv_with_data_sequence_reddit_device():
    """The executor's SPMV_WITH_DATA sequence twice on the full Reddit-shaped
    graph (232,965 nodes, 114.8M edges, F = 128) on the MI355X, with
    ``A_data.requires_grad``: output and dH equal the oracle's weighted fma
    chains bit for bit, d(A_data) is within 1e-5·Σ|dC·H| of the float64 dot
    (a seeded sample of 2M edges plus both ends), and the second call builds
    no CSR, sort or plan."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from dgl import data
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(scale=1, seed=0, device=dev)
    idx = torch.stack([dst, src])
    m, F = src.numel(), 128
    adj, _ = B.sparse_matrix(torch.ones(m, device=dev), ("coo", idx), (n, n))
    s_np, d_np = src.cpu().numpy(), dst.cpu().numpy()
    fwd = O.coo_to_csr(n, d_np, s_np)
    bwd = O.coo_to_csr(n, s_np, d_np)
    gen = torch.Generator(device=dev).manual_seed(7)
    rng = np.random.default_rng(7)
    sample = np.concatenate([[0, m - 1], rng.integers(0, m, 2_000_000)])
    for call in range(2):
        before = B.builds
        w = (torch.rand(m, 1, generator=gen, device=dev)).requires_grad_(True)
        h = (torch.rand(n, F, generator=gen, device=dev) * 2 - 1).requires_grad_(True)
        dc = torch.rand(n, F, generator=gen, device=dev) * 2 - 1
        out = _executor_spmv_with_data(adj, w, h)
        out.backward(dc)
        torch.cuda.synchronize()
        if call == 1:
            assert B.builds == before
        else:
            assert B.builds == before + 2  # forward + transpose, once
        w_np = w.detach().squeeze(1).cpu().numpy()
        h_np, dc_np = h.detach().cpu().numpy(), dc.cpu().numpy()
        assert np.array_equal(out.detach().cpu().numpy(),
                              O.spmm_csr(*fwd, h_np, val=w_np, num_threads=16))
        assert np.array_equal(h.grad.cpu().numpy(),
                              O.spmm_csr(*bwd, dc_np, val=w_np, num_threads=16))
        got = w.grad.squeeze(1).cpu().numpy()[sample]
        want, mag = _dot_bound(d_np[sample], s_np[sample], dc_np, h_np)
        assert np.all(np.abs(got - want) <= 1e-5 * mag + 1e-30)
