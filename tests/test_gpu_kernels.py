"""HIP kernels through the C-ABI vs the oracle, on the MI355X.

Bit-exact for integer CSR arrays and for the reference-arithmetic products
(copy_u / u_mul_e + sum, max); tolerance 1e-5 (north_star) for mean and the
SDDMM dot. Shapes sweep the kernel's (VEC, GROUP) specialisations, empty and
ragged inputs, multigraph duplicates and a Reddit-degree-scale row set.
"""
import ctypes

import numpy as np
import pytest
import torch

import dgl
from dgl import _ffi, kernel
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda", 0)


def rand_graph(rng, n_rows, n_cols, nnz, skew=False):
    if skew:  # power-law destinations: a few very long rows
        p = 1.0 / np.arange(1, n_rows + 1) ** 1.1
        row = rng.choice(n_rows, size=nnz, p=p / p.sum())
    else:
        row = rng.integers(0, n_rows, nnz)
    col = rng.integers(0, n_cols, nnz)
    return row.astype(np.int64), col.astype(np.int64)


@pytest.mark.parametrize("F", [1, 2, 3, 7, 16, 41, 64, 128, 256, 500])
def test_gspmm_copy_u_sum_exact(cuda, F):
    rng = np.random.default_rng(F)
    n = 3000
    row, col = rand_graph(rng, n, n, 40000, skew=True)
    H = rng.standard_normal((n, F)).astype(np.float32)
    adj = kernel.from_coo(n, n, row, col, kernel.ORDER_EID, cuda)
    out = kernel.gspmm(adj, "copy_u", "sum", torch.from_numpy(H).to(cuda))
    ref = O.spmm_coo(n, row, col, H)
    assert np.array_equal(out.cpu().numpy().reshape(n, F), ref)


@pytest.mark.parametrize("F", [1, 5, 100, 128, 200, 256, 602])
@pytest.mark.parametrize("edge_len", ["scalar", "vector"])
def test_gspmm_u_mul_e_sum(cuda, F, edge_len):
    """F = 100 / 200 / 602 leave lanes idle in the last feature pass; skewed
    rows run past the unroll depth many times."""
    rng = np.random.default_rng(7)
    n, m = 500, 20000  # many duplicate (row, col) pairs
    row, col = rand_graph(rng, n, 60, m, skew=True)
    H = rng.standard_normal((60, F)).astype(np.float32)
    W = rng.standard_normal((m, 1 if edge_len == "scalar" else F)).astype(np.float32)
    adj = kernel.from_coo(n, 60, row, col, kernel.ORDER_EID, cuda)
    out = kernel.gspmm(adj, "u_mul_e", "sum", torch.from_numpy(H).to(cuda),
                       torch.from_numpy(W).to(cuda)).cpu().numpy().reshape(n, F)
    if edge_len == "scalar":
        assert np.array_equal(out, O.spmm_coo(n, row, col, H, W[:, 0]))
    else:
        ref = np.zeros((n, F), np.float32)
        for f in range(F):
            ref[:, f] = O.spmm_coo(n, row, col, H[:, f:f + 1], W[:, f])[:, 0]
        assert np.array_equal(out, ref)


@pytest.mark.parametrize("F", [64, 128, 602])
def test_gspmm_slot_ordered_edge_values(cuda, F):
    """eid = NULL: edge values already in CSR slot order give the same bits as
    the eid-indexed call (copy_e and u_mul_e, sum and mean)."""
    rng = np.random.default_rng(F + 1)
    n = 400
    row, col = rand_graph(rng, n, n, 30000, skew=True)
    adj = kernel.from_coo(n, n, row, col, kernel.ORDER_EID, cuda)
    csr = adj.fwd
    H = torch.from_numpy(rng.standard_normal((n, F)).astype(np.float32)).to(cuda)
    W = torch.from_numpy(rng.standard_normal((len(row), 1)).astype(np.float32)).to(cuda)
    Ws = W.index_select(0, csr.eid).contiguous()
    stream = torch.cuda.current_stream(cuda).cuda_stream
    for msg in (1, 2):
        for red in (0, 2):
            outs = []
            for eid, w in ((csr.eid, W), (None, Ws)):
                o = torch.empty(n, F, device=cuda)
                _ffi.check_call(_ffi.LIB.dglhip_gspmm_device(
                    msg, red, n, F, _ffi.ptr(csr.indptr), _ffi.ptr(csr.indices),
                    None if eid is None else _ffi.ptr(eid), _ffi.ptr(H), _ffi.ptr(w), 1,
                    _ffi.ptr(o), None, None, stream))
                outs.append(o)
            torch.cuda.synchronize()
            assert torch.equal(outs[0], outs[1]), (msg, red)
    ref = O.spmm_coo(n, row, col, H.cpu().numpy(), W.cpu().numpy()[:, 0])
    o = torch.empty(n, F, device=cuda)
    _ffi.check_call(_ffi.LIB.dglhip_gspmm_device(1, 0, n, F, _ffi.ptr(csr.indptr),
                                                 _ffi.ptr(csr.indices), None, _ffi.ptr(H),
                                                 _ffi.ptr(Ws), 1, _ffi.ptr(o), None, None,
                                                 stream))
    torch.cuda.synchronize()
    assert np.array_equal(o.cpu().numpy(), ref)


def test_gspmm_max_and_mean(cuda):
    rng = np.random.default_rng(11)
    n, F = 700, 33
    row, col = rand_graph(rng, n, n, 9000, skew=True)
    H = rng.standard_normal((n, F)).astype(np.float32)
    adj = kernel.from_coo(n, n, row, col, kernel.ORDER_EID, cuda)
    Hd = torch.from_numpy(H).to(cuda)
    mx = kernel.gspmm(adj, "copy_u", "max", Hd).cpu().numpy()
    assert np.array_equal(mx, O.max_mailbox(n, row, H[col]))
    mn = kernel.gspmm(adj, "copy_u", "mean", Hd).cpu().numpy()
    np.testing.assert_allclose(mn, O.mean_mailbox(n, row, H[col]), rtol=1e-5, atol=1e-6)


def test_empty_and_degenerate(cuda):
    for n, nnz in ((0, 0), (5, 0), (1, 1)):
        row = np.zeros(nnz, np.int64)
        adj = kernel.from_coo(n, max(n, 1), row, row, kernel.ORDER_EID, cuda)
        H = torch.ones(max(n, 1), 4, device=cuda)
        out = kernel.gspmm(adj, "copy_u", "sum", H)
        assert out.shape == (n, 4)
        assert out.sum().item() == float(nnz * 4)


@pytest.mark.parametrize("order", [kernel.ORDER_EID, kernel.ORDER_COL])
def test_device_csr_builder_matches_host(cuda, order):
    rng = np.random.default_rng(5)
    # the last shape's (row, col) keys need more than 32 bits: the 64-bit sort
    for n_rows, n_cols, nnz in ((1, 1, 0), (10, 7, 100), (5000, 3000, 200000),
                                (70000, 70000, 300000)):
        row, col = rand_graph(rng, n_rows, n_cols, nnz)
        h = kernel.build_csr(n_rows, n_cols, row, col, order, "cpu")
        d = kernel.build_csr(n_rows, n_cols, row, col, order, cuda)
        assert torch.equal(h.indptr, d.indptr.cpu())
        assert torch.equal(h.indices, d.indices.cpu())
        assert torch.equal(h.eid, d.eid.cpu())
        assert torch.equal(h.row_order, d.row_order.cpu())
        if order == kernel.ORDER_EID and nnz:
            ip, ix, pos = O.coo_to_csr(n_rows, row, col)
            assert np.array_equal(h.indptr.numpy(), ip)
            assert np.array_equal(h.indices.numpy().astype(np.int64), ix)
            assert np.array_equal(h.eid.numpy(), pos)


def test_backward_transposed(cuda):
    rng = np.random.default_rng(9)
    n, F = 2000, 128
    row, col = rand_graph(rng, n, n, 50000, skew=True)
    H = torch.from_numpy(rng.standard_normal((n, F)).astype(np.float32)).to(cuda)
    G = rng.standard_normal((n, F)).astype(np.float32)
    W = rng.standard_normal(len(row)).astype(np.float32)
    adj = kernel.from_coo(n, n, row, col, kernel.ORDER_EID, cuda)
    Hr = H.clone().requires_grad_(True)
    kernel.gspmm(adj, "copy_u", "sum", Hr).backward(torch.from_numpy(G).to(cuda))
    assert np.array_equal(Hr.grad.cpu().numpy(), O.spmm_coo(n, col, row, G))
    Hr = H.clone().requires_grad_(True)
    Wd = torch.from_numpy(W).to(cuda).requires_grad_(True)
    kernel.gspmm(adj, "u_mul_e", "sum", Hr, Wd).backward(torch.from_numpy(G).to(cuda))
    assert np.array_equal(Hr.grad.cpu().numpy(), O.spmm_coo(n, col, row, G, W))
    np.testing.assert_allclose(Wd.grad.cpu().numpy(),
                               O.sddmm_dot(row, col, G, H.cpu().numpy()), rtol=1e-5, atol=1e-4)


def test_large_reddit_scale_rows(cuda):
    """Long power-law rows at F=128 (the bench shape). With the bit-exact
    switch (row split "off") exact vs the OpenMP oracle. Row 0 holds ~1M of
    the 8M slots, so the default policy ("auto") cuts it into chunks: that
    result must stay within 1e-5 of the oracle's chain, measured against the
    row's condition scale sum_k |H[col_k]| (the summation error bound)."""
    rng = np.random.default_rng(1)
    n = 200000
    row, col = rand_graph(rng, n, n, 8_000_000, skew=True)
    H = rng.uniform(-1, 1, (n, 128)).astype(np.float32)
    adj = kernel.from_coo(n, n, row, col, kernel.ORDER_EID, cuda)
    Hd = torch.from_numpy(H).to(cuda)
    ip, ix, pos = O.coo_to_csr(n, row, col)
    ref = O.spmm_csr(ip, ix, pos, H, num_threads=16)
    old = kernel.set_row_split("off")
    try:
        out = kernel.gspmm(adj, "copy_u", "sum", Hd).cpu().numpy()
    finally:
        kernel.set_row_split(old)
    assert np.array_equal(out, ref)
    old = kernel.set_row_split("auto")
    try:
        assert kernel._split_threshold(adj.fwd) > 0
        out = kernel.gspmm(adj, "copy_u", "sum", Hd).cpu().numpy()
    finally:
        kernel.set_row_split(old)
    scale = O.spmm_csr(ip, ix, pos, np.abs(H), num_threads=16)
    assert np.all(np.abs(out - ref) <= 1e-5 * scale + 1e-30)


def test_packed_func_on_device(cuda):
    rng = np.random.default_rng(2)
    n = 100
    row, col = rand_graph(rng, n, n, 1000)
    csr = kernel.build_csr(n, n, row, col, kernel.ORDER_EID, cuda)
    H = torch.from_numpy(rng.standard_normal((n, 8)).astype(np.float32)).to(cuda)
    out = torch.empty(n, 8, device=cuda)
    stream = torch.cuda.current_stream().cuda_stream
    _ffi.call_packed("dglhip._CAPI_GSpMM", 0, 0, csr.indptr, csr.indices, csr.eid, H, None,
                     out, None, csr.row_order, ("handle", stream))
    assert np.array_equal(out.cpu().numpy(), O.spmm_coo(n, row, col, H.cpu().numpy()))


def test_timing_hooks(cuda):
    n = 1000
    row = np.arange(n, dtype=np.int64)
    adj = kernel.from_coo(n, n, row, row, kernel.ORDER_EID, cuda)
    H = torch.ones(n, 128, device=cuda)
    kernel.timing_enable(True)
    for _ in range(3):
        kernel.gspmm(adj, "copy_u", "sum", H)
    ms, launches = kernel.timing_read()
    kernel.timing_enable(False)
    assert launches == 3 and ms > 0


@pytest.mark.parametrize("msg", ["copy_u", "u_mul_e"])
@pytest.mark.parametrize("reduce", ["sum", "mean"])
def test_heavy_row_split(cuda, msg, reduce):
    """Chunked heavy rows: deterministic, within the north-star 1e-5 of the
    exact chain; light rows stay bit-exact."""
    rng = np.random.default_rng(13)
    n, F = 4000, 128
    row, col = rand_graph(rng, n, n, 300000, skew=True)
    H = rng.uniform(-1, 1, (n, F)).astype(np.float32)
    W = rng.uniform(0.5, 1.5, len(row)).astype(np.float32)
    adj = kernel.from_coo(n, n, row, col, kernel.ORDER_EID, cuda)
    Hd, Wd = torch.from_numpy(H).to(cuda), torch.from_numpy(W).to(cuda)
    ef = Wd if msg == "u_mul_e" else None
    exact = kernel.gspmm(adj, msg, reduce, Hd, ef).cpu().numpy()
    old = kernel.set_row_split(1000)
    try:
        split1 = kernel.gspmm(adj, msg, reduce, Hd, ef).cpu().numpy()
        split2 = kernel.gspmm(adj, msg, reduce, Hd, ef).cpu().numpy()
    finally:
        kernel.set_row_split(old)
    assert np.array_equal(split1, split2)  # deterministic
    deg = np.bincount(row, minlength=n)
    assert (deg > 1000).sum() > 0
    light = deg <= 1000
    assert np.array_equal(split1[light], exact[light])
    scale = np.abs(exact).max()
    np.testing.assert_allclose(split1, exact, rtol=1e-5, atol=1e-5 * scale)


@pytest.mark.parametrize("F", [128, 41])
def test_full_reddit_bench_graph_bit_exact(cuda, F):
    """The bench workload at full size (BASELINE configs[1] shape: 232,965 nodes,
    114.8M edges; F=128, and GCN's 41-class layer) through update_all on the
    MI355X == the oracle's multi-core restatement, bit for bit: the forward
    and the backward dH = A^T dC (both on the source-blocked schedule)."""
    import dgl.function as fn
    from dgl import data
    src, dst, n = data.reddit_like(scale=1, seed=0, device=cuda)
    gen = torch.Generator(device=cuda).manual_seed(1)
    h = (torch.rand(n, F, generator=gen, device=cuda) * 2 - 1).requires_grad_(True)
    dc = torch.rand(n, F, generator=gen, device=cuda) * 2 - 1
    g = dgl.DGLGraph((src.cpu(), dst.cpu()))
    g.ndata["h"] = h
    g.update_all(fn.copy_src("h", "m"), fn.sum("m", "o"))
    g.ndata["o"].backward(dc)
    out = g.ndata["o"].detach().cpu().numpy()
    s_np, d_np = src.cpu().numpy(), dst.cpu().numpy()
    ip, ix, pos = O.coo_to_csr(n, d_np, s_np)
    ref = O.spmm_csr(ip, ix, pos, h.detach().cpu().numpy(), num_threads=16)
    assert np.array_equal(out, ref)
    ip, ix, pos = O.coo_to_csr(n, s_np, d_np)  # the transpose, slots in edge-id order
    ref_grad = O.spmm_csr(ip, ix, pos, dc.cpu().numpy(), num_threads=16)
    assert np.array_equal(h.grad.cpu().numpy(), ref_grad)


@pytest.mark.parametrize("F,H", [(32, 1), (64, 8), (128, 1), (128, 2), (128, 4), (128, 8),
                                 (128, 32), (64, 2),
                                 (256, 2), (512, 4), (5, 1), (48, 3), (96, 3), (256, 64)])
def test_gsddmm_dot_heads(cuda, F, H):
    """Per-head dot products out[eid, h] = <lhs[row, h], rhs[col, h]>: the
    8-lanes-per-slot kernel (F = 32 * {1,2,4,8,16}, head width 4/8/16 or a
    multiple of 32) and the per-slot kernel for other shapes, vs float64,
    deterministic across calls; skewed rows run through many slot groups and
    empty rows write nothing."""
    rng = np.random.default_rng(F * 31 + H)
    n = 600
    row, col = rand_graph(rng, n, n, 20000, skew=True)
    A = rng.standard_normal((n, F)).astype(np.float32)
    B = rng.standard_normal((n, F)).astype(np.float32)
    adj = kernel.from_coo(n, n, row, col, kernel.ORDER_EID, cuda)
    Ad, Bd = torch.from_numpy(A).to(cuda), torch.from_numpy(B).to(cuda)
    out = kernel.gsddmm_dot(adj, Ad, Bd, len(row), H).cpu().numpy()
    again = kernel.gsddmm_dot(adj, Ad, Bd, len(row), H).cpu().numpy()
    assert np.array_equal(out, again)
    D = F // H
    ref = (A[row].astype(np.float64).reshape(-1, H, D) *
           B[col].astype(np.float64).reshape(-1, H, D)).sum(-1)
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-4)


def test_rows_beyond_one_grid_dimension(cuda):
    """2^26 + 5 rows of one in-edge each at F = 16 (one wave per row): the
    launch folds into a 2-D grid (a 1-D grid of 2^26 waves is 2^32 lanes, past
    the per-dimension limit; RMAT-26 without heavy-row chunking hit it). Every
    row's result is checked: sum, mean, max (one slot each = the source row)
    and the per-edge g-SDDMM dot."""
    n = (1 << 26) + 5
    g = torch.Generator(device=cuda).manual_seed(3)
    col = torch.randperm(n, generator=g, device=cuda)
    row = torch.arange(n, device=cuda)
    adj = kernel.from_coo(n, n, row, col, kernel.ORDER_EID, cuda)
    H = torch.rand(n, 16, generator=g, device=cuda)
    expect = H.index_select(0, col)
    for red in ("sum", "mean", "max"):
        out = kernel.gspmm(adj, "copy_u", red, H)
        assert torch.equal(out, expect), red
        del out
    dots = kernel.gsddmm_dot(adj, H, H, n, 1)
    ref = (H * expect).sum(1, keepdim=True)
    torch.testing.assert_close(dots, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("F", [24, 41, 50])
@pytest.mark.parametrize("case", ["copy_u-sum", "copy_u-mean", "u_mul_e-sum"])
def test_padded_stride_gather(cuda, F, case):
    """Source rows that straddle cache lines (F = 24, 41, 50) are gathered
    from a padded copy (kernel.padded_width) once the table exceeds the L2s:
    the same chains, so the result equals the in-place gather bit for bit
    (and the oracle for sum)."""
    msg, red = case.split("-")
    rng = np.random.default_rng(F)
    n = (kernel.schedule_policy()["pad_min_bytes"] // (4 * F)) + 1000
    row, col = rand_graph(rng, n, n, 400_000, skew=True)
    H = rng.uniform(-1, 1, (n, F)).astype(np.float32)
    W = rng.uniform(-1, 1, (400_000, 1)).astype(np.float32)
    adj = kernel.from_coo(n, n, row, col, kernel.ORDER_EID, cuda)
    old_split = kernel.set_row_split("off")  # every row one chain: the padded path
    Hd = torch.from_numpy(H).to(cuda)
    Wd = torch.from_numpy(W).to(cuda) if msg == "u_mul_e" else None
    assert kernel.padded_width(F) > F
    assert kernel._pad_rows(kernel._MSG_NAMES[msg], kernel._RED_NAMES[red], Hd, F)
    padded = kernel.gspmm(adj, msg, red, Hd, Wd)
    old = kernel.set_pad_rows("off")
    try:
        plain = kernel.gspmm(adj, msg, red, Hd, Wd)
    finally:
        kernel.set_pad_rows(old)
    kernel.set_row_split(old_split)
    assert torch.equal(padded, plain)
    if case == "copy_u-sum":
        assert np.array_equal(padded.cpu().numpy(), O.spmm_coo(n, row, col, H))


@pytest.mark.parametrize("F", [41, 24])
@pytest.mark.parametrize("red", ["sum", "mean"])
def test_padded_stride_with_split_and_tiers(cuda, F, red):
    """The padded-stride gather composes with the heavy-row split (chunked
    entry) and the short-row tiers (GraphSAGE's F = 41 layer on RMAT takes all
    three): every combination of the three switches gives the same bits as
    the plain gather under the same split setting, and the oracle for sum
    without the split."""
    rng = np.random.default_rng(F + 7)
    n = 300_000
    row, col = rand_graph(rng, n, n, 900_000, skew=True)
    H = rng.uniform(-1, 1, (n, F)).astype(np.float32)
    adj = kernel.from_coo(n, n, row, col, kernel.ORDER_EID, cuda)
    Hd = torch.from_numpy(H).to(cuda)
    assert kernel._pad_rows(kernel._MSG_NAMES["copy_u"], kernel._RED_NAMES[red], Hd, F)
    outs = {}
    for split in ("off", 2000):
        for pad in ("auto", "off"):
            for tiered in (True, False):
                old_s, old_p = kernel.set_row_split(split), kernel.set_pad_rows(pad)
                old_t = kernel.set_short_rows(tiered)
                try:
                    outs[(split, pad, tiered)] = kernel.gspmm(adj, "copy_u", red, Hd)
                finally:
                    kernel.set_row_split(old_s)
                    kernel.set_pad_rows(old_p)
                    kernel.set_short_rows(old_t)
    for split in ("off", 2000):
        ref = outs[(split, "off", False)]
        for key, o in outs.items():
            if key[0] == split:
                assert torch.equal(o, ref), key
    if red == "sum":
        assert np.array_equal(outs[("off", "auto", True)].cpu().numpy(), O.spmm_coo(n, row, col, H))


@pytest.mark.parametrize("red", ["sum", "mean"])
@pytest.mark.parametrize("F", [128, 41, 2])
def test_short_row_tiers(cuda, red, F):
    """Rows of <= 8 slots and rows without slots go to the batched short-row
    kernel (kernel.CSR.tiers): the same chains, so the result equals the
    one-wave-per-row kernel bit for bit (and the oracle for sum), with and
    without the heavy-row split."""
    rng = np.random.default_rng(F)
    n = 300_000
    row, col = rand_graph(rng, n, n, 900_000, skew=True)
    H = rng.uniform(-1, 1, (n, F)).astype(np.float32)
    adj = kernel.from_coo(n, n, row, col, kernel.ORDER_EID, cuda)
    Hd = torch.from_numpy(H).to(cuda)
    n_long, tail = adj.fwd.tiers()
    assert sum(t[2] for t in tail) >= kernel.schedule_policy()["tier_min_rows"]
    assert {t[0] for t in tail} == {0, 4, 8}
    outs = {}
    for split in ("off", 2000):
        old_s = kernel.set_row_split(split)
        try:
            for tiered in (True, False):
                old = kernel.set_short_rows(tiered)
                try:
                    outs[(split, tiered)] = kernel.gspmm(adj, "copy_u", red, Hd)
                finally:
                    kernel.set_short_rows(old)
        finally:
            kernel.set_row_split(old_s)
    assert torch.equal(outs[("off", True)], outs[("off", False)])
    assert torch.equal(outs[(2000, True)], outs[(2000, False)])
    if red == "sum":
        assert np.array_equal(outs[("off", True)].cpu().numpy().reshape(n, F),
                              O.spmm_coo(n, row, col, H))


def test_short_row_tiers_accumulate_and_bf16(cuda):
    """SUM_ACCUM (empty rows skipped, the others continued from out) and bf16
    source rows through the short-row tiers: bit-identical to the untiered path."""
    rng = np.random.default_rng(3)
    n, F = 250_000, 64
    row, col = rand_graph(rng, n, n, 700_000, skew=True)
    csr = kernel.build_csr(n, n, row, col, kernel.ORDER_EID, cuda)
    H = torch.from_numpy(rng.uniform(-1, 1, (n, F)).astype(np.float32)).to(cuda)
    base = torch.from_numpy(rng.uniform(-1, 1, (n, F)).astype(np.float32)).to(cuda)
    for src in (H, H.to(torch.bfloat16)):
        res = []
        for tiered in (True, False):
            old = kernel.set_short_rows(tiered)
            try:
                o = base.clone()
                kernel.gspmm_into(csr, o, src, accumulate=True)
                res.append(o)
            finally:
                kernel.set_short_rows(old)
        assert torch.equal(res[0], res[1])


@pytest.mark.gpu
def test_per_call_timing_counts_calls():
    """kernel.timing_enable(per_call=True): one event pair per g-SpMM call on
    the launch stream (bench.py's kernel ms), whatever the call's launch
    count; the per-launch mode still counts launches."""
    from dgl import kernel
    dev = torch.device("cuda", 0)
    n = 5000
    g = torch.Generator().manual_seed(0)
    src = torch.randint(0, n, (200_000,), generator=g)
    dst = torch.randint(0, n, (200_000,), generator=g)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    h = torch.rand(n, 64, device=dev)
    kernel.gspmm(adj, "copy_u", "sum", h)
    kernel.timing_enable(True, per_call=True)
    for _ in range(3):
        kernel.gspmm(adj, "copy_u", "sum", h)
    ms, calls = kernel.timing_read()
    kernel.timing_enable(False)
    assert calls == 3 and ms > 0
    kernel.timing_enable(True)
    kernel.gspmm(adj, "copy_u", "sum", h)
    ms1, launches = kernel.timing_read()
    kernel.timing_enable(False)
    assert launches >= 1 and ms1 > 0
