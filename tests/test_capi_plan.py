"""The g-SpMM launch plan behind the C-ABI (dglhip_spmm_plan_*, the registry's
dglhip._CAPI_GSpMM with a plan argument; csrc/spmm_plan.*).

The reference's own stack reaches the product through F.spmm
(python/dgl/backend/pytorch/tensor.py:145-146, SPMVExecutor.run at
runtime/ir/executor.py:452-473) or through _init_api -> DGLFuncCall
(python/dgl/_ffi/function.py:267-306). These tests drive the plan the way
such a caller does — through DGLFuncCall with DLTensor arguments — and check
that it runs the engine's benchmarked schedule (the source-blocked launches,
the heavy-row split) with the oracle's bits, on the host and on the MI355X.
"""
import numpy as np
import pytest
import torch

from dgl import _ffi, kernel
from oracle import oracle as O


def _graph(n, m, seed, sorted_src=True, skew=False):
    rng = np.random.default_rng(seed)
    if skew:  # power-law destinations: a few very long rows
        p = 1.0 / np.arange(1, n + 1) ** 1.1
        dst = rng.choice(n, size=m, p=p / p.sum())
    else:
        dst = rng.integers(0, n, m)
    src = rng.integers(0, n, m)
    if sorted_src:  # edges numbered source-major
        o = np.lexsort((dst, src))
        src, dst = src[o], dst[o]
    return src.astype(np.int64), dst.astype(np.int64)


def _create(csr, stream=None):
    return _ffi.call_packed("dglhip._CAPI_SpmmPlanCreate", csr.indptr, csr.indices, csr.num_cols,
                            csr.row_order, stream)


def _free(plan):
    _ffi.call_packed("dglhip._CAPI_SpmmPlanFree", ("handle", plan))


def test_plan_exports_and_policy_roundtrip():
    names = set(_ffi.list_global_names())
    for n in ("SpmmPlanCreate", "SpmmPlanFree", "SpmmPlanSchedule", "SpmmPlanBlocked",
              "SpmmPlanCuts", "SpmmPlanSplit", "SpmmPlanTiers", "GSpMM"):
        assert "dglhip._CAPI_" + n in names
    pol = kernel.schedule_policy()
    assert pol["row_split"] == -1 or "DGLHIP_ROW_SPLIT" in __import__("os").environ
    with kernel.scheduled(block_bytes=1 << 20, block_min_slots=7):
        p = kernel.schedule_policy()
        assert p["block_bytes"] == 1 << 20 and p["block_min_slots"] == 7
    assert kernel.schedule_policy() == pol
    with pytest.raises(kernel.DGLError):
        kernel.set_schedule_policy(block_bytes=0)
    assert kernel.schedule_policy() == pol


def test_padded_width_rule():
    assert kernel.padded_width(128) == 128
    assert kernel.padded_width(41) == 48
    assert kernel.padded_width(24) == 32
    assert kernel.padded_width(16) == 16


def test_capi_gspmm_host_with_plan():
    """_CAPI_GSpMM on host arrays with a plan: the oracle's bits, for copy_u
    and u_mul_e (edge ids, slot order, a map) and max."""
    n, m = 1500, 60_000
    src, dst = _graph(n, m, 3)
    csr = kernel.build_csr(n, n, torch.from_numpy(dst), torch.from_numpy(src),
                           kernel.ORDER_EID, "cpu")
    gen = torch.Generator().manual_seed(4)
    H = torch.randn(n, 32, generator=gen)
    w = torch.rand(m, 1, generator=gen)
    plan = _create(csr)
    try:
        out = torch.empty(n, 32)
        _ffi.call_packed("dglhip._CAPI_GSpMM", 0, 0, csr.indptr, csr.indices, None, H, None,
                         out, None, None, None, ("handle", plan))
        assert np.array_equal(out.numpy(), O.spmm_coo(n, dst, src, H.numpy()))
        _ffi.call_packed("dglhip._CAPI_GSpMM", 1, 0, csr.indptr, csr.indices, csr.eid, H, w,
                         out, None, None, None, ("handle", plan))
        assert np.array_equal(out.numpy(), O.spmm_coo(n, dst, src, H.numpy(), w.numpy().ravel()))
        # slot order: the weights permuted into the CSR's slots, no edge ids
        ws = w[csr.eid]
        o2 = torch.empty(n, 32)
        _ffi.call_packed("dglhip._CAPI_GSpMM", 1, 0, csr.indptr, csr.indices, None, H, ws,
                         o2, None, None, None, ("handle", plan), 0)
        assert torch.equal(o2, out)
        # a map: rows of a reversed copy
        wr = torch.flip(w, [0]).contiguous()
        emap = (m - 1 - csr.eid).contiguous()
        _ffi.call_packed("dglhip._CAPI_GSpMM", 1, 0, csr.indptr, csr.indices, emap, H, wr,
                         o2, None, None, None, ("handle", plan), 2)
        assert torch.equal(o2, out)
    finally:
        _free(plan)


def test_capi_gspmm_without_plan_is_one_launch():
    """No plan argument: one launch over the CSR, no schedule built (same
    bits as the planned product)."""
    n, m = 800, 20_000
    src, dst = _graph(n, m, 5)
    csr = kernel.build_csr(n, n, torch.from_numpy(dst), torch.from_numpy(src),
                           kernel.ORDER_EID, "cpu")
    H = torch.randn(n, 16, generator=torch.Generator().manual_seed(6))
    out = torch.empty(n, 16)
    _ffi.call_packed("dglhip._CAPI_GSpMM", 0, 2, csr.indptr, csr.indices, None, H, None, out,
                     None, csr.row_order, None)
    ref = kernel.gspmm(kernel.from_coo(n, n, dst, src), "copy_u", "mean", H)
    assert torch.equal(out, ref)


def test_plan_rejects_another_csr():
    n = 300
    src, dst = _graph(n, 3000, 7)
    a = kernel.build_csr(n, n, torch.from_numpy(dst), torch.from_numpy(src), kernel.ORDER_EID,
                         "cpu")
    b = kernel.build_csr(n, n, torch.from_numpy(src), torch.from_numpy(dst), kernel.ORDER_EID,
                         "cpu")
    plan = _create(a)
    try:
        with pytest.raises(kernel.DGLError, match="another CSR"):
            _ffi.call_packed("dglhip._CAPI_GSpMM", 0, 0, b.indptr, b.indices, None,
                             torch.randn(n, 4), None, torch.empty(n, 4), None, None, None,
                             ("handle", plan))
    finally:
        _free(plan)


def test_host_plan_blocked_structures():
    """The host plan builds the same blocked schedule the device plan does
    (the walk and the scatter as host loops): items longest first, each
    row's slots block after block in its own order, suffixes last; the cuts
    bound the same ranges."""
    n, m = 2000, 200_000
    src, dst = _graph(n, m, 0)
    csr = kernel.build_csr(n, n, torch.from_numpy(dst), torch.from_numpy(src),
                           kernel.ORDER_EID, "cpu")
    with kernel.scheduled(block_table_min=0, block_bytes=1 << 16):
        plan = kernel._block_plan(csr, torch.empty(2, 128), 128)
        cuts = kernel._block_cuts(csr, 128 * 4, 1 << 16)
    assert plan is not None and len(plan) == plan.B and not plan.has_suffix
    assert len(cuts) == plan.B + 1
    ip = csr.indptr
    for b, it in enumerate(plan):
        cnt = it.ptr[1:] - it.ptr[:-1]
        assert bool((cnt[:-1] >= cnt[1:]).all())
        # item i of block b holds row rows[i]'s slots [cuts[b], cuts[b+1])
        r = it.rows.long()
        assert torch.equal(cnt, cuts[b + 1][r] - cuts[b][r])
        first = torch.repeat_interleave(cuts[b][r], cnt)
        within = torch.arange(it.nnz) - torch.repeat_interleave(it.ptr[:-1] - it.off, cnt)
        assert torch.equal(it.pos.long(), first + within)
    assert torch.equal(cuts[0], ip[:-1]) and torch.equal(cuts[-1], ip[1:])


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda", 0)


def _events_ms(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


@pytest.mark.gpu
def test_capi_gspmm_without_plan_under_stream_capture(cuda):
    """A plan-less dglhip._CAPI_GSpMM enqueues one kernel and nothing else (no
    allocation, no host sync), so it can be captured into a HIP graph: the
    replayed graph gives the oracle's bits, and so does a replay after the
    operand is overwritten in place."""
    n, m, F = 5000, 200_000, 64
    src, dst = _graph(n, m, 11)
    csr = kernel.build_csr(n, n, torch.from_numpy(dst).to(cuda), torch.from_numpy(src).to(cuda),
                           kernel.ORDER_EID, cuda)
    gen = torch.Generator(device=cuda).manual_seed(12)
    H = torch.rand(n, F, generator=gen, device=cuda)
    out = torch.empty(n, F, device=cuda)
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(cuda)
    side.wait_stream(torch.cuda.current_stream(cuda))
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            _ffi.call_packed("dglhip._CAPI_GSpMM", 0, 0, csr.indptr, csr.indices, None, H, None,
                             out, None, None, ("handle", side.cuda_stream))
    ip, ix, pos = O.coo_to_csr(n, dst, src)
    for _ in range(2):
        out.zero_()
        graph.replay()
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), O.spmm_csr(ip, ix, pos, H.cpu().numpy()))
        H.copy_(torch.rand(n, F, generator=gen, device=cuda))


@pytest.mark.gpu
def test_capi_planned_full_reddit_bit_exact_and_fast(cuda):
    """The headline graph (configs[1] shape: 232,965 nodes, 114.8M edges,
    F = 128) through dglhip._CAPI_GSpMM with a plan, as the reference's FFI
    would call it: the source-blocked schedule (19 launches per call), the
    oracle's bits forward and through the transposed CSR (the backward dH =
    A^T dC), and within 3 % of the engine's own Python path."""
    from dgl import data
    src, dst, n = data.reddit_like(scale=1, seed=0, device=cuda)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, cuda)
    s_np, d_np = src.cpu().numpy(), dst.cpu().numpy()
    del src, dst
    gen = torch.Generator(device=cuda).manual_seed(1)
    h = torch.rand(n, 128, generator=gen, device=cuda) * 2 - 1
    dc = torch.rand(n, 128, generator=gen, device=cuda) * 2 - 1
    stream = ("handle", torch.cuda.current_stream().cuda_stream)
    fwd, bwd = adj.fwd, adj.bwd
    pf, pb = _create(fwd, stream), _create(bwd, stream)
    try:
        sched = _ffi.call_packed("dglhip._CAPI_SpmmPlanSchedule", ("handle", pf), 0, 0, 128, 0,
                                 n, 0, 0, stream)
        assert sched >> 32 == kernel.PLAN_PATH_BLOCKED and sched & 0xffffffff == 19
        out = torch.empty(n, 128, device=cuda)
        dh = torch.empty(n, 128, device=cuda)

        def capi_fwd():
            _ffi.call_packed("dglhip._CAPI_GSpMM", 0, 0, fwd.indptr, fwd.indices, None, h, None,
                             out, None, fwd.row_order, stream, ("handle", pf))

        def capi_bwd():
            _ffi.call_packed("dglhip._CAPI_GSpMM", 0, 0, bwd.indptr, bwd.indices, None, dc, None,
                             dh, None, bwd.row_order, stream, ("handle", pb))
        capi_fwd()
        capi_bwd()
        kernel.timing_enable(True)
        capi_fwd()
        _, launches = kernel.timing_read()
        kernel.timing_enable(False)
        assert launches == 19
        ip, ix, pos = O.coo_to_csr(n, d_np, s_np)
        assert np.array_equal(out.cpu().numpy(), O.spmm_csr(ip, ix, pos, h.cpu().numpy(),
                                                            num_threads=16))
        ip, ix, pos = O.coo_to_csr(n, s_np, d_np)
        assert np.array_equal(dh.cpu().numpy(), O.spmm_csr(ip, ix, pos, dc.cpu().numpy(),
                                                           num_threads=16))
        py_out = torch.empty_like(out)

        def py_fwd():
            kernel.gspmm_into(fwd, py_out, h)
        t_capi, t_py = [], []
        for _ in range(3):  # interleaved rounds
            t_capi.append(_events_ms(capi_fwd, 20))
            t_py.append(_events_ms(py_fwd, 20))
        assert torch.equal(py_out, out)
        assert min(t_capi) <= 1.03 * min(t_py), (t_capi, t_py)
    finally:
        _free(pf)
        _free(pb)


@pytest.mark.gpu
def test_capi_planned_heavy_rows_power_law(cuda):
    """A 1M-row power-law graph whose hub rows are the launch's critical
    path: the plan's native heavy-row split (chunks added in order) — the
    oracle within 1e-5 of each row's sum |x| (the chain's summation bound),
    deterministic, and the Python operators' bits (one plan code)."""
    n, m = 1_000_000, 16_000_000
    src, dst = _graph(n, m, 11, sorted_src=False, skew=True)
    adj = kernel.from_coo(n, n, torch.from_numpy(dst), torch.from_numpy(src),
                          kernel.ORDER_EID, cuda)
    fwd = adj.fwd
    stream = ("handle", torch.cuda.current_stream().cuda_stream)
    H = torch.from_numpy(np.random.default_rng(12).uniform(-1, 1, (n, 128)).astype(np.float32))
    Hd = H.to(cuda)
    pf = _create(fwd, stream)
    try:
        thr = kernel._split_threshold(fwd)
        assert thr > 0
        st = fwd.plan.stats()
        assert st["heavy_threshold"] == thr and st["max_degree"] > thr
        out = torch.empty(n, 128, device=cuda)
        _ffi.call_packed("dglhip._CAPI_GSpMM", 0, 0, fwd.indptr, fwd.indices, None, Hd, None,
                         out, None, fwd.row_order, stream, ("handle", pf))
        again = torch.empty_like(out)
        _ffi.call_packed("dglhip._CAPI_GSpMM", 0, 0, fwd.indptr, fwd.indices, None, Hd, None,
                         again, None, fwd.row_order, stream, ("handle", pf))
        assert torch.equal(out, again)
        assert torch.equal(out, kernel.gspmm(adj, "copy_u", "sum", Hd))
        ip, ix, pos = O.coo_to_csr(n, dst, src)
        ref = O.spmm_csr(ip, ix, pos, H.numpy(), num_threads=16)
        scale = O.spmm_csr(ip, ix, pos, np.abs(H.numpy()), num_threads=16)
        got = out.cpu().numpy()
        assert np.all(np.abs(got - ref) <= 1e-5 * scale + 1e-30)
        deg = np.diff(ip)
        light = deg <= thr
        assert np.array_equal(got[light], ref[light])  # unchunked rows: one exact chain
    finally:
        _free(pf)


@pytest.mark.gpu
def test_device_plan_equals_host_plan(cuda):
    """The device build (walk and scatter kernels) gives the host build's
    arrays, blocked items and cuts, with and without suffixes."""
    n = 3000
    for case in ("source_major", "self_loops", "random_order"):
        src, dst = _graph(n, 300_000, 21, sorted_src=case != "random_order")
        if case == "self_loops":  # appended after the edges: one suffix slot per row
            loops = np.arange(n, dtype=np.int64)
            src, dst = np.concatenate([src, loops]), np.concatenate([dst, loops])
        h_csr = kernel.build_csr(n, n, torch.from_numpy(dst), torch.from_numpy(src),
                                 kernel.ORDER_EID, "cpu")
        d_csr = kernel.build_csr(n, n, torch.from_numpy(dst), torch.from_numpy(src),
                                 kernel.ORDER_EID, cuda)
        with kernel.scheduled(block_table_min=0, block_bytes=1 << 17):
            hp = kernel._block_plan(h_csr, torch.empty(2, 128), 128)
            dp = kernel._block_plan(d_csr, torch.empty(2, 128, device=cuda), 128)
            hc = kernel._block_cuts(h_csr, 512, 1 << 17)
            dc = kernel._block_cuts(d_csr, 512, 1 << 17)
        assert (hp is None) == (dp is None) == (case == "random_order")
        if hp is None:
            continue
        assert hp.has_suffix == (case == "self_loops")
        assert hp.has_suffix == dp.has_suffix and len(hp) == len(dp)
        assert torch.equal(hp.indices, dp.indices.cpu()) and torch.equal(hp.pos, dp.pos.cpu())
        for a, b in zip(hp, dp):
            assert torch.equal(a.rows, b.rows.cpu()) and torch.equal(a.ptr, b.ptr.cpu())
        assert all(torch.equal(a, b.cpu()) for a, b in zip(hc, dc))
