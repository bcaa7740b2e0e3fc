"""The source-swept g-SpMM (csrc/sweep.hip, dglhip_gspmm_sweep_device,
DESIGN.md §4.1 "Source sweep"): each wave keeps its rows' running sums in LDS
and walks their slots block by block, always in slot order, so the sum is the
row's chain — the oracle's bits — for any edge order, any block size and
any rows-per-wave, with rows spread over several launches when they exceed
one launch's LDS. Checked bit for bit against the oracle's COO chain (sum;
mean = that sum over the in-degree by IEEE division), on source-sorted and
random-order graphs.
"""
import ctypes

import numpy as np
import pytest
import torch

from dgl import kernel
from dgl._ffi import LIB, check_call, ptr
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda", 0)


def _graph(n, m, seed, order):
    rng = np.random.default_rng(seed)
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n, m)
    if order == "sorted":
        o = np.lexsort((dst, src))
        src, dst = src[o], dst[o]
    return src, dst


def _sweep(csr, h, out, n_blocks, rpw, mean=False):
    n, F = h.shape
    lo = int(csr.indices.min()) if csr.nnz else 0
    hi = int(csr.indices.max()) + 1 if csr.nnz else 1
    bs = max(1, -(-(hi - lo) // n_blocks))
    stream = ctypes.c_void_p(torch.cuda.current_stream(h.device).cuda_stream)
    check_call(LIB.dglhip_gspmm_sweep_device(
        csr.num_rows, F, ptr(csr.indptr), ptr(csr.indices) if csr.nnz else None, ptr(h),
        ptr(out), ptr(csr.row_order), lo, bs, n_blocks, 1 if mean else 0, rpw, stream))
    torch.cuda.synchronize()


@pytest.mark.parametrize("order", ["sorted", "random"])
@pytest.mark.parametrize("F,rpw", [(128, 10), (128, 20), (64, 40), (256, 5)])
def test_sweep_bits_any_order(order, F, rpw):
    dev = _dev()
    n, m = 20_000, 600_000
    src, dst = _graph(n, m, 1, order)
    csr = kernel.build_csr(n, n, torch.from_numpy(dst).to(dev), torch.from_numpy(src).to(dev),
                           kernel.ORDER_EID, dev)
    H = torch.randn(n, F, generator=torch.Generator().manual_seed(2))
    ref = O.spmm_coo(n, dst, src, H.numpy())
    h = H.to(dev)
    for nb in (1, 7, 64):
        out = torch.full((n, F), float("nan"), device=dev)
        _sweep(csr, h, out, nb, rpw)
        assert np.array_equal(out.cpu().numpy(), ref), (nb, rpw)


def test_sweep_mean_empty_rows_and_generations():
    """More rows than one launch holds (several launches), isolated rows
    (written as zeros), a hub row of 20,000 slots kept as one chain; mean is
    the chain's sum over the in-degree by IEEE division."""
    dev = _dev()
    n, m = 300_000, 2_000_000
    rng = np.random.default_rng(3)
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n // 2, m)          # rows n/2.. have no in-edges
    dst[:20_000] = 7                          # a hub row
    csr = kernel.build_csr(n, n, torch.from_numpy(dst).to(dev), torch.from_numpy(src).to(dev),
                           kernel.ORDER_EID, dev)
    H = torch.randn(n, 128, generator=torch.Generator().manual_seed(6))
    ref = O.spmm_coo(n, dst, src, H.numpy())
    deg = np.bincount(dst, minlength=n).astype(np.float32)[:, None]
    ref_mean = np.where(deg > 1, ref / np.maximum(deg, 1), ref).astype(np.float32)
    h = H.to(dev)
    for mean, want in ((False, ref), (True, ref_mean)):
        out = torch.full((n, 128), float("nan"), device=dev)
        _sweep(csr, h, out, 5, 10, mean)
        got = out.cpu().numpy()
        assert np.array_equal(got, want), mean
        assert not got[n // 2:].any()


def test_sweep_tiny_graphs():
    """One row per wave (no chunk prefetch), a single row, rows longer than
    one 64-slot chunk per block."""
    dev = _dev()
    for n, m in ((1, 200), (5, 3), (3, 1000)):
        src, dst = _graph(n, m, 4, "random")
        csr = kernel.build_csr(n, n, torch.from_numpy(dst).to(dev),
                               torch.from_numpy(src).to(dev), kernel.ORDER_EID, dev)
        H = torch.randn(n, 128, generator=torch.Generator().manual_seed(5))
        ref = O.spmm_coo(n, dst, src, H.numpy())
        for nb in (1, 2, 3):
            out = torch.full((n, 128), float("nan"), device=dev)
            _sweep(csr, H.to(dev), out, nb, 20)
            assert np.array_equal(out.cpu().numpy(), ref), (n, m, nb)


def _study_tool():
    import importlib.util
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "tools", "r05", "sweep_study.py")
    spec = importlib.util.spec_from_file_location("sweep_study", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("lag", [0, 2])
@pytest.mark.parametrize("rpw", [10, 19, 35, 51])
def test_sweep_stream_bits(lag, rpw):
    """The streamed layout (rows' block runs back to back per wave) and its
    soft barrier: the oracle's bits, sum and mean, with and without the
    barrier; a random-order graph has no such layout. 35 and 51 rows per
    wave hold 16 / 32 of them in registers (r06)."""
    dev = _dev()
    n, m = 50_000, 1_500_000
    src, dst = _graph(n, m, 7, "sorted")
    csr = kernel.build_csr(n, n, torch.from_numpy(dst).to(dev), torch.from_numpy(src).to(dev),
                           kernel.ORDER_EID, dev)
    H = torch.randn(n, 128, generator=torch.Generator().manual_seed(8))
    ref = O.spmm_coo(n, dst, src, H.numpy())
    deg = np.bincount(dst, minlength=n).astype(np.float32)[:, None]
    ref_mean = np.where(deg > 1, ref / np.maximum(deg, 1), ref).astype(np.float32)
    tool = _study_tool()
    lo, hi = int(csr.indices.min()), int(csr.indices.max()) + 1
    lt = tool.stream_layout(csr, 128, lo, hi, csr.row_order, 1, rpw)  # 1-MiB slices: 25 blocks
    assert lt is not None and lt["B"] > 8
    arrive = torch.zeros(lt["launches"] * (lt["B"] * 8 + 1) * 32, dtype=torch.int32, device=dev)
    h = H.to(dev)
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    for mean, want in ((0, ref), (1, ref_mean)):
        out = torch.full((n, 128), float("nan"), device=dev)
        check_call(LIB.dglhip_gspmm_sweep_stream_device(
            n, lt["W"], ptr(csr.row_order), ptr(lt["counts"]), lt["B"], ptr(lt["seg"]),
            ptr(lt["lay"]), ptr(csr.indptr), ptr(h), ptr(out), mean, rpw, 0, ptr(arrive),
            arrive.numel(), lag, 2000,
            stream))
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), want), mean
    src, dst = _graph(n, m, 7, "random")
    rnd = kernel.build_csr(n, n, torch.from_numpy(dst).to(dev), torch.from_numpy(src).to(dev),
                           kernel.ORDER_EID, dev)
    assert tool.stream_layout(rnd, 128, lo, hi, rnd.row_order, 1, rpw) is None


def test_plan_takes_the_sweep_for_large_tables():
    """A source table past the sweep's threshold (here lowered to 32 MiB):
    the plan schedules the sweep (path 4) for copy_u sum and mean of 128
    floats; update_all's forward and backward keep the oracle's bits, the
    same as with the sweep off; a 64-float table and a random-order graph
    stay on the other schedules."""
    import dgl
    import dgl.function as fn
    dev = _dev()
    n_src, n_dst, m = 120_000, 12_000, 2_000_000   # 61 MB source table, 167 slots per row
    rng = np.random.default_rng(11)
    src = rng.integers(0, n_src, m)
    dst = rng.integers(0, n_dst, m)
    o = np.lexsort((dst, src))
    src, dst = src[o], dst[o]
    H = torch.randn(n_src, 128, generator=torch.Generator().manual_seed(12))
    G = torch.randn(n_src, 128, generator=torch.Generator().manual_seed(13))
    ref = O.spmm_coo(n_src, dst, src, H.numpy())
    old = kernel.set_sweep_schedule(table_min=32 << 20, block_bytes=2 << 20)
    try:
        adj = kernel.from_coo(n_src, n_src, torch.from_numpy(dst).to(dev),
                              torch.from_numpy(src).to(dev), kernel.ORDER_EID, dev)
        path, launches = adj.fwd.plan.schedule(kernel.MSG_COPY_U, kernel.RED_SUM, 128, 0, n_src)
        assert path == kernel.PLAN_PATH_SWEEP and launches >= 1
        path64, _ = adj.fwd.plan.schedule(kernel.MSG_COPY_U, kernel.RED_SUM, 64, 0, n_src)
        assert path64 != kernel.PLAN_PATH_SWEEP
        res = {}
        for on in (True, False):
            kernel.set_sweep_schedule(on=on)
            g = dgl.DGLGraph((torch.from_numpy(src), torch.from_numpy(dst)))
            h = H.to(dev).requires_grad_(True)
            g.ndata["h"] = h
            g.update_all(fn.copy_src("h", "m"), fn.sum("m", "o"))
            g.ndata["o"].backward(G.to(dev))
            o_sum = g.ndata["o"].detach().cpu()
            g.update_all(fn.copy_src("h", "m"), fn.mean("m", "o"))
            res[on] = (o_sum, g.ndata["o"].detach().cpu(), h.grad.cpu())
        assert np.array_equal(res[True][0].numpy(), ref)
        for a, b in zip(res[True], res[False]):
            assert torch.equal(a, b)
        # the C-ABI route (DGLFuncCall with a plan handle) takes it too; a
        # plan-less call is one launch, the same bits
        kernel.set_sweep_schedule(on=True)
        from dgl import _ffi
        fwd = adj.fwd
        stream = ("handle", torch.cuda.current_stream().cuda_stream)
        plan = _ffi.call_packed("dglhip._CAPI_SpmmPlanCreate", fwd.indptr, fwd.indices, n_src,
                                fwd.row_order, stream)
        try:
            for extra in ((("handle", plan),), ()):
                out = torch.full((n_src, 128), float("nan"), device=dev)
                _ffi.call_packed("dglhip._CAPI_GSpMM", 0, 0, fwd.indptr, fwd.indices, None,
                                 H.to(dev), None, out, None, fwd.row_order, stream, *extra)
                torch.cuda.synchronize()
                assert np.array_equal(out.cpu().numpy(), ref)
        finally:
            _ffi.call_packed("dglhip._CAPI_SpmmPlanFree", ("handle", plan))
        rnd = rng.permutation(m)
        adj_r = kernel.from_coo(n_src, n_src, torch.from_numpy(dst[rnd]).to(dev),
                                torch.from_numpy(src[rnd]).to(dev), kernel.ORDER_EID, dev)
        path_r, _ = adj_r.fwd.plan.schedule(kernel.MSG_COPY_U, kernel.RED_SUM, 128, 0, n_src)
        assert path_r != kernel.PLAN_PATH_SWEEP
    finally:
        kernel.set_sweep_schedule(**old)


def test_accumulating_sweep_continues_the_chains():
    """SUM_ACCUM (the pipelined multi-GPU segments) through the plan's sweep:
    each non-empty row's chain continues from its value in out, rows without
    slots keep theirs; the same bits as the other schedules."""
    dev = _dev()
    n_src, n_dst, m = 120_000, 12_000, 2_000_000
    rng = np.random.default_rng(21)
    src = rng.integers(0, n_src, m)
    dst = rng.integers(0, n_dst // 2, m)     # half the rows have no slots
    o = np.lexsort((dst, src))
    src, dst = src[o], dst[o]
    csr = kernel.build_csr(n_dst, n_src, torch.from_numpy(dst).to(dev),
                           torch.from_numpy(src).to(dev), kernel.ORDER_EID, dev)
    h = torch.randn(n_src, 128, generator=torch.Generator().manual_seed(22)).to(dev)
    base = torch.randn(n_dst, 128, generator=torch.Generator().manual_seed(23)).to(dev)
    old = kernel.set_sweep_schedule(accum_table_min=32 << 20, block_bytes=2 << 20)
    try:
        path, _ = csr.plan.schedule(kernel.MSG_COPY_U, kernel.RED_SUM_ACCUM, 128, 0, n_src)
        assert path == kernel.PLAN_PATH_SWEEP
        res = []
        for on in (True, False):
            kernel.set_sweep_schedule(on=on)
            out = base.clone()
            kernel.gspmm_into(csr, out, h, accumulate=True)
            torch.cuda.synchronize()
            res.append(out.cpu())
        assert torch.equal(res[0], res[1])
        assert torch.equal(res[0][n_dst // 2:], base[n_dst // 2:].cpu())
        # a schedule order that is not degree-descending (empty rows first):
        # the sweep deals every row, same bits
        kernel.set_sweep_schedule(on=True)
        rev = kernel.build_csr(n_dst, n_src, torch.from_numpy(dst).to(dev),
                               torch.from_numpy(src).to(dev), kernel.ORDER_EID, dev)
        rev.row_order = torch.arange(n_dst - 1, -1, -1, dtype=torch.int32, device=dev)
        path, _ = rev.plan.schedule(kernel.MSG_COPY_U, kernel.RED_SUM_ACCUM, 128, 0, n_src)
        assert path == kernel.PLAN_PATH_SWEEP
        out = base.clone()
        kernel.gspmm_into(rev, out, h, accumulate=True)
        torch.cuda.synchronize()
        assert torch.equal(out.cpu(), res[1])
    finally:
        kernel.set_sweep_schedule(**old)


def test_accumulating_sweep_beside_an_occupying_kernel():
    """The default multi-GPU configuration runs the accumulating sweep's soft
    barrier (sweep_wait: it waits only for workgroups that have begun, and
    gives up after max_spin polls) beside RCCL kernels that hold CUs. Here a
    stream of 8192^2 GEMMs on a second stream holds the CUs while the sweep
    runs on the first: the oracle's bits (the sweep-off chains), bounded wall
    time, and the count of waits that ran out, read through the C-ABI. With
    max_spin = 1 waits do run out (the counter counts) and the bits stay."""
    import time
    dev = _dev()
    n_src, n_dst, m = 240_000, 24_000, 6_000_000   # 123 MB source table
    rng = np.random.default_rng(31)
    src = rng.integers(0, n_src, m)
    dst = rng.integers(0, n_dst, m)
    o = np.lexsort((dst, src))
    src, dst = src[o], dst[o]
    csr = kernel.build_csr(n_dst, n_src, torch.from_numpy(dst).to(dev),
                           torch.from_numpy(src).to(dev), kernel.ORDER_EID, dev)
    h = torch.randn(n_src, 128, generator=torch.Generator().manual_seed(32)).to(dev)
    base = torch.randn(n_dst, 128, generator=torch.Generator().manual_seed(33)).to(dev)
    old = kernel.set_sweep_schedule(accum_table_min=32 << 20, block_bytes=2 << 20)
    try:
        path, _ = csr.plan.schedule(kernel.MSG_COPY_U, kernel.RED_SUM_ACCUM, 128, 0, n_src)
        assert path == kernel.PLAN_PATH_SWEEP
        kernel.set_sweep_schedule(on=False)
        want = base.clone()
        kernel.gspmm_into(csr, want, h, accumulate=True)
        torch.cuda.synchronize()
        kernel.set_sweep_schedule(on=True)
        a = torch.randn(8192, 8192, device=dev)
        side = torch.cuda.Stream(dev)
        counts = {}
        for spin in (old["max_spin"], 1):
            kernel.set_sweep_schedule(max_spin=spin)
            kernel.sweep_barrier_expiries(reset=True)
            outs = [base.clone() for _ in range(4)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(12):
                    a = torch.mm(a, a) * 1e-4
            for out in outs:  # enqueued while the GEMMs hold the CUs
                kernel.gspmm_into(csr, out, h, accumulate=True)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            counts[spin] = kernel.sweep_barrier_expiries()
            print("max_spin %d: %d waits ran out over 4 calls beside the GEMMs, %.3f s"
                  % (spin, counts[spin], wall))
            assert wall < 30.0
            for out in outs:
                assert torch.equal(out, want)
        assert counts[1] > 0
    finally:
        kernel.set_sweep_schedule(**old)


def test_sweep_layout_follows_the_kernel_knobs():
    """The cached sweep layout is dealt over the waves one launch of the
    kernel that runs holds; a gathers-in-flight or rows-per-wave knob changed
    after the plan was built (its occupancy may differ) gets a layout of its
    own rather than a geometry mismatch at launch: same bits at
    16 and 32 gathers in flight and at 19, 35 and 51 rows per wave (16 / 32
    of them in registers), sum and the accumulating mode."""
    dev = _dev()
    n_src, n_dst, m = 120_000, 12_000, 2_000_000
    rng = np.random.default_rng(41)
    src = rng.integers(0, n_src, m)
    dst = rng.integers(0, n_dst, m)
    o = np.lexsort((dst, src))
    src, dst = src[o], dst[o]
    csr = kernel.build_csr(n_dst, n_src, torch.from_numpy(dst).to(dev),
                           torch.from_numpy(src).to(dev), kernel.ORDER_EID, dev)
    h = torch.randn(n_src, 128, generator=torch.Generator().manual_seed(42)).to(dev)
    base = torch.randn(n_dst, 128, generator=torch.Generator().manual_seed(43)).to(dev)
    ref = O.spmm_coo(n_dst, dst, src, h.cpu().numpy())
    old = kernel.set_sweep_schedule(table_min=32 << 20, accum_table_min=32 << 20,
                                    block_bytes=2 << 20)
    rows0 = ctypes.c_int()
    check_call(LIB.dglhip_get_sweep_rows(ctypes.byref(rows0)))
    try:
        res = {}
        for unroll, rows in ((16, 19), (32, 19), (16, 51), (16, 35), (32, 51), (16, 19)):
            check_call(LIB.dglhip_set_sweep_unroll(unroll))
            check_call(LIB.dglhip_set_sweep_rows(rows))
            out = torch.full((n_dst, 128), float("nan"), device=dev)
            kernel.gspmm_into(csr, out, h)
            acc = base.clone()
            kernel.gspmm_into(csr, acc, h, accumulate=True)
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy(), ref), (unroll, rows)
            res.setdefault("acc", acc.cpu())
            assert torch.equal(acc.cpu(), res["acc"]), (unroll, rows)
        path, _ = csr.plan.schedule(kernel.MSG_COPY_U, kernel.RED_SUM_ACCUM, 128, 0, n_src)
        assert path == kernel.PLAN_PATH_SWEEP
    finally:
        check_call(LIB.dglhip_set_sweep_unroll(16))
        check_call(LIB.dglhip_set_sweep_rows(rows0.value))
        kernel.set_sweep_schedule(**old)
