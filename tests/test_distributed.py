"""Multi-rank path (dgl.distributed) on CPU with gloo: each rank's rows of the
partitioned update_all equal the single-process product bit for bit, and the
backward (reduce-scatter of the transposed products) matches the oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _assert_chain_close(got, ref, scale):
    """A reassociated fp32 chain (segments, chunks, reduce-scatter) against
    the oracle's: within 1e-5 of the row's condition scale sum_k |x_k| (the
    summation error bound's yardstick), elementwise."""
    err = np.abs(np.asarray(got, dtype=np.float64) - ref)
    assert np.all(err <= 1e-5 * scale + 1e-6), float((err - 1e-5 * scale).max())


def _banded(n, width, seed):
    """Graph with locality: every source within `width` ids of its destination."""
    gen = torch.Generator().manual_seed(seed)
    dst = torch.randint(0, n, (12 * n,), generator=gen)
    src = (dst + torch.randint(-width, width + 1, dst.shape, generator=gen)).clamp(0, n - 1)
    return src, dst, n


def _worker(rank, world, port, n, F, halo="auto", graph="chung_lu"):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "dgl-1_amd")]
    from dgl import data
    from dgl.distributed import PartitionedGraph, balanced_bounds
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if graph == "banded":
            src, dst, n = _banded(n, 40, seed=3)
        else:
            src, dst, n = data.chung_lu(n, 40 * n, 30.0, seed=3)  # same graph on every rank
        bounds = balanced_bounds(torch.bincount(dst, minlength=n), world)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        sel = (dst >= lo) & (dst < hi)
        pg = PartitionedGraph(n, src[sel], dst[sel], bounds, "cpu", halo=halo)
        expect = {"auto": "alltoall" if graph == "banded" else "allgather"}.get(halo, halo)
        assert pg.halo_mode == expect, pg.halo_mode
        if expect == "alltoall":
            remote = src[sel][(src[sel] < lo) | (src[sel] >= hi)]
            assert pg.num_halo == torch.unique(remote).numel()
        gen = torch.Generator().manual_seed(7)
        H = torch.rand(n, F, generator=gen) * 2 - 1
        G = torch.randn(n, F, generator=gen)
        h_local = H[lo:hi].clone().requires_grad_(True)
        out = pg.update_all(h_local)
        ref = O.spmm_coo(n, dst.numpy(), src.numpy(), H.numpy())
        assert np.array_equal(out.detach().numpy(), ref[lo:hi]), "forward rows differ"
        out.backward(G[lo:hi])
        gref = O.spmm_coo(n, src.numpy(), dst.numpy(), G.numpy())
        np.testing.assert_allclose(h_local.grad.numpy(), gref[lo:hi], rtol=1e-5, atol=1e-5)
        assert pg.num_local == hi - lo and pg.num_edges == int(sel.sum())
        # mean_add (out + mean in the g-SpMM's store) == the sum of the two tensors
        base = torch.randn(hi - lo, F, generator=gen)
        h1 = H[lo:hi].clone().requires_grad_(True)
        o1 = pg.mean_add(h1, base.clone())
        o1.backward(G[lo:hi])
        h2 = H[lo:hi].clone().requires_grad_(True)
        o2 = base + pg.update_all(h2, "copy_u", "mean")
        o2.backward(G[lo:hi])
        assert torch.equal(o1.detach(), o2.detach()) and torch.equal(h1.grad, h2.grad)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_update_all(world):
    mp.spawn(_worker, args=(world, _free_port(), 3000, 16), nprocs=world, join=True)


@pytest.mark.parametrize("world,halo,graph", [(2, "alltoall", "chung_lu"),
                                              (3, "auto", "banded"),
                                              (3, "allgather", "banded")])
def test_partitioned_halo_modes(world, halo, graph):
    """All-to-allv halo (only the referenced remote rows): forward rows are
    bit-identical, backward (reverse all-to-allv + sum-on-receive) within
    1e-5; auto picks it for a banded graph, all-gather for a power-law one."""
    mp.spawn(_worker, args=(world, _free_port(), 3000, 16, halo, graph), nprocs=world, join=True)


def test_balanced_bounds():
    from dgl.distributed import balanced_bounds
    deg = torch.tensor([5, 1, 1, 1, 1, 1, 0, 10, 0, 0])
    b = balanced_bounds(deg, 2)
    assert b.tolist()[0] == 0 and b.tolist()[-1] == 10
    assert all(x <= y for x, y in zip(b.tolist(), b.tolist()[1:]))
    assert balanced_bounds(torch.zeros(0, dtype=torch.int64), 4).tolist() == [0, 0, 0, 0, 0]


def _sage_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "dgl-1_amd"), os.path.join(root, "tests")]
    from conftest import load_example
    sage = load_example("graphsage/train.py", "sage_train")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        args = sage.parser().parse_args(["--graph", "rmat", "--rmat-scale", "11", "--gpu", "-1",
                                         "--dist", "--n-epochs", "3", "--in-feats", "16",
                                         "--n-hidden", "16", "--n-classes", "5"])
        res = sage.run(args)
        if rank == 0:
            q.put({k: v.numpy() for k, v in res["state"].items()})
    finally:
        dist.destroy_process_group()


def test_graphsage_distributed_matches_single():
    """Three training steps of GraphSAGE-mean on 2 gloo ranks (halo all-gather,
    reduce-scatter backward, DDP all-reduce) == the single-process run."""
    from conftest import load_example
    sage = load_example("graphsage/train.py", "sage_train")
    args = sage.parser().parse_args(["--graph", "rmat", "--rmat-scale", "11", "--gpu", "-1",
                                     "--n-epochs", "3", "--in-feats", "16", "--n-hidden", "16",
                                     "--n-classes", "5"])
    single = sage.run(args)["state"]
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.spawn(_sage_worker, args=(2, _free_port(), q), nprocs=2, join=True)
    multi = q.get()
    for k, v in single.items():
        np.testing.assert_allclose(multi[k], v.numpy(), rtol=1e-4, atol=1e-5, err_msg=k)


def _pipe_worker(rank, world, port, graph="chung_lu"):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "dgl-1_amd")]
    from dgl import data
    from dgl.distributed import PartitionedGraph, balanced_bounds
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, F = 2500, 8
        if graph == "banded":  # halo well under an all-gather: auto takes the all-to-allv
            src, dst, n = _banded(n, 60, seed=5)
        else:
            src, dst, n = data.chung_lu(n, 30 * n, 30.0, seed=5)  # edge ids in (src, dst) order
        bounds = balanced_bounds(torch.bincount(dst, minlength=n), world)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        sel = (dst >= lo) & (dst < hi)
        H = torch.rand(n, F, generator=torch.Generator().manual_seed(2)) * 2 - 1
        ref = O.spmm_coo(n, dst.numpy(), src.numpy(), H.numpy())[lo:hi]
        for chunks in (1, 3):
            pg = PartitionedGraph(n, src[sel], dst[sel], bounds, "cpu", pipeline_chunks=chunks)
            assert pg.halo_mode == ("alltoall" if graph == "banded" else "allgather")
            out = pg.update_all(H[lo:hi].contiguous()).numpy()
            np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-5)
            if graph == "banded":
                # exactly the chain over (own sources first, then the received rows
                # chunk by chunk; edge id): chunk c holds part c of every owner's
                # request list, cut at (len * c) // C
                s, d = src[sel], dst[sel]
                remote = ((s < lo) | (s >= hi)).numpy()
                need = np.unique(s.numpy()[remote])
                owner = np.searchsorted(bounds.numpy(), need, side="right") - 1
                chunk_of = {}
                for p in range(world):
                    ids = need[owner == p]
                    for jj, v in enumerate(ids):
                        chunk_of[int(v)] = sum(jj >= (len(ids) * c) // chunks
                                               for c in range(1, chunks))
                seg = np.array([1 + chunk_of[int(v)] if r else 0
                                for v, r in zip(s.numpy(), remote)])
                order = np.lexsort((np.arange(len(s)), seg))
                exact = O.spmm_coo(n, d.numpy()[order], s.numpy()[order], H.numpy())[lo:hi]
                assert np.array_equal(out, exact)
            # deterministic
            assert np.array_equal(out, pg.update_all(H[lo:hi].contiguous()).numpy())
            # trainable: sum and mean, forward + backward (transposed segments,
            # chunked reverse exchange) against the oracle, deterministic
            G = torch.randn(n, F, generator=torch.Generator().manual_seed(3))
            deg = torch.bincount(dst, minlength=n).clamp(min=1).float().unsqueeze(1)
            fscale = O.spmm_coo(n, dst.numpy(), src.numpy(), np.abs(H.numpy()))[lo:hi]
            for reduce in ("sum", "mean"):
                h = H[lo:hi].clone().requires_grad_(True)
                o = pg.update_all(h, "copy_u", reduce)
                dv = 1.0 if reduce == "sum" else deg[lo:hi].numpy()
                _assert_chain_close(o.detach().numpy(), ref / dv, fscale / dv)
                o.backward(G[lo:hi])
                Gs = G if reduce == "sum" else G / deg
                gref = O.spmm_coo(n, src.numpy(), dst.numpy(), Gs.numpy())[lo:hi]
                gscale = O.spmm_coo(n, src.numpy(), dst.numpy(), np.abs(Gs.numpy()))[lo:hi]
                _assert_chain_close(h.grad.numpy(), gref, gscale)
                h2 = H[lo:hi].clone().requires_grad_(True)
                pg.update_all(h2, "copy_u", reduce).backward(G[lo:hi])
                assert torch.equal(h.grad, h2.grad)
            # mean_add: base + mean in the division's pass, the same bits and
            # gradients as the sum of the two tensors
            base = torch.randn(hi - lo, F, generator=torch.Generator().manual_seed(4))
            h3 = H[lo:hi].clone().requires_grad_(True)
            b3 = base.clone().requires_grad_(True)
            o3 = pg.mean_add(h3, b3.clone())
            o3.backward(G[lo:hi])
            h4 = H[lo:hi].clone().requires_grad_(True)
            o4 = base + pg.update_all(h4, "copy_u", "mean")
            o4.backward(G[lo:hi])
            assert torch.equal(o3.detach(), o4.detach())
            assert torch.equal(h3.grad, h4.grad) and torch.equal(b3.grad, G[lo:hi])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,graph", [(2, "chung_lu"), (3, "chung_lu"), (4, "chung_lu"),
                                         (2, "banded"), (3, "banded"), (4, "banded")])
def test_pipelined_forward(world, graph):
    """Pipelined halo (chunked exchange overlapped with the segments) in both
    halo modes: forward within 1e-5 (exactly the (segment, eid) chain for the
    all-to-allv), and trainable — sum and mean, backward within 1e-5 of the
    oracle's transposed product, deterministic."""
    mp.spawn(_pipe_worker, args=(world, _free_port(), graph), nprocs=world, join=True)


@pytest.mark.gpu
def test_single_rank_rccl_group_all_modes():
    """The RCCL code path of PartitionedGraph on the one GPU this pool gives:
    a world-size-1 nccl (RCCL) group, every halo mode and the pipelined
    forward with its comm stream, forward rows bit-exact and backward against
    the oracle. Multi-rank RCCL runs only in the driver's 8-GPU bench; this
    pins the collective calls' device placement, split lists and stream use."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "dgl-1_amd")]
    from dgl import data
    from dgl.distributed import PartitionedGraph
    from oracle import oracle as O

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(), rank=0,
                            world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        src, dst, n = data.chung_lu(4000, 40 * 4000, 30.0, seed=3)
        bounds = torch.tensor([0, n])
        gen = torch.Generator().manual_seed(7)
        H = torch.rand(n, 16, generator=gen) * 2 - 1
        G = torch.randn(n, 16, generator=gen)
        ref = O.spmm_coo(n, dst.numpy(), src.numpy(), H.numpy())
        gref = O.spmm_coo(n, src.numpy(), dst.numpy(), G.numpy())
        # bf16 halo: at world size 1 every source is an own row, so the results stay
        # exact; the runs pin the float16-view wire buffers through RCCL
        for halo, chunks, hd in (("auto", 0, None), ("allgather", 0, None),
                                 ("alltoall", 0, None), ("allgather", 2, None),
                                 ("alltoall", 2, None), ("allgather", 0, torch.bfloat16),
                                 ("alltoall", 0, torch.bfloat16),
                                 ("allgather", 2, torch.bfloat16),
                                 ("alltoall", 2, torch.bfloat16)):
            pg = PartitionedGraph(n, src, dst, bounds, dev, halo=halo, pipeline_chunks=chunks,
                                  halo_dtype=hd)
            h = H.to(dev).requires_grad_(True)
            out = pg.update_all(h)
            torch.cuda.synchronize()
            if chunks == 0:
                assert np.array_equal(out.detach().cpu().numpy(), ref), (halo, chunks)
            else:
                np.testing.assert_allclose(out.detach().cpu().numpy(), ref, rtol=1e-5,
                                           atol=1e-5)
            # the pipelined backward: reverse exchanges on the comm stream
            out.backward(G.to(dev))
            torch.cuda.synchronize()
            np.testing.assert_allclose(h.grad.cpu().numpy(), gref, rtol=1e-5, atol=1e-5)
        t = torch.ones(1, device=dev)
        dist.all_reduce(t)
        dist.barrier()
        assert t.item() == 1.0
    finally:
        dist.destroy_process_group()


def _bf16_worker(rank, world, port, halo, chunks):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "dgl-1_amd")]
    from dgl import data
    from dgl.distributed import PartitionedGraph, balanced_bounds
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if halo == "alltoall":
            src, dst, n = _banded(2400, 50, seed=9)
        else:
            src, dst, n = data.chung_lu(2400, 30 * 2400, 30.0, seed=9)
        bounds = balanced_bounds(torch.bincount(dst, minlength=n), world)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        sel = (dst >= lo) & (dst < hi)
        gen = torch.Generator().manual_seed(4)
        H = torch.rand(n, 12, generator=gen) * 2 - 1
        G = torch.randn(n, 12, generator=gen)
        # what the rank computes on: its own rows exact, remote rows rounded to bf16
        Heff = H.to(torch.bfloat16).float()
        Heff[lo:hi] = H[lo:hi]
        pg = PartitionedGraph(n, src[sel], dst[sel], bounds, "cpu", halo=halo,
                              pipeline_chunks=chunks, halo_dtype=torch.bfloat16)
        assert pg.halo_mode == halo
        h = H[lo:hi].clone().requires_grad_(True)
        out = pg.update_all(h)
        ref = O.spmm_coo(n, dst.numpy(), src.numpy(), Heff.numpy())[lo:hi]
        if chunks == 0:
            # same chain as the fp32 exchange, on the rounded remote rows: bit-exact
            assert np.array_equal(out.detach().numpy(), ref)
        else:
            np.testing.assert_allclose(out.detach().numpy(), ref, rtol=1e-5, atol=1e-5)
        # gradients travel in fp32 in every mode: the fp32 transposed product
        out.backward(G[lo:hi])
        gref = O.spmm_coo(n, src.numpy(), dst.numpy(), G.numpy())[lo:hi]
        np.testing.assert_allclose(h.grad.numpy(), gref, rtol=1e-5, atol=1e-5)
        # and the halving costs bf16 accuracy only: within 1 % of the fp32 product
        full = O.spmm_coo(n, dst.numpy(), src.numpy(), H.numpy())[lo:hi]
        np.testing.assert_allclose(out.detach().numpy(), full, rtol=2e-2, atol=2e-2)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("halo,chunks", [("allgather", 0), ("alltoall", 0), ("allgather", 2),
                                         ("alltoall", 3)])
def test_bf16_halo(halo, chunks):
    """Opt-in bf16 halo: remote rows travel rounded to bf16 as
    a float16 view, own rows stay exact; the forward equals the oracle on
    those inputs bit for bit (pipelined: within 1e-5), the backward and the
    result stay within bf16 accuracy of the fp32 product."""
    mp.spawn(_bf16_worker, args=(2, _free_port(), halo, chunks), nprocs=2, join=True)


def _switch_worker(rank, world, port):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "dgl-1_amd")]
    from dgl import data
    from dgl.distributed import PartitionedGraph, balanced_bounds

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        src, dst, n = data.chung_lu(1500, 20 * 1500, 20.0, seed=5)
        bounds = balanced_bounds(torch.bincount(dst, minlength=n), world)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        sel = (dst >= lo) & (dst < hi)
        H = torch.rand(n, 8, generator=torch.Generator().manual_seed(2)) * 2 - 1
        pg = PartitionedGraph(n, src[sel], dst[sel], bounds, "cpu", pipeline_chunks=2)
        a = pg.update_all(H[lo:hi].contiguous())
        pg.set_halo_dtype(torch.bfloat16)  # bench.py's secondary leg
        b = pg.update_all(H[lo:hi].contiguous())
        pg.set_halo_dtype(None)
        c = pg.update_all(H[lo:hi].contiguous())
        assert torch.equal(a, c)
        assert not torch.equal(a, b)
        torch.testing.assert_close(a, b, rtol=2e-2, atol=2e-2)
    finally:
        dist.destroy_process_group()


def test_switch_halo_dtype():
    """set_halo_dtype: bf16 then back to fp32 on one partition gives the fp32
    rows again, bit for bit (buffers reallocated for each wire type)."""
    mp.spawn(_switch_worker, args=(2, _free_port()), nprocs=2, join=True)


def _overlap_worker(rank, world, port, graph, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "dgl-1_amd")]
    from dgl import data
    from dgl.distributed import PartitionedGraph, balanced_bounds
    from oracle import oracle as O

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, F = 6000, 32
        if graph == "banded":
            src, dst, n = _banded(n, 80, seed=9)
        else:
            src, dst, n = data.chung_lu(n, 40 * n, 30.0, seed=9)
        bounds = balanced_bounds(torch.bincount(dst, minlength=n), world)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        sel = (dst >= lo) & (dst < hi)
        gen = torch.Generator().manual_seed(11)
        H = torch.rand(n, F, generator=gen) * 2 - 1
        G = torch.randn(n, F, generator=gen)
        ref = O.spmm_coo(n, dst.numpy(), src.numpy(), H.numpy())[lo:hi]
        fscale = O.spmm_coo(n, dst.numpy(), src.numpy(), np.abs(H.numpy()))[lo:hi]
        gref = O.spmm_coo(n, src.numpy(), dst.numpy(), G.numpy())[lo:hi]
        gscale = O.spmm_coo(n, src.numpy(), dst.numpy(), np.abs(G.numpy()))[lo:hi]
        for chunks in (2, 3):
            side = PartitionedGraph(n, src[sel], dst[sel], bounds, dev, pipeline_chunks=chunks,
                                    overlap=True)
            inline = PartitionedGraph(n, src[sel], dst[sel], bounds, dev,
                                      pipeline_chunks=chunks, overlap=False)
            assert side.comm_stream is not None and inline.comm_stream is None
            assert side.halo_mode == ("alltoall" if graph == "banded" else "allgather")
            for it in range(4):  # repeated calls: buffers reused across steps
                scale = float(it + 1)
                outs, grads = [], []
                for pg in (side, inline):
                    h = (H[lo:hi] * scale).to(dev).requires_grad_(True)
                    o = pg.update_all(h)
                    o.backward((G[lo:hi] * scale).to(dev))
                    torch.cuda.synchronize()
                    outs.append(o.detach().cpu())
                    grads.append(h.grad.cpu())
                assert torch.equal(outs[0], outs[1]), (graph, chunks, it)
                assert torch.equal(grads[0], grads[1]), (graph, chunks, it)
                _assert_chain_close(outs[0].numpy() / scale, ref, fscale)
                _assert_chain_close(grads[0].numpy() / scale, gref, gscale)
        q.put((rank, "ok"))
    except Exception as e:  # report to the parent, then fail the worker
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _sweep_segments_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "dgl-1_amd")]
    from dgl import data, kernel
    from dgl.distributed import PartitionedGraph, balanced_bounds

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, F = 20000, 128
        src, dst, n = data.chung_lu(n, 60 * n, 30.0, seed=13)
        bounds = balanced_bounds(torch.bincount(dst, minlength=n), world)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        sel = (dst >= lo) & (dst < hi)
        gen = torch.Generator().manual_seed(17)
        H = torch.rand(n, F, generator=gen) * 2 - 1
        G = torch.randn(n, F, generator=gen)
        res = {}
        for on in (True, False):
            # the accumulating sweep's floors lowered to this small graph
            old = kernel.set_sweep_schedule(on=on, accum_table_min=0, accum_min_slots=1,
                                            block_bytes=256 << 10)
            try:
                pg = PartitionedGraph(n, src[sel], dst[sel], bounds, dev, pipeline_chunks=2,
                                      overlap=True)
                if on:  # the halo chunks' segments take the sweep
                    seg = pg.seg_csrs[-1]
                    path, _ = seg.plan.schedule(kernel.MSG_COPY_U, kernel.RED_SUM_ACCUM, F, 0,
                                                seg.num_cols)
                    assert path == kernel.PLAN_PATH_SWEEP, path
                outs = []
                for it in range(3):
                    h = (H[lo:hi] * float(it + 1)).to(dev).requires_grad_(True)
                    o = pg.update_all(h)
                    o.backward((G[lo:hi] * float(it + 1)).to(dev))
                    torch.cuda.synchronize()
                    outs.append((o.detach().cpu(), h.grad.cpu()))
                res[on] = outs
            finally:
                kernel.set_sweep_schedule(**old)
        for (a, ga), (b, gb) in zip(res[True], res[False]):
            assert torch.equal(a, b) and torch.equal(ga, gb)
        q.put((rank, "ok"))
    except Exception as e:  # report to the parent, then fail the worker
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_pipelined_segments_on_the_accumulating_sweep():
    """Two gloo ranks on the one GPU, F = 128, the pipelined exchange on its
    side stream: with the accumulating sweep's floors lowered the halo
    chunks' SUM_ACCUM segments run the source sweep; forward rows and
    backward gradients over three steps equal the other schedules' bit for
    bit."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.spawn(_sweep_segments_worker, args=(2, _free_port(), q), nprocs=2, join=True)
    got = sorted(q.get(timeout=5) for _ in range(2))
    assert got == [(0, "ok"), (1, "ok")], got


@pytest.mark.gpu
@pytest.mark.parametrize("graph", ["chung_lu", "banded"])
def test_pipelined_comm_stream_two_gloo_ranks_one_gpu(graph):
    """The pipelined exchange on its side stream (the RCCL path's events,
    waits and record_stream bookkeeping), driven by two gloo ranks on the one
    GPU of the pool: gloo orders its device copies against the stream a
    collective is issued on, as RCCL does. Forward rows and backward gradients
    over four reused steps equal the inline path's bit for bit in both halo
    modes (all-gather chunks with the reduce-scatter backward; all-to-allv
    chunks with the reverse all-to-allv), and the oracle's within 1e-5."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.spawn(_overlap_worker, args=(2, _free_port(), graph, q), nprocs=2, join=True)
    got = sorted(q.get(timeout=5) for _ in range(2))
    assert got == [(0, "ok"), (1, "ok")], got
