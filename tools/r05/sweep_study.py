"""Source-swept g-SpMM (csrc/sweep.hip) against the engine's schedule on the
Reddit-shaped graph (copy_u + sum, F = 128): bits vs the one-launch kernel
and per-call ms (one event pair around each call), for a grid of source
block sizes and rows per wave, interleaved rounds.

  python tools/r05/sweep_study.py [--mib 2 3 4 6] [--rpw 10 20] [--rounds 3]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import data, kernel  # noqa: E402
from dgl._ffi import LIB, check_call, ptr  # noqa: E402


def timed(fn, iters):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(iters)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in ev) / iters


def stream_layout(csr, F, lo, hi, order, mib, rpw):
    """Slots laid out per (launch, block, wave, row), as the stream kernel
    (dglhip_gspmm_sweep_stream_device) reads them: the kernel deals row i of
    ``order`` to wave (i // W odd ? W - 1 - i % W : i % W) as its row i // W,
    and reads wave w's block-b run at seg[w, b]. None when a row's source
    blocks go back down (the layout keeps each row's block-b slots together)."""
    dev = csr.indptr.device
    n = csr.num_rows
    bs = max(1, int(mib * (1 << 20)) // (F * 4))
    B = max(1, -(-(hi - lo) // bs))
    deg = csr.indptr[1:] - csr.indptr[:-1]
    rows = torch.repeat_interleave(torch.arange(n, device=dev), deg)
    blk = (csr.indices.long() - lo) // bs
    if bool(((rows[1:] == rows[:-1]) & (blk[1:] < blk[:-1])).any()):
        return None
    wpl = ctypes.c_int64()
    check_call(LIB.dglhip_gspmm_sweep_stream_geometry(rpw, 0, ctypes.byref(wpl)))
    wpl = wpl.value
    L = -(-n // (wpl * rpw))
    W = L * wpl
    i = torch.arange(n, device=dev)
    j, pos = i // W, i % W
    wave = torch.where(j % 2 == 1, W - 1 - pos, pos)
    ro = order.long() if order is not None else i
    wave_of = torch.empty(n, dtype=torch.int64, device=dev)
    j_of = torch.empty(n, dtype=torch.int64, device=dev)
    wave_of[ro] = wave
    j_of[ro] = j
    key = (((wave_of[rows] // wpl) * B + blk) * W + wave_of[rows]) * rpw + j_of[rows]
    skey, perm = torch.sort(key, stable=True)
    lay = csr.indices[perm].contiguous()
    w_all = torch.arange(W, device=dev)
    q = (((w_all[:, None] // wpl) * B + torch.arange(B, device=dev)[None, :]) * W
         + w_all[:, None]) * rpw
    seg = torch.searchsorted(skey, q.reshape(-1)).contiguous()
    counts = torch.bincount(rows * B + blk, minlength=n * B).to(torch.int32)
    return {"W": W, "B": B, "lay": lay, "seg": seg, "counts": counts, "launches": L}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=float, nargs="+", default=[2, 3, 4, 6])
    ap.add_argument("--rpw", type=int, nargs="+", default=[10, 20])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--order", default="eid", choices=["eid", "random"])
    ap.add_argument("--out", default=None)
    ap.add_argument("--stream", action="store_true", help="also the streamed layout kernel")
    ap.add_argument("--lag", type=int, nargs="+", default=[0, 1, 2])
    ap.add_argument("--per-cu", type=int, default=0, help="workgroups per CU (0: occupancy)")
    ap.add_argument("--unroll", type=int, default=16)
    ap.add_argument("--scale", type=int, default=1, help="weak-scaled graph, rank 0's rows")
    ap.add_argument("--no-cursor", action="store_true", help="skip the cursor kernel")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(scale=args.scale, device=dev)
    n_src = n
    if args.scale > 1:
        # rank 0 of a weak-scaled N-rank row split: its rows' in-edges, sources
        # over all N x 232,965 nodes (the table N times the headline's)
        n = n // args.scale
        keep = dst < n
        src, dst = src[keep], dst[keep]
        o = torch.argsort(src * n + dst)  # source-major, as the generator numbers them
        src, dst = src[o], dst[o]
        del keep, o
    if args.order == "random":
        g = torch.Generator(device=dev).manual_seed(5)
        p = torch.randperm(src.numel(), device=dev, generator=g)
        src, dst = src[p], dst[p]
    adj = kernel.from_coo(n, n_src, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    csr = adj.fwd
    F = 128
    h = torch.rand(n_src, F, device=dev) * 2 - 1
    out = torch.empty(n, F, device=dev)
    old = kernel.set_blocked("off")
    kernel.gspmm_into(csr, out, h)
    ref = out.clone()
    kernel.set_blocked(old)
    lo = int(csr.indices.min())
    hi = int(csr.indices.max()) + 1
    order = csr.row_order
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    def sweep(mib, rpw):
        bs = max(1, int(mib * (1 << 20)) // (F * 4))
        nb = max(1, -(-(hi - lo) // bs))
        check_call(LIB.dglhip_gspmm_sweep_device(
            n, F, ptr(csr.indptr), ptr(csr.indices), ptr(h), ptr(out), ptr(order), lo, bs, nb,
            0, rpw, stream))
        return nb

    def layout(mib, rpw):
        return stream_layout(csr, F, lo, hi, order, mib, rpw)

    arrive = torch.zeros(1 << 22, dtype=torch.int32, device=dev)

    def stream_run(lt, rpw, lag):
        check_call(LIB.dglhip_gspmm_sweep_stream_device(
            n, lt["W"], ptr(order), ptr(lt["counts"]), lt["B"], ptr(lt["seg"]), ptr(lt["lay"]),
            ptr(csr.indptr), ptr(h), ptr(out), 0, rpw, 0, ptr(arrive), arrive.numel(), lag, 2000,
            stream))

    res = {"graph": "reddit_like", "order": args.order, "rounds": []}
    layouts = {}
    if args.per_cu:
        check_call(LIB.dglhip_set_sweep_per_cu(args.per_cu))
    check_call(LIB.dglhip_set_sweep_unroll(args.unroll))
    if args.stream:
        for mib in args.mib:
            for rpw in args.rpw:
                layouts[(mib, rpw)] = layout(mib, rpw)
    for _ in range(args.rounds):
        row = {"engine_ms": timed(lambda: kernel.gspmm_into(csr, out, h), args.iters)}
        torch.cuda.synchronize()
        row["engine_bits_equal"] = bool(torch.equal(out, ref))
        for mib in ([] if args.no_cursor else args.mib):
            for rpw in sorted({20 if r == 19 else r for r in args.rpw}):  # cursor: 10 or 20
                out.fill_(float("nan"))
                nb = sweep(mib, rpw)
                torch.cuda.synchronize()
                same = bool(torch.equal(out, ref))
                ms = timed(lambda: sweep(mib, rpw), args.iters)
                row["sweep_%gMiB_rpw%d" % (mib, rpw)] = {"ms": ms, "blocks": nb,
                                                         "bits_equal": same}
        for (mib, rpw), lt in layouts.items():
            if lt is None:
                continue
            for lag in args.lag:
                out.fill_(float("nan"))
                stream_run(lt, rpw, lag)
                torch.cuda.synchronize()
                same = bool(torch.equal(out, ref))
                ms = timed(lambda: stream_run(lt, rpw, lag), args.iters)
                row["stream_%gMiB_rpw%d_lag%d" % (mib, rpw, lag)] = {
                    "ms": ms, "blocks": lt["B"], "launches": lt["launches"], "bits_equal": same}
        res["rounds"].append(row)
        print(json.dumps(row), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
