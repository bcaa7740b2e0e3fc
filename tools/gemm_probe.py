"""The GCN's dense products at configs[1]'s shapes (and R-GCN's 11,816 x 500 x 500) on each BLAS backend torch
offers on ROCm (hipBLASLt, rocBLAS): forward X·W (232,965 x 602 x 128), the
weight gradient Xᵀ·dA, and layer 2's (x 128 x 41) pair; ms per call by
events.

  python tools/gemm_probe.py
"""
import json

import torch


def ms(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def host_us(fn, iters=200):
    """Host time per call while the GPU keeps up (enqueue only)."""
    import time
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    t = (time.perf_counter() - t0) / iters * 1e6
    torch.cuda.synchronize()
    return t


def main():
    dev = torch.device("cuda", 0)
    n = 232965
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(n, 602, generator=g, device=dev)
    w1 = torch.randn(602, 128, generator=g, device=dev)
    da1 = torch.randn(n, 128, generator=g, device=dev)
    h1 = torch.randn(n, 128, generator=g, device=dev)
    w2 = torch.randn(128, 41, generator=g, device=dev)
    da2 = torch.randn(n, 41, generator=g, device=dev)
    hr = torch.randn(11816, 500, generator=g, device=dev)
    wr = torch.randn(500, 500, generator=g, device=dev)
    sm = torch.randn(64, 64, generator=g, device=dev)
    res = {}
    for lib in ("cublaslt", "cublas"):
        try:
            torch.backends.cuda.preferred_blas_library(lib)
        except Exception as err:  # noqa: BLE001
            res[lib] = str(err)
            continue
        r = {"fwd1 x@w1": ms(lambda: torch.mm(x, w1)),
             "dw1 x^T@da1": ms(lambda: torch.mm(x.t(), da1)),
             "fwd2 h1@w2": ms(lambda: torch.mm(h1, w2)),
             "dw2 h1^T@da2": ms(lambda: torch.mm(h1.t(), da2)),
             "dh1 da2@w2^T": ms(lambda: torch.mm(da2, w2.t())),
             "rgcn h@W (11816x500x500)": ms(lambda: torch.mm(hr, wr)),
             "rgcn h^T@d": ms(lambda: torch.mm(hr.t(), hr)),
             "host_us rgcn h@W": host_us(lambda: torch.mm(hr, wr)),
             "host_us small 64x64": host_us(lambda: torch.mm(sm, sm))}
        res[lib] = r
    # the weight gradients as split-K batched GEMMs (row chunks, partials summed)
    def splitk(a, b, chunks):
        n = a.shape[0]
        k = n // chunks
        m = k * chunks
        out = torch.bmm(a[:m].reshape(chunks, k, a.shape[1]).transpose(1, 2),
                        b[:m].reshape(chunks, k, b.shape[1])).sum(0)
        if m < n:
            out = out + a[m:].t().matmul(b[m:])
        return out
    torch.backends.cuda.preferred_blas_library("cublaslt")
    sk = {}
    for c in (8, 16, 32, 64, 128, 256):
        sk["dw1 chunks %d" % c] = ms(lambda: splitk(x, da1, c))
        sk["dw2 chunks %d" % c] = ms(lambda: splitk(h1, da2, c))
    res["splitk_hipblaslt"] = sk
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
