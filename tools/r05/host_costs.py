"""r05: host (enqueue) microseconds of the R-GCN step's building blocks on
the device, no synchronisation inside the timed loop."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import kernel  # noqa: E402


def host_us(fn, n=200):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    host = (time.perf_counter() - t) / n * 1e6
    torch.cuda.synchronize()
    return round(host, 1)


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    E, N, R = 30000, 11800, 474
    row = torch.randint(0, N, (E,), generator=g, device=dev)
    col = torch.randint(0, N, (E,), generator=g, device=dev)
    rel = torch.randint(0, R, (E,), generator=g, device=dev)
    rowc, colc = row.cpu(), col.cpu()
    res = {}
    res["build_csr device (validate=False)"] = host_us(
        lambda: kernel.build_csr(N, N, row, col, kernel.ORDER_EID, dev, schedule=False,
                                 validate=False))
    res["build_csr device (validate=True: one sync)"] = host_us(
        lambda: kernel.build_csr(N, N, row, col, kernel.ORDER_EID, dev, schedule=False))
    res["build_csr from host arrays (pinned upload)"] = host_us(
        lambda: kernel.build_csr(N, N, rowc, colc, kernel.ORDER_EID, dev, schedule=False,
                                 validate=False))
    c = kernel.build_csr(N, N, row, col, kernel.ORDER_EID, dev, schedule=False, validate=False)
    res["_typed_items"] = host_us(lambda: kernel._typed_items(c.indptr, E))
    res["_position_groups (2n)"] = host_us(lambda: kernel._position_groups(torch.cat([row, col]), N))
    res["torch.sort stable 60k"] = host_us(lambda: torch.sort(torch.cat([row, col]), stable=True))
    res["coo_to_csr_workspace_bytes"] = host_us(
        lambda: kernel.LIB.dglhip_coo_to_csr_workspace_bytes(N, N, E, 0))
    a = torch.randn(N, 500, device=dev)
    w = torch.randn(500, 500, device=dev)
    res["mm 11800x500x500 (default blas)"] = host_us(lambda: a @ w)
    try:
        old = torch.backends.cuda.preferred_blas_library()
        torch.backends.cuda.preferred_blas_library("cublas")
        res["mm (rocBLAS)"] = host_us(lambda: a @ w)
        res["mm t (rocBLAS)"] = host_us(lambda: a.t() @ a)
        torch.backends.cuda.preferred_blas_library("cublaslt")
        res["mm (hipBLASLt)"] = host_us(lambda: a @ w)
        res["mm t (hipBLASLt)"] = host_us(lambda: a.t() @ a)
        torch.backends.cuda.preferred_blas_library(old)
    except Exception as e:  # noqa: BLE001
        res["blas switch"] = str(e)
    res["index_select 30k rows"] = host_us(lambda: a.index_select(0, row))
    res["elementwise mul"] = host_us(lambda: a * 2.0)
    res["empty"] = host_us(lambda: torch.empty(1000, device=dev))
    for k, v in res.items():
        print("%-45s %s" % (k, v), flush=True)


if __name__ == "__main__":
    main()
