"""The C runtime entry points the reference's ctypes layer binds
(python/dgl/_ffi: DGLArray*, DLPack exchange, DGLFunc*, callbacks, streams,
modules), on libdgl_hip.so through capi_client.py. The GPU case runs the
engine's g-SpMM on library-allocated ROCm arrays through the registry."""
import ctypes

import numpy as np
import pytest
import torch

import capi_client as C

from oracle import oracle as O


def test_array_alloc_copy_roundtrip():
    x = np.arange(12, dtype=np.float32).reshape(3, 4)
    a = C.array(x)
    assert a.shape == (3, 4) and a.dtype == np.float32 and a.device_type == C.CPU
    assert np.array_equal(a.numpy(), x)
    b = C.empty((3, 4), np.float32)
    C.check(C.LIB.DGLArrayCopyFromTo(a.handle, b.handle, None))
    assert np.array_equal(b.numpy(), x)
    with pytest.raises(C.CAPIError, match="byte count"):
        C.check(C.LIB.DGLArrayCopyFromBytes(a.handle, x.ctypes.data_as(ctypes.c_void_p),
                                            ctypes.c_size_t(4)))
    c = C.empty((2, 2), np.float32)
    with pytest.raises(C.CAPIError, match="different byte sizes"):
        C.check(C.LIB.DGLArrayCopyFromTo(a.handle, c.handle, None))
    e = C.empty((0,), np.int64)  # empty arrays are valid
    assert e.numpy().shape == (0,)


def test_dlpack_zero_copy_both_ways():
    t = torch.arange(10, dtype=torch.int64)
    a = C.from_torch(t)
    assert a.numpy().tolist() == list(range(10))
    t[3] = 42  # shares memory with the torch tensor
    assert a.numpy()[3] == 42
    back = a.to_torch()
    back[0] = -1
    assert t[0] == -1
    del a, back
    assert t.sum().item() == sum(range(10)) - 3 + 42 - 1
    # library-owned array exported to torch outlives its Python handle
    b = C.array(np.array([1.5, 2.5], dtype=np.float32))
    tb = b.to_torch()
    del b
    assert tb.tolist() == [1.5, 2.5]


def test_returned_arrays_and_functions_are_owned():
    f = C.get_global("graph_index._CAPI_DGLGraphGetAdj")
    g = C.get_global("graph_index._CAPI_DGLGraphCreateMutable")(False)
    C.GI._CAPI_DGLGraphAddVertices(g, 3)
    C.GI._CAPI_DGLGraphAddEdges(g, C.ids([0, 1]), C.ids([1, 2]))
    adj = f(g, False, "coo")
    assert isinstance(adj, C.Function) and not adj.is_global
    idx = adj(0)
    del adj  # the array keeps its own reference
    assert idx.numpy().tolist() == [1, 2, 0, 1]
    with pytest.raises(C.CAPIError, match="invalid choice"):
        f(g, False, "coo")(2)
    C.GI._CAPI_DGLGraphFree(g)


def test_python_callback_roundtrip_and_errors():
    seen = []

    def add(a, b):
        seen.append((a, b))
        return a + b

    fn = C.convert_func(add)
    assert fn(2, 3) == 5 and seen == [(2, 3)]
    assert C.convert_func(lambda s: s + "!")("hi") == "hi!"
    # an array argument is received (DGLCbArgToReturn) and returned (DGLCFuncSetReturn)
    arr = C.array(np.array([7, 8], dtype=np.int64))
    ident = C.convert_func(lambda x: x)
    out = ident(arr)
    assert isinstance(out, C.NDArray) and out.numpy().tolist() == [7, 8]
    del arr
    assert out.numpy().tolist() == [7, 8]

    def boom():
        raise ValueError("callback failed")

    with pytest.raises(C.CAPIError, match="callback failed"):
        C.convert_func(boom)()


def test_register_global_override_and_names():
    C.register_global("test.capi.double", lambda x: 2 * x)
    assert "test.capi.double" in C.global_names()
    assert C.get_global("test.capi.double")(21) == 42
    with pytest.raises(C.CAPIError, match="already registered"):
        C.register_global("test.capi.double", lambda x: x)
    C.register_global("test.capi.double", lambda x: 3 * x, override=True)
    assert C.get_global("test.capi.double")(2) == 6
    # a packed function passed as an argument is callable from the callee
    apply = C.convert_func(lambda f, v: f(v))
    assert apply(C.get_global("test.capi.double"), 5) == 15


def test_modules_streams_and_ext_types_on_cpu():
    h = ctypes.c_void_p()
    with pytest.raises(C.CAPIError, match="compiled into"):
        C.check(C.LIB.DGLModLoadFromFile(b"x.so", b"so", ctypes.byref(h)))
    assert C.LIB.DGLModFree(None) == 0
    assert C.LIB.DGLExtTypeFree(None, 15) == 0
    with pytest.raises(C.CAPIError):
        C.check(C.LIB.DGLModGetFunction(None, b"f", 0, ctypes.byref(h)))
    # CPU streams are no-ops
    C.check(C.LIB.DGLStreamCreate(C.CPU, 0, ctypes.byref(h)))
    assert h.value is None
    C.check(C.LIB.DGLSynchronize(C.CPU, 0, None))
    C.check(C.LIB.DGLStreamFree(C.CPU, 0, None))


def test_device_attr_cpu():
    attr = C.get_global("_GetDeviceAttr")
    assert attr(C.CPU, 0, 0) == 1  # kExist


@pytest.mark.gpu
def test_device_attr_rocm():
    attr = C.get_global("_GetDeviceAttr")
    assert attr(C.ROCM, 0, 0) == 1 and attr(C.ROCM, 4096, 0) == 0
    assert attr(C.ROCM, 0, 2) == 64  # wavefront width
    assert attr(C.ROCM, 0, 5).startswith("gfx950")
    assert attr(C.ROCM, 0, 7) == torch.cuda.get_device_properties(0).multi_processor_count


@pytest.mark.gpu
def test_device_arrays_gspmm_through_registry():
    """Library-allocated ROCm arrays, host<->device copies, a library stream
    made current with DGLSetStream, and the g-SpMM registry call on it; the
    result equals the oracle bit for bit."""
    torch.cuda.init()
    rng = np.random.default_rng(0)
    n, m, F = 500, 6000, 32
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n, m)
    H = rng.standard_normal((n, F)).astype(np.float32)
    indptr = np.empty(n + 1, np.int64)
    indices = np.empty(m, np.int32)
    eid = np.empty(m, np.int64)
    row, col = C.array(dst.astype(np.int64)), C.array(src.astype(np.int64))
    hp, hi, he = C.empty((n + 1,)), C.empty((m,), np.int32), C.empty((m,))
    C.get_global("dglhip._CAPI_COOToCSR")(n, n, row, col, 0, hp, hi, he)
    indptr, indices, eid = hp.numpy(), hi.numpy(), he.numpy()
    d_ptr, d_idx, d_eid = (C.array(x, C.ROCM, 0) for x in (indptr, indices, eid))
    d_h = C.array(H, C.ROCM, 0)
    d_out = C.empty((n, F), np.float32, C.ROCM, 0)
    s = ctypes.c_void_p()
    C.check(C.LIB.DGLStreamCreate(C.ROCM, 0, ctypes.byref(s)))
    C.check(C.LIB.DGLSetStream(C.ROCM, 0, s))
    try:
        C.get_global("dglhip._CAPI_GSpMM")(0, 0, d_ptr, d_idx, d_eid, d_h, None, d_out, None,
                                           None, None)
        C.check(C.LIB.DGLSynchronize(C.ROCM, 0, s))
        got = d_out.numpy()
        # device -> device copy, then read back
        d_copy = C.empty((n, F), np.float32, C.ROCM, 0)
        C.check(C.LIB.DGLArrayCopyFromTo(d_out.handle, d_copy.handle, s))
        C.check(C.LIB.DGLSynchronize(C.ROCM, 0, s))
        assert np.array_equal(d_copy.numpy(), got)
    finally:
        C.check(C.LIB.DGLSetStream(C.ROCM, 0, None))
        C.check(C.LIB.DGLStreamFree(C.ROCM, 0, s))
    assert np.array_equal(got, O.spmm_coo(n, dst, src, H))
    # a torch ROCm tensor enters through DLPack without a copy
    t = torch.from_numpy(H).cuda()
    a = C.from_torch(t)
    assert a.device_type == C.ROCM and a.dl.data == t.data_ptr()
