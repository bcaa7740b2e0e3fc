"""Test-side ctypes client of libdgl_hip's PackedFunc runtime.

It binds the library the way the reference's Python FFI binds libdgl
(python/dgl/_ffi/_ctypes/function.py:80-190: arguments packed as a DGLValue
union plus type codes; returns decoded by type code; arrays held as
NDARRAY_CONTAINER handles freed with DGLArrayFree; returned functions freed
with DGLFuncFree; Python callbacks wrapped with DGLFuncCreateFromCFunc), so the
tests exercise exactly the calling convention a reference build would use
against this library. Written for the tests; not imported by the package.
"""
import ctypes

import numpy as np
import torch
import torch.utils.dlpack

from dgl import _ffi

INT, UINT, FLOAT, HANDLE, NULL = 0, 1, 2, 3, 4
ARRAY_HANDLE, FUNC_HANDLE, STR, BYTES, NDARRAY_CONTAINER = 7, 10, 11, 12, 13
CPU, ROCM = 1, 10


class DGLValue(ctypes.Union):
    _fields_ = [("v_int64", ctypes.c_int64), ("v_float64", ctypes.c_double),
                ("v_handle", ctypes.c_void_p), ("v_str", ctypes.c_char_p)]


class DLTensor(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("device_type", ctypes.c_int32),
                ("device_id", ctypes.c_int32), ("ndim", ctypes.c_int32),
                ("code", ctypes.c_uint8), ("bits", ctypes.c_uint8), ("lanes", ctypes.c_uint16),
                ("shape", ctypes.POINTER(ctypes.c_int64)),
                ("strides", ctypes.POINTER(ctypes.c_int64)), ("byte_offset", ctypes.c_uint64)]


PackedCFunc = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(DGLValue),
                               ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_void_p,
                               ctypes.c_void_p)
CFuncFinalizer = ctypes.CFUNCTYPE(None, ctypes.c_void_p)

LIB = ctypes.CDLL(_ffi.lib_path(), mode=ctypes.RTLD_GLOBAL)
LIB.DGLGetLastError.restype = ctypes.c_char_p
LIB.DGLAPISetLastError.argtypes = [ctypes.c_char_p]
LIB.DGLDLManagedTensorCallDeleter.argtypes = [ctypes.c_void_p]
LIB.DGLDLManagedTensorCallDeleter.restype = None


class CAPIError(RuntimeError):
    pass


def check(rc):
    if rc != 0:
        raise CAPIError(LIB.DGLGetLastError().decode())


_DTYPES = {np.dtype(np.int64): (0, 64), np.dtype(np.int32): (0, 32),
           np.dtype(np.float32): (2, 32), np.dtype(np.float64): (2, 64)}
_NP = {(0, 64): np.int64, (0, 32): np.int32, (2, 32): np.float32, (2, 64): np.float64}


class NDArray(object):
    """Owning handle of a library array (NDArrayBase, _ctypes/ndarray.py:52-90)."""

    def __init__(self, handle, is_view=False):
        self.handle = ctypes.c_void_p(handle)
        self.is_view = is_view

    def __del__(self):
        if not self.is_view and LIB is not None and self.handle:
            check(LIB.DGLArrayFree(self.handle))

    @property
    def dl(self):
        return ctypes.cast(self.handle, ctypes.POINTER(DLTensor)).contents

    @property
    def shape(self):
        d = self.dl
        return tuple(d.shape[i] for i in range(d.ndim))

    @property
    def device_type(self):
        return self.dl.device_type

    @property
    def dtype(self):
        d = self.dl
        return _NP[(d.code, d.bits)]

    def numpy(self):
        out = np.empty(self.shape, dtype=self.dtype)
        check(LIB.DGLArrayCopyToBytes(self.handle, out.ctypes.data_as(ctypes.c_void_p),
                                      ctypes.c_size_t(out.nbytes)))
        return out

    def to_torch(self):
        """Zero-copy torch view (zerocopy_from_dgl_ndarray: DGLArrayToDLPack)."""
        ptr = ctypes.c_void_p()
        check(LIB.DGLArrayToDLPack(self.handle, ctypes.byref(ptr)))
        capsule = _capsule_new(ptr)
        return torch.utils.dlpack.from_dlpack(capsule)


def empty(shape, dtype=np.int64, device_type=CPU, device_id=0):
    code, bits = _DTYPES[np.dtype(dtype)]
    sh = (ctypes.c_int64 * len(shape))(*shape)
    h = ctypes.c_void_p()
    check(LIB.DGLArrayAlloc(sh, len(shape), code, bits, 1, device_type, device_id,
                            ctypes.byref(h)))
    return NDArray(h.value)


def array(x, device_type=CPU, device_id=0):
    """nd.array: alloc + DGLArrayCopyFromBytes (python/dgl/_ffi/ndarray.py:105-240)."""
    x = np.ascontiguousarray(x)
    a = empty(x.shape, x.dtype, device_type, device_id)
    check(LIB.DGLArrayCopyFromBytes(a.handle, x.ctypes.data_as(ctypes.c_void_p),
                                    ctypes.c_size_t(x.nbytes)))
    return a


ctypes.pythonapi.PyCapsule_New.restype = ctypes.py_object
ctypes.pythonapi.PyCapsule_New.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]
ctypes.pythonapi.PyCapsule_GetPointer.restype = ctypes.c_void_p
ctypes.pythonapi.PyCapsule_GetPointer.argtypes = [ctypes.py_object, ctypes.c_char_p]
ctypes.pythonapi.PyCapsule_SetName.argtypes = [ctypes.py_object, ctypes.c_char_p]
ctypes.pythonapi.PyCapsule_SetDestructor.argtypes = [ctypes.py_object, ctypes.c_void_p]
ctypes.pythonapi.PyCapsule_IsValid.argtypes = [ctypes.py_object, ctypes.c_char_p]
_Destructor = ctypes.CFUNCTYPE(None, ctypes.c_void_p)


@_Destructor
def _capsule_deleter(capsule):
    cap = ctypes.cast(capsule, ctypes.py_object)
    if ctypes.pythonapi.PyCapsule_IsValid(cap, b"dltensor"):
        LIB.DGLDLManagedTensorCallDeleter(ctypes.pythonapi.PyCapsule_GetPointer(cap, b"dltensor"))


def _capsule_new(ptr):
    return ctypes.pythonapi.PyCapsule_New(ptr, b"dltensor",
                                          ctypes.cast(_capsule_deleter, ctypes.c_void_p))


def from_torch(t):
    """zerocopy_to_dgl_ndarray: torch DLPack capsule -> DGLArrayFromDLPack."""
    cap = torch.utils.dlpack.to_dlpack(t.contiguous())
    ptr = ctypes.pythonapi.PyCapsule_GetPointer(cap, b"dltensor")
    h = ctypes.c_void_p()
    check(LIB.DGLArrayFromDLPack(ctypes.c_void_p(ptr), ctypes.byref(h)))
    ctypes.pythonapi.PyCapsule_SetName(cap, b"used_dltensor")
    ctypes.pythonapi.PyCapsule_SetDestructor(cap, None)
    return NDArray(h.value)


def ids(x):
    return array(np.asarray(x, dtype=np.int64).reshape(-1))


class Function(object):
    """Packed function handle (FunctionBase, _ctypes/function.py:150-190)."""

    def __init__(self, handle, is_global):
        self.handle = ctypes.c_void_p(handle)
        self.is_global = is_global

    def __del__(self):
        if not self.is_global and LIB is not None and self.handle:
            check(LIB.DGLFuncFree(self.handle))

    def __call__(self, *args):
        values, codes, keep = pack_args(args)
        ret = DGLValue()
        code = ctypes.c_int()
        check(LIB.DGLFuncCall(self.handle, values, codes, ctypes.c_int(len(args)),
                              ctypes.byref(ret), ctypes.byref(code)))
        del keep
        return decode(ret, code.value)


class ByteArray(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("size", ctypes.c_size_t)]


def decode(v, code):
    if code == INT:
        return v.v_int64
    if code == FLOAT:
        return v.v_float64
    if code == HANDLE:
        return ctypes.c_void_p(v.v_handle)
    if code == NULL:
        return None
    if code == STR:
        return v.v_str.decode()
    if code == BYTES:
        ba = ctypes.cast(v.v_handle, ctypes.POINTER(ByteArray)).contents
        return ctypes.string_at(ba.data, ba.size)
    if code == NDARRAY_CONTAINER:
        return NDArray(v.v_handle)
    if code == ARRAY_HANDLE:
        return NDArray(v.v_handle, is_view=True)
    if code == FUNC_HANDLE:
        return Function(v.v_handle, False)
    raise TypeError("unknown return type code %d" % code)


def pack_args(args):
    n = len(args)
    values = (DGLValue * n)()
    codes = (ctypes.c_int * n)()
    keep = []
    for i, a in enumerate(args):
        if a is None:
            values[i].v_handle = None
            codes[i] = NULL
        elif isinstance(a, NDArray):
            values[i].v_handle = a.handle
            codes[i] = ARRAY_HANDLE if a.is_view else NDARRAY_CONTAINER
        elif isinstance(a, bool):
            values[i].v_int64 = int(a)
            codes[i] = INT
        elif isinstance(a, (int, np.integer)):
            values[i].v_int64 = int(a)
            codes[i] = INT
        elif isinstance(a, float):
            values[i].v_float64 = a
            codes[i] = FLOAT
        elif isinstance(a, str):
            b = a.encode()
            keep.append(b)
            values[i].v_str = b
            codes[i] = STR
        elif isinstance(a, ctypes.c_void_p):
            values[i].v_handle = a
            codes[i] = HANDLE
        elif isinstance(a, Function):
            values[i].v_handle = a.handle
            codes[i] = FUNC_HANDLE
        elif callable(a):
            f = convert_func(a)
            keep.append(f)
            values[i].v_handle = f.handle
            codes[i] = FUNC_HANDLE
        else:
            raise TypeError("cannot pass %r" % type(a))
    return values, codes, keep


_live_callbacks = {}


@CFuncFinalizer
def _finalize(resource):
    _live_callbacks.pop(resource, None)


def convert_func(pyfunc):
    """Python callable -> packed function (convert_to_dgl_func, function.py:31-79)."""

    def cfun(args, type_codes, num_args, ret, _resource):
        pyargs = []
        for i in range(num_args):
            code = type_codes[i]
            if code in (NDARRAY_CONTAINER, FUNC_HANDLE):
                check(LIB.DGLCbArgToReturn(ctypes.byref(args[i]), code))
            pyargs.append(decode(args[i], code))
        try:
            rv = pyfunc(*pyargs)
        except Exception as e:  # noqa: BLE001
            LIB.DGLAPISetLastError(str(e).encode())
            return -1
        if rv is not None:
            values, codes, keep = pack_args((rv,))
            check(LIB.DGLCFuncSetReturn(ctypes.c_void_p(ret), values, codes, ctypes.c_int(1)))
            del keep
        return 0

    f = PackedCFunc(cfun)
    key = id(f)
    _live_callbacks[key] = f
    h = ctypes.c_void_p()
    check(LIB.DGLFuncCreateFromCFunc(f, ctypes.c_void_p(key), _finalize, ctypes.byref(h)))
    return Function(h.value, False)


def get_global(name):
    h = ctypes.c_void_p()
    check(LIB.DGLFuncGetGlobal(name.encode(), ctypes.byref(h)))
    if not h.value:
        raise CAPIError("no global function %s" % name)
    return Function(h.value, True)


def register_global(name, f, override=False):
    if not isinstance(f, Function):
        f = convert_func(f)
    check(LIB.DGLFuncRegisterGlobal(name.encode(), f.handle, int(override)))
    return f


def global_names():
    size = ctypes.c_int()
    arr = ctypes.POINTER(ctypes.c_char_p)()
    check(LIB.DGLFuncListGlobalNames(ctypes.byref(size), ctypes.byref(arr)))
    return [arr[i].decode() for i in range(size.value)]


class CAPI(object):
    """Attribute access to ``<namespace>._CAPI_<name>`` (the reference's
    _init_api, python/dgl/_ffi/function.py:267-306)."""

    def __init__(self, namespace):
        self._ns = namespace

    def __getattr__(self, name):
        return get_global("%s.%s" % (self._ns, name))


GI = CAPI("graph_index")
DB = CAPI("runtime.degree_bucketing")


def edge_triple(f):
    """(src, dst, id) numpy arrays from an EdgeArray packed function."""
    return tuple(f(i).numpy() for i in range(3))
