"""ctypes binding of libdgl_hip.so (the engine's C-ABI, include/dgl_hip.h).

Mirrors the reference's FFI layer (python/dgl/_ffi/base.py:31-62): the shared
library is located (``DGL_LIBRARY_PATH`` first, then the in-tree build), loaded
once, and every call goes through :func:`check_call`, which turns a -1 return
into ``DGLError(DGLGetLastError())``.

There is no fallback: if the library cannot be loaded every kernel entry
point raises. Build it with ``make -C dgl-1_amd/csrc`` (or
``__graft_entry__.build()``).
"""
from __future__ import absolute_import

import ctypes
import os

import torch  # noqa: F401  (loads the HIP runtime torch links against first)

from .base import DGLError

__all__ = ["LIB", "check_call", "lib_path", "tensor_arg", "call_packed", "list_global_names",
           "PackedFunction", "get_global_func", "CAPINamespace"]

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIBNAME = "libdgl_hip.so"


def lib_path():
    """Candidate location of libdgl_hip.so (python/dgl/_ffi/libinfo.py:7-60)."""
    cands = []
    env = os.environ.get("DGL_LIBRARY_PATH")
    if env:
        for d in env.split(os.pathsep):
            cands.append(os.path.join(d, _LIBNAME) if os.path.isdir(d) else d)
    cands.append(os.path.join(os.path.dirname(_HERE), "lib", _LIBNAME))
    for c in cands:
        if os.path.isfile(c):
            return c
    raise DGLError("cannot find %s (looked in %s); build it with "
                   "`make -C dgl-1_amd/csrc`" % (_LIBNAME, ", ".join(cands)))


_c_i64 = ctypes.c_int64
_c_int = ctypes.c_int
_vp = ctypes.c_void_p
_c_float = ctypes.c_float
_c_u64 = ctypes.c_uint64


def _load():
    lib = ctypes.CDLL(lib_path(), mode=ctypes.RTLD_GLOBAL)
    sig = {
        "DGLGetLastError": (ctypes.c_char_p, []),
        "dglhip_abi_version": (_c_int, []),
        "dglhip_build_info": (ctypes.c_char_p, []),
        "dglhip_coo_to_csr_host": (_c_int, [_c_i64, _c_i64, _c_i64, _vp, _vp, _c_int, _vp, _vp, _vp]),
        "dglhip_rows_by_degree_host": (_c_int, [_c_i64, _vp, _vp]),
        "dglhip_coo_to_csr_workspace_bytes": (_c_i64, [_c_i64, _c_i64, _c_i64, _c_int]),
        "dglhip_coo_to_csr_device": (_c_int, [_c_i64, _c_i64, _c_i64, _vp, _vp, _c_int, _vp, _vp,
                                              _vp, _vp, _c_i64, _vp]),
        "dglhip_gspmm_device": (_c_int, [_c_int, _c_int, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp,
                                         _c_i64, _vp, _vp, _vp, _vp]),
        "dglhip_gspmm_chunked_device": (_c_int, [_c_int, _c_int, _c_i64, _vp, _vp, _vp, _vp, _vp,
                                                 _c_i64, _vp, _c_i64, _vp, _c_i64, _vp, _vp,
                                                 _c_i64, _vp, _vp, _vp, _c_i64, _vp]),
        "dglhip_gspmm_ranges_device": (_c_int, [_c_int, _c_i64, _c_i64, _vp, _vp, _c_int, _vp, _vp,
                                                _vp, _vp, _c_i64, _vp, _vp]),
        "dglhip_gspmm_ranges_host": (_c_int, [_c_int, _c_i64, _c_i64, _vp, _vp, _c_int, _vp, _vp,
                                              _vp, _vp, _c_i64, _vp, _c_int]),
        "dglhip_gat_backward_t_ok": (_c_int, [_c_i64, _c_i64]),
        "dglhip_gat_backward_t_device": (_c_int, [_c_i64, _vp, _vp, _vp, _c_int, _c_int] +
                                         [_c_i64] * 4 + [_vp] * 7 +
                                         [_c_float, _c_float, _c_float, _c_int, _c_float,
                                          _c_u64, _vp, _vp, _vp, _vp, _vp]),
        "dglhip_gat_backward_t_packed_device": (_c_int, [_c_i64, _vp, _vp, _vp, _c_int, _c_int] +
                                                [_c_i64] * 4 + [_vp] * 6 +
                                                [_c_float, _c_float, _c_float, _c_int, _c_float,
                                                 _c_u64, _vp, _vp, _vp, _vp, _vp]),
        "dglhip_rowsum_heads8_device": (_c_int, [_c_i64, _vp, _vp, _vp, _vp, _vp]),
        "dglhip_gat_attention_grad_keep_ranges_device": (
            _c_int, [_c_i64, _c_i64, _c_i64] + [_vp] * 8 +
            [_c_float, _c_float, _c_float, _c_int, _c_float, _c_u64, _vp, _vp, _vp, _vp]),
        "dglhip_gat_attention_grad_logits_ranges_device": (
            _c_int, [_c_i64, _c_i64, _c_i64] + [_vp] * 11 +
            [_c_float, _c_float, _c_float, _c_int, _c_float, _c_float, _c_u64, _vp, _vp, _vp,
             _vp]),
        "dglhip_set_typed_block_width": (_c_int, [_c_int]),
        "dglhip_typed_items_workspace_bytes": (_c_i64, [_c_i64]),
        "dglhip_typed_items_device": (_c_int, [_c_i64, _vp, _c_i64, _vp, _vp, _vp, _c_i64, _vp]),
        "dglhip_distmult_score_device": (_c_int, [_c_i64] * 4 + [_vp] * 7),
        "dglhip_distmult_score_host": (_c_int, [_c_i64] * 4 + [_vp] * 6 + [_c_int]),
        "dglhip_distmult_grad_device": (_c_int, [_c_int] + [_c_i64] * 6 + [_vp] * 13),
        "dglhip_distmult_grad_host": (_c_int, [_c_int] + [_c_i64] * 5 + [_vp] * 9 + [_c_int]),
        "dglhip_distmult_loss_workspace_floats": (_c_i64, [_c_i64] * 4),
        "dglhip_distmult_loss_fwd_device": (_c_int, [_c_i64] * 4 + [_vp] * 6 + [_c_float] +
                                            [_vp] * 3 + [_c_i64, _vp]),
        "dglhip_distmult_loss_grad_device": (_c_int, [_c_int] + [_c_i64] * 6 + [_vp] * 10 +
                                             [_c_float] + [_vp] * 5),
        "dglhip_typed_block_spmm_device": (_c_int, [_c_i64] * 5 + [_vp] * 3 + [_c_i64] +
                                           [_vp] * 9),
        "dglhip_typed_block_spmm_host": (_c_int, [_c_i64] * 4 + [_vp] * 7 + [_c_int]),
        "dglhip_typed_block_wgrad_device": (_c_int, [_c_i64] * 5 + [_vp] * 3 + [_c_i64] +
                                            [_vp] * 9),
        "dglhip_typed_block_wgrad_host": (_c_int, [_c_i64] * 4 + [_vp] * 7 + [_c_int]),
        "dglhip_group_positions_workspace_bytes": (_c_i64, [_c_i64, _c_i64]),
        "dglhip_group_positions_device": (_c_int, [_c_i64, _c_i64, _vp, _c_i64] + [_vp] * 5 +
                                          [_c_i64, _vp]),
        "dglhip_relation_groups_workspace_bytes": (_c_i64, [_c_i64, _c_i64]),
        "dglhip_relation_groups_device": (_c_int, [_c_i64] * 3 + [_vp] * 4 + [_c_i64] +
                                          [_vp] * 7 + [_c_i64, _vp]),
        "dglhip_set_blocked_mean_add": (_c_int, [_c_int]),
        "dglhip_node_epilogue_parts": (_c_i64, [_c_i64]),
        "dglhip_node_epilogue_fwd_device": (_c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _c_int, _vp,
                                                     _vp]),
        "dglhip_node_epilogue_bwd_device": (_c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _c_int, _vp,
                                                     _vp, _vp]),
        "dglhip_typed_block_msg_ok": (_c_int, [_c_i64] * 3),
        "dglhip_set_typed_block_messages": (_c_int, [_c_int]),
        "dglhip_typed_block_msg_device": (_c_int, [_c_i64] * 5 + [_vp] * 8 + [_c_int] +
                                          [_vp] * 2),
        "dglhip_typed_msg_sum_device": (_c_int, [_c_i64] * 3 + [_vp] * 3 + [_c_i64] +
                                        [_vp] * 8),
        "dglhip_typed_block_wgrad_scaled_device": (_c_int, [_c_i64] * 5 + [_vp] * 3 + [_c_i64] +
                                                   [_vp] * 10),
        "dglhip_gsddmm_attention_device": (_c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp,
                                                    ctypes.c_float, ctypes.c_float,
                                                    ctypes.c_float, _c_int, _vp, _vp]),
        "dglhip_gsddmm_attention_host": (_c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp,
                                                  ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                                  _c_int, _vp, _c_int]),
        "dglhip_gat_aggregate_device": (_c_int, [_c_i64, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp,
                                                 _vp, _vp,
                                                 _vp, ctypes.c_float, ctypes.c_float,
                                                 ctypes.c_float, _c_int, ctypes.c_float,
                                                 ctypes.c_uint64, _vp, _vp, _vp, _vp, _vp, _vp]),
        "dglhip_gat_aggregate_logits_ranges_device": (
            _c_int, [_c_i64] * 4 + [_vp, _vp, _c_int] + [_vp] * 6 +
            [ctypes.c_float, ctypes.c_float, ctypes.c_float, _c_int, ctypes.c_float,
             ctypes.c_uint64] + [_vp] * 6),
        "dglhip_gat_logits_device": (_c_int, [_c_i64] * 3 + [_vp] * 6),
        "dglhip_gat_logits_host": (_c_int, [_c_i64] * 3 + [_vp] * 5 + [_c_int]),
        "dglhip_set_gat_logit_recompute": (_c_int, [_c_int]),
        "dglhip_gat_aggregate_ranges_device": (_c_int, [_c_i64, _c_i64, _c_i64, _c_i64, _vp,
                                                        _vp, _c_int, _vp, _vp, _vp, _vp, _vp,
                                                        ctypes.c_float, ctypes.c_float,
                                                        ctypes.c_float, _c_int, ctypes.c_float,
                                                        ctypes.c_uint64, _vp, _vp, _vp, _vp, _vp,
                                                        _vp]),
        "dglhip_set_gat_variant": (_c_int, [_c_int]),
        "dglhip_set_gat_bwd_variant": (_c_int, [_c_int]),
        "dglhip_gat_attention_grad_device": (_c_int, [_c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp,
                                                      _vp, _vp, _vp, ctypes.c_float,
                                                      ctypes.c_float, ctypes.c_float, _c_int,
                                                      ctypes.c_float, _vp, _vp]),
        "dglhip_gspmm_items_device": (_c_int, [_c_int, _c_i64, _c_i64, _vp, _vp, _c_int, _vp, _vp,
                                               _vp, _c_i64, _vp, _c_i64, _vp, _vp]),
        "dglhip_gspmm_sweep_device": (_c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _c_i64,
                                               _c_i64, _c_int, _c_int, _c_int, _vp]),
        "dglhip_gspmm_sweep_stream_geometry": (_c_int, [_c_int, _c_int, _vp]),
        "dglhip_set_sweep_per_cu": (_c_int, [_c_int]),
        "dglhip_sweep_barrier_expiries": (_c_int, [_c_int, _vp]),
        "dglhip_set_sweep_rows": (_c_int, [_c_int]),
        "dglhip_set_pair_slots": (_c_int, [_c_int]),
        "dglhip_gspmm_pair_items_ok": (_c_int, [_c_int, _c_i64, _c_i64, _c_i64]),
        "dglhip_get_sweep_rows": (_c_int, [_vp]),
        "dglhip_set_sweep_schedule": (_c_int, [_c_int, _c_i64, _c_i64, _c_int, _c_int, _c_i64,
                                               _c_i64, _c_int]),
        "dglhip_get_sweep_schedule": (_c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
        "dglhip_set_gat_fwd_waves": (_c_int, [_c_int]),
        "dglhip_set_sweep_unroll": (_c_int, [_c_int]),
        "dglhip_gspmm_sweep_stream_device": (_c_int, [_c_i64, _c_i64, _vp, _vp, _c_int, _vp, _vp,
                                                      _vp, _vp, _vp, _c_int, _c_int, _c_int, _vp,
                                                      _c_i64, _c_int, _c_int, _vp]),
        "dglhip_gspmm_max_ranges_device": (_c_int, [_c_int, _c_i64, _c_i64, _vp, _vp, _vp, _c_int,
                                                    _vp, _vp, _vp, _vp, _c_i64, _vp, _vp, _vp,
                                                    _vp]),
        "dglhip_gsddmm_ranges_device": (_c_int, [_c_int, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp,
                                                 _vp, _vp, _vp, _vp, _vp, _vp]),
        "dglhip_gat_attention_grad_ranges_device": (_c_int, [_c_i64, _c_i64, _c_i64, _vp, _vp,
                                                             _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                                             ctypes.c_float, ctypes.c_float,
                                                             ctypes.c_float, _c_int,
                                                             ctypes.c_float, _vp, _vp]),
        "dglhip_gat_attention_grad_rowsum_ok": (_c_int, [_c_i64, _c_i64]),
        "dglhip_gat_attention_grad_rowsum_ranges_device": (
            _c_int, [_c_i64, _c_i64, _c_i64] + [_vp] * 9 +
            [ctypes.c_float, ctypes.c_float, ctypes.c_float, _c_int, ctypes.c_float, _vp, _vp,
             _vp]),
        "dglhip_gat_dropout_mask_host": (_c_int, [_c_i64, _c_i64, ctypes.c_float, ctypes.c_uint64,
                                                  _vp]),
        "dglhip_degree_bucketing_host": (_c_int, [_c_i64, _vp, _c_i64, _vp, _vp, _vp, _vp, _vp]),
        "dglhip_gspmm_host": (_c_int, [_c_int, _c_int, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp,
                                       _c_i64, _vp, _vp, _c_int]),
        "dglhip_gsddmm_device": (_c_int, [_c_int, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp,
                                          _vp, _vp]),
        "dglhip_gsddmm_host": (_c_int, [_c_int, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp,
                                        _vp, _c_int]),
        "dglhip_timing_enable": (_c_int, [_c_int]),
        "dglhip_gspmm_resident_waves": (_c_int, [_c_int, ctypes.POINTER(_c_i64)]),
        "dglhip_set_spmm_variant": (_c_int, [_c_int, _c_int, _c_int, _c_int]),
        "dglhip_set_cache_policy": (_c_int, [_c_int]),
        "dglhip_set_row_policy": (_c_int, [_c_int]),
        "dglhip_set_gather_mode": (_c_int, [_c_int]),
        "dglhip_set_sddmm_variant": (_c_int, [_c_int]),
        "dglhip_gspmm_short_rows_device": (_c_int, [_c_int, _c_int, _c_i64, _c_i64, _c_i64,
                                                    _c_i64, _vp, _vp, _vp, _vp, _vp, _c_i64, _vp]),
        "dglhip_gspmm_strided_device": (_c_int, [_c_int, _c_int, _c_i64, _c_i64, _c_i64, _vp,
                                                 _vp, _vp, _vp, _vp, _c_i64, _vp, _vp, _vp]),
        "dglhip_node_linear_device": (_c_int, [_c_i64, _c_i64, _vp, _c_i64, _c_i64, _vp, _vp,
                                               _vp, _c_i64, _c_i64, _vp, _vp, _vp, _c_i64, _vp]),
        "dglhip_node_linear_cat_device": (_c_int, [_c_i64, _c_i64, _vp, _c_i64, _vp, _c_i64,
                                                   _c_i64, _vp, _vp, _vp, _vp, _c_i64, _c_int,
                                                   _vp]),
        "dglhip_set_node_linear_variant": (_c_int, [_c_int, _c_int]),
        "dglhip_node_linear_dgrad_device": (_c_int, [_c_i64, _c_i64, _c_i64, _vp, _c_i64, _vp,
                                                     _c_i64, _vp, _c_i64, _vp, _vp, _c_i64, _vp,
                                                     _c_i64, _vp, _vp, _vp]),
        "dglhip_node_linear_dgrad_workspace_floats": (_c_i64, [_c_i64]),
        "dglhip_div_rows_device": (_c_int, [_c_i64, _c_i64, _vp, _c_i64, _vp, _vp, _c_i64, _vp]),
        "dglhip_xent_workspace_floats": (_c_int, []),
        "dglhip_xent_fwd_device": (_c_int, [_c_i64, _c_i64, _vp, _c_i64, _vp, _vp, _vp, _vp, _vp]),
        "dglhip_xent_bwd_device": (_c_int, [_c_i64, _c_i64, _vp, _c_i64, _vp, _vp, _vp, _vp,
                                            _c_i64, _vp]),
        "dglhip_xent_colsum_workspace_floats": (_c_int, [_c_i64]),
        "dglhip_xent_bwd_ex_device": (_c_int, [_c_i64, _c_i64, _vp, _c_i64, _vp, _vp, _vp, _vp,
                                               _c_i64, _vp, _vp, _vp, _vp, _c_i64, _vp]),
        "dglhip_timing_read": (_c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_c_i64)]),
        "dglhip_spmm_get_policy": (_c_int, [_vp]),
        "dglhip_spmm_set_policy": (_c_int, [_vp]),
        "dglhip_spmm_split_threshold": (_c_int, [_c_i64, _c_i64, _c_i64, ctypes.POINTER(_c_i64)]),
        "dglhip_spmm_padded_width": (_c_int, [_c_i64, ctypes.POINTER(_c_i64)]),
        "dglhip_spmm_plan_create": (_c_int, [_c_int, _c_int, _c_i64, _c_i64, _c_i64, _vp, _vp,
                                             _vp, _vp, _vp, ctypes.POINTER(_vp)]),
        "dglhip_spmm_plan_free": (_c_int, [_vp]),
        "dglhip_spmm_plan_workspace": (_c_int, [_vp, _c_int, _c_int, _c_i64, _c_i64, _c_i64,
                                                _c_i64, _c_int, _vp, _vp, ctypes.POINTER(_c_i64)]),
        "dglhip_spmm_plan_run": (_c_int, [_vp, _c_int, _c_int, _c_i64, _vp, _c_i64, _c_i64, _vp,
                                          _c_i64, _c_int, _vp, _vp, _vp, _vp, _c_i64, _vp]),
        "dglhip_spmm_plan_schedule": (_c_int, [_vp, _c_int, _c_int, _c_i64, _c_i64, _c_i64,
                                               _c_i64, _c_int, _vp, _vp, ctypes.POINTER(_c_int),
                                               ctypes.POINTER(_c_i64)]),
        "dglhip_spmm_plan_stats": (_c_int, [_vp, ctypes.POINTER(_c_i64)]),
        "DGLFuncGetGlobal": (_c_int, [ctypes.c_char_p, ctypes.POINTER(_vp)]),
        "DGLFuncListGlobalNames": (_c_int, [ctypes.POINTER(_c_int),
                                            ctypes.POINTER(ctypes.POINTER(ctypes.c_char_p))]),
        "DGLFuncCall": (_c_int, [_vp, _vp, ctypes.POINTER(_c_int), _c_int, _vp, ctypes.POINTER(_c_int)]),
        "DGLFuncFree": (_c_int, [_vp]),
        "DGLArrayFree": (_c_int, [_vp]),
        "DGLArrayToDLPack": (_c_int, [_vp, ctypes.POINTER(_vp)]),
        "DGLDLManagedTensorCallDeleter": (None, [_vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


class _LazyLib(object):
    """Loads the library on first use so that `import dgl` works for docs/tests
    of pure-host logic; any kernel call without the library raises."""

    def __init__(self):
        self._lib = None
        self._err = None

    def _get(self):
        if self._lib is None:
            if self._err is not None:
                raise DGLError(self._err)
            try:
                self._lib = _load()
            except (OSError, DGLError) as err:  # pragma: no cover - depends on build
                self._err = "libdgl_hip.so unavailable: %s" % err
                raise DGLError(self._err)
        return self._lib

    def __getattr__(self, name):
        fn = getattr(self._get(), name)
        # kept on the instance: later lookups skip this hook (≈40 library
        # calls per R-GCN step went through it)
        setattr(self, name, fn)
        return fn

    @property
    def loaded(self):
        try:
            self._get()
            return True
        except DGLError:
            return False


LIB = _LazyLib()


def check_call(ret):
    """Raise DGLError with the library's last error if ``ret`` != 0."""
    if ret != 0:
        raise DGLError(LIB.DGLGetLastError().decode("utf-8", "replace"))


def ptr(t):
    """Raw data pointer of a tensor (None for None)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


# --------------------------------------------------------------------------
# PackedFunc calling convention (include/dgl_hip.h, csrc/registry.cc)
# --------------------------------------------------------------------------
_TC_INT, _TC_HANDLE, _TC_NULL, _TC_ARRAY = 0, 3, 4, 7


class _DGLHipTensor(ctypes.Structure):
    _fields_ = [("data", _vp), ("device_type", ctypes.c_int32), ("device_id", ctypes.c_int32),
                ("ndim", ctypes.c_int32), ("dtype_code", ctypes.c_uint8),
                ("dtype_bits", ctypes.c_uint8), ("dtype_lanes", ctypes.c_uint16),
                ("shape", ctypes.POINTER(_c_i64)), ("strides", ctypes.POINTER(_c_i64)),
                ("byte_offset", ctypes.c_uint64)]


class _DGLHipValue(ctypes.Union):
    _fields_ = [("v_int64", _c_i64), ("v_float64", ctypes.c_double), ("v_handle", _vp),
                ("v_str", ctypes.c_char_p)]


_DTYPE_CODE = {torch.int64: (0, 64), torch.int32: (0, 32), torch.float32: (2, 32)}


_ARRAY_TYPES = {}


def _array_type(ctype, n):
    """``ctype * n``, made once per (type, length): a fresh array type per call
    is a cyclic object that only the garbage collector frees."""
    key = (ctype, n)
    t = _ARRAY_TYPES.get(key)
    if t is None:
        t = _ARRAY_TYPES[key] = ctype * n
    return t


def tensor_arg(t):
    """Wrap a torch tensor as a non-owning DGLHipTensor (src/c_api_common.cc:16-23)."""
    code, bits = _DTYPE_CODE[t.dtype]
    shape = _array_type(_c_i64, t.dim())(*t.shape)
    strides = _array_type(_c_i64, t.dim())(*t.stride())
    dev = 10 if t.is_cuda else 1
    st = _DGLHipTensor(t.data_ptr(), dev, t.device.index or 0, t.dim(), code, bits, 1,
                       shape, strides, 0)
    st._keep = (shape, strides, t)  # keep alive for the duration of the call
    return st


def list_global_names():
    """Names registered in the engine's PackedFunc table."""
    n = _c_int()
    arr = ctypes.POINTER(ctypes.c_char_p)()
    check_call(LIB.DGLFuncListGlobalNames(ctypes.byref(n), ctypes.byref(arr)))
    return [arr[i].decode() for i in range(n.value)]


def call_packed(name, *args):
    """Call a registered function by name with ints, tensors, None or
    ``("handle", int)`` stream handles — the DGLFuncCall convention; returns
    the decoded result (see :class:`PackedFunction`)."""
    return get_global_func(name)(*args)


_TC_FLOAT, _TC_FUNC, _TC_STR, _TC_NDARRAY = 2, 10, 11, 13

ctypes.pythonapi.PyCapsule_New.restype = ctypes.py_object
ctypes.pythonapi.PyCapsule_New.argtypes = [_vp, ctypes.c_char_p, _vp]
ctypes.pythonapi.PyCapsule_GetPointer.restype = _vp
ctypes.pythonapi.PyCapsule_GetPointer.argtypes = [ctypes.py_object, ctypes.c_char_p]
ctypes.pythonapi.PyCapsule_IsValid.argtypes = [ctypes.py_object, ctypes.c_char_p]


@ctypes.CFUNCTYPE(None, _vp)
def _dltensor_capsule_deleter(capsule):
    # a capsule torch never consumed still owns its DGLHipManagedTensor
    cap = ctypes.cast(capsule, ctypes.py_object)
    if ctypes.pythonapi.PyCapsule_IsValid(cap, b"dltensor"):
        LIB.DGLDLManagedTensorCallDeleter(ctypes.pythonapi.PyCapsule_GetPointer(cap, b"dltensor"))


# the deleter's address, taken once (a cast per call would link the function
# object's keep-alive dict to a new object every time)
_DELETER_ADDR = ctypes.cast(_dltensor_capsule_deleter, _vp).value


def _ndarray_to_torch(handle):
    """Library-owned NDArray container -> torch tensor without a copy
    (zerocopy_from_dgl_ndarray: DGLArrayToDLPack, then the container's own
    reference is dropped; the DLPack manager keeps the storage alive)."""
    import torch.utils.dlpack
    mt = _vp()
    try:
        check_call(LIB.DGLArrayToDLPack(handle, ctypes.byref(mt)))
    finally:
        check_call(LIB.DGLArrayFree(handle))
    cap = ctypes.pythonapi.PyCapsule_New(mt, b"dltensor", _DELETER_ADDR)
    return torch.utils.dlpack.from_dlpack(cap)


class PackedFunction(object):
    """A function of the library's PackedFunc table, or one it returned
    (python/dgl/_ffi/_ctypes/function.py:150-190). Calls take ints, bools,
    floats, strings, torch tensors (passed as non-owning arrays), None and
    ``("handle", int)``; results come back decoded by type code: ints,
    floats, strings, handles (ints), torch tensors for returned arrays
    (zero-copy) and PackedFunction for returned functions (freed with
    DGLFuncFree when collected)."""

    __slots__ = ("handle", "_owned")

    def __init__(self, handle, owned):
        self.handle = handle
        self._owned = owned

    def __del__(self):
        if self._owned and self.handle:
            try:
                LIB.DGLFuncFree(self.handle)
            except Exception:  # noqa: BLE001 - interpreter shutdown
                pass

    def __call__(self, *args):
        # raw addresses (ctypes.addressof), not ctypes.cast / pointer objects:
        # a cast links the two objects' keep-alive dicts into a reference
        # cycle, so every tensor argument stayed alive until a garbage
        # collection (r05: the bench graph's 0.9-GB edge arrays were freed by a
        # collection inside the timed region, a 170-ms host stall)
        n = len(args)
        vals = _array_type(_DGLHipValue, max(n, 1))()
        codes = _array_type(_c_int, max(n, 1))()
        keep = []
        for i, a in enumerate(args):
            if a is None:
                codes[i] = _TC_NULL
            elif isinstance(a, torch.Tensor):
                st = tensor_arg(a)
                keep.append(st)
                vals[i].v_handle = ctypes.addressof(st)
                codes[i] = _TC_ARRAY
            elif isinstance(a, tuple) and a[0] == "handle":
                vals[i].v_handle = a[1]
                codes[i] = _TC_HANDLE
            elif isinstance(a, str):
                b = a.encode()
                keep.append(b)
                vals[i].v_str = b
                codes[i] = _TC_STR
            elif isinstance(a, float):
                vals[i].v_float64 = a
                codes[i] = _TC_FLOAT
            else:
                vals[i].v_int64 = int(a)
                codes[i] = _TC_INT
        ret = _DGLHipValue()
        rc = _c_int()
        check_call(LIB.DGLFuncCall(self.handle, ctypes.addressof(vals), codes, n,
                                   ctypes.addressof(ret), ctypes.byref(rc)))
        del keep
        code = rc.value
        if code == _TC_INT:
            return ret.v_int64
        if code == _TC_FLOAT:
            return ret.v_float64
        if code == _TC_NULL:
            return None
        if code == _TC_HANDLE:
            return ret.v_handle
        if code == _TC_STR:
            return ret.v_str.decode()
        if code == _TC_NDARRAY:
            return _ndarray_to_torch(ret.v_handle)
        if code == _TC_FUNC:
            return PackedFunction(ret.v_handle, True)
        raise DGLError("unsupported return type code %d" % code)


_GLOBALS = {}


def get_global_func(name):
    """The registered function ``name`` (cached; DGLFuncGetGlobal)."""
    f = _GLOBALS.get(name)
    if f is None:
        h = _vp()
        check_call(LIB.DGLFuncGetGlobal(name.encode(), ctypes.byref(h)))
        if not h.value:
            raise DGLError("global function %s is not registered" % name)
        f = _GLOBALS[name] = PackedFunction(h.value, False)
    return f


class CAPINamespace(object):
    """``ns._CAPI_<name>`` attribute access to the registry, as the reference's
    _init_api binds a module's functions (python/dgl/_ffi/function.py:267-306)."""

    def __init__(self, namespace):
        self._ns = namespace

    def __getattr__(self, name):
        f = get_global_func("%s.%s" % (self._ns, name))
        setattr(self, name, f)
        return f
