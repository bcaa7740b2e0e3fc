"""Sparse adjacency objects and the g-SpMM / g-SDDMM operators.

This module is the engine's replacement for what the reference delegates to
the tensor framework:

* ``F.sparse_matrix`` + ``F.spmm`` = ``torch.sparse_coo_tensor`` +
  ``torch.sparse.mm`` (python/dgl/backend/pytorch/tensor.py:45-51,145-146),
  driven by SPMVExecutor / SPMVWithDataExecutor
  (python/dgl/runtime/ir/executor.py:452-473,535-566);
* the adjacency index built by ``Graph::GetAdj`` (src/graph/graph.cc:506-554)
  and copied to the device on first use (python/dgl/graph_index.py:575-579).

A :class:`SparseAdj` holds a destination-major CSR (rows = reduce targets)
plus, built lazily, the source-major CSR of the transpose used by the
backward. Slot order within a row is the order in which torch's CPU sparse
product consumes the reference's uncoalesced COO (edge-id order for mutable
graphs), so the HIP kernels reproduce the reference's results bit for bit.

Every compute call goes to libdgl_hip.so (HIP kernels for tensors on a ROCm
device, the library's host kernels for CPU tensors). There is no other path.
Each CSR's schedules (the source-blocked plan, the heavy-row split, the
short-row tiers) live in its native launch plan (csrc/spmm_plan.*,
dglhip_spmm_plan_*): this module passes tensors to it and wraps what it
hands back, so the C-ABI and these operators run one schedule choice.
"""
from __future__ import absolute_import

import contextlib
import ctypes
import os
import weakref

import numpy as np
import torch

from . import _ffi, _handoff
from ._ffi import LIB, check_call, ptr
from .base import DGLError

__all__ = ["CSR", "SparseAdj", "build_csr", "gspmm", "gsddmm_dot",
           "MSG_COPY_U", "MSG_U_MUL_E", "MSG_COPY_E", "RED_SUM", "RED_MAX", "RED_MEAN"]

MSG_COPY_U, MSG_U_MUL_E, MSG_COPY_E = 0, 1, 2
MSG_COPY_U_BF16 = 3  # copy_u over bf16 source rows, widened exactly to fp32 (dgl_hip.h)
RED_SUM, RED_MAX, RED_MEAN = 0, 1, 2
RED_SUM_ACCUM = 3  # out += sum, each row's chain continued from out (include/dgl_hip.h)
RED_MEAN_ACCUM = 4  # out = out + mean (include/dgl_hip.h)
_ACCUM = (RED_SUM_ACCUM, RED_MEAN_ACCUM)
ORDER_EID, ORDER_COL = 0, 1
# edge values laid out in the forward CSR's slot order (edge_order="slot"):
# kernels read / write slot k at row k, no eid indirection
SLOT = "slot"

_MSG_NAMES = {"copy_src": MSG_COPY_U, "copy_u": MSG_COPY_U, "src_mul_edge": MSG_U_MUL_E,
              "u_mul_e": MSG_U_MUL_E, "copy_edge": MSG_COPY_E, "copy_e": MSG_COPY_E}
_RED_NAMES = {"sum": RED_SUM, "max": RED_MAX, "mean": RED_MEAN}



# ---------------------------------------------------------------------------
# Schedule policy: the native launch plan's (dglhip_spmm_get_policy /
# dglhip_spmm_set_policy, include/dgl_hip.h). One policy serves the engine's
# own operators and every C-ABI / PackedFunc caller of the plan.
#
# Heavy-row policy ("row_split") of the sum / mean kernels, sized from the
# device: R = the headline kernel's resident waves
# (dglhip_gspmm_resident_waves: compute units x waves per CU at its occupancy;
# MI355X 256 x 28 = 7,168).
#   "auto" : (default) a row is one wave's sequential chain, a launch spreads
#            its slots over the R resident waves and rows start longest-first,
#            so a row longer than twice a wave's share (nnz / (R / 2) slots)
#            outlasts the rest of the launch. Only then — and only for rows
#            longer than 16,384 slots (~1.5 ms of chained gathers), below which
#            the loss is bounded and every row stays one exact chain — are the
#            rows longer than max(4096, (7168 / 12000) x nnz / R) slots (nnz /
#            12,000 on MI355X) cut into chunks, sized to spread their slots
#            over 4R/7 waves (4,096 on MI355X). A floor of 65,536 left the
#            60k-slot hub rows of RMAT-26's pipelined segments at 1/8 unsplit:
#            13.2 -> 24.3 ms per step (bench.py --emulate-world 8 --workload rmat).
#            RMAT-26 (max in-degree ~855k, 2.9x the share) is split: GraphSAGE-
#            mean epoch 0.693 -> 0.640 s (profiles/r02/graphsage_rmat26_row_split.log);
#            Reddit (max 21,657 <= 114.8M / 3584 = 32,045) is not, and stays
#            bit-exact. A part with fewer resident waves has a longer share per
#            wave and splits less.
#   "off"  : every row is one sequential chain — bit-exact with the reference
#            on every graph (the documented bit-exact switch)
#   <int>  : explicit chunk length, applied whenever some row is longer
# (DGLHIP_ROW_SPLIT sets it from the environment.)
# ---------------------------------------------------------------------------
_REF_WAVES = 7168       # MI355X (and the host path, which never splits)
_WAVES = {}


class _Policy(ctypes.Structure):
    _fields_ = [("row_split", ctypes.c_int64), ("blocked", ctypes.c_int32),
                ("short_rows", ctypes.c_int32), ("pad_rows", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("block_bytes", ctypes.c_int64),
                ("block_table_min", ctypes.c_int64), ("block_table_max", ctypes.c_int64),
                ("block_min_slots", ctypes.c_int64), ("block_max_stretch", ctypes.c_double),
                ("block_max_suffix", ctypes.c_double), ("block_min_row_bytes", ctypes.c_int64),
                ("tier_min_rows", ctypes.c_int64), ("pad_min_bytes", ctypes.c_int64)]


_POLICY_KEYS = tuple(n for n, _ in _Policy._fields_ if n != "reserved")
# bumped at every policy change: part of the keys of the Python-side caches
# of native plan structures (a new policy may give a CSR another schedule)
_POLICY_GEN = [0]


def schedule_policy():
    """The g-SpMM schedule policy as a dict (row_split -1 auto / 0 off / a
    chunk length, blocked, short_rows, pad_rows, block_bytes, block_table_min,
    block_table_max, block_min_slots, block_max_stretch, block_max_suffix,
    block_min_row_bytes, tier_min_rows, pad_min_bytes)."""
    p = _Policy()
    check_call(LIB.dglhip_spmm_get_policy(ctypes.addressof(p)))
    return {k: getattr(p, k) for k in _POLICY_KEYS}


def set_schedule_policy(**changes):
    """Change fields of the schedule policy; returns the old policy (a dict
    that set_schedule_policy(**old) restores)."""
    p = _Policy()
    check_call(LIB.dglhip_spmm_get_policy(ctypes.addressof(p)))
    old = {k: getattr(p, k) for k in _POLICY_KEYS}
    for k, v in changes.items():
        if k not in _POLICY_KEYS:
            raise DGLError("unknown schedule policy field %r" % (k,))
        setattr(p, k, v)
    check_call(LIB.dglhip_spmm_set_policy(ctypes.addressof(p)))
    _POLICY_GEN[0] += 1
    return old


@contextlib.contextmanager
def scheduled(**changes):
    """Context manager: the schedule policy with ``changes`` for its body."""
    old = set_schedule_policy(**changes)
    try:
        yield
    finally:
        set_schedule_policy(**old)


def sweep_schedule():
    """The source-sweep schedule's knobs (DESIGN.md §4.1 "Source sweep"):
    {"on", "table_min", "block_bytes", "lag", "max_spin", "accum_table_min",
    "accum_min_slots", "accum_per_cu"}."""
    on, lag, spin, apc = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    tmin, bb, atm, ams = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    check_call(LIB.dglhip_get_sweep_schedule(ctypes.byref(on), ctypes.byref(tmin),
                                             ctypes.byref(bb), ctypes.byref(lag),
                                             ctypes.byref(spin), ctypes.byref(atm),
                                             ctypes.byref(ams), ctypes.byref(apc)))
    return {"on": bool(on.value), "table_min": tmin.value, "block_bytes": bb.value,
            "lag": lag.value, "max_spin": spin.value, "accum_table_min": atm.value,
            "accum_min_slots": ams.value, "accum_per_cu": apc.value}


def sweep_barrier_expiries(reset=False):
    """Waits of the accumulating sweep's soft barrier that ran out of polls
    (max_spin) on the current device since the last reset (a synchronous read;
    ``reset`` zeroes the count after reading). Results never depend on them."""
    v = ctypes.c_int64()
    check_call(LIB.dglhip_sweep_barrier_expiries(1 if reset else 0, ctypes.byref(v)))
    return int(v.value)


def set_sweep_schedule(**changes):
    """Change the source-sweep knobs; returns the old ones (for restoring).
    A plan keeps the sweep layouts it built; the choice is made per call."""
    old = sweep_schedule()
    new = dict(old, **changes)
    unknown = set(changes) - set(old)
    if unknown:
        raise DGLError("unknown sweep knobs: %s" % sorted(unknown))
    check_call(LIB.dglhip_set_sweep_schedule(int(bool(new["on"])), int(new["table_min"]),
                                             int(new["block_bytes"]), int(new["lag"]),
                                             int(new["max_spin"]), int(new["accum_table_min"]),
                                             int(new["accum_min_slots"]),
                                             int(new["accum_per_cu"])))
    return old


def _resident_waves(device=None):
    """R: the headline g-SpMM kernel's resident waves on ``device`` (queried
    once per device from the library); _REF_WAVES for host / unknown devices."""
    if device is None or torch.device(device).type != "cuda":
        return _REF_WAVES
    idx = torch.device(device).index
    idx = torch.cuda.current_device() if idx is None else idx
    if idx not in _WAVES:
        w = ctypes.c_int64()
        check_call(LIB.dglhip_gspmm_resident_waves(idx, ctypes.byref(w)))
        _WAVES[idx] = int(w.value)
    return _WAVES[idx]


def _row_split_name(v):
    return "auto" if v < 0 else ("off" if v == 0 else str(v))


def get_row_split():
    """The heavy-row policy: "auto", "off" or a chunk length (as a string)."""
    return _row_split_name(schedule_policy()["row_split"])


def set_row_split(policy):
    """Set the heavy-row policy ("auto", "off" or a chunk length); returns the old one."""
    pol = str(policy)
    if pol == "auto":
        v = -1
    elif pol in ("off", "0", "", "none", "None"):
        v = 0
    else:
        v = int(pol)
    return _row_split_name(set_schedule_policy(row_split=v)["row_split"])


def _split_threshold(csr, waves=None):
    """Rows longer than this many slots are chunked (0: none), for a launch
    over ``csr`` on a part with ``waves`` resident waves (None: csr's device):
    the native plan's gate (dglhip_spmm_split_threshold)."""
    R = waves if waves is not None else _resident_waves(getattr(csr, "device", None))
    t = ctypes.c_int64()
    check_call(LIB.dglhip_spmm_split_threshold(int(csr.nnz), int(csr.max_degree), int(R),
                                               ctypes.byref(t)))
    return int(t.value)



def _stream_of(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class CSR(object):
    """CSR matrix: indptr int64[R+1], indices int32[nnz], eid int64[nnz].

    ``row_order`` (int32[R], optional) is the degree-descending launch
    schedule handed to the HIP kernel.
    """

    def __init__(self, indptr, indices, eid, num_cols, row_order=None, host_indptr=None,
                 lazy_order=False):
        self.indptr = indptr
        self.indices = indices
        self._eid = eid
        self._eid_host = None
        self.num_rows = indptr.numel() - 1
        self.num_cols = int(num_cols)
        self._row_order = row_order
        # a device CSR's schedule is sorted on first use: products that never
        # launch by rows (the typed-block items, the blocked items) skip it
        self._lazy_order = bool(lazy_order) and row_order is None
        self._row_ids = None
        self._host_indptr = host_indptr
        self._plans = {}
        self._max_degree = None
        self._num_nonempty = None
        self._slot_eid = False  # not computed yet
        self._eid_loc = None
        self._native = None  # the native launch plan (built on first use)

    @property
    def row_order(self):
        """int32[R]: rows by degree, descending, ties by row id (a stable sort:
        the host builder's counting sort gives the same order); None when the
        CSR was built without a schedule."""
        if self._row_order is None and self._lazy_order:
            self._lazy_order = False
            if self.num_rows > 0:
                deg = self.indptr[1:] - self.indptr[:-1]
                self._row_order = torch.sort(deg, descending=True,
                                             stable=True)[1].to(torch.int32)
        return self._row_order

    @row_order.setter
    def row_order(self, value):
        self._row_order, self._lazy_order = value, False

    @property
    def eid(self):
        """int64[nnz], the edge id of each slot; brought back to the device
        (once) if offload_eid moved it to host memory."""
        if self._eid is None and self._eid_host is not None:
            self._eid = self._eid_host.to(self.indptr.device)
            self._eid_host = None
        return self._eid

    @eid.setter
    def eid(self, value):
        self._eid, self._eid_host = value, None

    def offload_eid(self):
        """Move ``eid`` (8 bytes per slot: 8.6 GB at 1.07B edges) to host
        memory until something reads it again. copy_u / copy_e-by-slot work
        (sum, mean, max; the transposed backward; the short-row and heavy-row
        plans) never reads it; edge-feature messages bring it back."""
        if self._eid is not None and self._eid.device.type != "cpu":
            self._eid_host = self._eid.cpu()
            self._eid = None
            if self._slot_eid is not None and self._slot_eid is not False:
                self._slot_eid = False  # recomputed (from the host copy) on demand

    @property
    def host_indptr(self):
        if self._host_indptr is None:
            self._host_indptr = self.indptr.cpu()
        return self._host_indptr

    @property
    def max_degree(self):
        if self._max_degree is None:
            ip = self.host_indptr
            self._max_degree = int((ip[1:] - ip[:-1]).max()) if self.num_rows else 0
        return self._max_degree

    @property
    def slot_eid(self):
        """``eid`` for the g-SpMM entry points, or None when the slots already
        run in edge-id order (eid == arange): the kernels then index edge
        features by slot and skip the eid indirection (include/dgl_hip.h).
        Checked once per CSR, in bounded chunks."""
        if self._slot_eid is False:
            ident = True
            n = self.eid.numel()
            step = 1 << 26
            for b in range(0, n, step):
                e = min(n, b + step)
                if not torch.equal(self.eid[b:e],
                                   torch.arange(b, e, dtype=self.eid.dtype,
                                                device=self.eid.device)):
                    ident = False
                    break
            self._slot_eid = None if ident else self.eid
        return self._slot_eid

    @property
    def eid_locality(self):
        """Fraction of consecutive slots whose edge ids are consecutive (1.0
        when the slots walk edge-id order); how sequential per-edge stores at
        out[eid] are along this CSR. Computed once, in bounded chunks."""
        if self._eid_loc is None:
            n = self.eid.numel()
            runs, step = 0, 1 << 26
            for b in range(0, n - 1, step):
                e = min(n - 1, b + step)
                runs += int((self.eid[b + 1:e + 1] == self.eid[b:e] + 1).sum().item())
            self._eid_loc = 1.0 if n < 2 else runs / float(n - 1)
        return self._eid_loc

    @property
    def num_nonempty(self):
        """Rows holding at least one slot (a prefix of the degree-descending
        row_order)."""
        if self._num_nonempty is None:
            ip = self.host_indptr
            self._num_nonempty = int((ip[1:] > ip[:-1]).sum()) if self.num_rows else 0
        return self._num_nonempty

    @property
    def plan(self):
        """The native launch plan of this CSR (dglhip_spmm_plan_*, built on
        first use): every g-SpMM over the CSR runs on it."""
        if self._native is None:
            self._native = _NativePlan(self)
        return self._native

    def split_plan(self, threshold, skip_empty=False, chunk=None):
        """The plan's heavy-row launch plan cutting rows longer than
        ``threshold`` slots into chunks of ``chunk`` slots (None: enough
        chunks to spread the heavy slots over 4R/7 waves, R the device's
        resident waves; at least 1,024 slots each, at most ``threshold``):
        dict of tensors light, heavy, chunk_ptr, beg, end and num_chunks, as
        dglhip_gspmm_chunked_device takes them. ``skip_empty`` leaves rows
        without slots out of the light list (accumulating launches need not
        touch them). The chunk launch runs alone before the light rows, so it
        must fill the chip: with chunks of ``threshold`` slots RMAT-26's 27 hub
        rows made 88 chunks, 88 waves chaining 89k gathers each for 6.6 ms of
        a 82 ms call."""
        p = self.plan
        f = _retry_oom(lambda: _capi("SpmmPlanSplit")(p.arg, int(threshold), 1 if skip_empty else 0,
                                                      int(chunk or 0), p.stream_arg()))
        meta = f(0).tolist()
        return {"light": f(1), "heavy": f(2), "chunk_ptr": f(3), "beg": f(4), "end": f(5),
                "num_chunks": int(meta[2])}

    def tiers(self, skip_empty=False, threshold=0):
        """The plan's short-row tiers of the degree-descending schedule (the
        first num_nonempty rows with ``skip_empty``), or with ``threshold`` of
        the heavy-row split's light rows: (n_long, [(max_deg, (rows, slot_ptr,
        slot_cols), n), ...]). Rows [0, n_long) of the list have more than 8
        slots; each tier lists rows of at most max_deg (8, 4, 0) slots as a
        compacted CSR of their own for dglhip_gspmm_short_rows_device
        (slot_ptr / slot_cols None for the empty tier)."""
        p = self.plan
        f = _retry_oom(lambda: _capi("SpmmPlanTiers")(p.arg, 1 if skip_empty else 0,
                                                      int(threshold), p.stream_arg()))
        meta = f(0).tolist()
        n_long, _, T = meta[:3]
        out = []
        for t in range(int(T)):
            maxd, n = int(meta[3 + 2 * t]), int(meta[4 + 2 * t])
            rows = f(1 + 3 * t)
            sp = f(2 + 3 * t) if maxd else None
            cols = f(3 + 3 * t) if maxd else None
            out.append((maxd, (rows, sp, cols), n))
        return int(n_long), out

    @property
    def nnz(self):
        return self.indices.numel()

    @property
    def device(self):
        return self.indptr.device

    def to(self, device):
        if self.device == torch.device(device):
            return self
        if self._row_order is None and self._lazy_order and torch.device(device).type == "cuda":
            return CSR(self.indptr.to(device), self.indices.to(device), self.eid.to(device),
                       self.num_cols, None, self._host_indptr, lazy_order=True)
        ro = None if self.row_order is None else self.row_order.to(device)
        return CSR(self.indptr.to(device), self.indices.to(device), self.eid.to(device),
                   self.num_cols, ro, self._host_indptr)

    def degrees(self):
        return self.indptr[1:] - self.indptr[:-1]

    def mean_divisor(self):
        """float32 (R, 1): each row's slot count, at least 1 (the mean's
        divisor, the reference's degree-bucketing ``mean``); cached."""
        if getattr(self, "_mean_div", None) is None:
            self._mean_div = self.degrees().clamp(min=1).to(torch.float32).unsqueeze(1)
        return self._mean_div

    def row_ids(self):
        """Row id of every slot (COO expansion), cached."""
        if self._row_ids is None:
            # output_size: no host sync for the total
            self._row_ids = torch.repeat_interleave(
                torch.arange(self.num_rows, device=self.device), self.degrees(),
                output_size=self.nnz)
        return self._row_ids


_PINNED_UPLOAD_MAX = 64 << 20


def _upload(t, device):
    """``t`` on ``device``; a small host tensor goes through pinned memory
    without blocking the host (a pageable copy waits for the stream's queued
    work: every sampled graph of an R-GCN step paid that wait)."""
    if (t.device.type == "cpu" and device.type == "cuda" and
            t.numel() * t.element_size() <= _PINNED_UPLOAD_MAX):
        return t.contiguous().pin_memory().to(device, non_blocking=True)
    return t.to(device)


def build_csr(num_rows, num_cols, row, col, order=ORDER_EID, device=None, schedule=True,
              validate=True):
    """Build a CSR over ``num_rows`` rows from COO (row[e], col[e]).

    Slot k of row r holds ``col`` of the k-th edge of r in ``order``; its
    ``eid`` is that edge's position in the input arrays. On a ROCm device the
    build runs on the GPU (stable radix sort), on CPU in the library's host
    builder; both produce identical arrays. ``validate`` checks the endpoints
    against the shape (one host sync on a device); edges the graph index
    already validated skip it. On a device the degree-descending schedule is
    sorted there too, so the build itself waits on nothing (R-GCN builds
    three CSRs per sampled graph: r05, Weak 5 of the r04 verdict).
    """
    row = torch.as_tensor(row, dtype=torch.int64)
    col = torch.as_tensor(col, dtype=torch.int64)
    nnz = row.numel()
    if col.numel() != nnz:
        raise DGLError("row/col length mismatch: %d vs %d" % (nnz, col.numel()))
    device = torch.device(device) if device is not None else row.device
    if device.type == "cuda":
        row = _upload(row, device).contiguous()
        col = _upload(col, device).contiguous()
        # (no host sync is possible while a HIP graph is being captured: a
        # captured build takes its edges as validated by whoever filled them)
        if nnz and validate and not torch.cuda.is_current_stream_capturing():
            b = torch.stack([row.min(), col.min(), row.max(), col.max()]).cpu().tolist()
            if min(b[0], b[1]) < 0 or b[2] >= num_rows or b[3] >= num_cols:
                raise DGLError("edge endpoints out of range for a %dx%d matrix"
                               % (num_rows, num_cols))
        indptr = torch.empty(num_rows + 1, dtype=torch.int64, device=device)
        indices = torch.empty(nnz, dtype=torch.int32, device=device)
        eid = torch.empty(nnz, dtype=torch.int64, device=device)
        ws_bytes = LIB.dglhip_coo_to_csr_workspace_bytes(num_rows, num_cols, nnz, order)
        if ws_bytes < 0:
            check_call(-1)
        ws = torch.empty(max(int(ws_bytes), 1), dtype=torch.uint8, device=device)
        check_call(LIB.dglhip_coo_to_csr_device(
            num_rows, num_cols, nnz, ptr(row), ptr(col), order, ptr(indptr), ptr(indices),
            ptr(eid), ptr(ws), int(ws_bytes), _stream_of(device)))
        del ws
        host_indptr = None  # fetched when something needs it (CSR.host_indptr)
        # the degree-descending schedule: sorted on the device at first use
        return CSR(indptr, indices, eid, num_cols, None, host_indptr, lazy_order=schedule)
    else:
        row = row.cpu().contiguous()
        col = col.cpu().contiguous()
        indptr = torch.empty(num_rows + 1, dtype=torch.int64)
        indices = torch.empty(nnz, dtype=torch.int32)
        eid = torch.empty(nnz, dtype=torch.int64)
        check_call(LIB.dglhip_coo_to_csr_host(num_rows, num_cols, nnz, ptr(row), ptr(col),
                                              order, ptr(indptr), ptr(indices), ptr(eid)))
        host_indptr = indptr if schedule else None
    row_order = None
    if schedule and num_rows > 0:
        ro = torch.empty(num_rows, dtype=torch.int32)
        check_call(LIB.dglhip_rows_by_degree_host(num_rows, ptr(host_indptr), ptr(ro)))
        row_order = ro.to(device)
    return CSR(indptr, indices, eid, num_cols, row_order, host_indptr)


class SparseAdj(object):
    """A (num_rows x num_cols) sparse matrix for message passing.

    ``fwd`` is the row-major (destination) CSR; ``bwd`` is the transpose
    (source-major) CSR, built on first use by ``transpose_builder``.
    ``edge_map`` (optional int64[nnz]) maps the matrix's edge slots
    (``eid`` values) to positions of the edge-feature tensor; None = identity.
    Per-device copies are cached.
    """

    def __init__(self, fwd, transpose_builder, shape):
        self.fwd = fwd
        self._tb = transpose_builder
        self._bwd = None
        self.shape = tuple(int(s) for s in shape)
        self._dev = {}

    @property
    def bwd(self):
        if self._bwd is None:
            self._bwd = self._tb(self.fwd.device)
            if getattr(self, "_eid_offloaded", False):
                self._bwd.offload_eid()
        return self._bwd

    def offload_edge_ids(self):
        """Keep both CSRs' edge-id arrays in host memory until an edge-feature
        operation needs them (CSR.offload_eid): 17 GB of HBM at 1.07B edges
        for graphs whose messages read node features only."""
        self._eid_offloaded = True
        self.fwd.offload_eid()
        if self._bwd is not None:
            self._bwd.offload_eid()
        m = getattr(self, "_bwd_fslot", None)
        if m is not None:
            self._bwd_fslot = None
        return self

    def to(self, device):
        device = torch.device(device)
        if device.type == "cuda" and device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        if self.fwd.device == device:
            return self
        key = str(device)
        if key not in self._dev:
            other = SparseAdj(self.fwd.to(device), self._tb, self.shape)
            if self._bwd is not None:
                other._bwd = self._bwd.to(device)
            self._dev[key] = other
        return self._dev[key]


def coo_of(csr):
    """(row, col) int64 in edge-id order, recovered from a CSR built by
    build_csr (slot k holds edge eid[k] of row r): the inverse of the build."""
    ip = csr.indptr
    row = torch.repeat_interleave(torch.arange(csr.num_rows, device=ip.device),
                                  ip[1:] - ip[:-1], output_size=csr.nnz)
    r = torch.empty_like(row)
    r[csr.eid] = row
    del row
    c = torch.empty(csr.nnz, dtype=torch.int64, device=ip.device)
    c[csr.eid] = csr.indices.long()
    return r, c


def from_coo(num_rows, num_cols, row, col, order=ORDER_EID, device=None, validate=True):
    """SparseAdj whose forward CSR groups (row, col) by row and whose backward
    CSR groups the same edges by col, both in ``order``.

    The edge list is held only until the transposed CSR is first built (an
    int64 pair per edge: 17 GB at a billion edges); later builds (another
    device) recover it from the forward CSR."""
    row = torch.as_tensor(row, dtype=torch.int64)
    col = torch.as_tensor(col, dtype=torch.int64)
    dev = torch.device(device) if device is not None else row.device
    if (dev.type == "cuda" and row.device.type == "cpu" and col.device.type == "cpu" and
            row.numel() == col.numel() and 2 * row.numel() * 8 <= _PINNED_UPLOAD_MAX):
        # both endpoint arrays in one pinned copy, shared by the forward build
        # and the transpose's (was four uploads per sampled graph, r06)
        both = torch.empty(2, row.numel(), dtype=torch.int64, pin_memory=True)
        both[0].copy_(row)
        both[1].copy_(col)
        both = both.to(dev, non_blocking=True)
        row, col = both[0], both[1]
    fwd = build_csr(num_rows, num_cols, row, col, order, device, validate=validate)
    coo = [row, col]

    def tb(dev):
        r, c = coo if coo[0] is not None else coo_of(fwd)
        coo[0] = coo[1] = None
        # the same edges as the forward CSR's: already in range
        return build_csr(num_cols, num_rows, c, r, order, dev, validate=False)

    return SparseAdj(fwd, tb, (num_rows, num_cols))


# ---------------------------------------------------------------------------
# Raw kernel calls
# ---------------------------------------------------------------------------
def _edge_len(eshape, fshape):
    """Values per edge for an edge feature of trailing shape ``eshape`` against
    node features of trailing shape ``fshape``: 1 (scalar), F (same shape) or
    H (leading dims of fshape, broadcast over the rest: GAT's (H, 1) vs (H, D))."""
    eshape, fshape = tuple(eshape), tuple(fshape)
    F = int(np.prod(fshape)) if fshape else 1
    if all(d == 1 for d in eshape):  # (), (1,), (1, 1): one scalar per edge
        return 1
    if eshape == fshape:
        return F
    k = len(eshape)
    while k > 0 and eshape[k - 1] == 1:
        k -= 1
    if 0 < k < len(fshape) and eshape[:k] == fshape[:k] and \
            all(d == 1 for d in eshape[k:]) and len(eshape) <= len(fshape):
        return int(np.prod(fshape[:k]))
    raise DGLError("edge feature shape %s does not broadcast against node feature shape %s"
                   % (eshape, fshape))


# ---------------------------------------------------------------------------
# The native launch plan of a CSR (dglhip_spmm_plan_*, csrc/spmm_plan.*)
# ---------------------------------------------------------------------------
def _retry_oom(fn):
    """Run ``fn``; when the library's hipMalloc fails, hand torch's cached
    blocks back to the device once and retry (plan structures live in memory
    the library allocates beside torch's caching allocator)."""
    try:
        return fn()
    except DGLError as err:
        msg = str(err)
        if "hipMalloc" not in msg and "out of memory" not in msg.lower():
            raise
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
        return fn()


def _capi(name):
    return _ffi.get_global_func("dglhip._CAPI_" + name)


class _NativePlan(object):
    """Handle on a CSR's launch plan (dglhip_spmm_plan_create / _free). The
    plan borrows the CSR's indptr / indices / row_order (the CSR holds them for
    as long as it holds the plan) and keeps the schedules the g-SpMM runs over
    them, built natively on first use: the same object the
    C-ABI and dglhip._CAPI_GSpMM hand out, so one implementation serves the
    Python operators and every C / PackedFunc caller."""

    __slots__ = ("handle", "device", "_ws", "_cache", "__weakref__")

    def __init__(self, csr):
        dev = csr.device
        self.handle = None
        self.device = dev
        self._ws = {}
        self._cache = {}
        h = ctypes.c_void_p()
        if dev.type == "cuda":
            idx = dev.index if dev.index is not None else torch.cuda.current_device()
            kind, stream = (10, idx), _stream_of(dev)
            hip = csr._host_indptr
        else:
            kind, stream, hip = (1, 0), None, None

        def make():
            check_call(LIB.dglhip_spmm_plan_create(
                kind[0], kind[1], csr.num_rows, csr.num_cols, csr.nnz, ptr(csr.indptr),
                ptr(csr.indices) if csr.nnz else None, ptr(hip), ptr(csr.row_order), stream,
                ctypes.byref(h)))
        _retry_oom(make)
        self.handle = h.value

    @property
    def arg(self):
        return ("handle", self.handle)

    def stream(self):
        return _stream_of(self.device) if self.device.type == "cuda" else None

    def stream_arg(self):
        return ("handle", self.stream().value) if self.device.type == "cuda" else None

    def __del__(self):
        h, self.handle = self.handle, None
        if h:
            try:
                LIB.dglhip_spmm_plan_free(h)
            except Exception:  # noqa: BLE001 - interpreter shutdown
                pass

    def workspace(self, msg, red, F, ldu, urows, elen, emode, erow):
        key = (msg, red, F, ldu, urows, elen, emode, _POLICY_GEN[0])
        nbytes = self._ws.get(key)
        if nbytes is None:
            b = ctypes.c_int64()
            _retry_oom(lambda: check_call(LIB.dglhip_spmm_plan_workspace(
                self.handle, msg, red, F, ldu, urows, elen, emode, ptr(erow), self.stream(),
                ctypes.byref(b))))
            nbytes = self._ws[key] = int(b.value)
        return nbytes

    def schedule(self, msg, red, F, ldu=0, urows=0, elen=0, emode=0, erow=None):
        """(path, launches) a run with these arguments takes
        (DGLHIP_PLAN_PATH_*: 0 host, 1 rows, 2 blocked, 3 blocked max, 4 sweep)."""
        path, launches = ctypes.c_int(), ctypes.c_int64()
        _retry_oom(lambda: check_call(LIB.dglhip_spmm_plan_schedule(
            self.handle, msg, red, F, ldu, urows, elen, emode, ptr(erow), self.stream(),
            ctypes.byref(path), ctypes.byref(launches))))
        return int(path.value), int(launches.value)

    def stats(self):
        """dict: rows, cols, nnz, max_degree, nonempty, waves, heavy_threshold."""
        s = (ctypes.c_int64 * 7)()
        check_call(LIB.dglhip_spmm_plan_stats(self.handle, s))
        return dict(zip(("rows", "cols", "nnz", "max_degree", "nonempty", "waves",
                         "heavy_threshold"), list(s)))


PLAN_PATH_HOST, PLAN_PATH_ROWS, PLAN_PATH_BLOCKED, PLAN_PATH_MAX_BLOCKED, PLAN_PATH_SWEEP = \
    0, 1, 2, 3, 4
_EDGE_BY_SLOT, _EDGE_BY_EID, _EDGE_BY_MAP = 0, 1, 2


def _edge_layout(csr, msg, emap):
    """(layout, rows tensor) of the edge values for the plan: by slot, by the
    CSR's edge ids (the plan caches what it derives from them), or a map."""
    if msg in (MSG_COPY_U, MSG_COPY_U_BF16) or emap is SLOT:
        return _EDGE_BY_SLOT, None
    if emap is None:
        return _EDGE_BY_EID, csr.eid
    return _EDGE_BY_MAP, emap.contiguous()


def _run_gspmm(csr, msg, red, ufeat2, efeat2, elen, feat_len, want_arg, out=None, emap=None):
    """ufeat2: (num_cols, F) or None; efeat2: (E, elen) or None. Returns (out, arg).
    ``out`` (optional) receives the result; RED_SUM_ACCUM adds into it.
    ``emap`` says where slot k's edge values are: None = row eid[k] (edge-id
    order), SLOT = row k (efeat2 laid out in this CSR's slot order), or an
    int64 tensor of rows per slot."""
    dev = (ufeat2 if ufeat2 is not None else efeat2).device
    if _CALL_EVENTS is None or dev.type != "cuda":
        return _run_gspmm_call(csr, msg, red, ufeat2, efeat2, elen, feat_len, want_arg, out,
                               emap, dev)
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    start.record(torch.cuda.current_stream(dev))
    res = _run_gspmm_call(csr, msg, red, ufeat2, efeat2, elen, feat_len, want_arg, out, emap,
                          dev)
    end.record(torch.cuda.current_stream(dev))
    _CALL_EVENTS.append((start, end))
    return res


def _run_gspmm_call(csr, msg, red, ufeat2, efeat2, elen, feat_len, want_arg, out, emap, dev):
    """One product on the CSR's native plan (dglhip_spmm_plan_run): the plan
    picks the source-blocked schedule, the heavy-row split, the short-row
    tiers, the padded-stride copy and the edge values' order exactly as it
    does for a C-ABI caller."""
    if csr.device != dev:
        raise DGLError("adjacency on %s but features on %s" % (csr.device, dev))
    if out is None:
        out = torch.empty(csr.num_rows, feat_len, dtype=torch.float32, device=dev)
    arg = None
    if red == RED_MAX and want_arg:
        arg = torch.empty(csr.num_rows, feat_len, dtype=torch.int64, device=dev)
    plan = csr.plan
    emode, erow = _edge_layout(csr, msg, emap)
    ldu = 0
    if ufeat2 is not None and ufeat2.shape[0] > 1 and _row_strided(ufeat2, feat_len):
        ldu = ufeat2.stride(0)
    urows = 0 if ufeat2 is None else ufeat2.shape[0]
    elen = 0 if efeat2 is None else elen
    nbytes = plan.workspace(msg, red, feat_len, ldu, urows, elen, emode, erow)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev) if nbytes else None
    check_call(LIB.dglhip_spmm_plan_run(
        plan.handle, msg, red, feat_len, ptr(ufeat2), ldu, urows, ptr(efeat2), elen, emode,
        ptr(erow), ptr(out), ptr(arg), ptr(ws), nbytes, plan.stream()))
    return out, arg


def set_short_rows(on):
    """Route short / empty rows to the batched short-row kernel (default on);
    returns the old setting."""
    return bool(set_schedule_policy(short_rows=1 if on else 0)["short_rows"])


def set_blocked(policy):
    """Source-blocked schedule for copy_u / u_mul_e with sum / mean / max and
    the fused GAT layer: "auto" (default: where it keeps the chains
    bit-identical and the table size pays) or "off". Returns the old
    policy."""
    old = set_schedule_policy(blocked=0 if str(policy) == "off" else 1)
    return "auto" if old["blocked"] else "off"


def set_pad_rows(policy):
    """Padded-stride gathers for line-straddling rows: "auto" (default) or
    "off"; returns the old policy."""
    old = set_schedule_policy(pad_rows=1 if str(policy) == "auto" else 0)
    return "auto" if old["pad_rows"] else "off"


_PADDED = {}


def padded_width(F):
    """Row stride (floats) for the source rows of a g-SpMM gather: F itself,
    or F rounded up to 16 / 32 floats when that cuts the 128-B lines a row
    touches by at least 5 % (F = 41: 2.28 -> 2.0 lines at a 48-float stride;
    F = 24: 1.5 -> 1.0 at 32); the plan's rule (dglhip_spmm_padded_width)."""
    w = _PADDED.get(F)
    if w is None:
        o = ctypes.c_int64()
        check_call(LIB.dglhip_spmm_padded_width(int(F), ctypes.byref(o)))
        w = _PADDED[F] = int(o.value)
    return w


def _pad_rows(msg, red, ufeat2, feat_len):
    """Whether the plan gathers these rows from a padded copy (the same rule:
    callers that produce such rows write them padded instead)."""
    if msg not in (MSG_COPY_U, MSG_U_MUL_E) or red not in (RED_SUM, RED_MEAN) + _ACCUM or \
            ufeat2 is None or ufeat2.dtype != torch.float32:
        return False
    pol = schedule_policy()
    return (bool(pol["pad_rows"]) and ufeat2.numel() * 4 >= pol["pad_min_bytes"] and
            padded_width(feat_len) != feat_len)


# the fused GAT kernels' blocks: their per-row work (the attention through LDS)
# makes a row's pass per block dearer than copy_u's, so fewer, larger blocks
_GAT_BLOCK_BYTES = int(os.environ.get("DGLHIP_GAT_BLOCK_BYTES", 11 << 20))  # 11 MiB
# the fused forward when no attention is stored (inference, and training with
# the one-pass backward, which recomputes it): with the batch's logits loaded
# ahead of its row gathers the per-row pass got cheaper, so smaller blocks pay
# (Reddit-shaped 8 x 16: 4.96 ms at 7 MiB, 4.98 at 8, 5.22 at 9, 5.81 at 11;
# tools/gat_block_percall.py, profiles/r04/gat_bwd/fwd_block_sweep.log)
_GAT_BLOCK_BYTES_NOGRAD = int(os.environ.get("DGLHIP_GAT_BLOCK_BYTES_NOGRAD", 7 << 20))
# the one-pass GAT backward over the transpose (its own per-row work: the
# attention recomputed per pair, the dot's exchanges, the epilogue): larger
# slices, as the forward's (Reddit-shaped 8 x 16, forward + backward: 4 / 6 /
# 8 / 11 / 14 / 18 MiB 17.97 / 16.86 / 16.48 / 16.18 / 16.25 / 16.39 ms, the
# same bits; tools/gat_bwd_sweep.py, profiles/r04/gat_bwd_sweep.json); at 5
# waves per SIMD (r05) 6 / 8 / 11 / 14 / 18 / 24 MiB 14.63 / 14.30 / 14.15 /
# 14.06 / 14.29 / 14.65 ms (profiles/r05/gat_fwd/bwd_block_sweep_*.json)
_GAT_BWD_BLOCK_BYTES = int(os.environ.get("DGLHIP_GAT_BWD_BLOCK_BYTES", 14 << 20))


class _PlanLaunch(object):
    """One launch of the plan's source-blocked schedule (views of the plan's
    arrays): ``rows`` (int32) the rows with slots in the block, longest first
    (stable by row id); item i's slots are [ptr[i], ptr[i+1]) of the plan's
    global slot arrays (``ptr`` holds global offsets); ``indices`` / ``pos``
    this launch's slots (column ids, and the CSR slot each came from)."""
    __slots__ = ("rows", "ptr", "indices", "pos", "nnz", "off", "suffix")


class _BlockedSchedule(list):
    """The plan's source-blocked schedule: its launches (B blocks, then the
    suffix if any) plus the global arrays: ``indices`` / ``pos`` (plan
    order), ``absent`` (rows the first launch does not list)."""


def _blocked_native(csr, row_bytes, block_bytes, blocks=0):
    """The native plan's blocked schedule for gathered rows of ``row_bytes``
    in ``block_bytes`` slices (or exactly ``blocks`` blocks), as torch views
    of its arrays (cached per policy); None when none applies."""
    plan = csr.plan
    key = ("blocked", int(row_bytes), int(block_bytes), int(blocks), _POLICY_GEN[0])
    if key in plan._cache:
        return plan._cache[key]
    f = _retry_oom(lambda: _capi("SpmmPlanBlocked")(plan.arg, int(row_bytes), int(block_bytes),
                                                    int(blocks), plan.stream_arg()))
    res = None
    if f is not None:
        meta = f(0).tolist()
        B, sfx, _, L = meta[:4]
        res = _BlockedSchedule()
        res.indices, res.pos, res.absent = f(1), f(2), f(3)
        res.B, res.has_suffix = int(B), bool(sfx)
        for i in range(int(L)):
            n_items, nnz, off, suffix = meta[4 + 4 * i:8 + 4 * i]
            it = _PlanLaunch()
            it.rows, it.ptr = f(4 + 2 * i), f(5 + 2 * i)
            it.indices = res.indices[off:off + nnz]
            it.pos = res.pos[off:off + nnz]
            it.nnz, it.off, it.suffix = int(nnz), int(off), bool(suffix)
            res.append(it)
    plan._cache[key] = res
    return res


def _block_plan(csr, ufeat2, feat_len, block_bytes=None):
    """The blocked schedule the plan runs for these source rows (None when
    the product keeps one launch): the blocks cut the referenced column range
    evenly (``block_bytes`` of source rows each, default the policy's)."""
    ld = ufeat2.stride(0) if (ufeat2.dim() == 2 and ufeat2.shape[0] > 1) else feat_len
    row_bytes = max(ld, feat_len) * ufeat2.element_size()
    if csr.nnz == 0:
        return None
    return _blocked_native(csr, row_bytes, block_bytes or schedule_policy()["block_bytes"])


def _block_items(csr, blocks):
    """The plan's blocked schedule at exactly ``blocks`` source blocks (None:
    some rows' suffixes exceed the policy's share)."""
    return _blocked_native(csr, 0, 0, blocks)


def _column_span(csr):
    """(lo, hi): the range of columns the slots reference."""
    if csr.nnz == 0:
        return (0, 0)
    ind = csr.indices
    lo, hi = torch.aminmax(ind) if ind.is_cuda else (ind.min(), ind.max())
    return int(lo), int(hi) + 1


def _cuts_native(csr, row_bytes, block_bytes, blocks=0):
    plan = csr.plan
    key = ("cuts", int(row_bytes), int(block_bytes), int(blocks), _POLICY_GEN[0])
    if key in plan._cache:
        return plan._cache[key]
    arr = _retry_oom(lambda: _capi("SpmmPlanCuts")(plan.arg, int(row_bytes), int(block_bytes),
                                                   int(blocks), plan.stream_arg()))
    res = None if arr is None else [arr[i] for i in range(arr.shape[0])]
    plan._cache[key] = res
    return res


def _block_cuts(csr, row_bytes, block_bytes=None):
    """The blocked schedule as row ranges (the plan's, cached): B + 1 int64
    arrays (B + 2 when some rows have a suffix), row r's slots of range i
    being [cuts[i][r], cuts[i + 1][r]) of the CSR itself (cuts[0] =
    indptr[:-1], the last = indptr[1:]), for kernels that keep the CSR's slot
    indices (the fused GAT layer, the g-SDDMM). ``row_bytes``: bytes gathered
    per source. None when the schedule does not apply."""
    if csr.nnz == 0:
        return None
    return _cuts_native(csr, row_bytes, block_bytes or _GAT_BLOCK_BYTES)


def _plan_tag(plan):
    """(source blocks, has a suffix launch): the key of caches derived from a
    blocked plan. The plan's length alone is ambiguous: B blocks plus a suffix
    and B + 1 blocks without one are both B + 1 launches, and one CSR gets
    different B at different widths or dtypes."""
    sfx = bool(plan[-1].suffix)
    return (len(plan) - int(sfx), sfx)


def blocked_schedule(adj, ufeat):
    """The number of source-blocked launches the copy_u sum / mean g-SpMM of
    ``ufeat`` over ``adj`` runs in (0: one launch), as the plan schedules it."""
    adj = adj.to(ufeat.device)
    if ufeat.device.type != "cuda":
        return 0
    u2 = ufeat.reshape(ufeat.shape[0], -1)
    F = u2.shape[1]
    ldu = u2.stride(0) if (u2.shape[0] > 1 and _row_strided(u2, F)) else 0
    msg = MSG_COPY_U_BF16 if u2.dtype == torch.bfloat16 else MSG_COPY_U
    path, launches = adj.fwd.plan.schedule(msg, RED_SUM, F, ldu, u2.shape[0])
    return launches if path == PLAN_PATH_BLOCKED else 0


def _block_slots(csr, plan):
    """int64: for each slot of the blocked plan, blocks in order, the slot of
    ``csr`` it came from (cached; for edge-valued messages)."""
    key = ("blocked_slots",) + _plan_tag(plan)
    if key not in csr._plans:
        csr._plans[key] = plan.pos.long()
    return csr._plans[key]


def _block_edge_rows(csr, plan, emap):
    """Rows of the edge-value tensor for the blocked plan's slots, for the
    layout ``emap`` names (_run_gspmm): None = edge ids, SLOT = the CSR's
    slots, or a per-slot row tensor (e.g. the transpose's forward-slot map).
    Cached: per layout, and for a row tensor per tensor object (held weakly:
    a new tensor, or one changed in place, composes anew)."""
    tag = _plan_tag(plan)
    slots = _block_slots(csr, plan)
    if emap is SLOT or (emap is None and csr.slot_eid is None):
        return slots
    if emap is None:
        key = ("blocked_eid",) + tag
        if key not in csr._plans:
            csr._plans[key] = csr.slot_eid.index_select(0, slots)
        return csr._plans[key]
    key = ("blocked_emap",) + tag
    hit = csr._plans.get(key)
    if hit is not None and hit[0]() is emap and hit[1] == emap._version:
        return hit[2]
    rows = emap.index_select(0, slots)
    csr._plans[key] = (weakref.ref(emap), emap._version, rows)
    return rows


def segment_blocks(csrs, feat_len, dtypes):
    """Launches of the source-blocked schedule over CSRs gathered at
    ``feat_len`` features of the given row dtypes (one per CSR; a pipelined
    partition's own and halo segments), 0 for a CSR that keeps one launch."""
    total = 0
    for csr, dt in zip(csrs, dtypes):
        if csr.device.type != "cuda" or csr.nnz == 0:
            continue
        msg = MSG_COPY_U_BF16 if dt == torch.bfloat16 else MSG_COPY_U
        path, launches = csr.plan.schedule(msg, RED_SUM_ACCUM, feat_len, 0, csr.num_cols)
        total += launches if path == PLAN_PATH_BLOCKED else 0
    return total



def _run_sddmm_dot(csr, lhs2, rhs2, num_edges, heads=1, slot=False):
    """out[eid, h] = <lhs[row, head h], rhs[col, head h]>; returns (num_edges, heads).
    ``slot``: out[k] for slot k of ``csr`` instead (values in its slot order)."""
    dev = lhs2.device
    out = torch.zeros(num_edges, heads, dtype=torch.float32, device=dev)
    F = lhs2.shape[1]
    eid = None if slot else csr.eid
    if dev.type == "cuda":
        # rows longest-first; the gathered rows one source block at a time
        # where the CSR has a blocked schedule (per-edge values: same bits)
        cuts = (_block_cuts(csr, F * 4, schedule_policy()["block_bytes"]) or
                [csr.indptr, csr.indptr[1:]])
        for b in range(len(cuts) - 1):
            check_call(LIB.dglhip_gsddmm_ranges_device(
                0, csr.num_rows, F, heads, ptr(cuts[b]), ptr(cuts[b + 1]), ptr(csr.row_order),
                ptr(csr.indices), ptr(eid), ptr(lhs2), ptr(rhs2), ptr(out), _stream_of(dev)))
    else:
        check_call(LIB.dglhip_gsddmm_host(0, csr.num_rows, F, heads, ptr(csr.indptr),
                                          ptr(csr.indices), ptr(eid), ptr(lhs2), ptr(rhs2),
                                          ptr(out), 0))
    return out


def _fwd_slot_of_bwd(adj):
    """For each slot of the transposed CSR, the forward-CSR slot holding the
    same edge: how an edge tensor laid out in forward slot order is read along
    the transpose (backward of slot-ordered edge values). Cached on ``adj``."""
    m = getattr(adj, "_bwd_fslot", None)
    if m is None:
        fwd, bwd = adj.fwd, adj.bwd
        # (the identity check is a host sync: used only when already made)
        if fwd._slot_eid is None:  # forward slots known to run in edge-id order
            m = bwd.eid
        else:
            inv = torch.empty_like(fwd.eid)
            inv[fwd.eid] = torch.arange(fwd.nnz, dtype=fwd.eid.dtype, device=fwd.eid.device)
            m = inv.index_select(0, bwd.eid)
            del inv
        adj._bwd_fslot = m
    return m


def edge_order_of(adj, edge_order):
    """Validate an ``edge_order`` argument ("eid" or "slot")."""
    if edge_order not in ("eid", "slot"):
        raise DGLError("edge_order must be 'eid' or 'slot', got %r" % (edge_order,))
    return edge_order == "slot"


def slot_permutation(adj):
    """int64[nnz]: the edge id held by each forward-CSR slot of ``adj``. An
    edge tensor ``x`` in edge-id order is ``x[slot_permutation(adj)]`` in slot
    order; a slot-ordered ``y`` goes back with ``out[perm] = y``."""
    return adj.fwd.eid


def _eid_major(adj):
    """(csr, transposed): the CSR of ``adj`` whose slots walk the edge ids most
    nearly in order, for kernels that store one value per edge at out[eid]
    (g-SDDMM): the stores are then sequential instead of a scatter. The
    forward CSR unless the transpose's edge ids run clearly more in order
    (edges added source-major, as the (src, dst)-sorted loaders add them).
    Every per-edge value is symmetric in its two endpoint operands (a*b ==
    b*a, fma(a, b, c) == fma(b, a, c), a + b == b + a, all exact), so both
    walks give the same bits."""
    fwd = adj.fwd
    if fwd.slot_eid is None:
        return fwd, False
    bwd = adj.bwd
    if bwd.eid_locality > max(0.5, 2.0 * fwd.eid_locality):
        return bwd, True
    return fwd, False


def _row_strided(t, F):
    """A (rows, F) float32 view whose rows sit at an even stride > F (a
    row-padded buffer): the strided g-SpMM entries read it as it is."""
    return (t.dim() == 2 and t.dtype == torch.float32 and t.shape[1] == F and
            t.stride(1) == 1 and t.stride(0) > F and t.stride(0) % 2 == 0)


def _f32c(t):
    if t is None:
        return None
    if t.dtype != torch.float32:
        raise DGLError("g-SpMM computes in float32, got %s" % t.dtype)
    return t.contiguous()


def _mean_scaled(fwd, dout, padded_ok):
    """dC / deg, the mean reducer's backward ahead of the transposed product;
    with ``padded_ok`` (only the node gradient reads it) written straight into
    the padded rows that product gathers when the rows straddle lines (one pass
    instead of the division's and the padding copy's)."""
    deg = fwd.mean_divisor()
    F = dout.shape[1]
    if padded_ok and dout.is_cuda and _pad_rows(MSG_COPY_U, RED_SUM, dout, F):
        ld = padded_width(F)
        buf = dout.new_empty(dout.shape[0], ld)
        check_call(LIB.dglhip_div_rows_device(
            dout.shape[0], F, ptr(dout), dout.stride(0), ptr(deg), ptr(buf), ld,
            _stream_of(dout.device)))
        return buf[:, :F]
    return (dout / deg).contiguous()


class _GSpMM(torch.autograd.Function):
    """out = REDUCE over in-slots of MSG(ufeat[col], efeat[eid]).

    Backward (SUM/MEAN): dU = the same product over the transposed CSR (the
    reference's autograd of torch.sparse.mm computes Aᵀ·dC the same way,
    accumulating over out-edges in edge-id order); dE by g-SDDMM.

    ``slot``: efeat is laid out in the forward CSR's slot order (row k = slot
    k), so the forward reads it without the eid indirection and dE comes back
    in the same layout (the SDDMM walks the forward CSR, sequential stores)."""

    @staticmethod
    def forward(ctx, adj, msg, red, feat_len, num_edges, ufeat2, efeat2, slot=False):
        elen = 0 if efeat2 is None else efeat2.shape[1]
        need_arg = red == RED_MAX and (
            (ufeat2 is not None and ufeat2.requires_grad) or
            (efeat2 is not None and efeat2.requires_grad))
        out, arg = _run_gspmm(adj.fwd, msg, red, ufeat2, efeat2, elen, feat_len, need_arg,
                              emap=SLOT if slot else None)
        ctx.adj, ctx.msg, ctx.red, ctx.num_edges, ctx.slot = adj, msg, red, num_edges, slot
        # keep an operand alive only when the backward reads its values: the
        # node rows for u_mul_e's edge gradient, the edge values for its node
        # gradient. copy_u/copy_e + sum/mean save nothing (in a partitioned
        # layer ufeat2 is the whole gathered halo, GBs per layer)
        u_mul_e = msg == MSG_U_MUL_E
        need_u = ufeat2 is not None and ufeat2.requires_grad
        need_e = efeat2 is not None and efeat2.requires_grad
        ctx.ushape = None if ufeat2 is None else tuple(ufeat2.shape)
        ctx.eshape = None if efeat2 is None else tuple(efeat2.shape)
        ctx.save_for_backward(ufeat2 if (u_mul_e and need_e) else None,
                              efeat2 if (u_mul_e and need_u) else None, arg)
        return out

    @staticmethod
    def backward(ctx, dout):
        ufeat2, efeat2, arg = ctx.saved_tensors
        adj, msg, red, slot = ctx.adj, ctx.msg, ctx.red, ctx.slot
        dout = dout.contiguous()
        fwd = adj.fwd
        du = de = None
        need_u = ctx.needs_input_grad[5]
        need_e = ctx.needs_input_grad[6]
        F = dout.shape[1]
        if red == RED_MEAN:
            dout = _mean_scaled(fwd, dout, padded_ok=need_u and not need_e)
            red_b = RED_SUM
        else:
            red_b = red
        if red_b == RED_SUM:
            if need_u:
                elen = 0 if efeat2 is None else efeat2.shape[1]
                reads_e = msg == MSG_U_MUL_E
                du, _ = _run_gspmm(adj.bwd, msg if msg != MSG_COPY_E else MSG_COPY_U, RED_SUM,
                                   dout, efeat2 if reads_e else None, elen if reads_e else 0, F,
                                   False, emap=_fwd_slot_of_bwd(adj) if (slot and reads_e)
                                   else None)
            if need_e:
                rows = fwd.row_ids()
                if msg == MSG_COPY_E:
                    g = dout.index_select(0, rows)
                    if ctx.eshape[1] == 1:
                        g = g.sum(1, keepdim=True)
                elif ctx.eshape[1] < F:  # scalar or per-head weights: g-SDDMM dot
                    u2 = ufeat2.contiguous()
                    if slot:  # forward walk, de[k] stored in slot order
                        de = _run_sddmm_dot(fwd, dout, u2, ctx.num_edges, ctx.eshape[1],
                                            slot=True)
                    else:
                        csr, tr = _eid_major(adj)
                        de = _run_sddmm_dot(csr, u2 if tr else dout, dout if tr else u2,
                                            ctx.num_edges, ctx.eshape[1])
                    g = None
                else:
                    g = dout.index_select(0, rows) * ufeat2.index_select(0, fwd.indices.long())
                if g is not None:
                    if slot:
                        de = g.reshape(ctx.eshape)
                    else:
                        de = dout.new_zeros(ctx.eshape)
                        de.index_copy_(0, fwd.eid, g)
        else:  # MAX: route each output element's gradient to its argmax slot
            valid = arg >= 0
            slots = arg.clamp(min=0)
            rowsel = valid.nonzero(as_tuple=True)
            sl = slots[rowsel]
            g = dout[rowsel]
            fidx = rowsel[1]
            dpe = F // ctx.eshape[1] if ctx.eshape is not None else 1
            if need_u:
                src = fwd.indices.long()[sl]
                gu = g
                if msg == MSG_U_MUL_E:
                    e = sl if slot else fwd.eid[sl]
                    gu = g * efeat2[e, fidx // dpe]
                du = dout.new_zeros(ctx.ushape)
                du.index_put_((src, fidx), gu, accumulate=True)
            if need_e:
                e = sl if slot else fwd.eid[sl]
                ge = g
                if msg == MSG_U_MUL_E:
                    ge = g * ufeat2[fwd.indices.long()[sl], fidx]
                de = dout.new_zeros(ctx.eshape)
                de.index_put_((e, fidx // dpe), ge, accumulate=True)
        return None, None, None, None, None, du, de, None


def gspmm(adj, msg, reduce, ufeat=None, efeat=None, num_edges=None, edge_order="eid"):
    """Generalised SpMM over ``adj`` (a SparseAdj on the features' device).

    ufeat : (num_cols, *fshape) node features or None (copy_e)
    efeat : (num_edges,) / (num_edges, 1) scalar or (num_edges, *fshape) edge
            features indexed by the adjacency's eid, or None (copy_u)
    edge_order : "eid" (efeat row e = edge id e, the frame's layout) or
            "slot" (row k = the forward CSR's slot k, as edge_attention /
            gsddmm_dot return with edge_order="slot": no eid indirection)
    returns (num_rows, *fshape) float32
    """
    slot = edge_order_of(adj, edge_order)
    msg = _MSG_NAMES.get(msg, msg)
    red = _RED_NAMES.get(reduce, reduce)
    if msg != MSG_COPY_E and ufeat is None:
        raise DGLError("message needs source node features")
    if msg != MSG_COPY_U and efeat is None:
        raise DGLError("message needs edge features")
    if ufeat is not None:
        fshape = tuple(ufeat.shape[1:])
    else:
        fshape = tuple(efeat.shape[1:]) if efeat.dim() > 1 else ()
        if fshape == (1,):
            fshape = (1,)
    F = 1
    for s in fshape:
        F *= int(s)
    dev = (ufeat if ufeat is not None else efeat).device
    adj = adj.to(dev)
    if ufeat is not None and _row_strided(ufeat, F) and dev.type == "cuda" and \
            msg == MSG_COPY_U and red in (RED_SUM, RED_MEAN):
        u2 = ufeat  # rows at a padded stride: gathered in place (_run_gspmm)
    else:
        u2 = None if ufeat is None else _f32c(ufeat.reshape(ufeat.shape[0], F))
    e2 = None
    if efeat is not None:
        ne = efeat.shape[0]
        elen = _edge_len(efeat.shape[1:], fshape) if ufeat is not None else F
        e2 = _f32c(efeat.reshape(ne, elen))
    if num_edges is None:
        num_edges = 0 if e2 is None else e2.shape[0]
    out = _GSpMM.apply(adj, msg, red, F, num_edges, u2, e2, slot)
    shape = (adj.shape[0],) + fshape if fshape else (adj.shape[0],)
    # the product's own tensor when no reshape is needed: a view would make
    # a caller's in-place update of the result rebase its autograd graph
    # (CopySlices: a zero fill and a copy of the whole gradient)
    return out if tuple(out.shape) == shape else out.reshape(shape)


class _MeanAddInto(torch.autograd.Function):
    """out <- out + mean over in-slots of ufeat[col] (copy_u + mean whose
    store adds the row's mean to the value in ``out``, in place). Backward:
    the incoming gradient for ``out``'s old value, the mean's transposed
    product for ufeat."""

    @staticmethod
    def forward(ctx, adj, ufeat2, out, feat_len):
        _run_gspmm(adj.fwd, MSG_COPY_U, RED_MEAN_ACCUM, ufeat2, None, 0, feat_len, False,
                   out=out)
        ctx.mark_dirty(out)
        ctx.adj = adj
        # what the backward's operand dC / deg looks like when padded: a
        # producer of dC (the node-row loss kernel) can write it as it stores
        # dC and hand it over as ``prescaled`` (nn.pytorch.sage_dense)
        ctx.scale_spec = None
        if out.is_cuda and _pad_rows(MSG_COPY_U, RED_SUM, out, feat_len):
            ctx.scale_spec = (adj.fwd.mean_divisor(), padded_width(feat_len))
        ctx.prescaled = None
        return out

    @staticmethod
    def backward(ctx, dout):
        adj = ctx.adj
        dout = dout.contiguous()
        given, ctx.prescaled = ctx.prescaled, None
        du = None
        if ctx.needs_input_grad[1]:
            d = _handoff.take(given, dout)  # dC / deg, written by dC's producer
            if d is None:
                d = _mean_scaled(adj.fwd, dout, padded_ok=True)
            du, _ = _run_gspmm(adj.bwd, MSG_COPY_U, RED_SUM, d, None, 0, dout.shape[1], False)
        return None, du, dout if ctx.needs_input_grad[2] else None, None


def gspmm_mean_add(adj, ufeat, out):
    """out <- out + mean over in-edges of ufeat[src] (copy_u + mean), in place
    and differentiable: the value of ``out + gspmm(adj, "copy_u", "mean",
    ufeat)`` bit for bit (a sum of two terms; rows without in-edges keep their
    value), with the addition in the aggregation's own store instead of a pass
    over both tensors (GraphSAGE's fc_self(h) + mean(fc_neigh(h)),
    nn.pytorch.sage_dense). ``out``: contiguous float32 (num_rows, F) on the
    features' device; ufeat may be row-padded (F columns of a wider row)."""
    F = out.shape[1] if out.dim() == 2 else -1
    dev = ufeat.device
    if (out.dtype != torch.float32 or out.dim() != 2 or not out.is_contiguous() or
            out.device != dev or ufeat.dim() != 2 or ufeat.shape[1] != F):
        raise DGLError("gspmm_mean_add: out must be a contiguous float32 (num_rows, F) "
                       "tensor beside (num_cols, F) features")
    adj = adj.to(dev)
    if out.shape[0] != adj.shape[0] or ufeat.shape[0] < adj.shape[1]:
        raise DGLError("gspmm_mean_add: shapes do not match the adjacency")
    u2 = ufeat if (_row_strided(ufeat, F) and dev.type == "cuda") else _f32c(ufeat)
    return _MeanAddInto.apply(adj, u2, out, F)


def gsddmm_dot(adj, lhs, rhs, num_edges, heads=1, edge_order="eid"):
    """out[eid, h] = <lhs[row, h], rhs[col, h]> for every slot of ``adj``
    (rows of lhs are the adjacency's rows, of rhs its columns; no autograd).
    edge_order="slot" returns row k = forward CSR slot k instead."""
    slot = edge_order_of(adj, edge_order)
    dev = lhs.device
    adj = adj.to(dev)
    lhs2 = _f32c(lhs.reshape(lhs.shape[0], -1))
    rhs2 = _f32c(rhs.reshape(rhs.shape[0], -1))
    if slot:
        return _run_sddmm_dot(adj.fwd, lhs2, rhs2, num_edges, heads, slot=True)
    csr, tr = _eid_major(adj)
    return _run_sddmm_dot(csr, rhs2 if tr else lhs2, lhs2 if tr else rhs2, num_edges, heads)


def gspmm_into(csr, out, ufeat, accumulate=False):
    """Raw copy_u + sum over ``csr`` into ``out`` (num_rows, F), no autograd:
    out = A·ufeat (ufeat float32, or bfloat16 rows widened exactly to fp32 in
    the kernel), or with ``accumulate`` out += A·ufeat with every row's chain
    continued from the value already in ``out`` (one product evaluated segment
    by segment: dgl.distributed's pipelined forward). Degree-descending
    schedule and, under set_row_split, heavy rows cut into chunks whose
    partials are added in order (deterministic)."""
    if out.dtype != torch.float32 or not out.is_contiguous():
        raise DGLError("out must be a contiguous float32 tensor")
    if out.shape[0] != csr.num_rows or out.device != csr.device:
        raise DGLError("out does not match the adjacency")
    if ufeat.shape[0] < csr.num_cols:
        raise DGLError("ufeat has %d rows, the adjacency %d columns"
                       % (ufeat.shape[0], csr.num_cols))
    F = out.shape[1]
    if ufeat.dtype == torch.bfloat16:  # rows read as bf16, summed in fp32 (exact widening)
        u2, msg = ufeat.reshape(ufeat.shape[0], F).contiguous(), MSG_COPY_U_BF16
    else:
        u2, msg = _f32c(ufeat.reshape(ufeat.shape[0], F)), MSG_COPY_U
    _run_gspmm(csr, msg, RED_SUM_ACCUM if accumulate else RED_SUM, u2, None, 0, F,
               False, out=out)
    return out


def gspmm_ranges(msg, beg, end, accumulate, indices, out, ufeat=None, efeat=None, eid=None):
    """out[i] (=|+=) sum over slots [beg[i], end[i]) of MSG(ufeat[indices[k]], efeat[eid[k]]),
    each row one sequential chain (continued from ``out`` when ``accumulate``).
    Raw op without autograd (the pipelined distributed forward)."""
    msg = _MSG_NAMES.get(msg, msg)
    dev = out.device
    F = out.shape[1]
    elen = 0 if efeat is None else efeat.shape[1]
    args = (msg, beg.numel(), F, ptr(beg), ptr(end), 1 if accumulate else 0, ptr(indices),
            ptr(eid), ptr(ufeat), ptr(efeat), elen, ptr(out))
    if dev.type == "cuda":
        check_call(LIB.dglhip_gspmm_ranges_device(*(args + (_stream_of(dev),))))
    else:
        check_call(LIB.dglhip_gspmm_ranges_host(*(args + (0,))))
    return out


def set_gather_mode(mode):
    """Study knob: where the copy_u + sum kernel's row gathers go through
    buffer descriptors instead of global loads, a bit mask (bit 0 one-launch
    calls, bit 1 the blocked schedule's launches: the default, 2); True = 3,
    False = 0. Same values."""
    if isinstance(mode, bool):
        mode = 3 if mode else 0
    check_call(LIB.dglhip_set_gather_mode(int(mode)))


def set_sddmm_variant(alternate):
    """Study knob for the sliced g-SDDMM dot: bit 0 runs it at its
    alternative depth of slots in flight, bit 1 loads the GAT epilogue's
    per-slot operands after the dot product instead of with the slot's
    gathers; 0 (default) neither. Same bits."""
    check_call(LIB.dglhip_set_sddmm_variant(int(alternate)))


# per-call timing (timing_enable(per_call=True)): (start, end) event pairs
_CALL_EVENTS = None


def timing_enable(flag=True, per_call=False):
    """Bracket every g-SpMM/g-SDDMM launch with hipEvents (bench support).
    With ``per_call`` instead one event pair on the current stream around each
    g-SpMM call on a ROCm device (all of the call's launches and its output's
    zero fill, no markers between the launches: the blocked schedule's 19
    launches per call had paid 0.18 ms for them); timing_read then counts
    calls."""
    global _CALL_EVENTS
    _CALL_EVENTS = [] if (flag and per_call) else None
    check_call(LIB.dglhip_timing_enable(1 if (flag and not per_call) else 0))


def timing_read():
    """(total kernel ms, launches — calls under per-call timing) since the
    last timing_enable."""
    if _CALL_EVENTS is not None:
        for _, end in _CALL_EVENTS:
            end.synchronize()
        return sum(a.elapsed_time(b) for a, b in _CALL_EVENTS), len(_CALL_EVENTS)
    ms = ctypes.c_double()
    n = ctypes.c_int64()
    check_call(LIB.dglhip_timing_read(ctypes.byref(ms), ctypes.byref(n)))
    return ms.value, n.value


# ---------------------------------------------------------------------------
# Typed-edge block-diagonal g-SpMM (R-GCN block layer)
# ---------------------------------------------------------------------------
class _Segments(object):
    """A CSR-like view for the typed-block kernels: rows with slot ranges
    ``indptr`` over column ids ``indices`` (int32)."""

    def __init__(self, indptr, indices):
        self.indptr, self.indices = indptr, indices
        self.num_rows = indptr.numel() - 1
        self.nnz = indices.numel()
        self._plans = {}


class _GatherRows(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, idx):
        ctx.num_rows = x.shape[0]
        ctx.save_for_backward(idx)
        return x.index_select(0, idx)

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        m, n = idx.numel(), ctx.num_rows
        if m == 0:
            return dy.new_zeros((n,) + tuple(dy.shape[1:])), None
        dy2 = _f32c(dy.reshape(m, -1))
        F = dy2.shape[1]
        dev = dy2.device
        # positions grouped by row, in increasing position (a stable sort; the
        # counts by an integer scatter-add): no host sync
        ptr_, order = _position_groups(idx, n)
        # the sum per row as the typed-block kernel over F blocks of 1 x 1
        # ones (fma(1, x, acc) == acc + x): chains of TYPED_CHUNK positions,
        # the chunks of a long row added in order
        seg = _Segments(ptr_, order)
        ones = torch.ones(1, F, 1, 1, dtype=torch.float32, device=dev)
        rel = torch.zeros(m, dtype=torch.int32, device=dev)
        dx = _run_typed_block(seg, dy2, ones, rel, None, F, 1, 1)
        return dx.view((n,) + tuple(dy.shape[1:])), None


def gather_rows(x, idx):
    """``x[idx]`` (rows) whose gradient sums each row's duplicates
    deterministically: dx[r] = the dy[i] with idx[i] == r in increasing i, as
    chains of TYPED_CHUNK positions whose partials are added in order (the
    typed-block kernel with unit weights; no atomics, no host sync). torch's
    index backward accumulates duplicates in an implementation-defined order
    and walks a hub row's duplicates serially (R-GCN's DistMult decoder: 3 of
    the 8 ms step, tools/rgcn_step.py)."""
    idx = idx.to(device=x.device, dtype=torch.int64).reshape(-1)
    return _GatherRows.apply(x, idx)


TYPED_CHUNK = 64  # DGLHIP_TYPED_CHUNK: slots per chain of the typed-block kernels


def set_typed_block_width(slices):
    """Study knob: at most ``slices`` (1, 2, 4, 8) slices of 64 outputs per
    wave of the typed-block g-SpMM (default 1; 8 was slower at configs[4]).
    Same bits."""
    check_call(LIB.dglhip_set_typed_block_width(int(slices)))


_DEBUG_GROUPS = os.environ.get("DGLHIP_DEBUG_GROUPS", "0") not in ("", "0")


def _check_groups(ptr_, order, idx, num_rows):
    """DGLHIP_DEBUG_GROUPS=1: check a position grouping on the host before a
    kernel walks it (one sync; skipped under HIP-graph capture)."""
    if idx.is_cuda and torch.cuda.is_current_stream_capturing():
        return
    p, o, ix = ptr_.cpu(), order.cpu().long(), idx.cpu()
    m = ix.numel()
    problems = []
    if p.numel() != num_rows + 1 or int(p[0]) != 0 or int(p[-1]) != m:
        problems.append("ptr ends %s..%s for %d positions" % (p[:1].tolist(), p[-1:].tolist(), m))
    if bool((p[1:] < p[:-1]).any()):
        problems.append("ptr not monotone")
    if m and (int(o.min()) < 0 or int(o.max()) >= m or
              not torch.equal(torch.sort(o)[0], torch.arange(m))):
        problems.append("order is not a permutation of the positions")
    if m and (int(ix.min()) < 0 or int(ix.max()) >= num_rows):
        problems.append("ids span [%d, %d] for %d rows" % (int(ix.min()), int(ix.max()), num_rows))
    if problems:
        raise DGLError("malformed position grouping: " + "; ".join(problems))


def _position_groups_items(idx, num_rows):
    """_position_groups on a device with the typed-block item list over it,
    in one library call (dglhip_group_positions_device: ≈80 µs of host time
    as a CSR build plus _typed_items, r06): (ptr, order, item_ptr, item_row)."""
    dev = idx.device
    m = idx.numel()
    R = max(int(num_rows), 1)
    bound = R + -(-m // TYPED_CHUNK)
    nb = LIB.dglhip_group_positions_workspace_bytes(R, m)
    if nb < 0:
        check_call(-1)
    ptr_ = torch.empty(R + 1, dtype=torch.int64, device=dev)
    order = torch.empty(max(m, 1), dtype=torch.int32, device=dev)[:m]
    item_ptr = torch.empty(R + 1, dtype=torch.int64, device=dev)
    item_row = torch.empty(bound, dtype=torch.int32, device=dev)
    ws = torch.empty(max(int(nb), 1), dtype=torch.uint8, device=dev)
    check_call(LIB.dglhip_group_positions_device(
        R, m, ptr(idx.contiguous()), bound, ptr(ptr_), ptr(order), ptr(item_ptr),
        ptr(item_row), ptr(ws), int(nb), _stream_of(dev)))
    return ptr_, order, item_ptr, item_row


def _position_groups(idx, num_rows):
    """Positions of ``idx`` grouped by row in increasing position, no host
    sync: (ptr int64[R+1], order int32[m]). On a device, the library's CSR
    builder over (idx, position) — an LSD radix sort, stable, and each row's
    first slot found by the fill — instead of torch's merge sort, scatter-add
    and scan (a quarter of the launches); the same arrays."""
    m = idx.numel()
    if idx.is_cuda and m:
        return _position_groups_items(idx, num_rows)[:2]
    order = torch.sort(idx, stable=True)[1].to(torch.int32)
    counts = torch.zeros(num_rows, dtype=torch.int64, device=idx.device).scatter_add_(
        0, idx, torch.ones_like(idx))
    ptr_ = torch.zeros(num_rows + 1, dtype=torch.int64, device=idx.device)
    torch.cumsum(counts, 0, out=ptr_[1:])
    return ptr_, order


class _DistMult(torch.autograd.Function):
    """score[i] = sum_f (h[s_i] * w[r_i] * h[o_i])_f in one kernel (no
    [n, F] gathers or products), and its gradients as ordered chains per node
    and relation (dglhip_distmult_*): each position's term as torch's autograd
    of the three-way product computes it, chained as gather_rows' backward
    chains them, so dh and dw carry the bits of the torch formulation
    ``gather_rows(h, s) * gather_rows(w, r) * gather_rows(h, o)`` with its
    duplicates summed by gather_rows; the score's sum runs in the kernel's
    order (lane chains + butterfly) instead of torch's."""

    @staticmethod
    def forward(ctx, h, w, s, r, o):
        n, F = s.numel(), h.shape[1]
        score = torch.empty(n, dtype=torch.float32, device=h.device)
        args = (n, F, h.shape[0], w.shape[0], ptr(s), ptr(r), ptr(o), ptr(h), ptr(w), ptr(score))
        if h.is_cuda:
            check_call(LIB.dglhip_distmult_score_device(*(args + (_stream_of(h.device),))))
        else:
            check_call(LIB.dglhip_distmult_score_host(*(args + (0,))))
        ctx.save_for_backward(h, w, s, r, o)
        return score

    @staticmethod
    def backward(ctx, dscore):
        h, w, s, r, o = ctx.saved_tensors
        ds = _f32c(dscore.reshape(-1))
        n, F = s.numel(), h.shape[1]
        grads = [None, None]
        for task, (need, rows, idx) in enumerate(
                ((ctx.needs_input_grad[0], h.shape[0], lambda: torch.cat([s, o])),
                 (ctx.needs_input_grad[1], w.shape[0], lambda: r))):
            if not need:
                continue
            ix = idx()
            if h.is_cuda and ix.numel():
                ptr_, order, item_ptr, item_row = _position_groups_items(ix, rows)
            else:
                ptr_, order = _position_groups(ix, rows)
                item_ptr = item_row = None
            if _DEBUG_GROUPS:
                _check_groups(ptr_, order, ix, rows)
            out = torch.empty(rows, F, dtype=torch.float32, device=h.device)
            common = (n, h.shape[0], w.shape[0])
            tail = (ptr(order), ptr(s), ptr(r), ptr(o), ptr(ds), ptr(h), ptr(w), ptr(out))
            if h.is_cuda:
                if item_ptr is None:
                    item_ptr, item_row = _typed_items(ptr_, ix.numel())
                part = torch.empty(item_row.numel(), F, dtype=torch.float32, device=h.device)
                check_call(LIB.dglhip_distmult_grad_device(
                    task, rows, item_row.numel(), F, *common, ptr(ptr_), ptr(item_ptr),
                    ptr(item_row), *tail, ptr(part), _stream_of(h.device)))
            else:
                check_call(LIB.dglhip_distmult_grad_host(task, rows, F, *common, ptr(ptr_),
                                                         *tail, 0))
            grads[task] = out
        return grads[0], grads[1], None, None, None


def distmult_score(h, w_rel, subj, rel, obj):
    """DistMult scores of (subj, rel, obj) triples over node embeddings ``h``
    and relation vectors ``w_rel`` (the reference's calc_score,
    examples/pytorch/rgcn/link_predict.py:50-55) in one kernel; differentiable
    in h and w_rel with deterministic gradients (see _DistMult). Indices out of
    range raise IndexError, as the torch formulation's index_select does: ids
    given on the host are checked there before they move; ids already on a
    device are checked when ``set_validate_indices(True)`` (or
    DGLHIP_VALIDATE_INDICES=1) asks for it, with one min/max reduction and a
    host sync per call. Unchecked, the kernel never reads past its tables: an
    out-of-range position scores NaN and adds nothing to the gradients."""
    return _DistMult.apply(_f32c(h), _f32c(w_rel), *_distmult_ids(h, w_rel, subj, rel, obj))


def _distmult_ids(h, w_rel, subj, rel, obj):
    """The triples' ids as int64 on h's device, checked (distmult_score)."""
    dev = h.device
    if w_rel.shape[1:] != h.shape[1:] or h.dim() != 2:
        raise DGLError("distmult_score: h and w_rel must be 2-D of one width")
    trip = [torch.as_tensor(t) for t in (subj, rel, obj)]
    if not (trip[0].numel() == trip[1].numel() == trip[2].numel()):
        raise DGLError("distmult_score: subj, rel, obj lengths differ")
    on_host = all(t.device.type == "cpu" for t in trip)
    if trip[0].numel() and (on_host or (_VALIDATE_INDICES and not (
            dev.type == "cuda" and torch.cuda.is_current_stream_capturing()))):
        lo_hi = torch.stack([torch.stack([t.min(), t.max()]).to(torch.int64)
                             for t in trip]).tolist()
        for (lo, hi), bound, what in zip(lo_hi, (h.shape[0], w_rel.shape[0], h.shape[0]),
                                         ("subj", "rel", "obj")):
            if lo < 0 or hi >= bound:
                raise IndexError("distmult_score: %s ids span [%d, %d], out of range for %d rows"
                                 % (what, lo, hi, bound))
    # one stacking copy (the triples usually arrive as the columns of one
    # (n, 3) sample tensor: three strided views) instead of three
    ids = torch.stack([t.to(device=dev, dtype=torch.int64).reshape(-1) for t in trip])
    return [ids[0], ids[1], ids[2]]


class _DistMultLoss(torch.autograd.Function):
    """distmult_link_loss on a device: the loss and the scores in two
    launches, the gradients as _DistMult's chains with the BCE gradient formed
    in the kernel and the regulariser's term added to every row
    (dglhip_distmult_loss_*)."""

    @staticmethod
    def forward(ctx, h, w, s, r, o, labels, reg):
        n, F = s.numel(), h.shape[1]
        dev = h.device
        score = torch.empty(n, dtype=torch.float32, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        nws = LIB.dglhip_distmult_loss_workspace_floats(n, h.shape[0], w.shape[0], F)
        ws = torch.empty(max(int(nws), 1), dtype=torch.float32, device=dev)
        check_call(LIB.dglhip_distmult_loss_fwd_device(
            n, F, h.shape[0], w.shape[0], ptr(s), ptr(r), ptr(o), ptr(h), ptr(w), ptr(labels),
            float(reg), ptr(score), ptr(loss), ptr(ws), int(nws), _stream_of(dev)))
        ctx.save_for_backward(h, w, s, r, o, labels, score)
        ctx.reg = float(reg)
        return loss

    @staticmethod
    def backward(ctx, g):
        h, w, s, r, o, labels, score = ctx.saved_tensors
        g = g.detach().to(torch.float32).reshape(1).contiguous()
        n, F = s.numel(), h.shape[1]
        dev = h.device
        grads = [None, None]
        for task, (need, rows, idx) in enumerate(
                ((ctx.needs_input_grad[0], h.shape[0], lambda: torch.cat([s, o])),
                 (ctx.needs_input_grad[1], w.shape[0], lambda: r))):
            if not need:
                continue
            ptr_, order, item_ptr, item_row = _position_groups_items(idx(), rows)
            out = torch.empty(rows, F, dtype=torch.float32, device=dev)
            part = torch.empty(item_row.numel(), F, dtype=torch.float32, device=dev)
            check_call(LIB.dglhip_distmult_loss_grad_device(
                task, rows, item_row.numel(), F, n, h.shape[0], w.shape[0], ptr(ptr_),
                ptr(item_ptr), ptr(item_row), ptr(order), ptr(s), ptr(r), ptr(o), ptr(score),
                ptr(labels), ptr(g), ctx.reg, ptr(h), ptr(w), ptr(out), ptr(part),
                _stream_of(dev)))
            grads[task] = out
        return grads[0], grads[1], None, None, None, None, None


def distmult_link_loss(h, w_rel, subj, rel, obj, labels, reg):
    """The R-GCN link-prediction loss (the reference's get_loss,
    examples/pytorch/rgcn/link_predict.py:57-66):

        F.binary_cross_entropy_with_logits(distmult_score(h, w_rel, subj, rel, obj), labels)
            + reg * (h.pow(2).mean() + w_rel.pow(2).mean())

    On a ROCm device one forward launch pair and the decoder's gradient
    launches (the BCE and regulariser gradients formed inside them) instead of
    about twenty small kernels; values within fp32 rounding of that
    expression (its sums associate differently). Ids are checked as
    distmult_score checks them."""
    ids = _distmult_ids(h, w_rel, subj, rel, obj)
    labels = torch.as_tensor(labels)
    if (h.is_cuda and h.dtype == torch.float32 and w_rel.dtype == torch.float32 and
            ids[0].numel() > 0 and h.numel() > 0):
        lab = labels.to(device=h.device, dtype=torch.float32).reshape(-1).contiguous()
        if lab.numel() != ids[0].numel():
            raise DGLError("distmult_link_loss: %d labels for %d triples"
                           % (lab.numel(), ids[0].numel()))
        return _DistMultLoss.apply(_f32c(h), _f32c(w_rel), *ids, lab, float(reg))
    score = _DistMult.apply(_f32c(h), _f32c(w_rel), *ids)
    return (torch.nn.functional.binary_cross_entropy_with_logits(score, labels.to(score)) +
            reg * (h.pow(2).mean() + w_rel.pow(2).mean()))


_VALIDATE_INDICES = os.environ.get("DGLHIP_VALIDATE_INDICES", "0") not in ("", "0")


def set_validate_indices(on):
    """Check device-resident index arguments (distmult_score's triples,
    typed_block_spmm's relations) on the host before launching (one sync per
    call); returns the old setting. Host-resident ones are always checked."""
    global _VALIDATE_INDICES
    old, _VALIDATE_INDICES = _VALIDATE_INDICES, bool(on)
    return old


def _typed_items(rowptr, nnz):
    """The typed-block kernels' work items over a CSR-like ``rowptr`` with
    ``nnz`` slots, built on the device with no host sync (cached by the
    caller): (item_ptr int64[R+1] — each row's first item, a row of deg slots
    having max(1, ceil(deg / TYPED_CHUNK)) items —, item_row int32[I_max],
    I_max = R + ceil(nnz / TYPED_CHUNK) >= the item count, the entries past
    the last item = R (padding the kernels skip))."""
    R = rowptr.numel() - 1
    if rowptr.is_cuda:  # three launches in the library (nit, rocPRIM scan, search)
        bound = R + -(-nnz // TYPED_CHUNK)
        item_ptr = torch.empty(R + 1, dtype=torch.int64, device=rowptr.device)
        item_row = torch.empty(max(bound, 1), dtype=torch.int32, device=rowptr.device)[:bound]
        nb = LIB.dglhip_typed_items_workspace_bytes(R)
        if nb < 0:
            check_call(-1)
        ws = torch.empty(max(int(nb), 1), dtype=torch.uint8, device=rowptr.device)
        check_call(LIB.dglhip_typed_items_device(R, ptr(rowptr), bound,
                                                 ptr(item_ptr), ptr(item_row), ptr(ws), int(nb),
                                                 _stream_of(rowptr.device)))
        return item_ptr, item_row
    deg = rowptr[1:] - rowptr[:-1]
    nit = torch.clamp((deg + (TYPED_CHUNK - 1)) // TYPED_CHUNK, min=1)
    item_ptr = torch.zeros(R + 1, dtype=torch.int64, device=rowptr.device)
    torch.cumsum(nit, 0, out=item_ptr[1:])
    bound = R + -(-nnz // TYPED_CHUNK)
    item_row = torch.searchsorted(item_ptr[1:], torch.arange(bound, device=rowptr.device),
                                  right=True).to(torch.int32)
    return item_ptr, item_row


def _run_typed_block(csr, ufeat2, weight, slot_rel, slot_norm, nb, si, so):
    dev = ufeat2.device
    out = torch.empty(csr.num_rows, nb * so, dtype=torch.float32, device=dev)
    if dev.type == "cuda":
        items = csr._plans.get("typed_items")
        if items is None:
            items = csr._plans["typed_items"] = _typed_items(csr.indptr, csr.nnz)
        item_ptr, item_row = items
        part = torch.empty(item_row.numel(), nb * so, dtype=torch.float32, device=dev)
        check_call(LIB.dglhip_typed_block_spmm_device(
            csr.num_rows, item_row.numel(), nb, si, so, ptr(csr.indptr), ptr(item_ptr),
            ptr(item_row), csr.num_rows, None, ptr(csr.indices), ptr(slot_rel),
            ptr(slot_norm), ptr(ufeat2), ptr(weight), ptr(out), ptr(part), _stream_of(dev)))
    else:
        check_call(LIB.dglhip_typed_block_spmm_host(
            csr.num_rows, nb, si, so, ptr(csr.indptr), ptr(csr.indices), ptr(slot_rel),
            ptr(slot_norm), ptr(ufeat2), ptr(weight), ptr(out), 0))
    return out


def set_typed_block_messages(on):
    """The typed-block g-SpMM as relation-major messages + a slot-order sum,
    and its weight gradient with LDS-staged rows (csrc/typed_block.hip, r06),
    instead of the one-kernel forms; the same bits."""
    check_call(LIB.dglhip_set_typed_block_messages(1 if on else 0))


def _typed_msg_ok(nb, si, so):
    return LIB.dglhip_typed_block_msg_ok(nb, si, so) == 1


def _relation_groups(adj, etype, num_rels):
    g = getattr(adj, "_rel_groups", None)
    if g is None or not g.matches(etype):
        g = adj._rel_groups = _RelationGroups(adj.fwd, etype, num_rels)
    return g


def _run_typed_msg(csr, slot_map, groups, pos_row, ufeat2, weight, slot_norm, nb, si, so,
                   operand_scale=None, out_scale=None, weight_transposed=False):
    """out = the typed-block g-SpMM over ``csr`` in two launches: every edge's
    message (blockdiag(weight[r]) applied to ufeat2[pos_row], that row scaled
    by ``operand_scale[pos_row]`` when given) stored at its forward slot,
    walked relation-major; then each row's sum over its slots, reading message
    ``slot_map[k]`` (None: k) for slot k, times ``out_scale[row]``."""
    dev = ufeat2.device
    Fo = nb * so
    R = groups.ptr.numel() - 1
    msg = torch.empty(max(csr.nnz, 1), Fo, dtype=torch.float32, device=dev)
    g_ptr, g_rel = groups.items
    stream = _stream_of(dev)
    check_call(LIB.dglhip_typed_block_msg_device(
        R, g_rel.numel(), nb, si, so, ptr(groups.ptr), ptr(g_ptr), ptr(g_rel), ptr(pos_row),
        ptr(groups.slot), ptr(ufeat2), ptr(operand_scale), ptr(weight),
        1 if weight_transposed else 0, ptr(msg), stream))
    items = csr._plans.get("typed_items")
    if items is None:
        items = csr._plans["typed_items"] = _typed_items(csr.indptr, csr.nnz)
    item_ptr, item_row = items
    out = torch.empty(csr.num_rows, Fo, dtype=torch.float32, device=dev)
    part = torch.empty(item_row.numel(), Fo, dtype=torch.float32, device=dev)
    check_call(LIB.dglhip_typed_msg_sum_device(
        csr.num_rows, item_row.numel(), Fo, ptr(csr.indptr), ptr(item_ptr), ptr(item_row),
        csr.num_rows, None, ptr(slot_map), ptr(slot_norm), ptr(msg), ptr(out_scale), ptr(out),
        ptr(part), stream))
    return out


def _slot_values(csr, etype, enorm):
    """The per-edge relation (int32) and norm in ``csr``'s slot order."""
    rel = etype.index_select(0, csr.eid).to(torch.int32)
    nrm = None if enorm is None else enorm.index_select(0, csr.eid)
    return rel, nrm


class _RelationGroups(object):
    """Relation-major grouping of an adjacency's edges for the weight
    gradient: ptr[R+1], the source and destination of each edge (forward
    slot order within a relation), ``slot`` the forward slot each came from,
    and the chunked items (_typed_items)."""

    def __init__(self, fwd, etype, num_rels):
        # relations are checked where they were given (typed_block_spmm: host
        # ids always, device ids on request), not with a sync here; the
        # grouping never stores outside its arrays for any value
        if fwd.device.type == "cuda":
            self._build_device(fwd, etype, num_rels)
        else:
            rel_of_slot = etype.index_select(0, fwd.eid)
            rel = build_csr(num_rels, max(fwd.num_cols, 1), rel_of_slot, fwd.indices.long(),
                            ORDER_EID, fwd.device, schedule=False, validate=False)
            self.ptr = rel.indptr
            self.src = rel.indices
            self.slot = rel.eid  # forward slot of each relation-major position
            self.dst = fwd.row_ids().index_select(0, self.slot).to(torch.int32)
            self.items = None
        self.etype = etype  # the relations it was built for (held: see matches)
        self.version = etype._version

    def _build_device(self, fwd, etype, num_rels):
        """The same arrays in one library call (dglhip_relation_groups_device:
        ≈100 µs of host time as a CSR build, gathers, repeat_interleave and
        the item list, r06)."""
        dev, nnz, R = fwd.device, fwd.nnz, max(int(num_rels), 1)
        bound = R + -(-nnz // TYPED_CHUNK)
        nb = LIB.dglhip_relation_groups_workspace_bytes(R, nnz)
        if nb < 0:
            check_call(-1)
        self.ptr = torch.empty(R + 1, dtype=torch.int64, device=dev)
        self.src = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)[:nnz]
        self.slot = torch.empty(max(nnz, 1), dtype=torch.int64, device=dev)[:nnz]
        self.dst = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)[:nnz]
        item_ptr = torch.empty(R + 1, dtype=torch.int64, device=dev)
        item_rel = torch.empty(bound, dtype=torch.int32, device=dev)
        ws = torch.empty(max(int(nb), 1), dtype=torch.uint8, device=dev)
        check_call(LIB.dglhip_relation_groups_device(
            R, fwd.num_rows, nnz, ptr(etype), ptr(fwd.indptr), ptr(fwd.indices), ptr(fwd.eid),
            bound, ptr(self.ptr), ptr(self.src), ptr(self.slot), ptr(self.dst), ptr(item_ptr),
            ptr(item_rel), ptr(ws), int(nb), _stream_of(dev)))
        self.items = (item_ptr, item_rel)

    def matches(self, etype):
        # typed_block_spmm hands a new 1-D view of the relations at every call
        # (r04 ADVICE: compared by object, the cache never hit). The held
        # tensor keeps its memory from being reused, so the same address and
        # length is the same memory, and views share one version counter
        return (self.etype.device == etype.device and self.etype.numel() == etype.numel() and
                self.etype.data_ptr() == etype.data_ptr() and self.version == etype._version)


def _typed_scale_fused(dev, nb, si, so):
    """A destination row scale rides in the message path's kernels (forward
    sum, dH messages, staged dW) for these widths on a device."""
    return (dev.type == "cuda" and _typed_msg_ok(nb, si, so) and _typed_msg_ok(nb, so, si) and
            nb * si * so <= 4096)


class _TypedBlock(torch.autograd.Function):
    @staticmethod
    def forward(ctx, adj, etype, num_rels, ufeat2, weight, enorm, row_scale=None):
        R, nb, si, so = weight.shape
        if ufeat2.is_cuda and _typed_msg_ok(nb, si, so):
            g = _relation_groups(adj, etype, R)
            nrm = None if enorm is None else enorm.index_select(0, adj.fwd.eid)
            out = _run_typed_msg(adj.fwd, None, g, g.src, ufeat2, weight, nrm, nb, si, so,
                                 out_scale=row_scale)
        else:
            assert row_scale is None  # typed_block_spmm scales outside otherwise
            rel, nrm = _slot_values(adj.fwd, etype, enorm)
            out = _run_typed_block(adj.fwd, ufeat2, weight, rel, nrm, nb, si, so)
        ctx.adj, ctx.num_rels = adj, num_rels
        ctx.save_for_backward(etype, ufeat2, weight, enorm, row_scale)
        return out

    @staticmethod
    def backward(ctx, dout):
        etype, ufeat2, weight, enorm, row_scale = ctx.saved_tensors
        adj = ctx.adj
        R, nb, si, so = weight.shape
        dout = dout.contiguous()
        du = dw = None
        if ctx.needs_input_grad[3]:
            if dout.is_cuda and _typed_msg_ok(nb, so, si):
                # messages Wt[r] dout[dst] at the forward slots, read along the
                # transpose (the weight read transposed in the kernel)
                g = _relation_groups(adj, etype, R)
                nrm = None if enorm is None else enorm.index_select(0, adj.bwd.eid)
                du = _run_typed_msg(adj.bwd, _fwd_slot_of_bwd(adj), g, g.dst, dout, weight, nrm,
                                    nb, so, si, operand_scale=row_scale, weight_transposed=True)
            else:
                wt = weight.transpose(2, 3).contiguous()  # (R, nb, so, si)
                rel, nrm = _slot_values(adj.bwd, etype, enorm)
                du = _run_typed_block(adj.bwd, dout, wt, rel, nrm, nb, so, si)
        if ctx.needs_input_grad[4]:
            g = _relation_groups(adj, etype, R)
            fwd_nrm = None if enorm is None else enorm.index_select(0, adj.fwd.eid)
            nrm = None if fwd_nrm is None else fwd_nrm.index_select(0, g.slot)
            dw = torch.empty_like(weight)
            if dout.is_cuda:
                item_ptr, item_rel = g.items
                part = torch.empty(item_rel.numel(), nb * si * so, dtype=torch.float32,
                                   device=dout.device)
                check_call(LIB.dglhip_typed_block_wgrad_scaled_device(
                    R, item_rel.numel(), nb, si, so, ptr(g.ptr), ptr(item_ptr), ptr(item_rel),
                    R, None, ptr(g.src), ptr(g.dst), ptr(nrm), ptr(ufeat2), ptr(dout),
                    ptr(row_scale), ptr(dw), ptr(part), _stream_of(dout.device)))
            else:
                check_call(LIB.dglhip_typed_block_wgrad_host(
                    R, nb, si, so, ptr(g.ptr), ptr(g.src), ptr(g.dst), ptr(nrm), ptr(ufeat2),
                    ptr(dout), ptr(dw), 0))
        return None, None, None, du, dw, None, None


def typed_block_spmm(adj, ufeat, weight, etype, enorm=None, row_scale=None):
    """R-GCN block-diagonal message passing in one kernel:
    out[v] = sum_{e=(u->v)} enorm[e] * blockdiag(weight[etype[e]]) applied to ufeat[u].

    adj    : SparseAdj (rows = destinations) on the features' device
    ufeat  : (num_src, nb * si) float32
    weight : (num_rels, nb, si, so) float32 (autograd)
    etype  : (num_edges,) int64 relation of each edge id
    enorm  : optional (num_edges,) float32 per-edge scale (not differentiated)
    row_scale : optional (num_rows,) float32 scale of each output row (not
             differentiated): the value of ``out * row_scale.unsqueeze(1)`` —
             the R-GCN layer's 1 / in-degree, rounded as that product is —
             applied inside the kernels when the message path runs (no
             elementwise pass either way, r06), else by that product
    """
    dev = ufeat.device
    adj = adj.to(dev)
    R, nb, si, so = weight.shape
    if ufeat.shape[1] != nb * si:
        raise DGLError("ufeat width %d != num_blocks * in_block %d" % (ufeat.shape[1], nb * si))
    etype = torch.as_tensor(etype)
    if etype.numel() and (etype.device.type == "cpu" or (
            _VALIDATE_INDICES and not (dev.type == "cuda" and
                                       torch.cuda.is_current_stream_capturing()))):
        lo, hi = torch.stack([etype.min(), etype.max()]).tolist()
        if lo < 0 or hi >= R:
            raise IndexError("typed_block_spmm: relations span [%d, %d], out of range for %d "
                             "relation weights" % (lo, hi, R))
    etype = etype.to(device=dev, dtype=torch.int64).contiguous().reshape(-1)
    en = None if enorm is None else _f32c(enorm.to(dev).reshape(-1).detach())
    # one relation (and norm) per edge id: the kernels gather them by edge id
    E = adj.fwd.nnz
    if etype.numel() != E or (en is not None and en.numel() != E):
        raise DGLError("typed_block_spmm: %d edges but etype has %d and enorm %s entries"
                       % (E, etype.numel(), "no" if en is None else en.numel()))
    if row_scale is None:
        return _TypedBlock.apply(adj, etype, R, _f32c(ufeat), _f32c(weight), en)
    rs = _f32c(torch.as_tensor(row_scale).to(dev).reshape(-1).detach())
    if rs.numel() != adj.fwd.num_rows:
        raise DGLError("typed_block_spmm: row_scale has %d entries for %d rows"
                       % (rs.numel(), adj.fwd.num_rows))
    if _typed_scale_fused(dev, nb, si, so):
        return _TypedBlock.apply(adj, etype, R, _f32c(ufeat), _f32c(weight), en, rs)
    return _TypedBlock.apply(adj, etype, R, _f32c(ufeat), _f32c(weight), en) * rs.unsqueeze(1)


# ---------------------------------------------------------------------------
# GAT edge attention (fused u_add_v g-SDDMM + leaky_relu + exp + clamp)
# ---------------------------------------------------------------------------
class _EdgeAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, adj, num_edges, alpha, lo, hi, apply_exp, a_src, a_dst, slot=False):
        # lhs is gathered by column, rhs read per row: over the transpose the
        # roles swap (a_dst[v] + a_src[u] == a_src[u] + a_dst[v] exactly).
        # slot: the forward CSR, out[k] per slot (no eid, sequential stores)
        csr, tr = (adj.fwd, False) if slot else _eid_major(adj)
        H = a_src.shape[1]
        lhs, rhs = (a_dst, a_src) if tr else (a_src, a_dst)
        out = torch.empty(num_edges, H, dtype=torch.float32, device=a_src.device)
        args = (csr.num_rows, H, ptr(csr.indptr), ptr(csr.indices),
                ptr(None if slot else csr.eid), ptr(lhs), ptr(rhs), float(alpha), float(lo),
                float(hi), 1 if apply_exp else 0, ptr(out))
        if a_src.is_cuda:
            check_call(LIB.dglhip_gsddmm_attention_device(*(args + (_stream_of(a_src.device),))))
        else:
            check_call(LIB.dglhip_gsddmm_attention_host(*(args + (0,))))
        ctx.adj, ctx.alpha, ctx.lo, ctx.hi, ctx.apply_exp = adj, alpha, lo, hi, apply_exp
        ctx.slot, ctx.tr = slot, tr
        ctx.save_for_backward(out, a_src, a_dst)
        return out

    @staticmethod
    def backward(ctx, dout):
        out, a_src, a_dst = ctx.saved_tensors
        adj = ctx.adj
        # d/dx clamp(exp(lrelu(x))): out * lrelu'(x) where not clamped, the
        # slope alpha where the logit x <= 0 (x == 0 included), as torch's
        # leaky_relu backward: from x itself, recomputed in out's order
        # (out <= 1 would differ for 0 < x < 2^-24, where exp(x) rounds to 1)
        x = _edge_logits(adj, a_src, a_dst, ctx.slot, ctx.tr, out.shape[0])
        inside = (out > ctx.lo) & (out < ctx.hi)
        slope = torch.where(x <= 0, torch.full_like(out, ctx.alpha), torch.ones_like(out))
        g = dout * out * slope if ctx.apply_exp else dout * slope
        g = torch.where(inside, g, torch.zeros_like(g)).contiguous()
        # sum the per-edge gradient at the source (transposed CSR) and destination
        H = g.shape[1]
        d_src, _ = _run_gspmm(adj.bwd, MSG_COPY_E, RED_SUM, None, g, H, H, False,
                              emap=_fwd_slot_of_bwd(adj) if ctx.slot else None)
        d_dst, _ = _run_gspmm(adj.fwd, MSG_COPY_E, RED_SUM, None, g, H, H, False,
                              emap=SLOT if ctx.slot else None)
        return None, None, None, None, None, None, d_src, d_dst, None


def _edge_logits(adj, a_src, a_dst, slot, tr, num_edges):
    """x = a_src[u] + a_dst[v] per edge u -> v (the attention kernels' sum,
    float32): by forward slot, or by edge id through the CSR the forward ran
    over (tr: the transpose, whose rows are the sources)."""
    if slot:
        fwd = adj.fwd
        return a_src.index_select(0, fwd.indices.long()) + \
            a_dst.index_select(0, fwd.row_ids())
    csr, _ = _eid_major(adj)
    rows, cols = csr.row_ids(), csr.indices.long()
    u, v = (rows, cols) if tr else (cols, rows)
    x = torch.empty(num_edges, a_src.shape[1], dtype=torch.float32, device=a_src.device)
    x[csr.eid.long()] = a_src.index_select(0, u) + a_dst.index_select(0, v)
    return x


def edge_attention(adj, a_src, a_dst, num_edges, alpha=0.2, clamp=(-10.0, 10.0),
                   apply_exp=True, edge_order="eid"):
    """Per-edge, per-head GAT attention in one kernel:
    clamp(exp(leaky_relu(a_src[u] + a_dst[v], alpha))) for every edge u -> v,
    returned as (num_edges, H) indexed by edge id (edge_order="slot": by
    forward CSR slot, for gspmm(..., edge_order="slot")). Differentiable in
    a_src/a_dst."""
    slot = edge_order_of(adj, edge_order)
    dev = a_src.device
    adj = adj.to(dev)
    H = a_src.reshape(a_src.shape[0], -1).shape[1]
    return _EdgeAttention.apply(adj, int(num_edges), float(alpha), float(clamp[0]),
                                float(clamp[1]), bool(apply_exp),
                                _f32c(a_src.reshape(-1, H)), _f32c(a_dst.reshape(-1, H)), slot)


# ---------------------------------------------------------------------------
# Fused GAT aggregation: attention + dropout + normaliser + head-broadcast sum
# ---------------------------------------------------------------------------
_GAT_SEED = {}
# the GAT backward: "auto" (the one-pass transposed kernel where it applies,
# 8 heads x 16) or "three" (r03's three passes, the attention stored)
_GAT_BWD = os.environ.get("DGLHIP_GAT_BWD", "auto")


# the one-pass backward reads er and dz packed into one [rows, 2H] table
# (dglhip_gat_backward_t_packed_device); False: two tables (study knob)
_GAT_BWD_PACK = os.environ.get("DGLHIP_GAT_BWD_PACK", "on") != "off"


def set_gat_bwd_pack(on):
    """Study knob: er and dz packed into one table for the one-pass GAT
    backward (default on); returns the old setting. Same bits."""
    global _GAT_BWD_PACK
    old = _GAT_BWD_PACK
    _GAT_BWD_PACK = bool(on)
    return old


def set_gat_backward(policy):
    """Study / test knob for the fused GAT layer's backward: "auto" or
    "three"; returns the old policy. Same bits either way."""
    global _GAT_BWD
    old = _GAT_BWD
    _GAT_BWD = str(policy)
    return old


def _gat_seed_counter(dev):
    """The per-device int64 counter of captured calls. Made at the first call
    on the device outside a capture (the warm-up a capture needs anyway), so
    its zero fill is not part of any graph; made first inside a capture its
    start value is arbitrary (torch.empty: a captured fill would reset it at
    every replay)."""
    key = str(dev)
    if key not in _GAT_SEED:
        if torch.cuda.is_current_stream_capturing():
            _GAT_SEED[key] = torch.empty(1, dtype=torch.int64, device=dev)
        else:
            _GAT_SEED[key] = torch.zeros(1, dtype=torch.int64, device=dev)
    return _GAT_SEED[key]


def _gat_seed_offset(dev):
    """For a call captured in a HIP graph: a base seed from torch's generator
    (drawn at capture) and the device counter the fused kernel adds to it,
    advanced on the device at every replay: every replay draws a new mask
    with no host round trip."""
    off = _gat_seed_counter(dev)
    off.add_(1)
    return int(torch.randint(0, 1 << 62, (1,)).item()), off


def set_gat_variant(variant):
    """Study knob for the fused GAT kernel: 0 automatic (default), 1 the
    attention computed in every lane that consumes it, 2 once per (slot,
    head) through LDS (1/2/4/8/16 heads) with each batch's feature rows
    gathered after its attention, 3 the LDS kernel with them gathered before
    it (what 0 picks on two-float lanes). Same bits."""
    check_call(LIB.dglhip_set_gat_variant(int(variant)))


def gat_dropout_scale(p):
    """The kept attention's scale 1 / (1 - p) as the fused kernel computes it
    (float32 operands), so host compositions match its bits."""
    one = np.float32(1.0)
    return float(one / (one - np.float32(p)))


def gat_dropout_mask(num_slots, num_heads, p, seed):
    """bool (num_slots, num_heads): the (slot, head) pairs the fused kernel
    keeps at dropout probability ``p`` under seed ``seed`` (its counter hash,
    computed on the host)."""
    keep = torch.empty(num_slots, num_heads, dtype=torch.uint8)
    check_call(LIB.dglhip_gat_dropout_mask_host(num_slots, num_heads, float(p), int(seed),
                                                ptr(keep)))
    return keep.bool()


def _attention_slots(fwd, el, er, alpha, lo, hi, apply_exp):
    out = torch.empty(fwd.nnz, el.shape[1], dtype=torch.float32, device=el.device)
    args = (fwd.num_rows, el.shape[1], ptr(fwd.indptr), ptr(fwd.indices), None, ptr(el),
            ptr(er), float(alpha), float(lo), float(hi), 1 if apply_exp else 0, ptr(out))
    if el.is_cuda:
        check_call(LIB.dglhip_gsddmm_attention_device(*(args + (_stream_of(el.device),))))
    else:
        check_call(LIB.dglhip_gsddmm_attention_host(*(args + (0,))))
    return out


class _GATAggregate(torch.autograd.Function):
    """(ft_sum, z) = (sum_k w[k,h] ft[u_k, h, :], sum_k a[k,h]) per destination
    row and head, a = clamp(exp(leaky_relu(el[u] + er[v]))), w = dropout(a),
    all in one kernel on the device (dglhip_gat_aggregate_device); a and w are
    kept in CSR slot order only when a gradient is needed. The backward is the
    three-kernel path's (the u_mul_e product over the transpose, the g-SDDMM
    dot, the copy_e gather, the attention's backward): same bits."""

    @staticmethod
    def forward(ctx, adj, alpha, lo, hi, apply_exp, p, seed, seed_off, el, er, ft2, D, grad_mode,
                attn_l=None):
        fwd = adj.fwd
        H = el.shape[1]
        F = ft2.shape[1]
        dev = ft2.device
        # needs_input_grad follows requires_grad even under torch.no_grad():
        # the caller's grad mode decides whether a backward can follow
        need = grad_mode and any(ctx.needs_input_grad[8:11])
        a = w = None
        # the one-pass backward over the transpose recomputes the attention:
        # nothing per edge is stored (8 heads x 16, _gat_backward_t)
        ctx.use_t = (need and dev.type == "cuda" and _GAT_BWD == "auto" and
                     LIB.dglhip_gat_backward_t_ok(H, D) == 1 and ft2.data_ptr() % 8 == 0)
        if dev.type == "cuda":
            out_ft = torch.empty(fwd.num_rows, F, dtype=torch.float32, device=dev)
            out_z = torch.empty(fwd.num_rows, H, dtype=torch.float32, device=dev)
            if need and not ctx.use_t:
                a = torch.empty(fwd.nnz, H, dtype=torch.float32, device=dev)
                w = torch.empty_like(a) if p > 0 else None
            # source-blocked (exact where the blocks never decrease along a
            # row): one launch per block, both chains continued; with nothing
            # stored, smaller blocks (_GAT_BLOCK_BYTES_NOGRAD)
            cuts = _block_cuts(fwd, (F + H) * 4,
                               None if a is not None else _GAT_BLOCK_BYTES_NOGRAD)
            if cuts is None:
                cuts = [fwd.indptr, fwd.indptr[1:]]
            # attn_l (el known to be gat_logits(ft, attn_l)): the 8 x 16
            # blocked kernel recomputes each source's logit from its row
            for b in range(len(cuts) - 1):
                check_call(LIB.dglhip_gat_aggregate_logits_ranges_device(
                    fwd.num_rows, ft2.shape[0], H, D, ptr(cuts[b]), ptr(cuts[b + 1]),
                    1 if b else 0, ptr(fwd.indices), ptr(fwd.row_order), ptr(el), ptr(er),
                    ptr(ft2), ptr(attn_l), float(alpha), float(lo), float(hi),
                    1 if apply_exp else 0, float(p), int(seed), ptr(seed_off), ptr(out_ft),
                    ptr(out_z), ptr(a), ptr(w), _stream_of(dev)))
        else:  # host: the same per-edge values and chains from the host kernels
            a = _attention_slots(fwd, el, er, alpha, lo, hi, apply_exp)
            w = None
            if p > 0:
                keep = gat_dropout_mask(fwd.nnz, H, p, seed)
                w = torch.where(keep, a * gat_dropout_scale(p), torch.zeros_like(a))
            out_ft, _ = _run_gspmm(fwd, MSG_U_MUL_E, RED_SUM, ft2, w if p > 0 else a, H, F,
                                   False, emap=SLOT)
            out_z, _ = _run_gspmm(fwd, MSG_COPY_E, RED_SUM, None, a, H, H, False, emap=SLOT)
            if not need:
                a = w = None
        ctx.adj, ctx.alpha, ctx.lo, ctx.hi, ctx.apply_exp, ctx.p = adj, alpha, lo, hi, \
            apply_exp, p
        # the dropout seed as this call used it (a captured call's device
        # counter moves on at the next call): the backward recomputes keep bits
        ctx.seed = int(seed)
        ctx.seed_off = None if (seed_off is None or p == 0 or not need) else seed_off.clone()
        if ctx.use_t:
            ctx.D = D
            ctx.save_for_backward(ft2, el, er)
        else:  # (el, er: the logits' sign gives the leaky_relu slope)
            ctx.save_for_backward(ft2, a, w, el, er)
        return out_ft, out_z

    @staticmethod
    def backward(ctx, d_ft, d_z):
        if ctx.use_t:
            return _gat_backward_t(ctx, d_ft, d_z) + (None,)
        ft2, a, w, el, er = ctx.saved_tensors
        adj = ctx.adj
        fwd = adj.fwd
        H = a.shape[1]
        F = ft2.shape[1]
        need_el, need_er, need_ft = ctx.needs_input_grad[8:11]
        d_el = d_er = d_ft2 = None
        d_ft = torch.zeros_like(ft2) if d_ft is None else d_ft.contiguous()
        wt = w if w is not None else a
        if need_ft:
            # (source-blocked where the transpose qualifies: _run_gspmm)
            d_ft2, _ = _run_gspmm(adj.bwd, MSG_U_MUL_E, RED_SUM, d_ft, wt, H, F, False,
                                  emap=_fwd_slot_of_bwd(adj))
        if need_el or need_er:
            scale = gat_dropout_scale(ctx.p) if w is not None else 1.0
            if ft2.is_cuda:
                # the dot, dropout, normaliser and activation gradients in one
                # pass (the g-SDDMM dot with the GAT epilogue): the torch ops
                # below, fused, same bits
                g = torch.empty_like(a)
                dz = None if d_z is None else d_z.contiguous()
                # every slot's value is its own: the source blocks' sub-ranges
                # (ft rows of one block at a time) give the same bits
                cuts = _block_cuts(fwd, F * 4) or [fwd.indptr, fwd.indptr[1:]]
                ft2c = ft2.contiguous()
                # er's gradient (the copy_edge sum of g over each row's slots)
                # summed in the same pass, in slot order across the blocks:
                # the same chain as the separate sum, one E x H read less
                fuse_er = (need_er and LIB.dglhip_gat_attention_grad_rowsum_ok(F, H) == 1 and
                           d_ft.data_ptr() % 16 == 0 and ft2c.data_ptr() % 16 == 0)
                er_sum = (torch.zeros(fwd.num_rows, H, dtype=torch.float32, device=ft2.device)
                          if fuse_er else None)
                # keep bits from the forward's hash (drop_p), not w != 0; the
                # slope from the logits el[u] + er[v]
                p_hash = float(ctx.p) if w is not None else 0.0
                for b in range(len(cuts) - 1):
                    check_call(LIB.dglhip_gat_attention_grad_logits_ranges_device(
                        fwd.num_rows, F, H, ptr(cuts[b]), ptr(cuts[b + 1]),
                        ptr(fwd.row_order), ptr(fwd.indices), ptr(d_ft), ptr(ft2c), ptr(a),
                        None, ptr(dz), ptr(el), ptr(er), float(ctx.alpha), float(ctx.lo),
                        float(ctx.hi), 1 if ctx.apply_exp else 0, 1.0, p_hash, ctx.seed,
                        ptr(ctx.seed_off), ptr(g), ptr(er_sum), _stream_of(ft2.device)))
                if fuse_er:
                    d_er = er_sum
            else:
                d_a = _run_sddmm_dot(fwd, d_ft, ft2.contiguous(), fwd.nnz, H, slot=True)
                if w is not None:  # dropout's backward: the kept pairs (the hash), scaled
                    keep = gat_dropout_mask(fwd.nnz, H, ctx.p, ctx.seed).to(d_a.device)
                    d_a = torch.where(keep, d_a * scale, torch.zeros_like(d_a))
                if d_z is not None:
                    d_a = d_a + d_z.contiguous().index_select(0, fwd.row_ids())
                # the attention's backward (_EdgeAttention.backward, slot order)
                x = _edge_logits(adj, el, er, True, False, fwd.nnz)
                inside = (a > ctx.lo) & (a < ctx.hi)
                slope = torch.where(x <= 0, torch.full_like(a, ctx.alpha), torch.ones_like(a))
                g = d_a * a * slope if ctx.apply_exp else d_a * slope
                g = torch.where(inside, g, torch.zeros_like(g)).contiguous()
            if need_el:
                d_el = _gat_el_grad(adj, g, H)
            if need_er and d_er is None:
                d_er, _ = _run_gspmm(fwd, MSG_COPY_E, RED_SUM, None, g, H, H, False, emap=SLOT)
        return (None,) * 8 + (d_el, d_er, d_ft2, None, None, None)


def _gat_backward_t(ctx, d_ft, d_z):
    """The GAT layer's backward as ONE pass over the transpose
    (dglhip_gat_backward_t_device): d_ft and d_el chained in the transpose's
    slot order — over its source-blocked plan when it has one, each block's
    launch continuing the chains — and the attention gradient g stored at its
    forward slot; d_er is the copy_e sum of g over the forward CSR. The
    attention and the dropout keep bits are recomputed from el, er and the
    seed, so the forward stored nothing per edge. Same bits as the r03
    three-pass backward (attention gradient over the CSR, d_ft and d_el over
    the transpose through the slot map)."""
    ft2, el, er = ctx.saved_tensors
    adj = ctx.adj
    fwd, bwd = adj.fwd, adj.bwd
    H, F, D = el.shape[1], ft2.shape[1], ctx.D
    need_el, need_er, need_ft = ctx.needs_input_grad[8:11]
    dev = ft2.device
    dout = (torch.zeros(fwd.num_rows, F, dtype=torch.float32, device=dev) if d_ft is None
            else _f32c(d_ft))
    dz = None if d_z is None else _f32c(d_z)
    emap = _fwd_slot_of_bwd(adj)
    d_ft2 = torch.empty(bwd.num_rows, F, dtype=torch.float32, device=dev)
    d_el = torch.empty(bwd.num_rows, H, dtype=torch.float32, device=dev)
    # the attention gradient at its forward slot, for d_er's sum (none when
    # er needs no gradient: the kernel then stores nothing)
    g = torch.empty(fwd.nnz, H, dtype=torch.float32, device=dev) if need_er else None
    common = (fwd.num_rows, ft2.shape[0], H, D)
    rest = (float(ctx.alpha), float(ctx.lo), float(ctx.hi), 1 if ctx.apply_exp else 0,
            float(ctx.p), ctx.seed, ptr(ctx.seed_off), ptr(d_ft2), ptr(d_el), ptr(g),
            _stream_of(dev))
    if dz is not None and _GAT_BWD_PACK:
        # er and dz side by side: a pair's two destination operands in one
        # 64-B run, one line per slot instead of two (same bits)
        erdz = torch.cat([er, dz], 1)
        tail = (ptr(ft2), ptr(el), ptr(erdz), ptr(dout)) + rest
        entry = LIB.dglhip_gat_backward_t_packed_device
    else:
        tail = (ptr(ft2), ptr(el), ptr(er), ptr(dz), ptr(dout)) + rest
        entry = LIB.dglhip_gat_backward_t_device
    plan = _block_plan(bwd, dout, F, _GAT_BWD_BLOCK_BYTES) if bwd.nnz else None
    if plan is None:
        check_call(entry(
            bwd.num_rows, ptr(bwd.row_order), ptr(bwd.indptr), ptr(bwd.indptr[1:]), 1, 0,
            *(common + (ptr(bwd.indices), ptr(emap)) + tail)))
    else:
        # the plan's launches over its global slot arrays: item offsets (ptr)
        # are global, so every launch takes the same column-id and map bases
        erows = _block_edge_rows(bwd, plan, emap)
        if plan.absent.numel():
            d_ft2.index_fill_(0, plan.absent.long(), 0.0)
            d_el.index_fill_(0, plan.absent.long(), 0.0)
        for i, it in enumerate(plan):
            check_call(entry(
                it.rows.numel(), ptr(it.rows), ptr(it.ptr), ptr(it.ptr[1:]), 0, 1 if i else 0,
                *(common + (ptr(plan.indices), ptr(erows)) + tail)))
    d_er = None
    if need_er:  # the copy_e sum of g over the CSR, one wave per row (same chain)
        d_er = torch.empty(fwd.num_rows, H, dtype=torch.float32, device=dev)
        check_call(LIB.dglhip_rowsum_heads8_device(fwd.num_rows, ptr(fwd.indptr),
                                                   ptr(fwd.row_order), ptr(g), ptr(d_er),
                                                   _stream_of(dev)))
    return ((None,) * 8 + (d_el if need_el else None, d_er, d_ft2 if need_ft else None, None,
                           None))


# el's gradient reads the E x H attention gradient (forward slot order)
# through the transpose's slot map: 32-B values at random forward slots, a
# 128-B line each. Cut by destination block, each launch's values come from
# one contiguous forward-slot range of about this many bytes, which the
# Infinity Cache holds (Reddit-shaped graph, 8 heads: one launch 3.72 ms;
# 32 / 128 / 256 / 512 MiB blocks 3.34 / 3.19 / 3.13 / 3.20 ms, the same
# bits; tools/el_grad_sweep.py)
_EL_GRAD_BLOCK_BYTES = int(os.environ.get("DGLHIP_EL_GRAD_BLOCK_BYTES", 256 << 20))


def _gat_el_grad(adj, g, H):
    """d_el[u, h] = sum of g[forward slot of k, h] over the transpose's slots k
    of source u, in slot order (the copy_edge sum of the attention gradient
    along the transpose). On a ROCm device with a graph numbered source-major
    it runs over destination blocks (row sub-ranges of the transpose, each
    continuing the rows' chains: the same bits); else in one launch."""
    bwd = adj.bwd
    emap = _fwd_slot_of_bwd(adj)
    cuts = None
    pol = schedule_policy()
    if g.is_cuda and pol["blocked"] and bwd.nnz and bwd.nnz < (1 << 31):
        B = -(-(g.numel() * g.element_size()) // _EL_GRAD_BLOCK_BYTES)
        B = min(B, bwd.nnz // (pol["block_min_slots"] * max(bwd.num_nonempty, 1)))
        if B >= 2:
            cuts = _cuts_native(bwd, 0, 0, B)
    if cuts is None:
        return _run_gspmm(bwd, MSG_COPY_E, RED_SUM, None, g, H, H, False, emap=emap)[0]
    out = torch.empty(bwd.num_rows, H, dtype=torch.float32, device=g.device)
    for b in range(len(cuts) - 1):
        gspmm_ranges(MSG_COPY_E, cuts[b], cuts[b + 1], b > 0, bwd.indices, out, efeat=g,
                     eid=emap)
    return out


def gat_aggregate(adj, ft, el, er, alpha=0.2, clamp=(-10.0, 10.0), attn_drop=0.0,
                  training=True, apply_exp=True, seed=None):
    """One GAT layer's aggregation in one kernel (examples/pytorch/gat/train.py:74-96):
    for every destination row v and head h, over v's in-edges u -> v in CSR
    slot order,

        a      = clamp(exp(leaky_relu(el[u, h] + er[v, h], alpha)), *clamp)
        ft_sum = sum a_drop * ft[u, h, :]    (a_drop = dropout(a), training only)
        z      = sum a

    returned as (ft_sum (R, H, D), z (R, H, 1)), differentiable in ft, el, er.
    ft (N, H, D); el (N, H[, 1]); er (R, H[, 1]). Equals edge_attention(...,
    edge_order="slot") followed by gspmm(u_mul_e, sum) and gspmm(copy_e, sum)
    bit for bit. The dropout mask is the kernel's counter hash of (seed,
    slot, head) (gat_dropout_mask), not torch's generator; ``seed`` None draws
    the seed from torch's generator at every call (inside a HIP graph capture:
    once per device, plus a device counter advanced at every replay)."""
    p = float(attn_drop) if training else 0.0
    if not 0.0 <= p < 1.0:
        raise DGLError("attention dropout must be in [0, 1), got %r" % (attn_drop,))
    dev = ft.device
    adj = adj.to(dev)
    N, H, D = ft.shape
    el2 = _f32c(el.reshape(el.shape[0], H))
    er2 = _f32c(er.reshape(er.shape[0], H))
    ft2 = _f32c(ft.reshape(N, H * D))
    if el2.shape[0] < adj.shape[1] or er2.shape[0] != adj.shape[0] or N < adj.shape[1]:
        raise DGLError("gat_aggregate: feature rows do not match the adjacency")
    seed_off = None
    if p > 0 and seed is None:
        if dev.type == "cuda" and torch.cuda.is_current_stream_capturing():
            seed, seed_off = _gat_seed_offset(dev)
        else:  # torch's generator, every call: torch.manual_seed repeats the masks
            if dev.type == "cuda":
                _gat_seed_counter(dev)  # ready for a later capture
            seed = int(torch.randint(0, 1 << 62, (1,)).item())
    ft_sum, z = _GATAggregate.apply(adj, float(alpha), float(clamp[0]), float(clamp[1]),
                                    bool(apply_exp), p, int(seed or 0), seed_off, el2, er2,
                                    ft2, D, torch.is_grad_enabled(), _logits_source(el, ft))
    return ft_sum.view(-1, H, D), z.view(-1, H, 1)


class _GATLogits(torch.autograd.Function):
    """(el, er) = ((ft * attn_l).sum(-1), (ft * attn_r).sum(-1)) per node and
    head in the library's fixed association (dglhip_gat_logits_*); backward
    in torch: d_ft = d_el * attn_l + d_er * attn_r, d_attn = sum_n d_e * ft."""

    @staticmethod
    def forward(ctx, ft, attn_l, attn_r):
        N, H, D = ft.shape
        el = torch.empty(N, H, dtype=torch.float32, device=ft.device)
        er = torch.empty_like(el)
        args = (N, H, D, ptr(ft), ptr(attn_l), ptr(attn_r), ptr(el), ptr(er))
        if ft.is_cuda:
            check_call(LIB.dglhip_gat_logits_device(*(args + (_stream_of(ft.device),))))
        else:
            check_call(LIB.dglhip_gat_logits_host(*(args + (0,))))
        ctx.save_for_backward(ft, attn_l, attn_r)
        return el, er

    @staticmethod
    def backward(ctx, d_el, d_er):
        ft, attn_l, attn_r = ctx.saved_tensors
        H, D = attn_l.shape
        d_el = torch.zeros(ft.shape[:2], device=ft.device) if d_el is None else d_el
        d_er = torch.zeros(ft.shape[:2], device=ft.device) if d_er is None else d_er
        d_ft = d_attn_l = d_attn_r = None
        if ctx.needs_input_grad[0]:
            d_ft = d_el.unsqueeze(-1) * attn_l + d_er.unsqueeze(-1) * attn_r
        if ctx.needs_input_grad[1]:
            d_attn_l = (d_el.unsqueeze(-1) * ft).sum(0)
        if ctx.needs_input_grad[2]:
            d_attn_r = (d_er.unsqueeze(-1) * ft).sum(0)
        return d_ft, d_attn_l, d_attn_r


def gat_logits(ft, attn_l, attn_r):
    """The GAT layer's attention logits (examples/pytorch/gat/train.py:66-67,
    ``bmm(head_ft, attn_l)``): el, er (N, H, 1) with el[n, h] = sum_d
    ft[n, h, d] * attn_l[h, d], in the library's association
    (dglhip_gat_logits_*). Differentiable in ft, attn_l and attn_r. When
    gat_aggregate is then given this el with the same ft, its 8-head x 16
    source-blocked forward recomputes each source's logit from the feature
    row it gathers anyway (same bits, a fifth fewer line requests)."""
    N, H, D = ft.shape
    ftc = _f32c(ft)
    al = _f32c(attn_l.reshape(H, D))
    ar = _f32c(attn_r.reshape(H, D))
    el, er = _GATLogits.apply(ftc, al, ar)
    el, er = el.view(N, H, 1), er.view(N, H, 1)
    # what the aggregation may recompute el from: this ft (data, shape,
    # version, and the tensor itself, held weakly: once it is freed its
    # address may come back as another tensor's) and attn_l's values at this
    # call; el's own version too (an in-place change of el voids the tag)
    el._dglhip_logits = (ftc.data_ptr(), tuple(ftc.shape), ftc._version, el._version,
                         al.detach().clone(), weakref.ref(ftc))
    return el, er


def _logits_source(el, ft):
    """attn_l when ``el`` came from gat_logits(ft, attn_l, ...) on this very ft
    (same data, shape and version) at 8 heads x 16 on a device, else None."""
    tag = getattr(el, "_dglhip_logits", None)
    if tag is None or not ft.is_cuda or tuple(ft.shape[1:]) != (8, 16):
        return None
    ptr_, shape, version, el_version, al, ref = tag
    if (ref() is None or ft.data_ptr() != ptr_ or tuple(ft.shape) != shape or
            ft._version != version or el._version != el_version):
        return None
    return al if al.device == ft.device else None
