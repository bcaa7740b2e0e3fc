// PackedFunc-style global function registry.
//
// The reference binds every native entry point by name through its
// TVM-derived runtime: DGL_REGISTER_GLOBAL (include/dgl/runtime/registry.h:
// 129-131) fills a global table (src/runtime/registry.cc:47), Python fetches a
// handle with DGLFuncGetGlobal (registry.cc:137) and calls it with
// DGLFuncCall(handle, values, type_codes, n, ret, ret_code)
// (src/runtime/c_runtime_api.cc:243-276), tensors travelling as DLTensor*
// (type code kArrayHandle) wrapped non-owning (src/c_api_common.cc:16-23).
// This file provides that calling convention for the engine's kernels so a
// ctypes binding written against libdgl can reach them unchanged; the typed
// C entry points in include/dgl_hip.h remain the fast path.
#include <cstdlib>
#include <initializer_list>
#include <memory>

#include "runtime.h"
#include "spmm_plan.h"

namespace dglhip {

using rt::Args;
using rt::RetValue;
using rt::check_compact;
using rt::data_as;
using rt::numel;
using rt::register_global;

namespace {

constexpr int kDeviceCPU = rt::kDLCPU;
constexpr int kDeviceROCM = rt::kDLROCM;

#define I64(t, w) data_as<int64_t>(t, 0, 64, w)
#define I32(t, w) data_as<int32_t>(t, 0, 32, w)
#define F32(t, w) data_as<float>(t, 2, 32, w)

void same_device(const DGLHipTensor* ref, std::initializer_list<const DGLHipTensor*> ts) {
  for (auto* t : ts) {
    if (!t) continue;
    DGLHIP_CHECK(t->device_type == ref->device_type && t->device_id == ref->device_id,
                 "tensors live on different devices");
  }
}

void throw_last(int rc) {
  if (rc != 0) throw Error(DGLGetLastError());
}

// NULL stream argument: the stream DGLSetStream made current on the device.
void* stream_or_current(void* s, const DGLHipTensor* t) {
  return s ? s : rt::current_stream(t->device_id);
}

}  // namespace

void register_kernel_functions() {
  // (msg, reduce, indptr, indices, eid|null, ufeat|null, efeat|null, out,
  //  arg_out|null, row_order|null, stream)
  // (msg, reduce, indptr, indices, eid|null, ufeat|null, efeat|null, out,
  //  arg_out|null, row_order|null, stream[, plan|null[, edge_layout]]):
  // the product on the plan's schedule when a plan made by
  // dglhip._CAPI_SpmmPlanCreate for this CSR is passed (a caller that runs
  // the product repeatedly keeps one, as the reference keeps its adjacency
  // per context, graph_index.py:537-585); without one, a single launch over
  // the CSR (no schedule build, no host sync; capturable). eid: the CSR's edge ids
  // (edge_layout BY_EID, the default; NULL = identity) or a per-slot map of
  // efeat rows (BY_MAP); efeat rows by slot with BY_SLOT.
  register_global("dglhip._CAPI_GSpMM", [](const Args& a, RetValue*) {
    const int msg = static_cast<int>(a.i64(0)), red = static_cast<int>(a.i64(1));
    auto* indptr = a.tensor(2);
    auto* indices = a.tensor(3);
    auto* eid = a.tensor(4, true);
    auto* uf = a.tensor(5, true);
    auto* ef = a.tensor(6, true);
    auto* out = a.tensor(7);
    auto* arg = a.tensor(8, true);
    auto* order = a.tensor(9, true);
    void* stream = a.handle(10);
    void* plan_h = a.size() > 11 ? a.handle(11) : nullptr;
    const int emode = a.size() > 12 ? static_cast<int>(a.i64(12)) : DGLHIP_EDGE_BY_EID;
    same_device(out, {indptr, indices, eid, uf, ef, arg, order});
    DGLHIP_CHECK(out->ndim == 2, "out must be 2-D [rows, feat]");
    const int64_t rows = out->shape[0], F = out->shape[1];
    DGLHIP_CHECK(numel(indptr) == rows + 1, "indptr length must be rows+1");
    int64_t elen = 0;
    if (ef) elen = ef->ndim == 1 ? 1 : numel(ef) / ef->shape[0];
    const bool dev = out->device_type == kDeviceROCM;
    DGLHIP_CHECK(dev || out->device_type == kDeviceCPU, "unsupported device type "
                                                           << out->device_type);
    int64_t ldu = 0, urows = 0;
    const void* ufp = nullptr;
    if (uf) {
      DGLHIP_CHECK(uf->ndim == 2 || uf->ndim == 1, "ufeat must be [rows, feat]");
      urows = uf->shape[0];
      const bool bf16 = msg == DGLHIP_MSG_COPY_U_BF16;
      DGLHIP_CHECK(uf->dtype_code == (bf16 ? 4 : 2) && uf->dtype_bits == (bf16 ? 16 : 32) ||
                       (bf16 && uf->dtype_code == 0 && uf->dtype_bits == 16) ||
                       (bf16 && uf->dtype_code == 1 && uf->dtype_bits == 16),
                   "ufeat dtype: float32 (bf16 bits for the bf16 message)");
      // rows at a padded stride (F columns of a wider row) or dense
      if (uf->ndim == 2 && uf->strides && uf->shape[0] > 1 && uf->strides[1] == 1 &&
          uf->strides[0] != uf->shape[1]) {
        ldu = uf->strides[0];
        DGLHIP_CHECK(uf->shape[1] == F, "strided ufeat must have feat_len columns");
      } else {
        check_compact(uf, "ufeat");
      }
      ufp = static_cast<const char*>(uf->data) + uf->byte_offset;
    }
    const int64_t nnz = numel(indices);
    std::unique_ptr<SpmmPlan> own;
    SpmmPlan* plan = static_cast<SpmmPlan*>(plan_h);
    hipStream_t s = static_cast<hipStream_t>(dev ? stream_or_current(stream, out) : nullptr);
    // No plan: the product is one launch (dglhip_gspmm_device / _strided /
    // _host), with no host sync, no allocation and no schedule build, so a
    // plan-less call costs what it did before plans existed and can be
    // captured into a HIP graph. Only a strided operand on the host, or a
    // row_order listing a subset of the rows, still takes a plan made for
    // the call.
    const bool full_order = !order || numel(order) == rows;
    if (!plan && full_order && (dev || ldu == 0)) {
      DGLHIP_CHECK(emode >= DGLHIP_EDGE_BY_SLOT && emode <= DGLHIP_EDGE_BY_MAP,
                   "unknown edge layout " << emode);
      const int64_t* erow = emode == DGLHIP_EDGE_BY_SLOT ? nullptr : I64(eid, "eid");
      DGLHIP_CHECK(!ef || erow || emode == DGLHIP_EDGE_BY_SLOT,
                   "edge layout " << emode << " needs eid");
      const float* u = static_cast<const float*>(ufp);
      int rc;
      if (!dev) {
        rc = dglhip_gspmm_host(msg, red, rows, F, I64(indptr, "indptr"), I32(indices, "indices"),
                               erow, u, F32(ef, "efeat"), elen, F32(out, "out"),
                               I64(arg, "arg_out"), 0);
      } else if (ldu != 0 && ldu != F) {
        DGLHIP_CHECK(!arg, "a strided operand takes no arg_out (sum / mean reducers)");
        rc = dglhip_gspmm_strided_device(msg, red, rows, F, ldu, I64(indptr, "indptr"),
                                         I32(indices, "indices"), erow, u, F32(ef, "efeat"),
                                         elen, F32(out, "out"), I32(order, "row_order"), s);
      } else {
        rc = dglhip_gspmm_device(msg, red, rows, F, I64(indptr, "indptr"),
                                 I32(indices, "indices"), erow, u, F32(ef, "efeat"), elen,
                                 F32(out, "out"), I64(arg, "arg_out"), I32(order, "row_order"),
                                 s);
      }
      throw_last(rc);
      return;
    }
    if (plan) {
      DGLHIP_CHECK(plan->on_device() == dev && (!dev || plan->device_id() == out->device_id),
                   "the plan lives on another device");
      DGLHIP_CHECK(plan->num_rows() == rows && plan->nnz() == nnz &&
                       plan->indptr() == I64(indptr, "indptr") &&
                       plan->indices() == I32(indices, "indices"),
                   "the plan was built for another CSR");
    } else {
      own.reset(new SpmmPlan(out->device_type, out->device_id, rows,
                             urows ? urows : rows, nnz, I64(indptr, "indptr"),
                             I32(indices, "indices"), nullptr, I32(order, "row_order"), s));
      plan = own.get();
    }
    PlanDevice guard(*plan);
    const int64_t* erow = I64(eid, "eid");
    const int64_t bytes = spmm_plan_workspace(*plan, msg, red, F, ldu, urows, elen, emode,
                                              erow, s);
    void* ws = nullptr;
    if (bytes > 0) {
      if (dev) DGLHIP_CHECK(hipMallocAsync(&ws, bytes, s) == hipSuccess, "workspace allocation");
      else ws = std::malloc(bytes);
    }
    try {
      spmm_plan_run(*plan, msg, red, F, ufp, ldu, urows, F32(ef, "efeat"), elen, emode, erow,
                    F32(out, "out"), I64(arg, "arg_out"), ws, bytes, s);
    } catch (...) {
      if (ws) { if (dev) (void)hipFreeAsync(ws, s); else std::free(ws); }
      throw;
    }
    if (ws) {
      if (dev) DGLHIP_CHECK(hipFreeAsync(ws, s) == hipSuccess, "workspace release");
      else std::free(ws);
    }
    // a plan made for this call owns arrays the enqueued launches read
    if (own && dev) DGLHIP_CHECK(hipStreamSynchronize(s) == hipSuccess, "stream synchronize");
  });
  // (indptr, indices, num_cols, row_order|null, stream) -> plan handle
  register_global("dglhip._CAPI_SpmmPlanCreate", [](const Args& a, RetValue* rv) {
    auto* indptr = a.tensor(0);
    auto* indices = a.tensor(1);
    const int64_t cols = a.i64(2);
    auto* order = a.tensor(3, true);
    void* stream = a.handle(4);
    same_device(indptr, {indices, order});
    const bool dev = indptr->device_type == kDeviceROCM;
    DGLHipSpmmPlan h = nullptr;
    throw_last(dglhip_spmm_plan_create(
        indptr->device_type, indptr->device_id, numel(indptr) - 1, cols, numel(indices),
        I64(indptr, "indptr"), I32(indices, "indices"), nullptr, I32(order, "row_order"),
        dev ? stream_or_current(stream, indptr) : nullptr, &h));
    rv->set_handle(h);
  });
  register_global("dglhip._CAPI_SpmmPlanFree", [](const Args& a, RetValue*) {
    throw_last(dglhip_spmm_plan_free(static_cast<DGLHipSpmmPlan>(a.handle(0))));
  });
  // (plan, msg, reduce, feat_len, ufeat_ld, num_src_rows, efeat_len,
  //  edge_layout, stream) -> path * 2^32 + launches
  register_global("dglhip._CAPI_SpmmPlanSchedule", [](const Args& a, RetValue* rv) {
    SpmmPlan* plan = static_cast<SpmmPlan*>(a.handle(0));
    DGLHIP_CHECK(plan, "null plan");
    PlanDevice guard(*plan);
    int64_t launches = 0;
    const int path = spmm_plan_path(*plan, static_cast<int>(a.i64(1)), static_cast<int>(a.i64(2)),
                                    a.i64(3), a.i64(4), a.i64(5), a.i64(6),
                                    static_cast<int>(a.i64(7)), nullptr,
                                    static_cast<hipStream_t>(a.handle(8)), &launches);
    rv->set_int((int64_t(path) << 32) + launches);
  });
  // (plan, row_bytes, block_bytes, blocks (0: from the sizes), stream)
  register_global("dglhip._CAPI_SpmmPlanBlocked", [](const Args& a, RetValue* rv) {
    SpmmPlan* plan = static_cast<SpmmPlan*>(a.handle(0));
    DGLHIP_CHECK(plan, "null plan");
    PlanDevice guard(*plan);
    hipStream_t s = static_cast<hipStream_t>(a.handle(4));
    const int64_t B = a.i64(3);
    std::shared_ptr<BlockedPlan> bp =
        B > 0 ? plan->blocked_for(static_cast<int>(B), s) : plan->blocked(a.i64(1), a.i64(2), s);
    if (!bp) {
      rv->set_handle(nullptr);
      return;
    }
    std::vector<int64_t> meta = {bp->B, bp->has_suffix ? 1 : 0, bp->n_absent,
                                 static_cast<int64_t>(bp->launches.size())};
    for (const BlockItems& it : bp->launches) {
      meta.push_back(it.n_items);
      meta.push_back(it.nnz);
      meta.push_back(it.off);
      meta.push_back(it.suffix ? 1 : 0);
    }
    std::vector<rt::NDArray> vec = {rt::NDArray::FromVector(meta), bp->indices, bp->pos,
                                    bp->absent};
    for (const BlockItems& it : bp->launches) {
      vec.push_back(it.rows);
      vec.push_back(it.ptr);
    }
    rv->set_func(rt::ndarray_vector_func(std::move(vec)));
  });
  // (plan, row_bytes, block_bytes, blocks (0: from the sizes), stream)
  register_global("dglhip._CAPI_SpmmPlanCuts", [](const Args& a, RetValue* rv) {
    SpmmPlan* plan = static_cast<SpmmPlan*>(a.handle(0));
    DGLHIP_CHECK(plan, "null plan");
    PlanDevice guard(*plan);
    hipStream_t s = static_cast<hipStream_t>(a.handle(4));
    const int64_t B = a.i64(3);
    std::shared_ptr<Cuts> c =
        B > 0 ? plan->cuts_for(static_cast<int>(B), s) : plan->cuts(a.i64(1), a.i64(2), s);
    if (!c) {
      rv->set_handle(nullptr);
      return;
    }
    rv->set_array(c->data);
  });
  // (plan, threshold, skip_empty, chunk (<= 0: sized to fill the part), stream)
  register_global("dglhip._CAPI_SpmmPlanSplit", [](const Args& a, RetValue* rv) {
    SpmmPlan* plan = static_cast<SpmmPlan*>(a.handle(0));
    DGLHIP_CHECK(plan, "null plan");
    PlanDevice guard(*plan);
    SplitPlan& sp = plan->split_plan(a.i64(1), a.b(2), a.i64(3),
                                     static_cast<hipStream_t>(a.handle(4)));
    std::vector<rt::NDArray> vec = {
        rt::NDArray::FromVector({sp.n_light, sp.n_heavy, sp.n_chunks}), sp.light, sp.heavy,
        sp.chunk_ptr, sp.beg, sp.end};
    rv->set_func(rt::ndarray_vector_func(std::move(vec)));
  });
  // (plan, skip_empty, threshold (0: the whole schedule; else a split's light rows), stream)
  register_global("dglhip._CAPI_SpmmPlanTiers", [](const Args& a, RetValue* rv) {
    SpmmPlan* plan = static_cast<SpmmPlan*>(a.handle(0));
    DGLHIP_CHECK(plan, "null plan");
    PlanDevice guard(*plan);
    hipStream_t s = static_cast<hipStream_t>(a.handle(3));
    const bool skip = a.b(1);
    const int64_t thr = a.i64(2);
    const Tiers& t = thr > 0 ? plan->tiers_light(plan->split_plan(thr, skip, -1, s), thr, skip, s)
                             : plan->tiers_plain(skip, s);
    std::vector<int64_t> meta = {t.n_long, t.n_tail, static_cast<int64_t>(t.tiers.size())};
    std::vector<rt::NDArray> vec;
    for (const Tier& tier : t.tiers) {
      meta.push_back(tier.maxd);
      meta.push_back(tier.n);
    }
    vec.push_back(rt::NDArray::FromVector(meta));
    for (const Tier& tier : t.tiers) {
      vec.push_back(tier.rows);
      vec.push_back(tier.maxd ? tier.sp : rt::NDArray::Ids(0));
      vec.push_back(tier.maxd ? tier.cols : rt::NDArray::Ids(0));
    }
    rv->set_func(rt::ndarray_vector_func(std::move(vec)));
  });
  // (op, num_heads, indptr, indices, eid, lhs, rhs, out, stream)
  register_global("dglhip._CAPI_GSDDMM", [](const Args& a, RetValue*) {
    const int op = static_cast<int>(a.i64(0));
    const int64_t heads = a.i64(1);
    auto* indptr = a.tensor(2);
    auto* indices = a.tensor(3);
    auto* eid = a.tensor(4);
    auto* lhs = a.tensor(5);
    auto* rhs = a.tensor(6);
    auto* out = a.tensor(7);
    void* stream = a.handle(8);
    same_device(out, {indptr, indices, eid, lhs, rhs});
    DGLHIP_CHECK(lhs->ndim == 2, "lhs must be 2-D");
    const int64_t rows = numel(indptr) - 1, F = lhs->shape[1];
    DGLHIP_CHECK(numel(out) >= heads, "out too small");
    if (out->device_type == kDeviceCPU) {
      throw_last(dglhip_gsddmm_host(op, rows, F, heads, I64(indptr, "indptr"),
                                    I32(indices, "indices"), I64(eid, "eid"),
                                    F32(lhs, "lhs"), F32(rhs, "rhs"),
                                    F32(out, "out"), 0));
    } else {
      throw_last(dglhip_gsddmm_device(op, rows, F, heads, I64(indptr, "indptr"),
                                      I32(indices, "indices"), I64(eid, "eid"),
                                      F32(lhs, "lhs"), F32(rhs, "rhs"),
                                      F32(out, "out"), stream_or_current(stream, out)));
    }
  });
  // (num_rows, num_cols, row, col, order, indptr, indices, eid) — host tensors
  register_global("dglhip._CAPI_COOToCSR", [](const Args& a, RetValue*) {
    const int64_t rows = a.i64(0), cols = a.i64(1);
    auto* row = a.tensor(2);
    auto* col = a.tensor(3);
    const int order = static_cast<int>(a.i64(4));
    auto* indptr = a.tensor(5);
    auto* indices = a.tensor(6);
    auto* eid = a.tensor(7);
    DGLHIP_CHECK(row->device_type == kDeviceCPU, "COOToCSR takes host tensors");
    same_device(row, {col, indptr, indices, eid});
    DGLHIP_CHECK(numel(row) == numel(col), "row/col length mismatch");
    throw_last(dglhip_coo_to_csr_host(rows, cols, numel(row), I64(row, "row"),
                                      I64(col, "col"), order, I64(indptr, "indptr"),
                                      I32(indices, "indices"), I64(eid, "eid")));
  });
  // (indptr, row_order) — host tensors
  register_global("dglhip._CAPI_RowsByDegree", [](const Args& a, RetValue*) {
    auto* indptr = a.tensor(0);
    auto* order = a.tensor(1);
    DGLHIP_CHECK(indptr->device_type == kDeviceCPU, "RowsByDegree takes host tensors");
    throw_last(dglhip_rows_by_degree_host(numel(indptr) - 1, I64(indptr, "indptr"),
                                          I32(order, "row_order")));
  });
}

}  // namespace dglhip
