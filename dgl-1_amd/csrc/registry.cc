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
#include <initializer_list>

#include "runtime.h"

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
    same_device(out, {indptr, indices, eid, uf, ef, arg, order});
    DGLHIP_CHECK(out->ndim == 2, "out must be 2-D [rows, feat]");
    const int64_t rows = out->shape[0], F = out->shape[1];
    DGLHIP_CHECK(numel(indptr) == rows + 1, "indptr length must be rows+1");
    int64_t elen = 0;
    if (ef) elen = ef->ndim == 1 ? 1 : numel(ef) / ef->shape[0];
    if (out->device_type == kDeviceCPU) {
      throw_last(dglhip_gspmm_host(msg, red, rows, F, I64(indptr, "indptr"),
                                   I32(indices, "indices"), I64(eid, "eid"),
                                   F32(uf, "ufeat"), F32(ef, "efeat"), elen,
                                   F32(out, "out"), I64(arg, "arg_out"), 0));
    } else {
      DGLHIP_CHECK(out->device_type == kDeviceROCM, "unsupported device type "
                                                        << out->device_type);
      throw_last(dglhip_gspmm_device(msg, red, rows, F, I64(indptr, "indptr"),
                                     I32(indices, "indices"), I64(eid, "eid"),
                                     F32(uf, "ufeat"), F32(ef, "efeat"), elen,
                                     F32(out, "out"), I64(arg, "arg_out"),
                                     I32(order, "row_order"), stream_or_current(stream, out)));
    }
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
