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
#include <cstring>
#include <functional>
#include <initializer_list>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/dgl_hip.h"
#include "common.h"

namespace dglhip {

namespace {

constexpr int kDeviceCPU = 1;
constexpr int kDeviceROCM = 10;

struct Args {
  DGLHipValue* values;
  int* codes;
  int n;

  void need(int i) const {
    DGLHIP_CHECK(i < n, "missing argument " << i << " (got " << n << ")");
  }
  int64_t i64(int i) const {
    need(i);
    DGLHIP_CHECK(codes[i] == DGLHIP_TC_INT || codes[i] == DGLHIP_TC_UINT,
                 "argument " << i << " must be an integer, type code " << codes[i]);
    return values[i].v_int64;
  }
  void* handle(int i) const {
    need(i);
    if (codes[i] == DGLHIP_TC_NULL) return nullptr;
    DGLHIP_CHECK(codes[i] == DGLHIP_TC_HANDLE,
                 "argument " << i << " must be a handle, type code " << codes[i]);
    return values[i].v_handle;
  }
  // Tensor argument; returns nullptr when the caller passed null.
  const DGLHipTensor* tensor(int i, bool optional = false) const {
    need(i);
    if (codes[i] == DGLHIP_TC_NULL) {
      DGLHIP_CHECK(optional, "argument " << i << " must not be null");
      return nullptr;
    }
    DGLHIP_CHECK(codes[i] == DGLHIP_TC_ARRAY_HANDLE,
                 "argument " << i << " must be a tensor, type code " << codes[i]);
    return static_cast<const DGLHipTensor*>(values[i].v_handle);
  }
};

int64_t numel(const DGLHipTensor* t) {
  int64_t n = 1;
  for (int d = 0; d < t->ndim; ++d) n *= t->shape[d];
  return n;
}

void check_compact(const DGLHipTensor* t, const char* what) {
  if (!t->strides) return;
  int64_t expect = 1;
  for (int d = t->ndim - 1; d >= 0; --d) {
    DGLHIP_CHECK(t->shape[d] == 1 || t->strides[d] == expect,
                 what << " must be contiguous");
    expect *= t->shape[d];
  }
}

template <typename T>
T* data_as(const DGLHipTensor* t, int code, int bits, const char* what) {
  if (!t) return nullptr;
  DGLHIP_CHECK(t->dtype_code == code && t->dtype_bits == bits && t->dtype_lanes == 1,
               what << " has dtype (" << int(t->dtype_code) << "," << int(t->dtype_bits)
                    << "), expected (" << code << "," << bits << ")");
  check_compact(t, what);
  return reinterpret_cast<T*>(static_cast<char*>(t->data) + t->byte_offset);
}

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

using Body = std::function<void(const Args&)>;

std::map<std::string, Body>& table() {
  static std::map<std::string, Body> t;
  return t;
}

std::vector<std::string>& names_cache() {
  static std::vector<std::string> v;
  return v;
}

void register_all() {
  auto& t = table();
  // (msg, reduce, indptr, indices, eid|null, ufeat|null, efeat|null, out,
  //  arg_out|null, row_order|null, stream)
  t["dglhip._CAPI_GSpMM"] = [](const Args& a) {
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
                                     I32(order, "row_order"), stream));
    }
  };
  // (op, num_heads, indptr, indices, eid, lhs, rhs, out, stream)
  t["dglhip._CAPI_GSDDMM"] = [](const Args& a) {
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
                                      F32(out, "out"), stream));
    }
  };
  // (num_rows, num_cols, row, col, order, indptr, indices, eid) — host tensors
  t["dglhip._CAPI_COOToCSR"] = [](const Args& a) {
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
  };
  // (indptr, row_order) — host tensors
  t["dglhip._CAPI_RowsByDegree"] = [](const Args& a) {
    auto* indptr = a.tensor(0);
    auto* order = a.tensor(1);
    DGLHIP_CHECK(indptr->device_type == kDeviceCPU, "RowsByDegree takes host tensors");
    throw_last(dglhip_rows_by_degree_host(numel(indptr) - 1, I64(indptr, "indptr"),
                                          I32(order, "row_order")));
  };
}

std::once_flag g_once;

std::map<std::string, Body>& registry() {
  std::call_once(g_once, register_all);
  return table();
}

}  // namespace
}  // namespace dglhip

using namespace dglhip;

extern "C" {

int DGLFuncGetGlobal(const char* name, DGLHipFunctionHandle* out) {
  API_BEGIN();
  DGLHIP_CHECK(name && out, "null argument");
  auto& r = registry();
  auto it = r.find(name);
  *out = it == r.end() ? nullptr : static_cast<void*>(&it->second);
  API_END();
}

int DGLFuncListGlobalNames(int* out_size, const char*** out_array) {
  API_BEGIN();
  static thread_local std::vector<const char*> ptrs;
  auto& r = registry();
  auto& names = names_cache();
  if (names.size() != r.size()) {
    names.clear();
    for (auto& kv : r) names.push_back(kv.first);
  }
  ptrs.clear();
  for (auto& s : names) ptrs.push_back(s.c_str());
  *out_size = static_cast<int>(ptrs.size());
  *out_array = ptrs.data();
  API_END();
}

int DGLFuncCall(DGLHipFunctionHandle func, DGLHipValue* arg_values,
                int* type_codes, int num_args, DGLHipValue* ret_val,
                int* ret_type_code) {
  API_BEGIN();
  DGLHIP_CHECK(func != nullptr, "null function handle");
  Args a{arg_values, type_codes, num_args};
  (*static_cast<Body*>(func))(a);
  if (ret_type_code) *ret_type_code = DGLHIP_TC_NULL;
  if (ret_val) ret_val->v_int64 = 0;
  API_END();
}

// Registry entries are owned by the library; freeing a global handle is a
// no-op, as for functions obtained from the reference's global table.
int DGLFuncFree(DGLHipFunctionHandle func) {
  (void)func;
  return 0;
}

}  // extern "C"
