// PackedFunc runtime of libdgl_hip: ref-counted NDArrays, function objects,
// argument/return values and the global registry.
//
// Restates the calling convention of the reference's TVM-derived runtime
// (include/dgl/runtime/c_runtime_api.h, packed_func.h, ndarray.h,
// src/runtime/c_runtime_api.cc, registry.cc) so that the reference's ctypes
// layer (python/dgl/_ffi/_ctypes/function.py:80-190, ndarray.py:20-90) can
// bind this library unchanged:
//   * an NDArray handle is a pointer to a container whose first member is the
//     DLTensor; returned arrays carry type code NDARRAY_CONTAINER and one
//     reference owned by the caller (freed with DGLArrayFree);
//   * a returned function carries FUNC_HANDLE and one reference (DGLFuncFree);
//   * graph objects travel as opaque HANDLEs.
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <string>
#include <utility>
#include <vector>

#include "../../include/dgl_hip.h"
#include "common.h"

namespace dglhip {
namespace rt {

constexpr int kDLCPU = 1;
constexpr int kDLROCM = 10;

struct NDContainer {
  DGLHipTensor dl;  // must stay the first member: DGLArrayHandle == &dl
  std::atomic<int> ref{1};
  std::vector<int64_t> shape;
  std::vector<int64_t> strides;
  enum Kind { kHost, kDevice, kExternal } kind = kHost;
  DGLHipManagedTensor* ext = nullptr;  // owner of external (DLPack) memory
};

void nd_incref(NDContainer* c);
void nd_decref(NDContainer* c);

// Intrusive reference to an NDContainer.
class NDArray {
 public:
  NDArray() = default;
  explicit NDArray(NDContainer* adopt) : c_(adopt) {}
  NDArray(const NDArray& o) : c_(o.c_) { if (c_) nd_incref(c_); }
  NDArray(NDArray&& o) noexcept : c_(o.c_) { o.c_ = nullptr; }
  NDArray& operator=(NDArray o) { std::swap(c_, o.c_); return *this; }
  ~NDArray() { if (c_) nd_decref(c_); }

  // Uninitialised array (host memory 64-B aligned, or hipMalloc on a ROCm device).
  static NDArray Empty(const std::vector<int64_t>& shape, int code, int bits,
                       int device_type = kDLCPU, int device_id = 0);
  // 1-D host int64 array.
  static NDArray Ids(int64_t n) { return Empty({n}, 0, 64); }
  static NDArray FromVector(const std::vector<int64_t>& v) {
    return FromIds(v.data(), static_cast<int64_t>(v.size()));
  }
  // 1-D host int64 copy of p[0, n) (parallel copy for large n).
  static NDArray FromIds(const int64_t* p, int64_t n);

  bool defined() const { return c_ != nullptr; }
  NDContainer* get() const { return c_; }
  NDContainer* release() { NDContainer* c = c_; c_ = nullptr; return c; }
  const DGLHipTensor* tensor() const { return &c_->dl; }
  int64_t numel() const;
  template <typename T> T* data() const {
    return reinterpret_cast<T*>(static_cast<char*>(c_->dl.data) + c_->dl.byte_offset);
  }

 private:
  NDContainer* c_ = nullptr;
};

struct RetValue;

// Positional arguments of a packed call.
struct Args {
  DGLHipValue* values;
  int* codes;
  int n;

  int size() const { return n; }
  int code(int i) const { need(i); return codes[i]; }
  void need(int i) const;
  int64_t i64(int i) const;
  double f64(int i) const;
  bool b(int i) const { return i64(i) != 0; }
  void* handle(int i) const;            // HANDLE or NULL
  std::string str(int i) const;
  // DLTensor argument (ARRAY_HANDLE or NDARRAY_CONTAINER); nullptr only when
  // `optional` and the caller passed NULL.
  const DGLHipTensor* tensor(int i, bool optional = false) const;
};

using Body = std::function<void(const Args&, RetValue*)>;

struct Func {
  Body body;
  std::atomic<int> ref{1};
  bool global = false;  // owned by the registry; DGLFuncFree never frees it
};

void func_incref(Func* f);
void func_decref(Func* f);

// Return slot of a packed call.
struct RetValue {
  int code = DGLHIP_TC_NULL;
  DGLHipValue v{};
  std::string s;
  NDArray arr;
  Func* fn = nullptr;  // one owned reference

  RetValue() = default;
  RetValue(const RetValue&) = delete;
  RetValue& operator=(const RetValue&) = delete;
  ~RetValue() { clear(); }

  void clear();
  void set_int(int64_t x) { clear(); code = DGLHIP_TC_INT; v.v_int64 = x; }
  void set_bool(bool x) { set_int(x ? 1 : 0); }
  void set_float(double x) { clear(); code = DGLHIP_TC_FLOAT; v.v_float64 = x; }
  void set_handle(void* h) { clear(); code = h ? DGLHIP_TC_HANDLE : DGLHIP_TC_NULL; v.v_handle = h; }
  void set_str(std::string x) { clear(); code = DGLHIP_TC_STR; s = std::move(x); }
  void set_array(NDArray a) { clear(); code = DGLHIP_TC_NDARRAY_CONTAINER; arr = std::move(a); }
  void set_func(Body body);
  // Copy a C value into this slot, taking a new reference to arrays and
  // functions (DGLCFuncSetReturn semantics).
  void assign_from_c(const DGLHipValue& value, int type_code);
  // Hand the value and its reference over to a C caller.
  void move_to_c(DGLHipValue* out, int* out_code);
};

// Closure returning vec[which] (ConvertNDArrayVectorToPackedFunc,
// src/c_api_common.cc:25-36; ConvertAdjToPackedFunc, graph_apis.cc:39-49).
Body ndarray_vector_func(std::vector<NDArray> vec);

// Registers `body` under `name` in the global table (built-in functions are
// registered once, on first lookup).
void register_global(const std::string& name, Body body);

// Host pointer helpers shared by the registered functions.
int64_t numel(const DGLHipTensor* t);
void check_compact(const DGLHipTensor* t, const char* what);
template <typename T>
T* data_as(const DGLHipTensor* t, int code, int bits, const char* what) {
  if (!t) return nullptr;
  DGLHIP_CHECK(t->dtype_code == code && t->dtype_bits == bits && t->dtype_lanes == 1,
               what << " has dtype (" << int(t->dtype_code) << "," << int(t->dtype_bits)
                    << "), expected (" << code << "," << bits << ")");
  check_compact(t, what);
  return reinterpret_cast<T*>(static_cast<char*>(t->data) + t->byte_offset);
}

// Thread-local current stream per device set by DGLSetStream (used by the
// registered kernels when their stream argument is NULL).
void* current_stream(int device_id);

}  // namespace rt

// Registration hooks of each translation unit (called once by the registry).
void register_kernel_functions();
void register_graph_index_functions();
void register_scheduler_functions();

}  // namespace dglhip
