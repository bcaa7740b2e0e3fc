// PackedFunc runtime of libdgl_hip (see runtime.h): NDArray containers,
// function objects, the global registry and every C runtime entry point the
// reference's ctypes layer binds (python/dgl/_ffi: base.py:62,
// function.py:67-229, ndarray.py:105-295, _ctypes/function.py:55-187,
// _ctypes/ndarray.py:32-84, _ctypes/types.py:54, runtime_ctypes.py:225).
//
// Semantics follow include/dgl/runtime/c_runtime_api.h: an entry point
// returns 0, or -1 with the message in DGLGetLastError(); returned arrays and
// functions carry one reference owned by the caller.
#include "runtime.h"

#include <hip/hip_runtime_api.h>

#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>

namespace dglhip {
namespace rt {

namespace {

void hip_check(hipError_t e, const char* what) {
  DGLHIP_CHECK(e == hipSuccess, what << ": " << hipGetErrorString(e));
}

// Runs fn with `device` as the current HIP device, restoring the previous one.
template <typename Fn>
void on_device(int device, Fn&& fn) {
  int prev = 0;
  hip_check(hipGetDevice(&prev), "hipGetDevice");
  if (prev != device) hip_check(hipSetDevice(device), "hipSetDevice");
  try {
    fn();
  } catch (...) {
    if (prev != device) (void)hipSetDevice(prev);
    throw;
  }
  if (prev != device) hip_check(hipSetDevice(prev), "hipSetDevice");
}

int64_t elem_bytes(const DGLHipTensor& t) {
  return (int64_t(t.dtype_bits) * t.dtype_lanes + 7) / 8;
}

int64_t nbytes_of(const DGLHipTensor& t) {
  int64_t n = 1;
  for (int d = 0; d < t.ndim; ++d) n *= t.shape[d];
  return n * elem_bytes(t);
}

void* data_ptr(const DGLHipTensor& t) {
  return static_cast<char*>(t.data) + t.byte_offset;
}

bool is_compact(const DGLHipTensor& t) {
  if (!t.strides) return true;
  int64_t expect = 1;
  for (int d = t.ndim - 1; d >= 0; --d) {
    if (t.shape[d] != 1 && t.strides[d] != expect) return false;
    expect *= t.shape[d];
  }
  return true;
}

// DGLByteArray (c_runtime_api.h:118-121).
struct ByteArray {
  const char* data;
  size_t size;
};

NDContainer* as_container(DGLHipArrayHandle h) {
  DGLHIP_CHECK(h != nullptr, "null array handle");
  return reinterpret_cast<NDContainer*>(h);
}

}  // namespace

// ---------------------------------------------------------------- NDArray
void nd_incref(NDContainer* c) { c->ref.fetch_add(1, std::memory_order_relaxed); }

void nd_decref(NDContainer* c) {
  if (c->ref.fetch_sub(1, std::memory_order_acq_rel) != 1) return;
  switch (c->kind) {
    case NDContainer::kHost:
      std::free(c->dl.data);
      break;
    case NDContainer::kDevice:
      (void)hipFree(c->dl.data);
      break;
    case NDContainer::kExternal:
      if (c->ext && c->ext->deleter) c->ext->deleter(c->ext);
      break;
  }
  delete c;
}

NDArray NDArray::Empty(const std::vector<int64_t>& shape, int code, int bits,
                       int device_type, int device_id) {
  auto* c = new NDContainer();
  NDArray out(c);  // owns c from here on
  c->shape = shape;
  c->dl.ndim = static_cast<int32_t>(shape.size());
  c->dl.shape = c->shape.data();
  c->dl.strides = nullptr;
  c->dl.byte_offset = 0;
  c->dl.dtype_code = static_cast<uint8_t>(code);
  c->dl.dtype_bits = static_cast<uint8_t>(bits);
  c->dl.dtype_lanes = 1;
  c->dl.device_type = device_type;
  c->dl.device_id = device_id;
  c->dl.data = nullptr;
  for (int64_t s : shape) DGLHIP_CHECK(s >= 0, "negative array extent " << s);
  const int64_t nbytes = nbytes_of(c->dl);
  if (device_type == kDLCPU) {
    c->kind = NDContainer::kHost;
    // 64-B aligned; never a zero-size request so data is never NULL.
    const size_t sz = static_cast<size_t>((std::max<int64_t>(nbytes, 1) + 63) / 64 * 64);
    c->dl.data = std::aligned_alloc(64, sz);
    DGLHIP_CHECK(c->dl.data != nullptr, "host allocation of " << nbytes << " bytes failed");
  } else {
    DGLHIP_CHECK(device_type == kDLROCM, "unsupported device type " << device_type);
    c->kind = NDContainer::kDevice;
    on_device(device_id, [&] {
      hip_check(hipMalloc(&c->dl.data, static_cast<size_t>(std::max<int64_t>(nbytes, 1))),
                "hipMalloc");
    });
  }
  return out;
}

NDArray NDArray::FromIds(const int64_t* p, int64_t n) {
  NDArray a = Ids(n);
  int64_t* dst = a.data<int64_t>();
  // threads share the first-touch page faults of the new buffer (10^9-id
  // exports of the graph index)
  parallel_for(n, default_num_threads(), [&](int64_t b, int64_t e, int) {
    std::memcpy(dst + b, p + b, static_cast<size_t>(e - b) * sizeof(int64_t));
  }, int64_t(1) << 18);
  return a;
}

int64_t NDArray::numel() const {
  int64_t n = 1;
  for (int d = 0; d < c_->dl.ndim; ++d) n *= c_->dl.shape[d];
  return n;
}

int64_t numel(const DGLHipTensor* t) {
  int64_t n = 1;
  for (int d = 0; d < t->ndim; ++d) n *= t->shape[d];
  return n;
}

void check_compact(const DGLHipTensor* t, const char* what) {
  DGLHIP_CHECK(is_compact(*t), what << " must be contiguous");
}

// ---------------------------------------------------------------- functions
void func_incref(Func* f) { f->ref.fetch_add(1, std::memory_order_relaxed); }

void func_decref(Func* f) {
  if (f->ref.fetch_sub(1, std::memory_order_acq_rel) == 1) delete f;
}

// ---------------------------------------------------------------- arguments
void Args::need(int i) const {
  DGLHIP_CHECK(i < n, "missing argument " << i << " (got " << n << ")");
}

int64_t Args::i64(int i) const {
  need(i);
  DGLHIP_CHECK(codes[i] == DGLHIP_TC_INT || codes[i] == DGLHIP_TC_UINT,
               "argument " << i << " must be an integer, type code " << codes[i]);
  return values[i].v_int64;
}

double Args::f64(int i) const {
  need(i);
  if (codes[i] == DGLHIP_TC_INT || codes[i] == DGLHIP_TC_UINT)
    return static_cast<double>(values[i].v_int64);
  DGLHIP_CHECK(codes[i] == DGLHIP_TC_FLOAT,
               "argument " << i << " must be a number, type code " << codes[i]);
  return values[i].v_float64;
}

void* Args::handle(int i) const {
  need(i);
  if (codes[i] == DGLHIP_TC_NULL) return nullptr;
  DGLHIP_CHECK(codes[i] == DGLHIP_TC_HANDLE,
               "argument " << i << " must be a handle, type code " << codes[i]);
  return values[i].v_handle;
}

std::string Args::str(int i) const {
  need(i);
  DGLHIP_CHECK(codes[i] == DGLHIP_TC_STR,
               "argument " << i << " must be a string, type code " << codes[i]);
  return values[i].v_str ? std::string(values[i].v_str) : std::string();
}

const DGLHipTensor* Args::tensor(int i, bool optional) const {
  need(i);
  if (codes[i] == DGLHIP_TC_NULL) {
    DGLHIP_CHECK(optional, "argument " << i << " must not be null");
    return nullptr;
  }
  DGLHIP_CHECK(codes[i] == DGLHIP_TC_ARRAY_HANDLE || codes[i] == DGLHIP_TC_NDARRAY_CONTAINER,
               "argument " << i << " must be a tensor, type code " << codes[i]);
  DGLHIP_CHECK(values[i].v_handle != nullptr, "argument " << i << " is a null tensor");
  return static_cast<const DGLHipTensor*>(values[i].v_handle);
}

// ---------------------------------------------------------------- return slot
void RetValue::clear() {
  if (fn) {
    func_decref(fn);
    fn = nullptr;
  }
  arr = NDArray();
  s.clear();
  code = DGLHIP_TC_NULL;
  v.v_int64 = 0;
}

void RetValue::set_func(Body body) {
  clear();
  fn = new Func();
  fn->body = std::move(body);
  code = DGLHIP_TC_FUNC_HANDLE;
}

void RetValue::assign_from_c(const DGLHipValue& value, int type_code) {
  switch (type_code) {
    case DGLHIP_TC_NDARRAY_CONTAINER: {
      auto* c = reinterpret_cast<NDContainer*>(value.v_handle);
      nd_incref(c);
      set_array(NDArray(c));
      break;
    }
    case DGLHIP_TC_FUNC_HANDLE: {
      auto* f = static_cast<Func*>(value.v_handle);
      func_incref(f);
      clear();
      fn = f;
      code = DGLHIP_TC_FUNC_HANDLE;
      break;
    }
    case DGLHIP_TC_STR:
      set_str(value.v_str ? value.v_str : "");
      break;
    case DGLHIP_TC_BYTES: {
      const auto* ba = static_cast<const ByteArray*>(value.v_handle);
      clear();
      s.assign(ba->data, ba->size);
      code = DGLHIP_TC_BYTES;
      break;
    }
    case DGLHIP_TC_MODULE_HANDLE:
      DGLHIP_CHECK(false, "modules are not supported by this runtime");
      break;
    default:  // POD values (int, float, handles, array views, contexts, types)
      clear();
      code = type_code;
      v = value;
      break;
  }
}

void RetValue::move_to_c(DGLHipValue* out, int* out_code) {
  // Per-thread storage for string / bytes results, valid until the thread's
  // next call (the reference's DGLFuncCall keeps them in its thread-local
  // return store, c_runtime_api.cc:136).
  static thread_local std::string ret_str;
  static thread_local ByteArray ret_bytes;
  DGLHipValue val{};
  int c = code;
  switch (code) {
    case DGLHIP_TC_NDARRAY_CONTAINER:
      val.v_handle = arr.release();
      break;
    case DGLHIP_TC_FUNC_HANDLE:
      val.v_handle = fn;
      fn = nullptr;
      break;
    case DGLHIP_TC_STR:
      ret_str = s;
      val.v_str = ret_str.c_str();
      break;
    case DGLHIP_TC_BYTES:
      ret_str = s;
      ret_bytes.data = ret_str.data();
      ret_bytes.size = ret_str.size();
      val.v_handle = &ret_bytes;
      break;
    default:
      val = v;
      break;
  }
  clear();
  if (out) {
    *out = val;
  } else if (c == DGLHIP_TC_NDARRAY_CONTAINER) {
    nd_decref(static_cast<NDContainer*>(val.v_handle));
  } else if (c == DGLHIP_TC_FUNC_HANDLE) {
    func_decref(static_cast<Func*>(val.v_handle));
  }
  if (out_code) *out_code = out ? c : DGLHIP_TC_NULL;
}

Body ndarray_vector_func(std::vector<NDArray> vec) {
  return [vec](const Args& a, RetValue* rv) {
    const int64_t which = a.i64(0);
    DGLHIP_CHECK(which >= 0 && which < static_cast<int64_t>(vec.size()),
                 "invalid choice " << which << " (have " << vec.size() << ")");
    rv->set_array(vec[which]);
  };
}

// ---------------------------------------------------------------- registry
namespace {

struct Registry {
  std::mutex mu;
  std::map<std::string, Func*> table;
  std::vector<std::string> names;
};

Registry& raw_registry() {
  static Registry* r = new Registry();  // never destroyed: handles outlive exit
  return *r;
}

std::once_flag g_builtin_once;

// _GetDeviceAttr (src/runtime/c_runtime_api.cc:391-408, device_api.h:18-28):
// (device_type, device_id, kind) for the Context properties of
// python/dgl/_ffi/runtime_ctypes.py:150-222.
void register_runtime_functions() {
  register_global("_GetDeviceAttr", [](const Args& a, RetValue* rv) {
    const int dev_type = static_cast<int>(a.i64(0));
    const int dev = static_cast<int>(a.i64(1));
    const int kind = static_cast<int>(a.i64(2));
    if (dev_type == kDLCPU) {
      if (kind == 0) rv->set_int(1);  // kExist; other CPU attributes are unset
      return;
    }
    DGLHIP_CHECK(dev_type == kDLROCM, "unsupported device type " << dev_type);
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
    if (kind == 0) {
      rv->set_int(dev >= 0 && dev < count ? 1 : 0);
      return;
    }
    DGLHIP_CHECK(dev >= 0 && dev < count, "no ROCm device " << dev);
    hipDeviceProp_t p;
    hip_check(hipGetDeviceProperties(&p, dev), "hipGetDeviceProperties");
    switch (kind) {
      case 1: rv->set_int(p.maxThreadsPerBlock); break;
      case 2: rv->set_int(p.warpSize); break;
      case 3: rv->set_int(static_cast<int64_t>(p.sharedMemPerBlock)); break;
      case 4: rv->set_str(std::to_string(p.major) + "." + std::to_string(p.minor)); break;
      case 5: rv->set_str(p.gcnArchName); break;
      case 6: rv->set_int(p.clockRate); break;
      case 7: rv->set_int(p.multiProcessorCount); break;
      case 8:
        rv->set_str("[" + std::to_string(p.maxThreadsDim[0]) + ", " +
                    std::to_string(p.maxThreadsDim[1]) + ", " +
                    std::to_string(p.maxThreadsDim[2]) + "]");
        break;
      default: DGLHIP_CHECK(false, "unknown device attribute " << kind);
    }
  });
}

Registry& registry() {
  std::call_once(g_builtin_once, [] {
    register_runtime_functions();
    register_kernel_functions();
    register_graph_index_functions();
    register_scheduler_functions();
  });
  return raw_registry();
}

}  // namespace

void register_global(const std::string& name, Body body) {
  auto& r = raw_registry();
  std::lock_guard<std::mutex> lk(r.mu);
  auto* f = new Func();
  f->body = std::move(body);
  f->global = true;
  auto it = r.table.find(name);
  if (it != r.table.end()) func_decref(it->second);
  r.table[name] = f;
}

// ---------------------------------------------------------------- streams
namespace {
thread_local std::map<int, void*> t_current_stream;
}

void* current_stream(int device_id) {
  auto it = t_current_stream.find(device_id);
  return it == t_current_stream.end() ? nullptr : it->second;
}

}  // namespace rt
}  // namespace dglhip

using namespace dglhip;
using namespace dglhip::rt;

extern "C" {

// ------------------------------------------------------------------ functions
int DGLFuncGetGlobal(const char* name, DGLHipFunctionHandle* out) {
  API_BEGIN();
  DGLHIP_CHECK(name && out, "null argument");
  auto& r = registry();
  std::lock_guard<std::mutex> lk(r.mu);
  auto it = r.table.find(name);
  *out = it == r.table.end() ? nullptr : static_cast<void*>(it->second);
  API_END();
}

int DGLFuncListGlobalNames(int* out_size, const char*** out_array) {
  API_BEGIN();
  static thread_local std::vector<const char*> ptrs;
  auto& r = registry();
  std::lock_guard<std::mutex> lk(r.mu);
  r.names.clear();
  for (auto& kv : r.table) r.names.push_back(kv.first);
  ptrs.clear();
  for (auto& s : r.names) ptrs.push_back(s.c_str());
  *out_size = static_cast<int>(ptrs.size());
  *out_array = ptrs.data();
  API_END();
}

int DGLFuncCall(DGLHipFunctionHandle func, DGLHipValue* arg_values, int* type_codes,
                int num_args, DGLHipValue* ret_val, int* ret_type_code) {
  API_BEGIN();
  DGLHIP_CHECK(func != nullptr, "null function handle");
  Args a{arg_values, type_codes, num_args};
  RetValue rv;
  static_cast<Func*>(func)->body(a, &rv);
  rv.move_to_c(ret_val, ret_type_code);
  API_END();
}

int DGLFuncFree(DGLHipFunctionHandle func) {
  API_BEGIN();
  auto* f = static_cast<Func*>(func);
  if (f && !f->global) func_decref(f);
  API_END();
}

int DGLFuncRegisterGlobal(const char* name, DGLHipFunctionHandle f, int override_) {
  API_BEGIN();
  DGLHIP_CHECK(name && f, "null argument");
  auto& r = registry();
  auto* fn = static_cast<Func*>(f);
  std::lock_guard<std::mutex> lk(r.mu);
  auto it = r.table.find(name);
  DGLHIP_CHECK(it == r.table.end() || override_,
               "Global PackedFunc " << name << " is already registered");
  func_incref(fn);
  if (it != r.table.end()) func_decref(it->second);
  r.table[name] = fn;
  API_END();
}

int DGLFuncCreateFromCFunc(DGLHipPackedCFunc func, void* resource_handle,
                           DGLHipPackedCFuncFinalizer fin, DGLHipFunctionHandle* out) {
  API_BEGIN();
  DGLHIP_CHECK(func && out, "null argument");
  // The finalizer runs when the last copy of the body goes away.
  std::shared_ptr<void> res(resource_handle, [fin](void* p) { if (fin) fin(p); });
  auto* f = new Func();
  f->body = [func, res](const Args& a, RetValue* rv) {
    if (func(a.values, a.codes, a.n, rv, res.get()) != 0)
      throw Error(DGLGetLastError());
  };
  *out = f;
  API_END();
}

int DGLCFuncSetReturn(DGLHipRetValueHandle ret, DGLHipValue* value, int* type_code,
                      int num_ret) {
  API_BEGIN();
  DGLHIP_CHECK(ret && value && type_code, "null argument");
  DGLHIP_CHECK(num_ret == 1, "a packed function returns exactly one value");
  static_cast<RetValue*>(ret)->assign_from_c(value[0], type_code[0]);
  API_END();
}

int DGLCbArgToReturn(DGLHipValue* value, int code) {
  API_BEGIN();
  DGLHIP_CHECK(value, "null argument");
  // The callee takes its own reference to arrays and functions it receives.
  if (code == DGLHIP_TC_NDARRAY_CONTAINER) {
    nd_incref(reinterpret_cast<NDContainer*>(value->v_handle));
  } else if (code == DGLHIP_TC_FUNC_HANDLE) {
    func_incref(static_cast<Func*>(value->v_handle));
  } else {
    DGLHIP_CHECK(code != DGLHIP_TC_MODULE_HANDLE, "modules are not supported by this runtime");
  }
  API_END();
}

// ------------------------------------------------------------------ arrays
int DGLArrayAlloc(const int64_t* shape, int ndim, int dtype_code, int dtype_bits,
                  int dtype_lanes, int device_type, int device_id, DGLHipArrayHandle* out) {
  API_BEGIN();
  DGLHIP_CHECK(out && (shape || ndim == 0) && ndim >= 0, "invalid arguments");
  DGLHIP_CHECK(dtype_lanes == 1, "vector dtypes (lanes=" << dtype_lanes << ") are not supported");
  DGLHIP_CHECK(dtype_bits % 8 == 0 && dtype_bits > 0, "dtype bits must be a multiple of 8");
  std::vector<int64_t> sh(shape, shape + ndim);
  NDArray a = NDArray::Empty(sh, dtype_code, dtype_bits, device_type, device_id);
  *out = &a.release()->dl;
  API_END();
}

int DGLArrayFree(DGLHipArrayHandle handle) {
  API_BEGIN();
  if (handle) nd_decref(as_container(handle));
  API_END();
}

int DGLArrayCopyFromBytes(DGLHipArrayHandle handle, void* data, size_t nbytes) {
  API_BEGIN();
  DGLHIP_CHECK(handle && (data || nbytes == 0), "null argument");
  DGLHIP_CHECK(is_compact(*handle), "array must be contiguous");
  const int64_t n = nbytes_of(*handle);
  DGLHIP_CHECK(static_cast<size_t>(n) == nbytes,
               "byte count " << nbytes << " does not match the array's " << n);
  if (nbytes == 0) return 0;
  if (handle->device_type == kDLCPU) {
    std::memcpy(data_ptr(*handle), data, nbytes);
  } else {
    on_device(handle->device_id, [&] {
      hip_check(hipMemcpy(data_ptr(*handle), data, nbytes, hipMemcpyHostToDevice), "hipMemcpy");
    });
  }
  API_END();
}

int DGLArrayCopyToBytes(DGLHipArrayHandle handle, void* data, size_t nbytes) {
  API_BEGIN();
  DGLHIP_CHECK(handle && (data || nbytes == 0), "null argument");
  DGLHIP_CHECK(is_compact(*handle), "array must be contiguous");
  const int64_t n = nbytes_of(*handle);
  DGLHIP_CHECK(static_cast<size_t>(n) == nbytes,
               "byte count " << nbytes << " does not match the array's " << n);
  if (nbytes == 0) return 0;
  if (handle->device_type == kDLCPU) {
    std::memcpy(data, data_ptr(*handle), nbytes);
  } else {
    on_device(handle->device_id, [&] {
      hip_check(hipMemcpy(data, data_ptr(*handle), nbytes, hipMemcpyDeviceToHost), "hipMemcpy");
    });
  }
  API_END();
}

int DGLArrayCopyFromTo(DGLHipArrayHandle from, DGLHipArrayHandle to, DGLHipStreamHandle stream) {
  API_BEGIN();
  DGLHIP_CHECK(from && to, "null argument");
  DGLHIP_CHECK(is_compact(*from) && is_compact(*to), "arrays must be contiguous");
  const int64_t n = nbytes_of(*from);
  DGLHIP_CHECK(n == nbytes_of(*to), "copy between arrays of different byte sizes ("
                                        << n << " vs " << nbytes_of(*to) << ")");
  if (n == 0) return 0;
  if (from->device_type == kDLCPU && to->device_type == kDLCPU) {
    std::memcpy(data_ptr(*to), data_ptr(*from), static_cast<size_t>(n));
  } else {
    const int dev = from->device_type == kDLROCM ? from->device_id : to->device_id;
    on_device(dev, [&] {
      auto s = static_cast<hipStream_t>(stream ? stream : current_stream(dev));
      hip_check(hipMemcpyAsync(data_ptr(*to), data_ptr(*from), static_cast<size_t>(n),
                               hipMemcpyDefault, s), "hipMemcpyAsync");
      // A copy that involves host memory completes before returning, as the
      // reference's device API does for its CPU<->GPU copies.
      if (from->device_type == kDLCPU || to->device_type == kDLCPU)
        hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    });
  }
  API_END();
}

int DGLArrayFromDLPack(DGLHipManagedTensor* from, DGLHipArrayHandle* out) {
  API_BEGIN();
  DGLHIP_CHECK(from && out, "null argument");
  auto* c = new NDContainer();
  c->kind = NDContainer::kExternal;
  c->ext = from;
  c->dl = from->dl_tensor;
  c->shape.assign(from->dl_tensor.shape, from->dl_tensor.shape + from->dl_tensor.ndim);
  c->dl.shape = c->shape.data();
  if (from->dl_tensor.strides) {
    c->strides.assign(from->dl_tensor.strides,
                      from->dl_tensor.strides + from->dl_tensor.ndim);
    c->dl.strides = c->strides.data();
  }
  *out = &c->dl;
  API_END();
}

int DGLArrayToDLPack(DGLHipArrayHandle from, DGLHipManagedTensor** out) {
  API_BEGIN();
  DGLHIP_CHECK(from && out, "null argument");
  NDContainer* c = as_container(from);
  nd_incref(c);
  auto* m = new DGLHipManagedTensor();
  m->dl_tensor = c->dl;
  m->manager_ctx = c;
  m->deleter = [](DGLHipManagedTensor* self) {
    nd_decref(static_cast<NDContainer*>(self->manager_ctx));
    delete self;
  };
  *out = m;
  API_END();
}

void DGLDLManagedTensorCallDeleter(DGLHipManagedTensor* dltensor) {
  if (dltensor && dltensor->deleter) dltensor->deleter(dltensor);
}

// ------------------------------------------------------------------ streams
int DGLStreamCreate(int device_type, int device_id, DGLHipStreamHandle* out) {
  API_BEGIN();
  DGLHIP_CHECK(out, "null argument");
  *out = nullptr;
  if (device_type == kDLCPU) return 0;
  DGLHIP_CHECK(device_type == kDLROCM, "unsupported device type " << device_type);
  on_device(device_id, [&] {
    hipStream_t s;
    hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
    *out = s;
  });
  API_END();
}

int DGLStreamFree(int device_type, int device_id, DGLHipStreamHandle stream) {
  API_BEGIN();
  if (device_type == kDLCPU || !stream) return 0;
  on_device(device_id, [&] {
    hip_check(hipStreamDestroy(static_cast<hipStream_t>(stream)), "hipStreamDestroy");
  });
  API_END();
}

int DGLSetStream(int device_type, int device_id, DGLHipStreamHandle handle) {
  API_BEGIN();
  if (device_type == kDLROCM) dglhip::rt::t_current_stream[device_id] = handle;
  API_END();
}

int DGLSynchronize(int device_type, int device_id, DGLHipStreamHandle stream) {
  API_BEGIN();
  if (device_type == kDLCPU) return 0;
  DGLHIP_CHECK(device_type == kDLROCM, "unsupported device type " << device_type);
  on_device(device_id, [&] {
    hip_check(hipStreamSynchronize(static_cast<hipStream_t>(stream)), "hipStreamSynchronize");
  });
  API_END();
}

int DGLStreamStreamSynchronize(int device_type, int device_id, DGLHipStreamHandle src,
                               DGLHipStreamHandle dst) {
  API_BEGIN();
  if (device_type == kDLCPU) return 0;
  on_device(device_id, [&] {
    hipEvent_t ev;
    hip_check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventRecord(ev, static_cast<hipStream_t>(src)), "hipEventRecord");
    hip_check(hipStreamWaitEvent(static_cast<hipStream_t>(dst), ev, 0), "hipStreamWaitEvent");
    hip_check(hipEventDestroy(ev), "hipEventDestroy");
  });
  API_END();
}

// ------------------------------------------------------------------ modules
int DGLModLoadFromFile(const char* file_name, const char* format, DGLHipModuleHandle* out) {
  API_BEGIN();
  (void)format;
  if (out) *out = nullptr;
  DGLHIP_CHECK(false, "cannot load module " << (file_name ? file_name : "(null)")
                      << ": kernels are compiled into libdgl_hip.so");
  API_END();
}

int DGLModImport(DGLHipModuleHandle mod, DGLHipModuleHandle dep) {
  API_BEGIN();
  (void)mod;
  (void)dep;
  DGLHIP_CHECK(false, "runtime modules are not supported by this runtime");
  API_END();
}

int DGLModGetFunction(DGLHipModuleHandle mod, const char* func_name, int query_imports,
                      DGLHipFunctionHandle* out) {
  API_BEGIN();
  (void)query_imports;
  if (out) *out = nullptr;
  DGLHIP_CHECK(mod == nullptr, "runtime modules are not supported by this runtime");
  DGLHIP_CHECK(false, "no module to look up " << (func_name ? func_name : "(null)"));
  API_END();
}

int DGLModFree(DGLHipModuleHandle mod) {
  API_BEGIN();
  DGLHIP_CHECK(mod == nullptr, "runtime modules are not supported by this runtime");
  API_END();
}

int DGLExtTypeFree(void* handle, int type_code) {
  API_BEGIN();
  DGLHIP_CHECK(handle == nullptr, "no extension type " << type_code << " is registered");
  API_END();
}

}  // extern "C"
