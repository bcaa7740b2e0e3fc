// Device-side COO -> CSR builder.
//
// Replaces the host adjacency build the reference performs before every first
// product on a device (Graph::GetAdj src/graph/graph.cc:506-554, copied to the
// device in python/dgl/graph_index.py:575-579) and, for rectangular
// send_and_recv / pull matrices, the per-call CPU rebuild in
// python/dgl/runtime/spmv.py:154-227.
//
// Algorithm: stable LSD radix sort (rocPRIM) of the edge ids keyed by row
// (ORDER_EID) or by (row, col) (ORDER_COL); a stable sort keeps ascending
// edge id as the final tie-break, which is exactly the slot order of the host
// builder. Then a gather of column ids and a boundary fill of indptr.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include "../../include/dgl_hip.h"
#include "common.h"

namespace dglhip {

#define HIP_CALL(expr)                                                        \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    DGLHIP_CHECK(_e == hipSuccess, #expr << " -> " << hipGetErrorString(_e)); \
  } while (0)

namespace {

__global__ void make_keys(int64_t nnz, const int64_t* __restrict__ row,
                          const int64_t* __restrict__ col, int64_t num_cols,
                          int order, uint64_t* __restrict__ keys,
                          int64_t* __restrict__ ids) {
  for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < nnz;
       e += int64_t(gridDim.x) * blockDim.x) {
    const uint64_t r = static_cast<uint64_t>(row[e]);
    keys[e] = order == DGLHIP_ORDER_COL ? r * uint64_t(num_cols) + uint64_t(col[e]) : r;
    ids[e] = e;
  }
}

__global__ void gather_cols(int64_t nnz, const int64_t* __restrict__ col,
                            const int64_t* __restrict__ eid,
                            int32_t* __restrict__ indices) {
  for (int64_t k = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; k < nnz;
       k += int64_t(gridDim.x) * blockDim.x)
    indices[k] = static_cast<int32_t>(col[eid[k]]);
}

// indptr[r] = first slot whose row >= r. Slot k writes the entries for the
// rows in (row[k-1], row[k]]; the last slot also closes the tail. Every entry
// is written exactly once.
__global__ void fill_indptr(int64_t nnz, int64_t num_rows,
                            const int64_t* __restrict__ row,
                            const int64_t* __restrict__ eid,
                            int64_t* __restrict__ indptr) {
  for (int64_t k = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; k < nnz;
       k += int64_t(gridDim.x) * blockDim.x) {
    const int64_t cur = row[eid[k]];
    const int64_t prev = k == 0 ? -1 : row[eid[k - 1]];
    for (int64_t r = prev + 1; r <= cur; ++r) indptr[r] = k;
    if (k == nnz - 1)
      for (int64_t r = cur + 1; r <= num_rows; ++r) indptr[r] = nnz;
  }
}

__global__ void fill_zero_indptr(int64_t n, int64_t* indptr) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x)
    indptr[i] = 0;
}

int key_bits(int64_t num_rows, int64_t num_cols, int order) {
  uint64_t maxkey = order == DGLHIP_ORDER_COL
                        ? uint64_t(num_rows) * uint64_t(std::max<int64_t>(num_cols, 1))
                        : uint64_t(num_rows);
  int bits = 1;
  while (bits < 64 && (uint64_t(1) << bits) < maxkey) ++bits;
  return bits;
}

size_t sort_temp_bytes(int64_t nnz, int bits) {
  size_t bytes = 0;
  uint64_t* k = nullptr;
  int64_t* v = nullptr;
  HIP_CALL(rocprim::radix_sort_pairs(nullptr, bytes, k, k, v, v, size_t(nnz), 0,
                                     unsigned(bits)));
  return bytes;
}

int64_t align256(int64_t x) { return (x + 255) & ~int64_t(255); }

unsigned grid_for(int64_t n) {
  return static_cast<unsigned>(std::min<int64_t>((n + 255) / 256, 65536));
}

}  // namespace
}  // namespace dglhip

using namespace dglhip;

extern "C" {

int64_t dglhip_coo_to_csr_workspace_bytes(int64_t num_rows, int64_t num_cols,
                                          int64_t nnz, int order) {
  try {
    const int bits = key_bits(num_rows, num_cols, order);
    return 3 * align256(nnz * 8) + align256(int64_t(sort_temp_bytes(nnz, bits)));
  } catch (const std::exception& e) {
    set_last_error(e.what());
    return -1;
  }
}

int dglhip_coo_to_csr_device(int64_t num_rows, int64_t num_cols, int64_t nnz,
                             const int64_t* row, const int64_t* col, int order,
                             int64_t* indptr, int32_t* indices, int64_t* eid,
                             void* workspace, int64_t workspace_bytes,
                             void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows >= 0 && num_cols >= 0 && nnz >= 0, "negative size");
  DGLHIP_CHECK(num_cols <= 0x7fffffff, "num_cols exceeds int32 column ids");
  DGLHIP_CHECK(order == DGLHIP_ORDER_EID || order == DGLHIP_ORDER_COL,
               "unknown order " << order);
  if (nnz == 0) {
    hipLaunchKernelGGL(fill_zero_indptr, dim3(grid_for(num_rows + 1)), dim3(256),
                       0, stream, num_rows + 1, indptr);
    HIP_CALL(hipGetLastError());
    return 0;
  }
  const int bits = key_bits(num_rows, num_cols, order);
  size_t temp = sort_temp_bytes(nnz, bits);
  const int64_t need = 3 * align256(nnz * 8) + align256(int64_t(temp));
  DGLHIP_CHECK(workspace && workspace_bytes >= need,
               "workspace too small: " << workspace_bytes << " < " << need);
  char* ws = static_cast<char*>(workspace);
  uint64_t* keys_in = reinterpret_cast<uint64_t*>(ws);
  uint64_t* keys_out = reinterpret_cast<uint64_t*>(ws + align256(nnz * 8));
  int64_t* ids_in = reinterpret_cast<int64_t*>(ws + 2 * align256(nnz * 8));
  void* tmp = ws + 3 * align256(nnz * 8);
  hipLaunchKernelGGL(make_keys, dim3(grid_for(nnz)), dim3(256), 0, stream, nnz,
                     row, col, num_cols, order, keys_in, ids_in);
  HIP_CALL(hipGetLastError());
  HIP_CALL(rocprim::radix_sort_pairs(tmp, temp, keys_in, keys_out, ids_in, eid,
                                     size_t(nnz), 0, unsigned(bits), stream));
  hipLaunchKernelGGL(gather_cols, dim3(grid_for(nnz)), dim3(256), 0, stream, nnz,
                     col, eid, indices);
  HIP_CALL(hipGetLastError());
  hipLaunchKernelGGL(fill_indptr, dim3(grid_for(nnz)), dim3(256), 0, stream, nnz,
                     num_rows, row, eid, indptr);
  HIP_CALL(hipGetLastError());
  API_END();
}

}  // extern "C"
