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

// Key of edge e: its row (ORDER_EID) or (row, col) flattened (ORDER_COL);
// the sort's values are the edge ids. K / V are 32-bit whenever the keys and
// the edge count fit (the narrow path: half the workspace at 1B edges).
template <typename K, typename V>
__global__ void make_keys(int64_t nnz, const int64_t* __restrict__ row,
                          const int64_t* __restrict__ col, int64_t num_cols,
                          int order, K* __restrict__ keys, V* __restrict__ ids) {
  for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < nnz;
       e += int64_t(gridDim.x) * blockDim.x) {
    const uint64_t r = static_cast<uint64_t>(row[e]);
    keys[e] = static_cast<K>(order == DGLHIP_ORDER_COL
                                 ? r * uint64_t(num_cols) + uint64_t(col[e]) : r);
    ids[e] = static_cast<V>(e);
  }
}

// Slot k: its edge id (widened to int64) and that edge's column.
template <typename V>
__global__ void gather_cols(int64_t nnz, const int64_t* __restrict__ col,
                            const V* __restrict__ sorted_ids,
                            int64_t* __restrict__ eid, int32_t* __restrict__ indices) {
  for (int64_t k = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; k < nnz;
       k += int64_t(gridDim.x) * blockDim.x) {
    const int64_t e = static_cast<int64_t>(sorted_ids[k]);
    eid[k] = e;
    indices[k] = static_cast<int32_t>(col[e]);
  }
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
    // rows clamped to [-1, num_rows]: an unvalidated out-of-range row gives a
    // wrong CSR, never a store outside indptr
    const int64_t cur = min(max(row[eid[k]], int64_t(-1)), num_rows);
    const int64_t prev = k == 0 ? -1 : min(max(row[eid[k - 1]], int64_t(-1)), num_rows);
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

// 32-bit keys and edge ids when both fit
bool narrow(int64_t nnz, int bits) { return bits <= 32 && nnz < (int64_t(1) << 31); }

template <typename K, typename V>
size_t sort_temp_bytes(int64_t nnz, int bits) {
  size_t bytes = 0;
  rocprim::double_buffer<K> k(nullptr, nullptr);
  rocprim::double_buffer<V> v(nullptr, nullptr);
  HIP_CALL(rocprim::radix_sort_pairs(nullptr, bytes, k, v, size_t(nnz), 0, unsigned(bits)));
  return bytes;
}

int64_t align256(int64_t x) { return (x + 255) & ~int64_t(255); }

// Workspace: key and value double buffers (the sort ping-pongs between them,
// no internal copies) + rocPRIM's small temporary storage. 16 B per edge on
// the narrow path (17 GB at RMAT-26's 1.07B edges), 32 B otherwise.
int64_t workspace_bytes(int64_t nnz, int bits) {
  if (narrow(nnz, bits))
    return 4 * align256(nnz * 4) + align256(int64_t(sort_temp_bytes<uint32_t, int32_t>(nnz, bits)));
  return 4 * align256(nnz * 8) + align256(int64_t(sort_temp_bytes<uint64_t, int64_t>(nnz, bits)));
}

unsigned grid_for(int64_t n) {
  return static_cast<unsigned>(std::min<int64_t>((n + 255) / 256, 65536));
}

template <typename K, typename V>
void build(int64_t num_rows, int64_t num_cols, int64_t nnz, const int64_t* row,
           const int64_t* col, int order, int bits, int64_t* indptr, int32_t* indices,
           int64_t* eid, char* ws, hipStream_t stream) {
  const int64_t kb = align256(nnz * int64_t(sizeof(K)));
  const int64_t vb = align256(nnz * int64_t(sizeof(V)));
  rocprim::double_buffer<K> keys(reinterpret_cast<K*>(ws), reinterpret_cast<K*>(ws + kb));
  rocprim::double_buffer<V> ids(reinterpret_cast<V*>(ws + 2 * kb),
                                reinterpret_cast<V*>(ws + 2 * kb + vb));
  void* tmp = ws + 2 * kb + 2 * vb;
  size_t temp = sort_temp_bytes<K, V>(nnz, bits);
  hipLaunchKernelGGL((make_keys<K, V>), dim3(grid_for(nnz)), dim3(256), 0, stream, nnz, row,
                     col, num_cols, order, keys.current(), ids.current());
  HIP_CALL(hipGetLastError());
  HIP_CALL(rocprim::radix_sort_pairs(tmp, temp, keys, ids, size_t(nnz), 0, unsigned(bits),
                                     stream));
  hipLaunchKernelGGL((gather_cols<V>), dim3(grid_for(nnz)), dim3(256), 0, stream, nnz, col,
                     ids.current(), eid, indices);
  HIP_CALL(hipGetLastError());
  hipLaunchKernelGGL(fill_indptr, dim3(grid_for(nnz)), dim3(256), 0, stream, nnz, num_rows,
                     row, eid, indptr);
  HIP_CALL(hipGetLastError());
}

}  // namespace
}  // namespace dglhip

using namespace dglhip;

extern "C" {

int64_t dglhip_coo_to_csr_workspace_bytes(int64_t num_rows, int64_t num_cols,
                                          int64_t nnz, int order) {
  try {
    return workspace_bytes(nnz, key_bits(num_rows, num_cols, order));
  } catch (const std::exception& e) {
    set_last_error(e.what());
    return -1;
  }
}

int dglhip_coo_to_csr_device(int64_t num_rows, int64_t num_cols, int64_t nnz,
                             const int64_t* row, const int64_t* col, int order,
                             int64_t* indptr, int32_t* indices, int64_t* eid,
                             void* workspace, int64_t workspace_bytes_given,
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
  const int64_t need = workspace_bytes(nnz, bits);
  DGLHIP_CHECK(workspace && workspace_bytes_given >= need,
               "workspace too small: " << workspace_bytes_given << " < " << need);
  char* ws = static_cast<char*>(workspace);
  if (narrow(nnz, bits))
    build<uint32_t, int32_t>(num_rows, num_cols, nnz, row, col, order, bits, indptr, indices,
                             eid, ws, stream);
  else
    build<uint64_t, int64_t>(num_rows, num_cols, nnz, row, col, order, bits, indptr, indices,
                             eid, ws, stream);
  API_END();
}

}  // extern "C"
