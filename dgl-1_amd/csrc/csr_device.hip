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

// ---- Groupings for the typed-block and DistMult kernels (r06) -------------
// One call each instead of a CSR build, index gathers, a repeat_interleave
// and the item list as separate host calls (≈100 µs of host time per
// relation grouping of a 30,000-edge sample, ≈80 per DistMult grouping).

// key of slot k = etype[fwd_eid[k]] (the relation of the forward CSR's slot
// k), value k; out-of-range relations are clamped into the key range (the
// grouping stays inside its arrays; typed_block_spmm checks relations where
// it is asked to)
template <typename K>
__global__ void relation_keys(int64_t nnz, int64_t num_rels, const int64_t* __restrict__ etype,
                              const int64_t* __restrict__ fwd_eid, K* __restrict__ keys,
                              int32_t* __restrict__ ids) {
  for (int64_t k = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; k < nnz;
       k += int64_t(gridDim.x) * blockDim.x) {
    const int64_t r = etype[fwd_eid[k]];
    keys[k] = static_cast<K>(r < 0 ? 0 : (r >= num_rels ? num_rels - 1 : r));
    ids[k] = static_cast<int32_t>(k);
  }
}

// keys[k] = idx[k] clamped into [0, num_rows), value k
template <typename K>
__global__ void position_keys(int64_t m, int64_t num_rows, const int64_t* __restrict__ idx,
                              K* __restrict__ keys, int32_t* __restrict__ ids) {
  for (int64_t k = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; k < m;
       k += int64_t(gridDim.x) * blockDim.x) {
    const int64_t r = idx[k];
    keys[k] = static_cast<K>(r < 0 ? 0 : (r >= num_rows ? num_rows - 1 : r));
    ids[k] = static_cast<int32_t>(k);
  }
}

// ptr[r] = first sorted position whose key >= r (keys sorted ascending)
template <typename K>
__global__ void fill_ptr_sorted(int64_t m, int64_t num_rows, const K* __restrict__ sorted,
                                int64_t* __restrict__ ptr) {
  for (int64_t k = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; k < m;
       k += int64_t(gridDim.x) * blockDim.x) {
    const int64_t cur = static_cast<int64_t>(sorted[k]);
    const int64_t prev = k == 0 ? -1 : static_cast<int64_t>(sorted[k - 1]);
    for (int64_t r = prev + 1; r <= cur; ++r) ptr[r] = k;
    if (k == m - 1)
      for (int64_t r = cur + 1; r <= num_rows; ++r) ptr[r] = m;
  }
}

// relation-major position p: the forward slot s it holds, the slot's column
// (source) and its row (destination: the row whose slot range holds s)
__global__ void relation_members(int64_t nnz, int64_t fwd_rows,
                                 const int32_t* __restrict__ sorted_slot,
                                 const int32_t* __restrict__ fwd_indices,
                                 const int64_t* __restrict__ fwd_indptr,
                                 int32_t* __restrict__ src, int64_t* __restrict__ slot,
                                 int32_t* __restrict__ dst) {
  for (int64_t p = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; p < nnz;
       p += int64_t(gridDim.x) * blockDim.x) {
    const int64_t s = sorted_slot[p];
    slot[p] = s;
    src[p] = fwd_indices[s];
    int64_t lo = 0, hi = fwd_rows - 1;  // the last row r with indptr[r] <= s
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (fwd_indptr[mid] <= s) lo = mid;
      else hi = mid - 1;
    }
    dst[p] = static_cast<int32_t>(lo);
  }
}

__global__ void copy_ids(int64_t m, const int32_t* __restrict__ from, int32_t* __restrict__ to) {
  for (int64_t k = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; k < m;
       k += int64_t(gridDim.x) * blockDim.x)
    to[k] = from[k];
}

// workspace of a grouping sort over m values with keys below num_rows:
// key and id double buffers (32-bit), rocPRIM's temporary storage, then the
// item list's scan workspace
int64_t group_sort_bytes(int64_t num_rows, int64_t m) {
  const int bits = key_bits(num_rows, 1, DGLHIP_ORDER_EID);
  return 4 * align256(m * 4) + align256(int64_t(sort_temp_bytes<uint32_t, int32_t>(m, bits)));
}

int64_t grouping_workspace_bytes(int64_t num_rows, int64_t m) {
  const int64_t items = dglhip_typed_items_workspace_bytes(num_rows);
  DGLHIP_CHECK(items >= 0, "item workspace query failed");
  return group_sort_bytes(num_rows, m) + align256(items);
}

// sort ids by key in the workspace (stable); returns the sorted key and id
// buffers through k_out / v_out
template <typename KeyFn>
void group_sort(int64_t num_rows, int64_t m, char* ws, hipStream_t stream, KeyFn&& make,
                uint32_t** k_out, int32_t** v_out) {
  const int bits = key_bits(num_rows, 1, DGLHIP_ORDER_EID);
  const int64_t kb = align256(m * 4);
  rocprim::double_buffer<uint32_t> keys(reinterpret_cast<uint32_t*>(ws),
                                        reinterpret_cast<uint32_t*>(ws + kb));
  rocprim::double_buffer<int32_t> ids(reinterpret_cast<int32_t*>(ws + 2 * kb),
                                      reinterpret_cast<int32_t*>(ws + 3 * kb));
  size_t temp = sort_temp_bytes<uint32_t, int32_t>(m, bits);
  make(keys.current(), ids.current());
  HIP_CALL(hipGetLastError());
  HIP_CALL(rocprim::radix_sort_pairs(ws + 4 * kb, temp, keys, ids, size_t(m), 0,
                                     unsigned(bits), stream));
  *k_out = keys.current();
  *v_out = ids.current();
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

int64_t dglhip_group_positions_workspace_bytes(int64_t num_rows, int64_t m) {
  try {
    return grouping_workspace_bytes(num_rows, m);
  } catch (const std::exception& e) {
    set_last_error(e.what());
    return -1;
  }
}

int dglhip_group_positions_device(int64_t num_rows, int64_t m, const int64_t* idx,
                                  int64_t bound, int64_t* ptr, int32_t* order,
                                  int64_t* item_ptr, int32_t* item_row, void* workspace,
                                  int64_t workspace_bytes_given, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows > 0 && m >= 0 && m < (int64_t(1) << 31), "bad sizes");
  DGLHIP_CHECK(bound >= num_rows + (m + DGLHIP_TYPED_CHUNK - 1) / DGLHIP_TYPED_CHUNK,
               "item bound " << bound << " below the item count's bound");
  DGLHIP_CHECK(ptr && item_ptr && item_row && workspace && (m == 0 || (idx && order)),
               "null pointer argument");
  const int64_t need = grouping_workspace_bytes(num_rows, m);
  DGLHIP_CHECK(workspace_bytes_given >= need,
               "workspace too small: " << workspace_bytes_given << " < " << need);
  char* ws = static_cast<char*>(workspace);
  const int64_t sb = group_sort_bytes(num_rows, m);
  if (m == 0) {
    hipLaunchKernelGGL(fill_zero_indptr, dim3(grid_for(num_rows + 1)), dim3(256), 0, stream,
                       num_rows + 1, ptr);
    HIP_CALL(hipGetLastError());
  } else {
    uint32_t* sk;
    int32_t* sv;
    group_sort(num_rows, m, ws, stream, [&](uint32_t* k, int32_t* v) {
      hipLaunchKernelGGL((position_keys<uint32_t>), dim3(grid_for(m)), dim3(256), 0, stream, m,
                         num_rows, idx, k, v);
    }, &sk, &sv);
    hipLaunchKernelGGL(copy_ids, dim3(grid_for(m)), dim3(256), 0, stream, m, sv, order);
    hipLaunchKernelGGL((fill_ptr_sorted<uint32_t>), dim3(grid_for(m)), dim3(256), 0, stream, m,
                       num_rows, sk, ptr);
    HIP_CALL(hipGetLastError());
  }
  const int rc = dglhip_typed_items_device(num_rows, ptr, bound, item_ptr, item_row, ws + sb,
                                           workspace_bytes_given - sb, stream);
  DGLHIP_CHECK(rc == 0, "item list failed");
  API_END();
}

int64_t dglhip_relation_groups_workspace_bytes(int64_t num_rels, int64_t nnz) {
  return dglhip_group_positions_workspace_bytes(num_rels, nnz);
}

int dglhip_relation_groups_device(int64_t num_rels, int64_t fwd_rows, int64_t nnz,
                                  const int64_t* etype, const int64_t* fwd_indptr,
                                  const int32_t* fwd_indices, const int64_t* fwd_eid,
                                  int64_t bound, int64_t* ptr, int32_t* src, int64_t* slot,
                                  int32_t* dst, int64_t* item_ptr, int32_t* item_rel,
                                  void* workspace, int64_t workspace_bytes_given,
                                  void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rels > 0 && fwd_rows >= 0 && nnz >= 0 && nnz < (int64_t(1) << 31),
               "bad sizes");
  DGLHIP_CHECK(bound >= num_rels + (nnz + DGLHIP_TYPED_CHUNK - 1) / DGLHIP_TYPED_CHUNK,
               "item bound " << bound << " below the item count's bound");
  DGLHIP_CHECK(ptr && item_ptr && item_rel && workspace &&
                   (nnz == 0 || (etype && fwd_indptr && fwd_indices && fwd_eid && src && slot &&
                                 dst && fwd_rows > 0)),
               "null pointer argument");
  const int64_t need = grouping_workspace_bytes(num_rels, nnz);
  DGLHIP_CHECK(workspace_bytes_given >= need,
               "workspace too small: " << workspace_bytes_given << " < " << need);
  char* ws = static_cast<char*>(workspace);
  const int64_t sb = group_sort_bytes(num_rels, nnz);
  if (nnz == 0) {
    hipLaunchKernelGGL(fill_zero_indptr, dim3(grid_for(num_rels + 1)), dim3(256), 0, stream,
                       num_rels + 1, ptr);
    HIP_CALL(hipGetLastError());
  } else {
    uint32_t* sk;
    int32_t* sv;
    group_sort(num_rels, nnz, ws, stream, [&](uint32_t* k, int32_t* v) {
      hipLaunchKernelGGL((relation_keys<uint32_t>), dim3(grid_for(nnz)), dim3(256), 0, stream,
                         nnz, num_rels, etype, fwd_eid, k, v);
    }, &sk, &sv);
    hipLaunchKernelGGL(relation_members, dim3(grid_for(nnz)), dim3(256), 0, stream, nnz,
                       fwd_rows, sv, fwd_indices, fwd_indptr, src, slot, dst);
    hipLaunchKernelGGL((fill_ptr_sorted<uint32_t>), dim3(grid_for(nnz)), dim3(256), 0, stream,
                       nnz, num_rels, sk, ptr);
    HIP_CALL(hipGetLastError());
  }
  const int rc = dglhip_typed_items_device(num_rels, ptr, bound, item_ptr, item_rel, ws + sb,
                                           workspace_bytes_given - sb, stream);
  DGLHIP_CHECK(rc == 0, "item list failed");
  API_END();
}

}  // extern "C"
