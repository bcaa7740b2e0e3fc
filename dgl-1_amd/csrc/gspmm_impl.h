// Shared part of the g-SpMM kernels (sum / mean / max, every message and
// edge-feature layout) and their launch logic. Included by gspmm.hip (the
// C-ABI, which only declares dispatch_sum_me / dispatch_max_me) and by
// gspmm_inst.hip, which is compiled once per (message, edge layout) pair
// (-DGSPMM_INST_MSG / -DGSPMM_INST_EM, see the Makefile) and instantiates
// them, so the kernel variants build in parallel translation units.
// Design notes: gspmm.hip header and DESIGN.md §4.1.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <initializer_list>
#include <mutex>
#include <vector>

#include "../../include/dgl_hip.h"
#include "common.h"
#include "launch.h"
#include "timing.h"

namespace dglhip {

// GAT attention dropout: keep(k, h) = hash(seed, k * H + h) >= threshold, a
// stateless counter hash shared by the fused forward (gat_fused.hip), the
// backward epilogues (gspmm.hip) and the host mask.
// lowbias32 (a 32-bit integer finaliser); two rounds over the 64-bit index
__host__ __device__ __forceinline__ uint32_t gat_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__host__ __device__ __forceinline__ bool gat_keep(uint64_t seed, int64_t idx, uint32_t thr) {
  const uint64_t i = static_cast<uint64_t>(idx);
  const uint32_t r = gat_mix32(gat_mix32(static_cast<uint32_t>(i) ^ static_cast<uint32_t>(seed)) ^
                               (static_cast<uint32_t>(i >> 32) + static_cast<uint32_t>(seed >> 32) +
                                0x9e3779b9u));
  return r >= thr;
}

// keep iff hash >= threshold: P(keep) = 1 - p
static inline uint32_t gat_drop_threshold(float p) {
  const double t = static_cast<double>(p) * 4294967296.0;
  return t >= 4294967295.0 ? 0xffffffffu : static_cast<uint32_t>(t);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int VEC> struct Vec;
template <> struct Vec<1> {
  typedef float T;
  static __device__ __forceinline__ T zero() { return 0.0f; }
  static __device__ __forceinline__ T splat(float x) { return x; }
  static __device__ __forceinline__ T fma(T a, T b, T c) { return __builtin_fmaf(a, b, c); }
  static __device__ __forceinline__ T max(T a, T b) { return a > b ? a : b; }
};
template <> struct Vec<2> {
  typedef f32x2 T;
  static __device__ __forceinline__ T zero() { return T{0.0f, 0.0f}; }
  static __device__ __forceinline__ T splat(float x) { return T{x, x}; }
  static __device__ __forceinline__ T fma(T a, T b, T c) {
    return T{__builtin_fmaf(a.x, b.x, c.x), __builtin_fmaf(a.y, b.y, c.y)};
  }
};
template <> struct Vec<4> {
  typedef f32x4 T;
  static __device__ __forceinline__ T zero() { return T{0.0f, 0.0f, 0.0f, 0.0f}; }
  static __device__ __forceinline__ T splat(float x) { return T{x, x, x, x}; }
  static __device__ __forceinline__ T fma(T a, T b, T c) {
    return T{__builtin_fmaf(a.x, b.x, c.x), __builtin_fmaf(a.y, b.y, c.y),
             __builtin_fmaf(a.z, b.z, c.z), __builtin_fmaf(a.w, b.w, c.w)};
  }
};

template <int VEC>
__device__ __forceinline__ typename Vec<VEC>::T ldv(const float* p) {
  return *reinterpret_cast<const typename Vec<VEC>::T*>(p);
}
template <int VEC>
__device__ __forceinline__ void stv(float* p, typename Vec<VEC>::T v) {
  *reinterpret_cast<typename Vec<VEC>::T*>(p) = v;
}

// DGLHIP_MSG_COPY_U_BF16: copy_u over source rows held as bf16 bits. Each
// value widens exactly to fp32 (bits << 16) before it enters the fp32 chain,
// so results equal the fp32 kernel on the widened rows, bit for bit.
__host__ __device__ constexpr bool copies_u(int msg) {
  return msg == DGLHIP_MSG_COPY_U || msg == DGLHIP_MSG_COPY_U_BF16;
}

template <int VEC>
__device__ __forceinline__ typename Vec<VEC>::T gather_bf16(const float* ufeat, int32_t col,
                                                            int64_t F, int64_t f0);
template <>
__device__ __forceinline__ float gather_bf16<1>(const float* ufeat, int32_t col, int64_t F,
                                                int64_t f0) {
  const uint16_t b = reinterpret_cast<const uint16_t*>(ufeat)[int64_t(col) * F + f0];
  return __uint_as_float(uint32_t(b) << 16);
}
template <>
__device__ __forceinline__ f32x2 gather_bf16<2>(const float* ufeat, int32_t col, int64_t F,
                                                int64_t f0) {
  // two consecutive bf16 values, element f0 in the low half (little endian)
  const uint32_t w = *reinterpret_cast<const uint32_t*>(
      reinterpret_cast<const uint16_t*>(ufeat) + int64_t(col) * F + f0);
  return f32x2{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
}
template <>
__device__ __forceinline__ f32x4 gather_bf16<4>(const float* ufeat, int32_t col, int64_t F,
                                                int64_t f0) {
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  const u32x2 w = *reinterpret_cast<const u32x2*>(
      reinterpret_cast<const uint16_t*>(ufeat) + int64_t(col) * F + f0);
  return f32x4{__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
               __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u)};
}

// Cache policy of the source-row gathers and output stores (POL template
// parameter; copy_u + sum at VEC 2 x 64 lanes, selected by dglhip_set_cache_policy):
//  POL_DEFAULT : default policy everywhere.
//  POL_NT      : every gather and the output store non-temporal.
//  POL_HOT     : column ids carry a "hot source" flag in bit 31 (set by the host on
//                the sources with the most out-edges); hot rows load with the
//                default policy, all other rows and the output non-temporal, so
//                once-read traffic does not evict the rows that are read again.
//  POL_NT_OUT  : only the output store non-temporal.
enum { POL_DEFAULT = 0, POL_NT = 1, POL_HOT = 2, POL_NT_OUT = 3 };

// BUF: the row is wave-uniform (a whole wave per row, the column id from the
// scalar slot stream): gather it through a buffer descriptor built from the
// row's address, so every gather in flight shares the lane's one 32-bit byte
// offset instead of holding a 64-bit address of its own (VGPRs -> waves per
// SIMD). Same loads, same values.
template <int VEC>
__device__ __forceinline__ typename Vec<VEC>::T gather_row_buf(const float* row, int64_t F,
                                                               int64_t f0) {
  typedef typename Vec<VEC>::T V;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(row), 0, static_cast<int>(F * int64_t(sizeof(float))), 0x00020000);
  const uint32_t off = static_cast<uint32_t>(f0 * int64_t(sizeof(float)));
  if (VEC == 4) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 w = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    return *reinterpret_cast<const V*>(&w);
  }
  if (VEC == 2) {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 w = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    return *reinterpret_cast<const V*>(&w);
  }
  const unsigned int w = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
  return *reinterpret_cast<const V*>(&w);
}

template <int VEC, int POL, bool BUF = false>
__device__ __forceinline__ typename Vec<VEC>::T gather_row(const float* __restrict__ ufeat,
                                                           int32_t col, int64_t F, int64_t f0) {
  typedef typename Vec<VEC>::T V;
  if (BUF && (POL == POL_DEFAULT || POL == POL_NT_OUT))
    return gather_row_buf<VEC>(ufeat + int64_t(col) * F, F, f0);
  if (POL == POL_NT) {
    return __builtin_nontemporal_load(reinterpret_cast<const V*>(ufeat + int64_t(col) * F + f0));
  } else if (POL == POL_HOT) {
    const V* p = reinterpret_cast<const V*>(ufeat + int64_t(col & 0x7fffffff) * F + f0);
    if (col < 0) return *p;  // wave-uniform: col comes from the scalar slot stream
    return __builtin_nontemporal_load(p);
  }
  return ldv<VEC>(ufeat + int64_t(col) * F + f0);
}

// Output rows: non-temporal under every policy but the default. The policy is
// a template parameter, not a runtime flag: the compiler merges a branch
// between a plain and a non-temporal store into one plain store.
template <int VEC, int POL>
__device__ __forceinline__ void store_row(float* p, typename Vec<VEC>::T v) {
  if (POL == POL_DEFAULT) stv<VEC>(p, v);
  else __builtin_nontemporal_store(v, reinterpret_cast<typename Vec<VEC>::T*>(p));
}

// Edge-feature layouts (EM template parameter):
//  EM_FULL   : one value per edge and feature, efeat[e, f]
//  EM_SCALAR : one scalar per edge broadcast over the row, efeat[e]
//  EM_HEAD   : one scalar per edge and head, efeat[e, f / D] with D = F / elen
//              (GAT's (E, H, 1) attention against (N, H, D) features)
enum { EM_FULL = 0, EM_SCALAR = 1, EM_HEAD = 2 };

// Message for slot k as a vector of VEC features starting at feature f0.
//  COPY_U : u                     U_MUL_E: w * u (fused into the reducer)
//  COPY_E : e
// `eoff` is the edge-feature column of f0 (f0, 0 or f0 / D by EM).
template <int VEC, int MSG, int EM, int POL = POL_DEFAULT, bool BUF = false>
struct SlotLoad {
  typedef typename Vec<VEC>::T V;
  V u;
  V e;
  __device__ __forceinline__ void load(const float* __restrict__ ufeat,
                                       const float* __restrict__ efeat, int64_t ldu,
                                       int64_t F, int64_t f0, int64_t elen, int64_t eoff,
                                       int32_t src, int64_t edge) {
    // ldu: row stride of ufeat in elements (F, or a padded width)
    if (MSG == DGLHIP_MSG_COPY_U_BF16) u = gather_bf16<VEC>(ufeat, src, ldu, f0);
    else if (MSG != DGLHIP_MSG_COPY_E) u = gather_row<VEC, POL, BUF>(ufeat, src, ldu, f0);
    if (!copies_u(MSG)) {
      if (EM == EM_FULL) e = ldv<VEC>(efeat + edge * F + f0);
      else e = Vec<VEC>::splat(efeat[edge * elen + eoff]);
    }
  }
};

// Sequential reduction of slots [beg, end) of one row for the VEC features at
// f0: the fma chain the reference's product runs (see the file header).
template <int VEC, int UNROLL, int MSG, int EM, bool USE_EID, int POL = POL_DEFAULT,
          bool BUF = false>
__device__ __forceinline__ typename Vec<VEC>::T reduce_range(
    typename Vec<VEC>::T acc, int64_t beg, int64_t end, int64_t ldu, int64_t F, int64_t f0,
    int64_t elen, int64_t eoff, const int32_t* __restrict__ indices,
    const int64_t* __restrict__ eid, const float* __restrict__ ufeat,
    const float* __restrict__ efeat) {
  int64_t k = beg;
  for (; k + UNROLL <= end; k += UNROLL) {
    SlotLoad<VEC, MSG, EM, POL, BUF> s[UNROLL];
#pragma unroll
    for (int j = 0; j < UNROLL; ++j)
      s[j].load(ufeat, efeat, ldu, F, f0, elen, eoff, indices[k + j],
                copies_u(MSG) ? 0 : (USE_EID ? eid[k + j] : k + j));
#pragma unroll
    for (int j = 0; j < UNROLL; ++j) {
      if (copies_u(MSG)) acc += s[j].u;
      else if (MSG == DGLHIP_MSG_COPY_E) acc += s[j].e;
      else acc = Vec<VEC>::fma(s[j].e, s[j].u, acc);
    }
  }
  // the last rem < UNROLL slots as one predicated batch: all their gathers in
  // flight together (a slot-by-slot tail would serialise up to UNROLL - 1
  // load latencies per row, which dominates rows shorter than UNROLL)
  const int64_t rem = end - k;
  if (rem > 0) {
    SlotLoad<VEC, MSG, EM, POL, BUF> s[UNROLL];
#pragma unroll
    for (int j = 0; j < UNROLL - 1; ++j)
      if (j < rem)
        s[j].load(ufeat, efeat, ldu, F, f0, elen, eoff, indices[k + j],
                  copies_u(MSG) ? 0 : (USE_EID ? eid[k + j] : k + j));
#pragma unroll
    for (int j = 0; j < UNROLL - 1; ++j) {
      if (j < rem) {
        if (copies_u(MSG)) acc += s[j].u;
        else if (MSG == DGLHIP_MSG_COPY_E) acc += s[j].e;
        else acc = Vec<VEC>::fma(s[j].e, s[j].u, acc);
      }
    }
  }
  return acc;
}

// Software-pipelined variant of reduce_range (copy_u only): the gathers of
// batch t+1 are issued before batch t is accumulated, so 2 x UNROLL row
// reads stay in flight across iterations instead of draining every batch.
// Same per-element operation order (bit-identical results).
template <int VEC, int UNROLL>
__device__ __forceinline__ typename Vec<VEC>::T reduce_range_pipelined(
    typename Vec<VEC>::T acc, int64_t beg, int64_t end, int64_t ldu, int64_t f0,
    const int32_t* __restrict__ indices, const float* __restrict__ ufeat) {
  typedef typename Vec<VEC>::T V;
  int64_t k = beg;
  if (k + UNROLL <= end) {
    V cur[UNROLL];
#pragma unroll
    for (int j = 0; j < UNROLL; ++j) cur[j] = ldv<VEC>(ufeat + int64_t(indices[k + j]) * ldu + f0);
    k += UNROLL;
    for (; k + UNROLL <= end; k += UNROLL) {
      V nxt[UNROLL];
#pragma unroll
      for (int j = 0; j < UNROLL; ++j)
        nxt[j] = ldv<VEC>(ufeat + int64_t(indices[k + j]) * ldu + f0);
#pragma unroll
      for (int j = 0; j < UNROLL; ++j) acc += cur[j];
#pragma unroll
      for (int j = 0; j < UNROLL; ++j) cur[j] = nxt[j];
    }
#pragma unroll
    for (int j = 0; j < UNROLL; ++j) acc += cur[j];
  }
  for (; k < end; ++k) acc += ldv<VEC>(ufeat + int64_t(indices[k]) * ldu + f0);
  return acc;
}

// Cache policy of the running output row of accumulating items (the
// blocked schedule's launches after the first read and rewrite each item's
// row: 30 % of the fabric bytes, streaming through the L2s that hold the
// gathered source block). RP (dglhip_set_row_policy, a study knob):
//   0  plain load and store;
//   1  non-temporal load and store;
//   2  non-temporal load, store with sc1 (the line leaves the XCD's L2): the
//      default (Reddit-shaped headline 3.83 -> 3.74 ms; policy 1 4.10; the
//      source rows keep the L2s);
//   3  load with sc0 sc1 and store with sc1 (system scope both ways);
//   4  plain load, store with sc1.
// With 2-4 the first launch (which only writes its rows) stores with sc1 too.
// Same values in every variant.
template <int VEC, int RP>
__device__ __forceinline__ typename Vec<VEC>::T load_out(const float* row, int64_t f0) {
  typedef typename Vec<VEC>::T V;
  if (RP == 1 || RP == 2) return __builtin_nontemporal_load(reinterpret_cast<const V*>(row + f0));
  if (RP == 3 && VEC == 2) {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(row), 0, 0x7fffffff, 0x00020000);
    const u32x2 w = __builtin_amdgcn_raw_buffer_load_b64(
        r, static_cast<uint32_t>(f0 * int64_t(sizeof(float))), 0, 1 | 16);
    return *reinterpret_cast<const V*>(&w);
  }
  return ldv<VEC>(row + f0);
}

template <int VEC, int RP>
__device__ __forceinline__ void store_out(float* row, int64_t f0, typename Vec<VEC>::T v) {
  typedef typename Vec<VEC>::T V;
  if (RP == 1) {
    __builtin_nontemporal_store(v, reinterpret_cast<V*>(row + f0));
    return;
  }
  if ((RP == 2 || RP == 3 || RP == 4) && VEC == 2) {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(row, 0, 0x7fffffff,
                                                                       0x00020000);
    __builtin_amdgcn_raw_buffer_store_b64(*reinterpret_cast<const u32x2*>(&v), r,
                                          static_cast<uint32_t>(f0 * int64_t(sizeof(float))),
                                          0, 16);
    return;
  }
  if ((RP == 2 || RP == 3 || RP == 4) && VEC == 4) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(row, 0, 0x7fffffff,
                                                                       0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(&v), r,
                                           static_cast<uint32_t>(f0 * int64_t(sizeof(float))),
                                           0, 16);
    return;
  }
  stv<VEC>(row + f0, v);
}

// Sum-reduce kernel (also MEAN). GROUP lanes per work item, VEC floats per
// lane. A work item is a whole row (CHUNKED = false: item i = row_order[i]),
// or a slot range [chunk_beg[i], chunk_end[i]) whose sum goes to out[i, :]
// (CHUNKED = true). With ACCUM the chain continues from the value already in
// out[i, :] (segment-by-segment evaluation of one sequential chain); with
// MEAN and ACCUM on whole rows the row's mean is added to the value in
// out[i, :] (out + mean: a sum of two terms, the same bits either way round).
template <int VEC, int GROUP, int UNROLL, int MSG, int EM, bool MEAN, bool CHUNKED,
          bool ACCUM, bool PIPE = false, int POL = POL_DEFAULT, bool BUF = false, int RP = 0>
__global__ __launch_bounds__(256) void gspmm_sum_kernel(
    int64_t num_items, int64_t F, int64_t elen, int64_t ldu,
    const int64_t* __restrict__ indptr,
    const int32_t* __restrict__ indices, const int64_t* __restrict__ eid,
    const float* __restrict__ ufeat, const float* __restrict__ efeat,
    float* __restrict__ out, const int32_t* __restrict__ row_order,
    const int64_t* __restrict__ chunk_beg, const int64_t* __restrict__ chunk_end) {
  typedef typename Vec<VEC>::T V;
  constexpr int ITEMS_PER_WAVE = 64 / GROUP;
  const int lane = threadIdx.x & 63;
  // wave index is uniform; make that explicit so slot data goes through SGPRs
  const int64_t wave =
      block_linear() * (blockDim.x >> 6) +
      __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int64_t it = wave * ITEMS_PER_WAVE + (GROUP == 64 ? 0 : lane / GROUP);
  if (it >= num_items) return;
  const int gl = GROUP == 64 ? lane : (lane % GROUP);
  int64_t row, beg, end;
  if (CHUNKED) {
    // item it: slots [chunk_beg[it], chunk_end[it]) into row row_order[it]
    // (the blocked schedule's items), or into partial row it (heavy-row
    // chunks, row ranges); the three loads are independent
    row = row_order ? row_order[it] : it;
    if (GROUP == 64) row = __builtin_amdgcn_readfirstlane(static_cast<int>(row));
    beg = chunk_beg[it];
    end = chunk_end[it];
  } else {
    row = row_order ? row_order[it] : it;
    if (GROUP == 64) row = __builtin_amdgcn_readfirstlane(static_cast<int>(row));
    beg = indptr[row];
    end = indptr[row + 1];
  }
  for (int64_t f0 = int64_t(gl) * VEC; f0 < F; f0 += int64_t(GROUP) * VEC) {
    const int64_t eoff = EM == EM_HEAD ? f0 / (F / elen) : (EM == EM_FULL ? f0 : 0);
    constexpr bool ADD_MEAN = MEAN && ACCUM && !CHUNKED;
    V acc = (ACCUM && !ADD_MEAN) ? load_out<VEC, RP>(out + row * F, f0) : Vec<VEC>::zero();
    if (PIPE && MSG == DGLHIP_MSG_COPY_U)
      acc = reduce_range_pipelined<VEC, UNROLL>(acc, beg, end, ldu, f0, indices, ufeat);
    else if (copies_u(MSG) || eid != nullptr)  // uniform branch
      acc = reduce_range<VEC, UNROLL, MSG, EM, true, POL, BUF && GROUP == 64>(
          acc, beg, end, ldu, F, f0, elen, eoff, indices, eid, ufeat, efeat);
    else
      acc = reduce_range<VEC, UNROLL, MSG, EM, false>(acc, beg, end, ldu, F, f0, elen, eoff, indices,
                                                      eid, ufeat, efeat);
    if (!CHUNKED && MEAN && end - beg > 1)
      acc = acc / Vec<VEC>::splat(static_cast<float>(end - beg));
    if (ADD_MEAN) acc = ldv<VEC>(out + row * F + f0) + acc;
    if (RP) store_out<VEC, RP>(out + row * F, f0, acc);
    else store_row<VEC, POL>(out + row * F + f0, acc);
  }
}

// Combine the chunk partials of each heavy row in chunk order:
// out[row] = ((p0 + p1) + p2) + ... (deterministic), then MEAN scaling; with
// ACCUM the row's running value comes first: out[row] = ((out[row] + p0) + p1) ...;
// with MEAN and ACCUM the mean is added to it: out[row] + (p0 + p1 + ...) / deg
template <bool MEAN, bool ACCUM>
__global__ __launch_bounds__(256) void gspmm_combine_kernel(
    int64_t num_heavy, int64_t F, const int64_t* __restrict__ indptr,
    const int32_t* __restrict__ heavy_rows, const int64_t* __restrict__ heavy_chunk_ptr,
    const float* __restrict__ partial, float* __restrict__ out) {
  const int64_t wave = block_linear() * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wave >= num_heavy) return;
  const int lane = threadIdx.x & 63;
  const int64_t row = heavy_rows[wave];
  const int64_t c0 = heavy_chunk_ptr[wave], c1 = heavy_chunk_ptr[wave + 1];
  const float deg = static_cast<float>(indptr[row + 1] - indptr[row]);
  for (int64_t f = lane; f < F; f += 64) {
    float acc = (ACCUM && !MEAN) ? out[row * F + f] + partial[c0 * F + f] : partial[c0 * F + f];
    for (int64_t c = c0 + 1; c < c1; ++c) acc += partial[c * F + f];
    if (MEAN && deg > 1.0f) acc = acc / deg;
    if (MEAN && ACCUM) acc = out[row * F + f] + acc;
    out[row * F + f] = acc;
  }
}

// Max-reduce kernel with argmax slot: first slot wins ties (a strict running
// max over the mailbox, seeded with the first message), 0 / -1 for rows
// without slots. Same lane mapping as the sum kernel (GROUP lanes per row,
// VEC features per lane, UNROLL gathers in flight); the compares then run
// slot by slot in CSR order, so the argmax is the one the sequential
// reduction picks.
template <int VEC, int UNROLL, int MSG, int EM, bool USE_EID>
__device__ __forceinline__ void max_row(int64_t row, int gl, int group, int64_t beg,
                                        int64_t end, int64_t F, int64_t elen,
                                        const int32_t* __restrict__ indices,
                                        const int64_t* __restrict__ eid,
                                        const float* __restrict__ ufeat,
                                        const float* __restrict__ efeat,
                                        float* __restrict__ out, int64_t* __restrict__ arg_out,
                                        bool prev = false) {
  typedef typename Vec<VEC>::T V;
  auto message = [](const SlotLoad<VEC, MSG, EM>& s) -> V {
    if (copies_u(MSG)) return s.u;
    if (MSG == DGLHIP_MSG_COPY_E) return s.e;
    return s.u * s.e;
  };
  auto edge = [&](int64_t k) -> int64_t {
    return copies_u(MSG) ? 0 : (USE_EID ? eid[k] : k);
  };
  for (int64_t f0 = int64_t(gl) * VEC; f0 < F; f0 += int64_t(group) * VEC) {
    const int64_t eoff = EM == EM_HEAD ? f0 / (F / elen) : (EM == EM_FULL ? f0 : 0);
    V best = Vec<VEC>::zero();
    int64_t arg[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) arg[i] = -1;
    int64_t k = beg;
    if (prev) {  // the row's earlier slots (a previous source block): continue from them
      best = ldv<VEC>(out + row * F + f0);
#pragma unroll
      for (int i = 0; i < VEC; ++i) arg[i] = arg_out ? arg_out[row * F + f0 + i] : -1;
    } else if (k < end) {
      SlotLoad<VEC, MSG, EM> s;
      s.load(ufeat, efeat, F, F, f0, elen, eoff, indices[k], edge(k));
      best = message(s);
#pragma unroll
      for (int i = 0; i < VEC; ++i) arg[i] = k;
      ++k;
    }
    for (; k + UNROLL <= end; k += UNROLL) {
      SlotLoad<VEC, MSG, EM> s[UNROLL];
#pragma unroll
      for (int j = 0; j < UNROLL; ++j)
        s[j].load(ufeat, efeat, F, F, f0, elen, eoff, indices[k + j], edge(k + j));
#pragma unroll
      for (int j = 0; j < UNROLL; ++j) {
        const V x = message(s[j]);
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const float xi = reinterpret_cast<const float*>(&x)[i];
          float& bi = reinterpret_cast<float*>(&best)[i];
          if (xi > bi) { bi = xi; arg[i] = k + j; }
        }
      }
    }
    const int64_t rem = end - k;  // the last < UNROLL slots: one predicated batch
    if (rem > 0) {
      SlotLoad<VEC, MSG, EM> s[UNROLL];
#pragma unroll
      for (int j = 0; j < UNROLL - 1; ++j)
        if (j < rem) s[j].load(ufeat, efeat, F, F, f0, elen, eoff, indices[k + j], edge(k + j));
#pragma unroll
      for (int j = 0; j < UNROLL - 1; ++j) {
        if (j < rem) {
          const V x = message(s[j]);
#pragma unroll
          for (int i = 0; i < VEC; ++i) {
            const float xi = reinterpret_cast<const float*>(&x)[i];
            float& bi = reinterpret_cast<float*>(&best)[i];
            if (xi > bi) { bi = xi; arg[i] = k + j; }
          }
        }
      }
    }
    stv<VEC>(out + row * F + f0, best);
    if (arg_out) {
#pragma unroll
      for (int i = 0; i < VEC; ++i) arg_out[row * F + f0 + i] = arg[i];
    }
  }
}

template <int VEC, int GROUP, int UNROLL, int MSG, int EM>
__global__ __launch_bounds__(256) void gspmm_max_kernel(
    int64_t num_rows, int64_t F, int64_t elen, const int64_t* __restrict__ indptr,
    const int32_t* __restrict__ indices, const int64_t* __restrict__ eid,
    const float* __restrict__ ufeat, const float* __restrict__ efeat,
    float* __restrict__ out, int64_t* __restrict__ arg_out,
    const int32_t* __restrict__ row_order, const int64_t* __restrict__ row_beg,
    const int64_t* __restrict__ row_end, int accumulate) {
  constexpr int ITEMS_PER_WAVE = 64 / GROUP;
  const int lane = threadIdx.x & 63;
  const int64_t wave =
      block_linear() * (blockDim.x >> 6) +
      __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int64_t it = wave * ITEMS_PER_WAVE + (GROUP == 64 ? 0 : lane / GROUP);
  if (it >= num_rows) return;
  const int gl = GROUP == 64 ? lane : (lane % GROUP);
  int64_t row = row_order ? row_order[it] : it;
  if (GROUP == 64) row = __builtin_amdgcn_readfirstlane(static_cast<int>(row));
  // row ranges (source-blocked schedule): the row's slots [row_beg, row_end)
  // of this block; with accumulate, continue from the earlier blocks' max
  const int64_t rs = indptr[row];
  const int64_t beg = row_beg ? row_beg[row] : rs;
  const int64_t end = row_end ? row_end[row] : indptr[row + 1];
  if (accumulate && beg == end) return;  // nothing new: the row keeps its value
  const bool prev = accumulate && beg > rs;
  if (copies_u(MSG) || eid != nullptr)  // uniform branch
    max_row<VEC, UNROLL, MSG, EM, true>(row, gl, GROUP, beg, end, F, elen, indices, eid, ufeat,
                                        efeat, out, arg_out, prev);
  else
    max_row<VEC, UNROLL, MSG, EM, false>(row, gl, GROUP, beg, end, F, elen, indices, eid,
                                         ufeat, efeat, out, arg_out, prev);
}

// ---------------------------------------------------------------------------
// Dispatch
// ---------------------------------------------------------------------------
// Widest per-lane vector the row length and every feature pointer allow.
static inline int pick_vec(int64_t F, std::initializer_list<const void*> ptrs) {
  auto aligned = [&](int bytes) {
    for (const void* p : ptrs)
      if (p && (reinterpret_cast<uintptr_t>(p) % bytes) != 0) return false;
    return true;
  };
  // no VEC 4 by default: at F=256 one 1-KB row per wave instruction (8 gathers
  // in flight) ran 16.3 ms against 15.7 ms for two VEC-2 passes with 16 in
  // flight (tools/feat_sweep.py, Reddit-shaped graph)
  if (F % 2 == 0 && F >= 4 && aligned(8)) return 2;
  return 1;
}

static inline int pick_group(int64_t F, int vec) {
  const int64_t lanes = (F + vec - 1) / vec;
  int g = 1;
  while (g < lanes && g < 64) g <<= 1;
  return g;
}

// Rows of 16..64 floats take a whole wave each (idle lanes) rather than
// sharing one: the slot stream is then wave-uniform (column ids through the
// scalar cache) instead of a per-lane index load ahead of every gather.
// tools/feat_sweep.py, Reddit-shaped graph: F=16 2.18 -> 1.73 ms, F=32
// 2.12 -> 1.74 ms, F=64 level.
static inline void one_row_per_wave(int64_t F, int& vec, int& group) {
  if (group < 64 && F >= 16) {
    vec = 1;
    group = 64;
  }
}

struct SumLaunch {
  int64_t num_items, F, elen;
  const int64_t* indptr;
  const int32_t* indices;
  const int64_t* eid;
  const float* ufeat;
  const float* efeat;
  float* out;
  const int32_t* row_order;
  const int64_t* chunk_beg;  // non-null: chunked launch (partials to `out`)
  const int64_t* chunk_end;
  bool accumulate;           // continue each item's chain from the value in `out`
  bool nt_out = false;       // non-temporal output stores (see stream_output)
  int64_t ldu = 0;           // ufeat row stride in elements (0: F)
};

// Outputs past twice the 256 MiB Infinity Cache are stored non-temporally
// (POL_NT_OUT): streamed out, they would evict the feature rows that are
// gathered again (RMAT-26, 34 GB out: 94.1 -> 89.5 ms,
// tools/cache_policy_study.py). Covers copy_u + sum at VEC 2 x 64 lanes.
static inline bool stream_output(int64_t rows, int64_t feat_len) {
  return rows * feat_len * int64_t(sizeof(float)) > (int64_t(512) << 20);
}

// Tuning override for the copy_u + sum shape (dglhip_set_spmm_variant);
// 0 = automatic choice.
extern int g_var_vec, g_var_group, g_var_unroll, g_var_pipe;
// Cache policy for copy_u + sum at VEC 2 x 64 lanes (dglhip_set_cache_policy).
// -1: automatic (non-temporal output past 512 MiB, default otherwise).
extern int g_cache_policy;
// Row gathers of copy_u + sum at VEC 2 x 64 lanes through buffer descriptors
// (dglhip_set_gather_mode), a bit mask: bit 0 the one-launch rows and the
// heavy-row chunk launches, bit 1 the blocked schedule's item launches, the
// first block's included (the default, 2); 0 global loads everywhere.
extern int g_gather_buf;
// Running-row cache policy of the blocked schedule's copy_u + sum item
// launches (load_out / store_out; dglhip_set_row_policy): 2 by default. It
// applies where no output cache policy does (g_cache_policy automatic with
// an output under twice the Infinity Cache, or 0): an explicit or automatic
// non-temporal output (POL_NT_OUT and the study policies) takes precedence.
extern int g_row_pol;

template <int VEC, int GROUP, int MSG, int EM, bool MEAN, int UNROLL_OVERRIDE = 0,
          bool PIPE = false>
static inline void launch_sum(const SumLaunch& a, hipStream_t stream) {
  // 16 row gathers in flight per lane group: measured +22% over 8 on HBM-bound
  // RMAT (tools/kernel_sweep.py), neutral on the MALL-resident Reddit table
  constexpr int UNROLL = UNROLL_OVERRIDE ? UNROLL_OVERRIDE : ((VEC == 4) ? 8 : 16);
  constexpr int ITEMS_PER_BLOCK = 4 * (64 / GROUP);
  const int64_t blocks = (a.num_items + ITEMS_PER_BLOCK - 1) / ITEMS_PER_BLOCK;
  DGLHIP_CHECK(blocks <= 0x7fffffff, "grid too large: " << blocks);
  if (blocks == 0) return;
  constexpr bool POL_OK = MSG == DGLHIP_MSG_COPY_U && VEC == 2 && GROUP == 64 && !MEAN &&
                         !PIPE && UNROLL_OVERRIDE == 0;
  const int pol = !POL_OK ? POL_DEFAULT
                  : g_cache_policy >= 0 ? g_cache_policy
                  : a.nt_out ? POL_NT_OUT : POL_DEFAULT;
  timed_launch(stream, [&] {
    // the running-row cache policy study (dglhip_set_row_policy): only the
    // shapes POL_OK covers are instantiated
    if constexpr (POL_OK) {
      // the blocked schedule's items only (item rows given; heavy-row chunk
      // and row-range launches keep their own policy: r04 ADVICE)
      if (a.chunk_beg && a.row_order && pol == POL_DEFAULT && g_row_pol > 0 &&
          (a.accumulate || g_row_pol >= 2)) {
#define DGLHIP_RP_LAUNCH_B(ACC, RPV, B)                                                         \
  hipLaunchKernelGGL((gspmm_sum_kernel<VEC, GROUP, UNROLL, MSG, EM, MEAN, true, ACC, false,     \
                                       POL_DEFAULT, B, RPV>),                                   \
                     grid_1d(blocks), dim3(256), 0, stream, a.num_items, a.F, a.elen,           \
                     a.ldu ? a.ldu : a.F, a.indptr, a.indices, a.eid, a.ufeat, a.efeat, a.out,  \
                     a.row_order, a.chunk_beg, a.chunk_end)
#define DGLHIP_RP_LAUNCH(ACC, RPV) DGLHIP_RP_LAUNCH_B(ACC, RPV, false)
        if ((g_gather_buf & 2) && g_row_pol == 2) {
          // the default: row gathers through per-row buffer descriptors (the
          // row base in SGPRs, one lane offset for all 16: 42 instead of 70
          // VGPRs, 8 waves per SIMD instead of 7; Reddit-shaped headline
          // 3.74 -> 3.61 ms, same bits, tools/gather_mode_ab.py)
          if (!a.accumulate) DGLHIP_RP_LAUNCH_B(false, 4, true);
          else DGLHIP_RP_LAUNCH_B(true, 2, true);
          return;
        }
        if (!a.accumulate) DGLHIP_RP_LAUNCH(false, 4);  // the first launch: stores only
        else if (g_row_pol == 1) DGLHIP_RP_LAUNCH(true, 1);
        else if (g_row_pol == 2) DGLHIP_RP_LAUNCH(true, 2);
        else if (g_row_pol == 3) DGLHIP_RP_LAUNCH(true, 3);
        else DGLHIP_RP_LAUNCH(true, 4);
#undef DGLHIP_RP_LAUNCH
#undef DGLHIP_RP_LAUNCH_B
        return;
      }
    }
#define DGLHIP_POL_LAUNCH_B(CH, P, B)                                                      \
  hipLaunchKernelGGL((gspmm_sum_kernel<VEC, GROUP, UNROLL, MSG, EM, false, CH, false, false, P, B>), \
                     grid_1d(blocks), dim3(256), 0, stream, a.num_items,   \
                     a.F, a.elen, a.ldu ? a.ldu : a.F, a.indptr, a.indices, a.eid, a.ufeat, a.efeat, a.out,         \
                     a.row_order, a.chunk_beg, a.chunk_end)
#define DGLHIP_POL_LAUNCH(CH, P) DGLHIP_POL_LAUNCH_B(CH, P, false)
    if (POL_OK && (g_gather_buf & 1) && !a.accumulate && (pol == POL_DEFAULT || pol == POL_NT_OUT)) {
      // row gathers through buffer descriptors (gather_row_buf)
      const bool ch = a.chunk_beg != nullptr;
      if (pol == POL_DEFAULT) { if (ch) DGLHIP_POL_LAUNCH_B(true, POL_DEFAULT, true); else DGLHIP_POL_LAUNCH_B(false, POL_DEFAULT, true); }
      else { if (ch) DGLHIP_POL_LAUNCH_B(true, POL_NT_OUT, true); else DGLHIP_POL_LAUNCH_B(false, POL_NT_OUT, true); }
    } else if (POL_OK && pol != POL_DEFAULT && !a.accumulate) {
      const bool ch = a.chunk_beg != nullptr;
      if (pol == POL_NT) { if (ch) DGLHIP_POL_LAUNCH(true, POL_NT); else DGLHIP_POL_LAUNCH(false, POL_NT); }
      else if (pol == POL_HOT) { if (ch) DGLHIP_POL_LAUNCH(true, POL_HOT); else DGLHIP_POL_LAUNCH(false, POL_HOT); }
      else { if (ch) DGLHIP_POL_LAUNCH(true, POL_NT_OUT); else DGLHIP_POL_LAUNCH(false, POL_NT_OUT); }
    } else if (a.chunk_beg && a.accumulate)
      hipLaunchKernelGGL((gspmm_sum_kernel<VEC, GROUP, UNROLL, MSG, EM, MEAN, true, true>),
                         grid_1d(blocks), dim3(256), 0, stream,
                         a.num_items, a.F, a.elen, a.ldu ? a.ldu : a.F, a.indptr, a.indices, a.eid, a.ufeat, a.efeat,
                         a.out, a.row_order, a.chunk_beg, a.chunk_end);
    else if (!a.chunk_beg && a.accumulate)
      hipLaunchKernelGGL((gspmm_sum_kernel<VEC, GROUP, UNROLL, MSG, EM, MEAN, false, true>),
                         grid_1d(blocks), dim3(256), 0, stream,
                         a.num_items, a.F, a.elen, a.ldu ? a.ldu : a.F, a.indptr, a.indices, a.eid, a.ufeat, a.efeat,
                         a.out, a.row_order, a.chunk_beg, a.chunk_end);
    else if (a.chunk_beg)
      hipLaunchKernelGGL((gspmm_sum_kernel<VEC, GROUP, UNROLL, MSG, EM, MEAN, true, false>),
                         grid_1d(blocks), dim3(256), 0, stream,
                         a.num_items, a.F, a.elen, a.ldu ? a.ldu : a.F, a.indptr, a.indices, a.eid, a.ufeat, a.efeat,
                         a.out, a.row_order, a.chunk_beg, a.chunk_end);
    else
      hipLaunchKernelGGL((gspmm_sum_kernel<VEC, GROUP, UNROLL, MSG, EM, MEAN, false, false, PIPE>),
                         grid_1d(blocks), dim3(256), 0, stream,
                         a.num_items, a.F, a.elen, a.ldu ? a.ldu : a.F, a.indptr, a.indices, a.eid, a.ufeat, a.efeat,
                         a.out, a.row_order, a.chunk_beg, a.chunk_end);
#undef DGLHIP_POL_LAUNCH
#undef DGLHIP_POL_LAUNCH_B
  });
}

template <int MSG, int EM, bool MEAN>
static inline bool dispatch_variant(const SumLaunch& a, hipStream_t stream) {
  if (MSG != DGLHIP_MSG_COPY_U || MEAN || g_var_vec == 0 || a.accumulate) return false;
  const int v = g_var_vec, gr = g_var_group, u = g_var_unroll, pp = g_var_pipe;
  if (int64_t(v) * gr < a.F && (a.F % (int64_t(v) * gr)) != 0) return false;
  if (a.F % v != 0) return false;
#define DGLHIP_VAR(V, G, U, P)                                                   \
  if (v == V && gr == G && u == U && pp == P) {                                \
    launch_sum<V, G, MSG, EM, MEAN, U, P>(a, stream);                          \
    return true;                                                               \
  }
  DGLHIP_VAR(2, 64, 4, 0) DGLHIP_VAR(2, 64, 8, 0) DGLHIP_VAR(2, 64, 16, 0)
  DGLHIP_VAR(2, 64, 32, 0) DGLHIP_VAR(4, 32, 8, 0) DGLHIP_VAR(4, 32, 16, 0)
  DGLHIP_VAR(4, 32, 32, 0) DGLHIP_VAR(2, 64, 8, 1) DGLHIP_VAR(2, 64, 16, 1)
  DGLHIP_VAR(4, 32, 8, 1) DGLHIP_VAR(4, 32, 16, 1)
  // narrow rows (F < 128, or F not a multiple of 2 x 64): tools/feat_sweep.py
  DGLHIP_VAR(1, 64, 8, 0) DGLHIP_VAR(1, 64, 16, 0) DGLHIP_VAR(1, 64, 32, 0)
  DGLHIP_VAR(2, 32, 16, 0) DGLHIP_VAR(2, 32, 32, 0) DGLHIP_VAR(1, 32, 32, 0)
#undef DGLHIP_VAR
  return false;
}

template <int MSG, int EM, bool MEAN>
static inline void dispatch_sum_shape(const SumLaunch& a, hipStream_t stream) {
  const int64_t F = a.F;
  if (dispatch_variant<MSG, EM, MEAN>(a, stream)) return;
  int vec = pick_vec(F, {a.ufeat, EM == EM_FULL ? a.efeat : nullptr, a.out});
  // per-head weights: a lane's VEC features must stay inside one head
  while (EM == EM_HEAD && vec > 1 && (F / a.elen) % vec != 0) vec >>= 1;
  int group = pick_group(F, vec);
  one_row_per_wave(F, vec, group);
#define DGLHIP_CASE(V, G)                                  \
  if (vec == V && group == G) {                            \
    launch_sum<V, G, MSG, EM, MEAN>(a, stream);            \
    return;                                                \
  }
  DGLHIP_CASE(2, 64) DGLHIP_CASE(2, 32) DGLHIP_CASE(2, 16) DGLHIP_CASE(2, 8)
  DGLHIP_CASE(2, 4) DGLHIP_CASE(2, 2)
  DGLHIP_CASE(1, 64) DGLHIP_CASE(1, 32) DGLHIP_CASE(1, 16) DGLHIP_CASE(1, 8)
  DGLHIP_CASE(1, 4) DGLHIP_CASE(1, 2) DGLHIP_CASE(1, 1)
#undef DGLHIP_CASE
  DGLHIP_CHECK(false, "no kernel for F=" << F << " vec=" << vec << " group=" << group);
}

static inline int edge_mode(int64_t elen, int64_t F) {
  return elen == F ? EM_FULL : (elen == 1 ? EM_SCALAR : EM_HEAD);
}


struct MaxLaunch {
  int64_t num_rows, F, elen;
  const int64_t* indptr;
  const int32_t* indices;
  const int64_t* eid;
  const float* ufeat;
  const float* efeat;
  float* out;
  int64_t* arg_out;
  const int32_t* row_order;
  const int64_t* row_beg = nullptr;  // row ranges (NULL: whole rows)
  const int64_t* row_end = nullptr;
  int accumulate = 0;
};


template <int MSG, int EM>
static inline void dispatch_max_shape(const MaxLaunch& a, hipStream_t stream) {
  const int64_t F = a.F;
  int vec = pick_vec(F, {a.ufeat, EM == EM_FULL ? a.efeat : nullptr, a.out});
  while (EM == EM_HEAD && vec > 1 && (F / a.elen) % vec != 0) vec >>= 1;
  int group = pick_group(F, vec);
  one_row_per_wave(F, vec, group);
#define DGLHIP_CASE(V, G)                                                            \
  if (vec == V && group == G) {                                                      \
    constexpr int ITEMS_PER_BLOCK = 4 * (64 / G);                                    \
    const int64_t blocks = (a.num_rows + ITEMS_PER_BLOCK - 1) / ITEMS_PER_BLOCK;     \
    DGLHIP_CHECK(blocks <= 0x7fffffff, "grid too large: " << blocks);                \
    timed_launch(stream, [&] {                                                       \
      hipLaunchKernelGGL((gspmm_max_kernel<V, G, 8, MSG, EM>),                       \
                         grid_1d(blocks), dim3(256), 0, stream,  \
                         a.num_rows, a.F, a.elen, a.indptr, a.indices, a.eid,        \
                         a.ufeat, a.efeat, a.out, a.arg_out, a.row_order, a.row_beg, \
                         a.row_end, a.accumulate);                                   \
    });                                                                              \
    return;                                                                          \
  }
  DGLHIP_CASE(2, 64) DGLHIP_CASE(2, 32) DGLHIP_CASE(2, 16) DGLHIP_CASE(2, 8)
  DGLHIP_CASE(2, 4) DGLHIP_CASE(2, 2)
  DGLHIP_CASE(1, 64) DGLHIP_CASE(1, 32) DGLHIP_CASE(1, 16) DGLHIP_CASE(1, 8)
  DGLHIP_CASE(1, 4) DGLHIP_CASE(1, 2) DGLHIP_CASE(1, 1)
#undef DGLHIP_CASE
  DGLHIP_CHECK(false, "no max kernel for F=" << F << " vec=" << vec << " group=" << group);
}


// One (message, edge layout) pair of the sum/mean and max reducers. Defined
// only in gspmm_inst.hip, which explicitly instantiates it per pair.
template <int MSG, int EM>
void dispatch_sum_me(bool mean, const SumLaunch& a, hipStream_t stream);
template <int MSG, int EM>
void dispatch_max_me(const MaxLaunch& a, hipStream_t stream);

#ifdef GSPMM_INST_MSG
template <int MSG, int EM>
void dispatch_sum_me(bool mean, const SumLaunch& a, hipStream_t stream) {
  if (mean) dispatch_sum_shape<MSG, EM, true>(a, stream);
  else dispatch_sum_shape<MSG, EM, false>(a, stream);
}
template <int MSG, int EM>
void dispatch_max_me(const MaxLaunch& a, hipStream_t stream) {
  dispatch_max_shape<MSG, EM>(a, stream);
}
#endif

}  // namespace dglhip
