// g-SpMM / g-SDDMM HIP kernels for gfx950 (MI355X, CDNA4).
//
// Replaces the reference's F.spmm = torch.sparse.mm on an uncoalesced COO
// (python/dgl/backend/pytorch/tensor.py:145-146) as driven by SPMVExecutor /
// SPMVWithDataExecutor (python/dgl/runtime/ir/executor.py:452-473,535-566),
// and the degree-bucketing UDF reduce for max/mean
// (python/dgl/runtime/degree_bucketing.py:13-190).
//
// Design:
//  * One lane GROUP (a whole 64-lane wave for F=128) owns one destination row.
//    Each lane holds VEC consecutive features of the row in registers, so the
//    gathered source row arrives as one coalesced wave-instruction
//    (64 lanes x 8 B = 512 B = one F=128 fp32 row) and no LDS round trip or
//    cross-lane reduction is needed: every output element is a sequential
//    fma chain over the row's CSR slots — the exact arithmetic of the
//    reference's CPU product, hence bit-exact parity.
//  * Memory-level parallelism comes from UNROLL (16) independent row gathers
//    in flight per wave plus several waves per SIMD. With a whole
//    wave per row the CSR slot stream is wave-uniform: column ids and edge
//    weights come through the scalar cache (s_load), not VGPRs.
//  * Rows are launched in degree-descending order (row_order) so the longest
//    sequential chains start first and the tail is short.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <initializer_list>
#include <mutex>
#include <vector>

#include "../../include/dgl_hip.h"
#include "common.h"

namespace dglhip {

#define HIP_CALL(expr)                                                      \
  do {                                                                      \
    hipError_t _e = (expr);                                                 \
    DGLHIP_CHECK(_e == hipSuccess, #expr << " -> " << hipGetErrorString(_e)); \
  } while (0)

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

template <int VEC, int POL>
__device__ __forceinline__ typename Vec<VEC>::T gather_row(const float* __restrict__ ufeat,
                                                           int32_t col, int64_t F, int64_t f0) {
  typedef typename Vec<VEC>::T V;
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
template <int VEC, int MSG, int EM, int POL = POL_DEFAULT>
struct SlotLoad {
  typedef typename Vec<VEC>::T V;
  V u;
  V e;
  __device__ __forceinline__ void load(const float* __restrict__ ufeat,
                                       const float* __restrict__ efeat,
                                       int64_t F, int64_t f0, int64_t elen, int64_t eoff,
                                       int32_t src, int64_t edge) {
    if (MSG != DGLHIP_MSG_COPY_E) u = gather_row<VEC, POL>(ufeat, src, F, f0);
    if (MSG != DGLHIP_MSG_COPY_U) {
      if (EM == EM_FULL) e = ldv<VEC>(efeat + edge * F + f0);
      else e = Vec<VEC>::splat(efeat[edge * elen + eoff]);
    }
  }
};

// Sequential reduction of slots [beg, end) of one row for the VEC features at
// f0: the fma chain the reference's product runs (see the file header).
template <int VEC, int UNROLL, int MSG, int EM, bool USE_EID, int POL = POL_DEFAULT>
__device__ __forceinline__ typename Vec<VEC>::T reduce_range(
    typename Vec<VEC>::T acc, int64_t beg, int64_t end, int64_t F, int64_t f0, int64_t elen,
    int64_t eoff, const int32_t* __restrict__ indices,
    const int64_t* __restrict__ eid, const float* __restrict__ ufeat,
    const float* __restrict__ efeat) {
  int64_t k = beg;
  for (; k + UNROLL <= end; k += UNROLL) {
    SlotLoad<VEC, MSG, EM, POL> s[UNROLL];
#pragma unroll
    for (int j = 0; j < UNROLL; ++j)
      s[j].load(ufeat, efeat, F, f0, elen, eoff, indices[k + j],
                MSG == DGLHIP_MSG_COPY_U ? 0 : (USE_EID ? eid[k + j] : k + j));
#pragma unroll
    for (int j = 0; j < UNROLL; ++j) {
      if (MSG == DGLHIP_MSG_COPY_U) acc += s[j].u;
      else if (MSG == DGLHIP_MSG_COPY_E) acc += s[j].e;
      else acc = Vec<VEC>::fma(s[j].e, s[j].u, acc);
    }
  }
  // the last rem < UNROLL slots as one predicated batch: all their gathers in
  // flight together (a slot-by-slot tail would serialise up to UNROLL - 1
  // load latencies per row, which dominates rows shorter than UNROLL)
  const int64_t rem = end - k;
  if (rem > 0) {
    SlotLoad<VEC, MSG, EM, POL> s[UNROLL];
#pragma unroll
    for (int j = 0; j < UNROLL - 1; ++j)
      if (j < rem)
        s[j].load(ufeat, efeat, F, f0, elen, eoff, indices[k + j],
                  MSG == DGLHIP_MSG_COPY_U ? 0 : (USE_EID ? eid[k + j] : k + j));
#pragma unroll
    for (int j = 0; j < UNROLL - 1; ++j) {
      if (j < rem) {
        if (MSG == DGLHIP_MSG_COPY_U) acc += s[j].u;
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
    typename Vec<VEC>::T acc, int64_t beg, int64_t end, int64_t F, int64_t f0,
    const int32_t* __restrict__ indices, const float* __restrict__ ufeat) {
  typedef typename Vec<VEC>::T V;
  int64_t k = beg;
  if (k + UNROLL <= end) {
    V cur[UNROLL];
#pragma unroll
    for (int j = 0; j < UNROLL; ++j) cur[j] = ldv<VEC>(ufeat + int64_t(indices[k + j]) * F + f0);
    k += UNROLL;
    for (; k + UNROLL <= end; k += UNROLL) {
      V nxt[UNROLL];
#pragma unroll
      for (int j = 0; j < UNROLL; ++j)
        nxt[j] = ldv<VEC>(ufeat + int64_t(indices[k + j]) * F + f0);
#pragma unroll
      for (int j = 0; j < UNROLL; ++j) acc += cur[j];
#pragma unroll
      for (int j = 0; j < UNROLL; ++j) cur[j] = nxt[j];
    }
#pragma unroll
    for (int j = 0; j < UNROLL; ++j) acc += cur[j];
  }
  for (; k < end; ++k) acc += ldv<VEC>(ufeat + int64_t(indices[k]) * F + f0);
  return acc;
}

// Sum-reduce kernel (also MEAN). GROUP lanes per work item, VEC floats per
// lane. A work item is a whole row (CHUNKED = false: item i = row_order[i]),
// or a slot range [chunk_beg[i], chunk_end[i]) whose sum goes to out[i, :]
// (CHUNKED = true). With ACCUM the chain continues from the value already in
// out[i, :] (segment-by-segment evaluation of one sequential chain).
template <int VEC, int GROUP, int UNROLL, int MSG, int EM, bool MEAN, bool CHUNKED,
          bool ACCUM, bool PIPE = false, int POL = POL_DEFAULT>
__global__ __launch_bounds__(256) void gspmm_sum_kernel(
    int64_t num_items, int64_t F, int64_t elen, const int64_t* __restrict__ indptr,
    const int32_t* __restrict__ indices, const int64_t* __restrict__ eid,
    const float* __restrict__ ufeat, const float* __restrict__ efeat,
    float* __restrict__ out, const int32_t* __restrict__ row_order,
    const int64_t* __restrict__ chunk_beg, const int64_t* __restrict__ chunk_end) {
  typedef typename Vec<VEC>::T V;
  constexpr int ITEMS_PER_WAVE = 64 / GROUP;
  const int lane = threadIdx.x & 63;
  // wave index is uniform; make that explicit so slot data goes through SGPRs
  const int64_t wave =
      int64_t(blockIdx.x) * (blockDim.x >> 6) +
      __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int64_t it = wave * ITEMS_PER_WAVE + (GROUP == 64 ? 0 : lane / GROUP);
  if (it >= num_items) return;
  const int gl = GROUP == 64 ? lane : (lane % GROUP);
  int64_t row, beg, end;
  if (CHUNKED) {
    row = it;
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
    V acc = ACCUM ? ldv<VEC>(out + row * F + f0) : Vec<VEC>::zero();
    if (PIPE && MSG == DGLHIP_MSG_COPY_U)
      acc = reduce_range_pipelined<VEC, UNROLL>(acc, beg, end, F, f0, indices, ufeat);
    else if (MSG == DGLHIP_MSG_COPY_U || eid != nullptr)  // uniform branch
      acc = reduce_range<VEC, UNROLL, MSG, EM, true, POL>(acc, beg, end, F, f0, elen, eoff,
                                                          indices, eid, ufeat, efeat);
    else
      acc = reduce_range<VEC, UNROLL, MSG, EM, false>(acc, beg, end, F, f0, elen, eoff, indices,
                                                      eid, ufeat, efeat);
    if (!CHUNKED && MEAN && end - beg > 1)
      acc = acc / Vec<VEC>::splat(static_cast<float>(end - beg));
    store_row<VEC, POL>(out + row * F + f0, acc);
  }
}

// Combine the chunk partials of each heavy row in chunk order:
// out[row] = ((p0 + p1) + p2) + ... (deterministic), then MEAN scaling; with
// ACCUM the row's running value comes first: out[row] = ((out[row] + p0) + p1) ...
template <bool MEAN, bool ACCUM>
__global__ __launch_bounds__(256) void gspmm_combine_kernel(
    int64_t num_heavy, int64_t F, const int64_t* __restrict__ indptr,
    const int32_t* __restrict__ heavy_rows, const int64_t* __restrict__ heavy_chunk_ptr,
    const float* __restrict__ partial, float* __restrict__ out) {
  const int64_t wave = int64_t(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wave >= num_heavy) return;
  const int lane = threadIdx.x & 63;
  const int64_t row = heavy_rows[wave];
  const int64_t c0 = heavy_chunk_ptr[wave], c1 = heavy_chunk_ptr[wave + 1];
  const float deg = static_cast<float>(indptr[row + 1] - indptr[row]);
  for (int64_t f = lane; f < F; f += 64) {
    float acc = ACCUM ? out[row * F + f] + partial[c0 * F + f] : partial[c0 * F + f];
    for (int64_t c = c0 + 1; c < c1; ++c) acc += partial[c * F + f];
    if (MEAN && deg > 1.0f) acc = acc / deg;
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
                                        float* __restrict__ out, int64_t* __restrict__ arg_out) {
  typedef typename Vec<VEC>::T V;
  auto message = [](const SlotLoad<VEC, MSG, EM>& s) -> V {
    if (MSG == DGLHIP_MSG_COPY_U) return s.u;
    if (MSG == DGLHIP_MSG_COPY_E) return s.e;
    return s.u * s.e;
  };
  auto edge = [&](int64_t k) -> int64_t {
    return MSG == DGLHIP_MSG_COPY_U ? 0 : (USE_EID ? eid[k] : k);
  };
  for (int64_t f0 = int64_t(gl) * VEC; f0 < F; f0 += int64_t(group) * VEC) {
    const int64_t eoff = EM == EM_HEAD ? f0 / (F / elen) : (EM == EM_FULL ? f0 : 0);
    V best = Vec<VEC>::zero();
    int64_t arg[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) arg[i] = -1;
    int64_t k = beg;
    if (k < end) {
      SlotLoad<VEC, MSG, EM> s;
      s.load(ufeat, efeat, F, f0, elen, eoff, indices[k], edge(k));
      best = message(s);
#pragma unroll
      for (int i = 0; i < VEC; ++i) arg[i] = k;
      ++k;
    }
    for (; k + UNROLL <= end; k += UNROLL) {
      SlotLoad<VEC, MSG, EM> s[UNROLL];
#pragma unroll
      for (int j = 0; j < UNROLL; ++j)
        s[j].load(ufeat, efeat, F, f0, elen, eoff, indices[k + j], edge(k + j));
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
        if (j < rem) s[j].load(ufeat, efeat, F, f0, elen, eoff, indices[k + j], edge(k + j));
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
    const int32_t* __restrict__ row_order) {
  constexpr int ITEMS_PER_WAVE = 64 / GROUP;
  const int lane = threadIdx.x & 63;
  const int64_t wave =
      int64_t(blockIdx.x) * (blockDim.x >> 6) +
      __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int64_t it = wave * ITEMS_PER_WAVE + (GROUP == 64 ? 0 : lane / GROUP);
  if (it >= num_rows) return;
  const int gl = GROUP == 64 ? lane : (lane % GROUP);
  int64_t row = row_order ? row_order[it] : it;
  if (GROUP == 64) row = __builtin_amdgcn_readfirstlane(static_cast<int>(row));
  const int64_t beg = indptr[row], end = indptr[row + 1];
  if (MSG == DGLHIP_MSG_COPY_U || eid != nullptr)  // uniform branch
    max_row<VEC, UNROLL, MSG, EM, true>(row, gl, GROUP, beg, end, F, elen, indices, eid, ufeat,
                                        efeat, out, arg_out);
  else
    max_row<VEC, UNROLL, MSG, EM, false>(row, gl, GROUP, beg, end, F, elen, indices, eid,
                                         ufeat, efeat, out, arg_out);
}

// SDDMM dot: one wave per row. One head (H == 1): per slot a wave-wide fma
// dot product of two feature rows reduced in a fixed butterfly order. Several
// heads: lane h computes head h's dot over its D = F / H features as one
// sequential fma chain. Both orders are fixed, so results are deterministic.
__global__ __launch_bounds__(256) void gsddmm_dot_kernel(
    int64_t num_rows, int64_t F, int64_t H, const int64_t* __restrict__ indptr,
    const int32_t* __restrict__ indices, const int64_t* __restrict__ eid,
    const float* __restrict__ lhs, const float* __restrict__ rhs,
    float* __restrict__ out) {
  const int64_t wave = int64_t(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wave >= num_rows) return;
  const int lane = threadIdx.x & 63;
  const float* a = lhs + wave * F;
  const int64_t D = F / H;
  for (int64_t k = indptr[wave]; k < indptr[wave + 1]; ++k) {
    const float* c = rhs + int64_t(indices[k]) * F;
    if (H == 1) {
      float acc = 0.0f;
      for (int64_t f = lane; f < F; f += 64) acc = __builtin_fmaf(a[f], c[f], acc);
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
      if (lane == 0) out[eid[k]] = acc;
    } else {
      for (int64_t h = lane; h < H; h += 64) {
        float acc = 0.0f;
        for (int64_t d = 0; d < D; ++d) acc = __builtin_fmaf(a[h * D + d], c[h * D + d], acc);
        out[eid[k] * H + h] = acc;
      }
    }
  }
}

// SDDMM dot for rows of NB x 32 floats (F = 32 * NB), one wave per row: the
// wave takes 8 slots at a time, 8 lanes per slot; lane j of a slot reads the
// 16 B at 32 i + 4 j of every 32-float column block i (one instruction = 8
// whole 128-B lines), UNROLL groups of 8 slots in flight. Per lane and block
// the partial is an fma chain over its 4 features (x, y, z, w); a head's
// total is the sum of its lanes' partials in block order, then an xor
// butterfly over the lanes sharing the head (both lanes of a pair add the
// same two values, so every lane ends with identical bits: deterministic).
//   D >= 32 (D % 32 == 0): a head spans D / 32 whole blocks, 8-lane butterfly;
//   D <  32 (D in 4, 8, 16): D / 4 lanes per head, butterfly within them.
template <int NB, int UNROLL>
__global__ __launch_bounds__(256) void gsddmm_dot_sliced_kernel(
    int64_t num_rows, int64_t H, int64_t D, const int64_t* __restrict__ indptr,
    const int32_t* __restrict__ indices, const int64_t* __restrict__ eid,
    const float* __restrict__ lhs, const float* __restrict__ rhs, float* __restrict__ out) {
  constexpr int F = NB * 32;
  const int64_t row = int64_t(blockIdx.x) * (blockDim.x >> 6) +
                      __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  if (row >= num_rows) return;
  const int lane = threadIdx.x & 63;
  const int s = lane >> 3, j = lane & 7;
  const int64_t beg = indptr[row], end = indptr[row + 1];
  if (beg == end) return;
  f32x4 a[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) a[i] = ldv<4>(lhs + row * F + 32 * i + 4 * j);
  const int lph = D >= 32 ? 8 : static_cast<int>(D >> 2);   // lanes sharing a head
  const int64_t dblk = D >= 32 ? D / 32 : 1;                 // blocks per head (D >= 32)
  for (int64_t k0 = beg; k0 < end; k0 += 8 * UNROLL) {
    f32x4 c[UNROLL][NB];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      int64_t k = k0 + 8 * u + s;
      k = k < end ? k : end - 1;  // idle slot lanes re-read the row's last slot
      const float* r = rhs + int64_t(indices[k]) * F + 4 * j;
#pragma unroll
      for (int i = 0; i < NB; ++i) c[u][i] = ldv<4>(r + 32 * i);
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t k = k0 + 8 * u + s;
      float p[NB];
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        float t = a[i].x * c[u][i].x;
        t = __builtin_fmaf(a[i].y, c[u][i].y, t);
        t = __builtin_fmaf(a[i].z, c[u][i].z, t);
        p[i] = __builtin_fmaf(a[i].w, c[u][i].w, t);
      }
      if (D >= 32) {
        float t = 0.0f;
#pragma unroll
        for (int i = 0; i < NB; ++i) {  // blocks in order; a head closes every dblk blocks
          t = (i % dblk == 0) ? p[i] : t + p[i];
          if ((i + 1) % dblk == 0) {
            float r = t;
            r += __shfl_xor(r, 4, 64);
            r += __shfl_xor(r, 2, 64);
            r += __shfl_xor(r, 1, 64);
            if (j == 0 && k < end) out[eid[k] * H + i / dblk] = r;
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          float t = p[i];
          if (lph >= 4) t += __shfl_xor(t, 2, 64);
          if (lph >= 2) t += __shfl_xor(t, 1, 64);
          const int64_t h = (32 * i + 4 * j) / D;
          if ((j % lph) == 0 && k < end) out[eid[k] * H + h] = t;
        }
      }
    }
  }
}

// GAT edge attention, one wave per destination row v (gat/train.py:90-96):
//   out[eid[k], h] = clamp(exp(leaky_relu(lhs[u, h] + rhs[v, h], alpha)), lo, hi)
// with u = indices[k]; lanes run over the row's (slot, head) pairs.
__global__ __launch_bounds__(256) void gsddmm_attention_kernel(
    int64_t num_rows, int64_t H, const int64_t* __restrict__ indptr,
    const int32_t* __restrict__ indices, const int64_t* __restrict__ eid,
    const float* __restrict__ lhs, const float* __restrict__ rhs, float alpha, float lo,
    float hi, int apply_exp, float* __restrict__ out) {
  const int64_t row = int64_t(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= num_rows) return;
  const int lane = threadIdx.x & 63;
  const int64_t beg = indptr[row], n = (indptr[row + 1] - beg) * H;
  for (int64_t idx = lane; idx < n; idx += 64) {
    const int64_t k = beg + idx / H, h = idx - (idx / H) * H;
    float x = lhs[int64_t(indices[k]) * H + h] + rhs[row * H + h];
    x = x > 0.0f ? x : alpha * x;
    if (apply_exp) x = __expf(x);
    out[eid[k] * H + h] = fminf(fmaxf(x, lo), hi);
  }
}

// ---------------------------------------------------------------------------
// Timing support: hipEvent pairs around each launch, on the launch stream.
// ---------------------------------------------------------------------------
struct Timing {
  std::mutex mu;
  bool enabled = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
  double total_ms = 0.0;
  int64_t launches = 0;
};
static Timing g_timing;

static std::pair<hipEvent_t, hipEvent_t> take_events() {
  if (!g_timing.pool.empty()) {
    auto p = g_timing.pool.back();
    g_timing.pool.pop_back();
    return p;
  }
  std::pair<hipEvent_t, hipEvent_t> p;
  HIP_CALL(hipEventCreate(&p.first));
  HIP_CALL(hipEventCreate(&p.second));
  return p;
}

template <typename LaunchFn>
static void timed_launch(hipStream_t stream, LaunchFn&& fn) {
  std::unique_lock<std::mutex> lk(g_timing.mu);
  if (!g_timing.enabled) {
    lk.unlock();
    fn();
    HIP_CALL(hipGetLastError());
    return;
  }
  auto ev = take_events();
  HIP_CALL(hipEventRecord(ev.first, stream));
  fn();
  HIP_CALL(hipGetLastError());
  HIP_CALL(hipEventRecord(ev.second, stream));
  g_timing.pending.push_back(ev);
}

// ---------------------------------------------------------------------------
// Dispatch
// ---------------------------------------------------------------------------
// Widest per-lane vector the row length and every feature pointer allow.
static int pick_vec(int64_t F, std::initializer_list<const void*> ptrs) {
  auto aligned = [&](int bytes) {
    for (const void* p : ptrs)
      if (p && (reinterpret_cast<uintptr_t>(p) % bytes) != 0) return false;
    return true;
  };
  if (F % 4 == 0 && F >= 256 && aligned(16)) return 4;
  if (F % 2 == 0 && F >= 4 && aligned(8)) return 2;
  return 1;
}

static int pick_group(int64_t F, int vec) {
  const int64_t lanes = (F + vec - 1) / vec;
  int g = 1;
  while (g < lanes && g < 64) g <<= 1;
  return g;
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
};

// Outputs past twice the 256 MiB Infinity Cache are stored non-temporally
// (POL_NT_OUT): streamed out, they would evict the feature rows that are
// gathered again (RMAT-26, 34 GB out: 94.1 -> 89.5 ms,
// tools/cache_policy_study.py). Covers copy_u + sum at VEC 2 x 64 lanes.
static bool stream_output(int64_t rows, int64_t feat_len) {
  return rows * feat_len * int64_t(sizeof(float)) > (int64_t(512) << 20);
}

// Tuning override for the copy_u + sum shape (dglhip_set_spmm_variant);
// 0 = automatic choice.
static int g_var_vec = 0, g_var_group = 0, g_var_unroll = 0, g_var_pipe = 0;
// Cache policy for copy_u + sum at VEC 2 x 64 lanes (dglhip_set_cache_policy).
// -1: automatic (non-temporal output past 512 MiB, default otherwise).
static int g_cache_policy = -1;

template <int VEC, int GROUP, int MSG, int EM, bool MEAN, int UNROLL_OVERRIDE = 0,
          bool PIPE = false>
static void launch_sum(const SumLaunch& a, hipStream_t stream) {
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
#define DGLHIP_POL_LAUNCH(CH, P)                                                           \
  hipLaunchKernelGGL((gspmm_sum_kernel<VEC, GROUP, UNROLL, MSG, EM, false, CH, false, false, P>), \
                     dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream, a.num_items,   \
                     a.F, a.elen, a.indptr, a.indices, a.eid, a.ufeat, a.efeat, a.out,         \
                     a.row_order, a.chunk_beg, a.chunk_end)
    if (POL_OK && pol != POL_DEFAULT && !a.accumulate) {
      const bool ch = a.chunk_beg != nullptr;
      if (pol == POL_NT) { if (ch) DGLHIP_POL_LAUNCH(true, POL_NT); else DGLHIP_POL_LAUNCH(false, POL_NT); }
      else if (pol == POL_HOT) { if (ch) DGLHIP_POL_LAUNCH(true, POL_HOT); else DGLHIP_POL_LAUNCH(false, POL_HOT); }
      else { if (ch) DGLHIP_POL_LAUNCH(true, POL_NT_OUT); else DGLHIP_POL_LAUNCH(false, POL_NT_OUT); }
    } else if (a.chunk_beg && a.accumulate)
      hipLaunchKernelGGL((gspmm_sum_kernel<VEC, GROUP, UNROLL, MSG, EM, MEAN, true, true>),
                         dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream,
                         a.num_items, a.F, a.elen, a.indptr, a.indices, a.eid, a.ufeat, a.efeat,
                         a.out, a.row_order, a.chunk_beg, a.chunk_end);
    else if (!a.chunk_beg && a.accumulate && !MEAN)
      hipLaunchKernelGGL((gspmm_sum_kernel<VEC, GROUP, UNROLL, MSG, EM, false, false, true>),
                         dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream,
                         a.num_items, a.F, a.elen, a.indptr, a.indices, a.eid, a.ufeat, a.efeat,
                         a.out, a.row_order, a.chunk_beg, a.chunk_end);
    else if (a.chunk_beg)
      hipLaunchKernelGGL((gspmm_sum_kernel<VEC, GROUP, UNROLL, MSG, EM, MEAN, true, false>),
                         dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream,
                         a.num_items, a.F, a.elen, a.indptr, a.indices, a.eid, a.ufeat, a.efeat,
                         a.out, a.row_order, a.chunk_beg, a.chunk_end);
    else
      hipLaunchKernelGGL((gspmm_sum_kernel<VEC, GROUP, UNROLL, MSG, EM, MEAN, false, false, PIPE>),
                         dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream,
                         a.num_items, a.F, a.elen, a.indptr, a.indices, a.eid, a.ufeat, a.efeat,
                         a.out, a.row_order, a.chunk_beg, a.chunk_end);
#undef DGLHIP_POL_LAUNCH
  });
}

template <int MSG, int EM, bool MEAN>
static bool dispatch_variant(const SumLaunch& a, hipStream_t stream) {
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
#undef DGLHIP_VAR
  return false;
}

template <int MSG, int EM, bool MEAN>
static void dispatch_sum_shape(const SumLaunch& a, hipStream_t stream) {
  const int64_t F = a.F;
  if (dispatch_variant<MSG, EM, MEAN>(a, stream)) return;
  int vec = pick_vec(F, {a.ufeat, EM == EM_FULL ? a.efeat : nullptr, a.out});
  // per-head weights: a lane's VEC features must stay inside one head
  while (EM == EM_HEAD && vec > 1 && (F / a.elen) % vec != 0) vec >>= 1;
  const int group = pick_group(F, vec);
#define DGLHIP_CASE(V, G)                                  \
  if (vec == V && group == G) {                            \
    launch_sum<V, G, MSG, EM, MEAN>(a, stream);            \
    return;                                                \
  }
  DGLHIP_CASE(4, 64)
  DGLHIP_CASE(2, 64) DGLHIP_CASE(2, 32) DGLHIP_CASE(2, 16) DGLHIP_CASE(2, 8)
  DGLHIP_CASE(2, 4) DGLHIP_CASE(2, 2)
  DGLHIP_CASE(1, 64) DGLHIP_CASE(1, 32) DGLHIP_CASE(1, 16) DGLHIP_CASE(1, 8)
  DGLHIP_CASE(1, 4) DGLHIP_CASE(1, 2) DGLHIP_CASE(1, 1)
#undef DGLHIP_CASE
  DGLHIP_CHECK(false, "no kernel for F=" << F << " vec=" << vec << " group=" << group);
}

static int edge_mode(int64_t elen, int64_t F) {
  return elen == F ? EM_FULL : (elen == 1 ? EM_SCALAR : EM_HEAD);
}

static void dispatch_sum(int msg_op, bool mean, const SumLaunch& a, hipStream_t stream) {
#define DGLHIP_SUM(M, E)                                      \
  do {                                                        \
    if (mean) dispatch_sum_shape<M, E, true>(a, stream);      \
    else dispatch_sum_shape<M, E, false>(a, stream);          \
  } while (0)
  const int em = edge_mode(a.elen, a.F);
  if (msg_op == DGLHIP_MSG_COPY_U) {
    DGLHIP_SUM(DGLHIP_MSG_COPY_U, EM_SCALAR);
  } else if (msg_op == DGLHIP_MSG_U_MUL_E) {
    if (em == EM_FULL) DGLHIP_SUM(DGLHIP_MSG_U_MUL_E, EM_FULL);
    else if (em == EM_SCALAR) DGLHIP_SUM(DGLHIP_MSG_U_MUL_E, EM_SCALAR);
    else DGLHIP_SUM(DGLHIP_MSG_U_MUL_E, EM_HEAD);
  } else {
    if (em == EM_FULL) DGLHIP_SUM(DGLHIP_MSG_COPY_E, EM_FULL);
    else if (em == EM_SCALAR) DGLHIP_SUM(DGLHIP_MSG_COPY_E, EM_SCALAR);
    else DGLHIP_SUM(DGLHIP_MSG_COPY_E, EM_HEAD);
  }
#undef DGLHIP_SUM
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
};

template <int MSG, int EM>
static void dispatch_max_shape(const MaxLaunch& a, hipStream_t stream) {
  const int64_t F = a.F;
  int vec = pick_vec(F, {a.ufeat, EM == EM_FULL ? a.efeat : nullptr, a.out});
  while (EM == EM_HEAD && vec > 1 && (F / a.elen) % vec != 0) vec >>= 1;
  const int group = pick_group(F, vec);
#define DGLHIP_CASE(V, G)                                                            \
  if (vec == V && group == G) {                                                      \
    constexpr int ITEMS_PER_BLOCK = 4 * (64 / G);                                    \
    const int64_t blocks = (a.num_rows + ITEMS_PER_BLOCK - 1) / ITEMS_PER_BLOCK;     \
    DGLHIP_CHECK(blocks <= 0x7fffffff, "grid too large: " << blocks);                \
    timed_launch(stream, [&] {                                                       \
      hipLaunchKernelGGL((gspmm_max_kernel<V, G, 8, MSG, EM>),                       \
                         dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream,  \
                         a.num_rows, a.F, a.elen, a.indptr, a.indices, a.eid,        \
                         a.ufeat, a.efeat, a.out, a.arg_out, a.row_order);           \
    });                                                                              \
    return;                                                                          \
  }
  DGLHIP_CASE(4, 64)
  DGLHIP_CASE(2, 64) DGLHIP_CASE(2, 32) DGLHIP_CASE(2, 16) DGLHIP_CASE(2, 8)
  DGLHIP_CASE(2, 4) DGLHIP_CASE(2, 2)
  DGLHIP_CASE(1, 64) DGLHIP_CASE(1, 32) DGLHIP_CASE(1, 16) DGLHIP_CASE(1, 8)
  DGLHIP_CASE(1, 4) DGLHIP_CASE(1, 2) DGLHIP_CASE(1, 1)
#undef DGLHIP_CASE
  DGLHIP_CHECK(false, "no max kernel for F=" << F << " vec=" << vec << " group=" << group);
}

static void dispatch_max(int msg_op, const MaxLaunch& a, hipStream_t stream) {
  const int em = edge_mode(a.elen, a.F);
  if (msg_op == DGLHIP_MSG_COPY_U) {
    dispatch_max_shape<DGLHIP_MSG_COPY_U, EM_SCALAR>(a, stream);
  } else if (msg_op == DGLHIP_MSG_U_MUL_E) {
    if (em == EM_FULL) dispatch_max_shape<DGLHIP_MSG_U_MUL_E, EM_FULL>(a, stream);
    else if (em == EM_SCALAR) dispatch_max_shape<DGLHIP_MSG_U_MUL_E, EM_SCALAR>(a, stream);
    else dispatch_max_shape<DGLHIP_MSG_U_MUL_E, EM_HEAD>(a, stream);
  } else {
    if (em == EM_FULL) dispatch_max_shape<DGLHIP_MSG_COPY_E, EM_FULL>(a, stream);
    else if (em == EM_SCALAR) dispatch_max_shape<DGLHIP_MSG_COPY_E, EM_SCALAR>(a, stream);
    else dispatch_max_shape<DGLHIP_MSG_COPY_E, EM_HEAD>(a, stream);
  }
}

}  // namespace dglhip

using namespace dglhip;

extern "C" {

int dglhip_gspmm_device(int msg_op, int reduce_op, int64_t num_rows,
                        int64_t feat_len, const int64_t* indptr,
                        const int32_t* indices, const int64_t* eid,
                        const float* ufeat, const float* efeat,
                        int64_t efeat_len, float* out, int64_t* arg_out,
                        const int32_t* row_order, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(msg_op >= 0 && msg_op <= 2, "unknown msg op " << msg_op);
  DGLHIP_CHECK(reduce_op >= 0 && reduce_op <= 3, "unknown reduce op " << reduce_op);
  DGLHIP_CHECK(num_rows >= 0 && feat_len >= 0, "negative size");
  if (num_rows == 0 || feat_len == 0) return 0;  // empty tensors may carry null pointers
  DGLHIP_CHECK(indptr != nullptr && out != nullptr, "null indptr/out");
  const bool use_u = msg_op != DGLHIP_MSG_COPY_E;
  const bool use_e = msg_op != DGLHIP_MSG_COPY_U;
  DGLHIP_CHECK(!use_u || ufeat, "ufeat is null");
  DGLHIP_CHECK(!use_e || efeat, "efeat is null");
  DGLHIP_CHECK(!use_e || (efeat_len >= 1 && feat_len % efeat_len == 0),
               "edge feature length " << efeat_len << " must divide feat_len " << feat_len);
  const int64_t elen = use_e ? efeat_len : 1;
  if (reduce_op == DGLHIP_REDUCE_MAX) {
    MaxLaunch m{num_rows, feat_len, elen, indptr, indices, eid, ufeat, efeat, out, arg_out,
                row_order};
    dispatch_max(msg_op, m, stream);
    return 0;
  }
  const bool mean = reduce_op == DGLHIP_REDUCE_MEAN;
  SumLaunch a{num_rows, feat_len, elen, indptr, indices, eid, ufeat, efeat, out, row_order,
              nullptr, nullptr, reduce_op == DGLHIP_REDUCE_SUM_ACCUM,
              stream_output(num_rows, feat_len)};
  dispatch_sum(msg_op, mean, a, stream);
  API_END();
}

int dglhip_gspmm_chunked_device(int msg_op, int reduce_op, int64_t feat_len,
                                const int64_t* indptr, const int32_t* indices,
                                const int64_t* eid, const float* ufeat,
                                const float* efeat, int64_t efeat_len, float* out,
                                int64_t num_light, const int32_t* light_rows,
                                int64_t num_chunks, const int64_t* chunk_beg,
                                const int64_t* chunk_end, int64_t num_heavy,
                                const int32_t* heavy_rows,
                                const int64_t* heavy_chunk_ptr, float* partial,
                                void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(msg_op >= 0 && msg_op <= 2, "unknown msg op " << msg_op);
  DGLHIP_CHECK(reduce_op == DGLHIP_REDUCE_SUM || reduce_op == DGLHIP_REDUCE_MEAN ||
                   reduce_op == DGLHIP_REDUCE_SUM_ACCUM,
               "chunked rows support sum/mean only");
  DGLHIP_CHECK(num_light >= 0 && num_chunks >= 0 && num_heavy >= 0, "negative size");
  if (feat_len == 0) return 0;
  const bool use_u = msg_op != DGLHIP_MSG_COPY_E;
  const bool use_e = msg_op != DGLHIP_MSG_COPY_U;
  DGLHIP_CHECK(!use_u || ufeat, "ufeat is null");
  DGLHIP_CHECK(!use_e || efeat, "efeat is null");
  DGLHIP_CHECK(!use_e || (efeat_len >= 1 && feat_len % efeat_len == 0),
               "edge feature length " << efeat_len << " must divide feat_len " << feat_len);
  DGLHIP_CHECK(num_chunks == 0 || (partial && chunk_beg && chunk_end), "null chunk plan");
  const int64_t elen = use_e ? efeat_len : 1;
  const bool mean = reduce_op == DGLHIP_REDUCE_MEAN;
  const bool accum = reduce_op == DGLHIP_REDUCE_SUM_ACCUM;
  if (num_chunks > 0) {  // heavy-row chunks first: the longest work starts first
    SumLaunch c{num_chunks, feat_len, elen, indptr, indices, eid, ufeat, efeat, partial,
                nullptr, chunk_beg, chunk_end, false};
    dispatch_sum(msg_op, false, c, stream);
  }
  if (num_light > 0) {
    SumLaunch l{num_light, feat_len, elen, indptr, indices, eid, ufeat, efeat, out,
                light_rows, nullptr, nullptr, accum,
                stream_output(num_light + num_heavy, feat_len)};
    dispatch_sum(msg_op, mean, l, stream);
  }
  if (num_heavy > 0) {
    const int64_t blocks = (num_heavy + 3) / 4;
    timed_launch(stream, [&] {
      if (mean)
        hipLaunchKernelGGL((gspmm_combine_kernel<true, false>),
                           dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream,
                           num_heavy, feat_len, indptr, heavy_rows, heavy_chunk_ptr, partial,
                           out);
      else if (accum)
        hipLaunchKernelGGL((gspmm_combine_kernel<false, true>),
                           dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream,
                           num_heavy, feat_len, indptr, heavy_rows, heavy_chunk_ptr, partial,
                           out);
      else
        hipLaunchKernelGGL((gspmm_combine_kernel<false, false>),
                           dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream,
                           num_heavy, feat_len, indptr, heavy_rows, heavy_chunk_ptr, partial,
                           out);
    });
  }
  API_END();
}

int dglhip_gspmm_ranges_device(int msg_op, int64_t num_items, int64_t feat_len,
                               const int64_t* item_beg, const int64_t* item_end,
                               int accumulate, const int32_t* indices, const int64_t* eid,
                               const float* ufeat, const float* efeat, int64_t efeat_len,
                               float* out, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(msg_op >= 0 && msg_op <= 2, "unknown msg op " << msg_op);
  DGLHIP_CHECK(num_items >= 0 && feat_len >= 0, "negative size");
  if (num_items == 0 || feat_len == 0) return 0;
  const bool use_u = msg_op != DGLHIP_MSG_COPY_E;
  const bool use_e = msg_op != DGLHIP_MSG_COPY_U;
  DGLHIP_CHECK(item_beg && item_end && out, "null ranges/out");
  DGLHIP_CHECK(!use_u || ufeat, "ufeat is null");
  DGLHIP_CHECK(!use_e || efeat, "efeat is null");
  DGLHIP_CHECK(!use_e || (efeat_len >= 1 && feat_len % efeat_len == 0),
               "edge feature length " << efeat_len << " must divide feat_len " << feat_len);
  SumLaunch a{num_items, feat_len, use_e ? efeat_len : 1, nullptr, indices, eid, ufeat, efeat,
              out, nullptr, item_beg, item_end, accumulate != 0,
              stream_output(num_items, feat_len)};
  dispatch_sum(msg_op, false, a, stream);
  API_END();
}

int dglhip_gsddmm_device(int op, int64_t num_rows, int64_t feat_len,
                         int64_t num_heads, const int64_t* indptr, const int32_t* indices,
                         const int64_t* eid, const float* lhs,
                         const float* rhs, float* out, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(op == DGLHIP_SDDMM_DOT, "unknown sddmm op " << op);
  DGLHIP_CHECK(num_rows >= 0 && feat_len >= 0, "negative size");
  DGLHIP_CHECK(num_heads >= 1 && feat_len % num_heads == 0,
               "num_heads " << num_heads << " must divide feat_len " << feat_len);
  if (num_rows == 0) return 0;
  DGLHIP_CHECK(indptr && indices && eid && lhs && rhs && out, "null pointer argument");
  const int64_t blocks = (num_rows + 3) / 4;
  DGLHIP_CHECK(blocks <= 0x7fffffff, "grid too large: " << blocks);
  const int64_t D = feat_len / num_heads;
  const bool aligned = (reinterpret_cast<uintptr_t>(lhs) % 16) == 0 &&
                       (reinterpret_cast<uintptr_t>(rhs) % 16) == 0;
  const bool head_ok = D >= 32 ? (D % 32 == 0) : (D == 4 || D == 8 || D == 16);
  const int64_t nb = feat_len % 32 == 0 ? feat_len / 32 : 0;
  const bool sliced = aligned && head_ok && (nb == 1 || nb == 2 || nb == 4 || nb == 8 ||
                                             nb == 16);
  timed_launch(stream, [&] {
#define DGLHIP_SDDMM(NB)                                                                   \
  hipLaunchKernelGGL((gsddmm_dot_sliced_kernel<NB, (NB >= 8 ? 1 : 2)>),                    \
                     dim3(static_cast<unsigned>(blocks)),                                  \
                     dim3(256), 0, stream, num_rows, num_heads, D, indptr, indices, eid, lhs, \
                     rhs, out)
    if (sliced && nb == 1) DGLHIP_SDDMM(1);
    else if (sliced && nb == 2) DGLHIP_SDDMM(2);
    else if (sliced && nb == 4) DGLHIP_SDDMM(4);
    else if (sliced && nb == 8) DGLHIP_SDDMM(8);
    else if (sliced && nb == 16) DGLHIP_SDDMM(16);
    else
      hipLaunchKernelGGL(gsddmm_dot_kernel, dim3(static_cast<unsigned>(blocks)),
                         dim3(256), 0, stream, num_rows, feat_len, num_heads, indptr,
                         indices, eid, lhs, rhs, out);
#undef DGLHIP_SDDMM
  });
  API_END();
}

int dglhip_set_spmm_variant(int vec, int group, int unroll, int pipelined) {
  API_BEGIN();
  DGLHIP_CHECK((vec == 0) || ((vec == 1 || vec == 2 || vec == 4) &&
                              (group == 32 || group == 64) &&
                              (unroll == 4 || unroll == 8 || unroll == 16 || unroll == 32)),
               "unsupported variant " << vec << "," << group << "," << unroll);
  g_var_vec = vec;
  g_var_group = group;
  g_var_unroll = unroll;
  g_var_pipe = pipelined ? 1 : 0;
  API_END();
}

int dglhip_set_cache_policy(int policy) {
  API_BEGIN();
  DGLHIP_CHECK(policy >= -1 && policy <= POL_NT_OUT, "unknown cache policy " << policy);
  g_cache_policy = policy;
  API_END();
}

int dglhip_gsddmm_attention_device(int64_t num_rows, int64_t num_heads,
                                   const int64_t* indptr, const int32_t* indices,
                                   const int64_t* eid, const float* lhs, const float* rhs,
                                   float alpha, float clamp_lo, float clamp_hi, int apply_exp,
                                   float* out, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows >= 0 && num_heads >= 1, "bad sizes");
  if (num_rows == 0) return 0;
  DGLHIP_CHECK(indptr && indices && eid && lhs && rhs && out, "null pointer argument");
  DGLHIP_CHECK((num_rows + 3) / 4 <= 0x7fffffff, "grid too large");
  timed_launch(stream, [&] {
    hipLaunchKernelGGL(gsddmm_attention_kernel, dim3(static_cast<unsigned>((num_rows + 3) / 4)),
                       dim3(256), 0, stream, num_rows, num_heads, indptr, indices, eid, lhs,
                       rhs, alpha, clamp_lo, clamp_hi, apply_exp, out);
  });
  API_END();
}

int dglhip_timing_enable(int enable) {
  API_BEGIN();
  std::lock_guard<std::mutex> lk(g_timing.mu);
  g_timing.enabled = enable != 0;
  g_timing.total_ms = 0.0;
  g_timing.launches = 0;
  for (auto& p : g_timing.pending) g_timing.pool.push_back(p);
  g_timing.pending.clear();
  API_END();
}

int dglhip_timing_read(double* total_ms, int64_t* launches) {
  API_BEGIN();
  std::lock_guard<std::mutex> lk(g_timing.mu);
  for (auto& p : g_timing.pending) {
    HIP_CALL(hipEventSynchronize(p.second));
    float ms = 0.0f;
    HIP_CALL(hipEventElapsedTime(&ms, p.first, p.second));
    g_timing.total_ms += ms;
    g_timing.launches += 1;
    g_timing.pool.push_back(p);
  }
  g_timing.pending.clear();
  if (total_ms) *total_ms = g_timing.total_ms;
  if (launches) *launches = g_timing.launches;
  API_END();
}

}  // extern "C"
