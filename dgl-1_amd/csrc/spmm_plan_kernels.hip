// Device kernels of the g-SpMM launch plan (spmm_plan.h): the E-sized passes
// of the plan build (the monotone-prefix walk over every row's slots, the
// scatter of the slots into item order, the short-row tiers' column ids) and
// the small per-call passes of a planned run (edge values into plan order,
// the first launch's absent rows, the mean's division).
//
// The walk and the scatter give each row one wave: 64 consecutive slots per
// step, coalesced; the source block of a slot is (col - lo) / bs, a decrease
// against the previous slot (DPP-free: __shfl_up, the previous step's last
// lane for lane 0) ends the row's monotone prefix, and run starts (a slot
// whose block differs from its predecessor's) come from one ballot per step.
// The prefix's blocks never decrease, so each (row, block) is one contiguous
// run of slots and its count / its item position are written exactly once.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "common.h"
#include "launch.h"
#include "spmm_plan.h"

namespace dglhip {

namespace {

inline void check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  DGLHIP_CHECK(e == hipSuccess, what << ": " << hipGetErrorString(e));
}

// blocks of 4 waves, one item per wave
inline dim3 wave_grid(int64_t items) { return grid_1d((items + 3) / 4); }

__global__ __launch_bounds__(256) void span_kernel(int64_t nnz, const int32_t* __restrict__ ind,
                                                   int32_t* lo_hi) {
  int lo = INT_MAX, hi = -1;
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < nnz; k += stride) {
    const int c = ind[k];
    lo = c < lo ? c : lo;
    hi = c > hi ? c : hi;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int a = __shfl_xor(lo, o, 64), b = __shfl_xor(hi, o, 64);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(lo_hi, lo);
    atomicMax(lo_hi + 1, hi);
  }
}

__global__ __launch_bounds__(256) void eid_identity_kernel(int64_t nnz,
                                                           const int64_t* __restrict__ eid,
                                                           int32_t* flag) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  bool diff = false;
  for (int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < nnz; k += stride)
    diff |= eid[k] != k;
  if (__ballot(diff) != 0 && (threadIdx.x & 63) == 0) *flag = 1;
}

__device__ __forceinline__ int slot_block(const int32_t* __restrict__ ind, int64_t k, bool valid,
                                          int64_t lo, int64_t bs) {
  return valid ? static_cast<int>((int64_t(ind[k]) - lo) / bs) : INT_MAX;
}

__global__ __launch_bounds__(256) void block_walk_kernel(int64_t R,
                                                         const int64_t* __restrict__ indptr,
                                                         const int32_t* __restrict__ ind,
                                                         int64_t lo, int64_t bs, int B,
                                                         int32_t* __restrict__ counts,
                                                         int64_t* __restrict__ pend) {
  const int64_t r = block_linear() * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const int lane = threadIdx.x & 63;
  const int64_t beg = indptr[r], end = indptr[r + 1];
  int32_t* cnt = counts + r * B;
  int64_t pe = end;
  int prev = -1;                // block of the previous step's last slot
  int run_b = -1;               // a run still open at the end of the previous step
  int64_t run_s = 0;
  for (int64_t base = beg; base < end; base += 64) {
    const int64_t k = base + lane;
    const bool valid = k < end;
    const int b = slot_block(ind, k, valid, lo, bs);
    int pb = __shfl_up(b, 1, 64);
    if (lane == 0) pb = prev;
    const bool dec = valid && k > beg && b < pb;
    const uint64_t decm = __ballot(dec);
    const int limit = decm ? __builtin_ctzll(decm) : 64;
    const bool inpre = valid && lane < limit;
    const bool st = inpre && (k == beg || b != pb);
    const uint64_t stm = __ballot(st);
    const bool term = limit < 64 || base + 64 >= end;
    const int64_t cend = base + limit < end ? base + limit : end;  // the prefix's end here
    if (run_b >= 0 && (stm != 0 || term)) {
      const int64_t close = stm ? base + __builtin_ctzll(stm) : cend;
      if (lane == 0) cnt[run_b] = static_cast<int32_t>(close - run_s);
      run_b = -1;
    }
    if (st) {
      const uint64_t higher = lane == 63 ? 0ull : (stm & (~0ull << (lane + 1)));
      if (higher) cnt[b] = __builtin_ctzll(higher) - lane;
      else if (term) cnt[b] = static_cast<int32_t>(cend - k);
    }
    if (!term && stm) {
      const int last = 63 - __builtin_clzll(stm);
      run_b = __shfl(b, last, 64);
      run_s = base + last;
    }
    if (limit < 64) {
      pe = base + limit;
      break;
    }
    prev = __shfl(b, 63, 64);
  }
  if (lane == 0) pend[r] = pe;
}

__global__ __launch_bounds__(256) void block_scatter_kernel(
    int64_t R, const int64_t* __restrict__ indptr, const int32_t* __restrict__ ind, int64_t lo,
    int64_t bs, int B, const int64_t* __restrict__ pend, const int64_t* __restrict__ item_start,
    const int64_t* __restrict__ sfx_start, int32_t* __restrict__ out_ind,
    int32_t* __restrict__ out_pos) {
  const int64_t r = block_linear() * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const int lane = threadIdx.x & 63;
  const int64_t beg = indptr[r], end = indptr[r + 1];
  const int64_t pe = pend[r];
  const int64_t* ist = item_start + r * B;
  int prev = -1;
  int64_t run_s = beg;
  for (int64_t base = beg; base < end; base += 64) {
    const int64_t k = base + lane;
    const bool valid = k < end;
    const bool inpre = valid && k < pe;
    const int b = slot_block(ind, k, inpre, lo, bs);
    int pb = __shfl_up(b, 1, 64);
    if (lane == 0) pb = prev;
    const bool st = inpre && (k == beg || b != pb);
    const uint64_t stm = __ballot(st);
    const uint64_t le = lane == 63 ? stm : (stm & ((2ull << lane) - 1));
    const int64_t s = le ? base + 63 - __builtin_clzll(le) : run_s;
    if (inpre) {
      const int64_t dst = ist[b] + (k - s);
      out_ind[dst] = ind[k];
      out_pos[dst] = static_cast<int32_t>(k);
    } else if (valid) {
      const int64_t dst = sfx_start[r] + (k - pe);
      out_ind[dst] = ind[k];
      out_pos[dst] = static_cast<int32_t>(k);
    }
    if (stm) run_s = base + 63 - __builtin_clzll(stm);
    prev = __shfl(b, 63, 64);
  }
}

__global__ __launch_bounds__(256) void tier_cols_kernel(int64_t n, const int32_t* __restrict__ rows,
                                                        const int64_t* __restrict__ indptr,
                                                        const int32_t* __restrict__ ind,
                                                        const int64_t* __restrict__ sp,
                                                        int32_t* __restrict__ cols) {
  const int64_t i = block_linear() * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t s = indptr[rows[i]];
  const int64_t o = sp[i], m = sp[i + 1] - o;
  for (int64_t j = 0; j < m; ++j) cols[o + j] = ind[s + j];
}

__global__ __launch_bounds__(256) void compose_kernel(int64_t n, const int32_t* __restrict__ pos,
                                                      const int64_t* __restrict__ map,
                                                      int64_t* __restrict__ out) {
  const int64_t j = block_linear() * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int64_t p = pos[j];
  out[j] = map ? map[p] : p;
}

__global__ __launch_bounds__(256) void gather_vals_kernel(int64_t n,
                                                          const int64_t* __restrict__ rows,
                                                          const float* __restrict__ vals,
                                                          float* __restrict__ out) {
  const int64_t j = block_linear() * blockDim.x + threadIdx.x;
  if (j < n) out[j] = vals[rows[j]];
}

__global__ __launch_bounds__(256) void zero_rows_kernel(int64_t n, const int32_t* __restrict__ rows,
                                                        int64_t F, float* __restrict__ out) {
  const int64_t i = block_linear() * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  float* o = out + int64_t(rows[i]) * F;
  for (int64_t f = threadIdx.x & 63; f < F; f += 64) o[f] = 0.0f;
}

__global__ __launch_bounds__(256) void div_degree_kernel(int64_t R, int64_t F,
                                                         const int64_t* __restrict__ indptr,
                                                         float* __restrict__ out) {
  const int64_t r = block_linear() * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const int64_t d = indptr[r + 1] - indptr[r];
  const float div = static_cast<float>(d > 1 ? d : 1);
  float* o = out + r * F;
  for (int64_t f = threadIdx.x & 63; f < F; f += 64) o[f] = o[f] / div;
}

// out[r] = out[r] + sums[r] / deg r for rows with in-edges (the one-launch
// mean_add store: the chain, divided when deg > 1, added to out; rows without
// in-edges keep out)
__global__ __launch_bounds__(256) void add_mean_kernel(int64_t R, int64_t F,
                                                       const int64_t* __restrict__ indptr,
                                                       const float* __restrict__ sums,
                                                       float* __restrict__ out) {
  const int64_t r = block_linear() * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const int64_t d = indptr[r + 1] - indptr[r];
  if (d == 0) return;
  const float div = static_cast<float>(d);
  const float* sr = sums + r * F;
  float* o = out + r * F;
  for (int64_t f = threadIdx.x & 63; f < F; f += 64) {
    const float m = d > 1 ? sr[f] / div : sr[f];
    o[f] = o[f] + m;
  }
}

// rows of F floats into rows padded to ld floats (the plan's line-aligned
// copy of a narrow source table): element-parallel, reads in order. (A 2-D
// hipMemcpy2DAsync of the same rows ran at ~0.25 TB/s: 155 us for F = 41 on
// the Reddit-shaped graph's 38 MB, r06.)
__global__ __launch_bounds__(256) void pad_rows_kernel(int64_t total, int64_t F, int64_t ld,
                                                       const float* __restrict__ src,
                                                       float* __restrict__ dst) {
  for (int64_t i = block_linear() * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t r = i / F;
    dst[r * ld + (i - r * F)] = src[i];
  }
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace

void plan_pad_rows_device(int64_t n, int64_t F, int64_t ld, const float* src, float* dst,
                          hipStream_t s) {
  const int64_t total = n * F;
  if (total == 0) return;
  const int64_t blocks = std::min<int64_t>(cdiv(total, 256), 65536);
  hipLaunchKernelGGL(pad_rows_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s, total,
                     F, ld, src, dst);
  check_launch("plan padded rows copy");
}

void plan_span_device(int64_t nnz, const int32_t* indices, int32_t* lo_hi, hipStream_t s) {
  if (nnz == 0) return;
  const int64_t blocks = std::min<int64_t>(cdiv(nnz, 256), 4096);
  hipLaunchKernelGGL(span_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s, nnz,
                     indices, lo_hi);
  check_launch("plan span");
}

void plan_eid_identity_device(int64_t nnz, const int64_t* eid, int32_t* flag, hipStream_t s) {
  if (nnz == 0) return;
  const int64_t blocks = std::min<int64_t>(cdiv(nnz, 256), 4096);
  hipLaunchKernelGGL(eid_identity_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s,
                     nnz, eid, flag);
  check_launch("plan eid identity");
}

void plan_block_walk_device(int64_t R, const int64_t* indptr, const int32_t* indices, int64_t lo,
                            int64_t bs, int B, int32_t* counts, int64_t* pend, hipStream_t s) {
  if (R == 0) return;
  hipLaunchKernelGGL(block_walk_kernel, wave_grid(R), dim3(256), 0, s, R, indptr, indices, lo, bs,
                     B, counts, pend);
  check_launch("plan block walk");
}

void plan_block_scatter_device(int64_t R, const int64_t* indptr, const int32_t* indices,
                               int64_t lo, int64_t bs, int B, const int64_t* pend,
                               const int64_t* item_start, const int64_t* sfx_start,
                               int32_t* out_indices, int32_t* out_pos, hipStream_t s) {
  if (R == 0) return;
  hipLaunchKernelGGL(block_scatter_kernel, wave_grid(R), dim3(256), 0, s, R, indptr, indices, lo,
                     bs, B, pend, item_start, sfx_start, out_indices, out_pos);
  check_launch("plan block scatter");
}

void plan_tier_cols_device(int64_t n, const int32_t* rows, const int64_t* indptr,
                           const int32_t* indices, const int64_t* sp, int32_t* cols,
                           hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(tier_cols_kernel, grid_1d(cdiv(n, 256)), dim3(256), 0, s, n, rows, indptr,
                     indices, sp, cols);
  check_launch("plan tier columns");
}

void plan_compose_device(int64_t n, const int32_t* pos, const int64_t* map, int64_t* out,
                         hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(compose_kernel, grid_1d(cdiv(n, 256)), dim3(256), 0, s, n, pos, map, out);
  check_launch("plan compose");
}

void plan_gather_vals_device(int64_t n, const int64_t* rows, const float* vals, float* out,
                             hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(gather_vals_kernel, grid_1d(cdiv(n, 256)), dim3(256), 0, s, n, rows, vals,
                     out);
  check_launch("plan gather values");
}

void plan_zero_rows_device(int64_t n, const int32_t* rows, int64_t F, float* out, hipStream_t s) {
  if (n == 0 || F == 0) return;
  hipLaunchKernelGGL(zero_rows_kernel, wave_grid(n), dim3(256), 0, s, n, rows, F, out);
  check_launch("plan zero rows");
}

void plan_div_degree_device(int64_t R, int64_t F, const int64_t* indptr, float* out,
                            hipStream_t s) {
  if (R == 0 || F == 0) return;
  hipLaunchKernelGGL(div_degree_kernel, wave_grid(R), dim3(256), 0, s, R, F, indptr, out);
  check_launch("plan mean division");
}

void plan_add_mean_device(int64_t R, int64_t F, const int64_t* indptr, const float* sums,
                          float* out, hipStream_t s) {
  if (R == 0 || F == 0) return;
  hipLaunchKernelGGL(add_mean_kernel, wave_grid(R), dim3(256), 0, s, R, F, indptr, sums, out);
  check_launch("plan mean addition");
}

}  // namespace dglhip
