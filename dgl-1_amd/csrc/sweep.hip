// Source-swept g-SpMM (copy_u + sum / mean, fp32 rows of 64 * VEC floats):
// one launch per "generation" of destination rows whose running sums live in
// LDS, each wave walking its rows' slots source block by source block.
//
// The source-blocked schedule (spmm_plan.cc) gets the L2 hit
// rate of small source slices by running one launch per slice; each launch
// re-reads and re-writes every row's running sum (19 passes over the 119 MB
// output on the Reddit-shaped graph) and ends on its longest items. Here a
// wave owns up to RPW rows for the whole launch and keeps their sums in LDS
// (160 KB per CU: 320 rows of 512 B), so a block boundary costs an LDS read and
// write instead of an HBM-side pass, and all waves of a launch sweep the same
// blocks in the same order (they start together and carry the same work per
// block, rows being dealt to waves in a snake over the degree-descending order).
//
// Chain order: every row's slots are taken strictly in slot order. In block b
// a wave advances a row's cursor over the slots whose source lies below block
// b's end, stopping at the first that does not; the last block takes the
// rest. So the sum is the one-launch kernel's chain for ANY edge order (a row
// whose sources go back down just does part of its work in a later block) —
// the blocked schedule's precondition (source-monotone chains) only decides
// how well the L2s serve the gathers, not the bits.
//
// Reference: the product this evaluates is the COO spmm of
// python/dgl/backend/pytorch/tensor.py:145-146 on the adjacency of
// src/graph/graph.cc:509-524; the chain is the oracle's
// (oracle/spmm_oracle.c).
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdlib>

#include "gspmm_impl.h"

namespace dglhip {
namespace {

constexpr int kSweepWaves = 4;  // waves per workgroup
constexpr int kMaxLagBlocks = 256;  // source blocks the soft barrier covers
constexpr int kShards = 8, kStride = 32;

// the soft barrier's two halves (once per block and wave)
__device__ __noinline__ void sweep_arrive(int* wg_done, int* arrive, int b) {
  const int lane = threadIdx.x & 63;
  int last = 0;
  if (lane == 0) last = atomicAdd(&wg_done[b], 1) == kSweepWaves - 1;
  if (__builtin_amdgcn_readfirstlane(last) && lane == 0)
    __hip_atomic_fetch_add(arrive + (int64_t(b) * kShards + blockIdx.x % kShards) * kStride, 1,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Waits until every workgroup of the launch that has STARTED (the counter
// `started`, one add per workgroup as it begins) has finished block b; a
// workgroup not yet resident (the CU held by another stream's kernel) is
// not waited for — it runs later, on its own. false when max_spin polls ran
// out (a safety net: the wave then stops waiting).
__device__ __noinline__ bool sweep_wait(const int* arrive, const int* started, int b,
                                        int max_spin) {
  const int lane = threadIdx.x & 63;
  const int* c = arrive + int64_t(b) * kShards * kStride;
  for (int spin = 0; spin < max_spin; ++spin) {
    int seen = lane < kShards ? __hip_atomic_load(c + lane * kStride, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT)
                              : 0;
    const int need =
        lane == kShards ? __hip_atomic_load(started, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                        : 0;
#pragma unroll
    for (int d = 1; d < kShards; d <<= 1) seen += __shfl_xor(seen, d);
    if (__builtin_amdgcn_readfirstlane(seen) >= __builtin_amdgcn_readlane(need, kShards))
      return true;
    __builtin_amdgcn_s_sleep(8);
  }
  return false;
}

// Waits that ran out of polls (sweep_wait returned false), over every launch
// on this device since the last reset; read through
// dglhip_sweep_barrier_expiries. One vector atomic per expiry (lane 0 of the
// wave that gave up), none on the waits that succeed.
__device__ unsigned long long g_sweep_expired = 0;

__device__ __forceinline__ int32_t lane_of(int32_t v, int j) {
  return __builtin_amdgcn_readlane(v, j);
}

// Kernel arguments: rows [0, num_rows) of the CSR (indptr, indices) are dealt
// to waves_total waves over all launches of one call; this launch runs waves
// [wave_base, wave_base + gridDim.x * 4). Source block b covers columns
// [lo + b * bs, lo + (b + 1) * bs); block nblocks - 1 takes everything left.
template <int VEC, int RPW, int UNROLL, bool MEAN>
__global__ __launch_bounds__(256) void gspmm_sweep_kernel(
    int64_t num_rows, int64_t waves_total, int64_t wave_base,
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const float* __restrict__ ufeat, float* __restrict__ out,
    const int32_t* __restrict__ row_order, int64_t lo, int64_t bs, int nblocks) {
  typedef typename Vec<VEC>::T V;
  constexpr int F = 64 * VEC;
  __shared__ float sums[kSweepWaves * RPW * F];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int64_t wv = wave_base + int64_t(blockIdx.x) * kSweepWaves + w;
  const int64_t f0 = int64_t(lane) * VEC;
  // lane j < RPW describes the wave's j-th row: round j of a snake deal of
  // the degree-descending rows over all waves (rows are a prefix of the lanes)
  int32_t row = -1, len = 0, cur = 0, beg_lo = 0, beg_hi = 0;
  if (lane < RPW && wv < waves_total) {
    const int64_t pos = (lane & 1) ? (waves_total - 1 - wv) : wv;
    const int64_t i = int64_t(lane) * waves_total + pos;
    if (i < num_rows) {
      row = row_order ? row_order[i] : static_cast<int32_t>(i);
      const int64_t b = indptr[row];
      len = static_cast<int32_t>(indptr[row + 1] - b);
      beg_lo = static_cast<int32_t>(b);
      beg_hi = static_cast<int32_t>(b >> 32);
    }
  }
  const int nrows = __builtin_popcountll(__ballot(row >= 0));
  float* my = sums + w * RPW * F;
  for (int j = 0; j < nrows; ++j) stv<VEC>(my + j * F + f0, Vec<VEC>::zero());

  // a row's slot chunk: the column ids of its next min(64, left) slots
  auto chunk = [&](int j, int32_t c, int32_t n_all) -> int32_t {
    const int64_t beg = (int64_t(lane_of(beg_hi, j)) << 32) |
                        static_cast<uint32_t>(lane_of(beg_lo, j));
    return lane < n_all - c ? indices[beg + c + lane] : INT_MAX;
  };
  // the next visit's first chunk is loaded before this visit's gathers, so
  // its latency hides behind them (not with one row: its cursor moves)
  int32_t pre = INT_MAX;
  bool have_pre = false;
  for (int b = 0; b < nblocks; ++b) {
    const int64_t bend = (b == nblocks - 1) ? INT64_MAX : lo + int64_t(b + 1) * bs;
    for (int j = 0; j < nrows; ++j) {
      const int32_t c0 = lane_of(cur, j);
      const int32_t n_all = lane_of(len, j);
      const bool had = have_pre;
      have_pre = false;
      if (c0 >= n_all) continue;
      int32_t col = had ? pre : chunk(j, c0, n_all);
      if (nrows > 1 && !(j + 1 == nrows && b + 1 == nblocks)) {
        const int jn = j + 1 < nrows ? j + 1 : 0;
        const int32_t cn = lane_of(cur, jn), ln = lane_of(len, jn);
        if (cn < ln) {
          pre = chunk(jn, cn, ln);
          have_pre = true;
        }
      }
      V acc = ldv<VEC>(my + j * F + f0);
      int32_t c = c0;
      while (true) {
        const int32_t avail = min(64, n_all - c);
        const uint64_t ok = __ballot(lane < avail && int64_t(col) < bend);
        const int n = ~ok == 0 ? 64 : __builtin_ctzll(~ok);
        int t = 0;
        for (; t + UNROLL <= n; t += UNROLL) {
          V s[UNROLL];
#pragma unroll
          for (int u = 0; u < UNROLL; ++u)
            s[u] = gather_row_buf<VEC>(ufeat + int64_t(lane_of(col, t + u)) * F, F, f0);
#pragma unroll
          for (int u = 0; u < UNROLL; ++u) acc += s[u];
        }
        if (t < n) {
          // the last n - t < UNROLL slots as one predicated batch
          const int rem = n - t;
          V s[UNROLL];
#pragma unroll
          for (int u = 0; u < UNROLL - 1; ++u)
            if (u < rem)
              s[u] = gather_row_buf<VEC>(ufeat + int64_t(lane_of(col, t + u)) * F, F, f0);
#pragma unroll
          for (int u = 0; u < UNROLL - 1; ++u)
            if (u < rem) acc += s[u];
        }
        c += n;
        if (n < avail || c >= n_all) break;
        col = chunk(j, c, n_all);
      }
      stv<VEC>(my + j * F + f0, acc);
      if (lane == j) cur = c;
    }
  }
  for (int j = 0; j < nrows; ++j) {
    const int32_t r = lane_of(row, j);
    V acc = ldv<VEC>(my + j * F + f0);
    if (MEAN) {
      const int32_t d = lane_of(len, j);
      if (d > 1) acc = acc / Vec<VEC>::splat(static_cast<float>(d));
    }
    stv<VEC>(out + int64_t(r) * F + f0, acc);
  }
}

// Streamed variant: the slots are laid out per (launch, block, wave, row) by
// the host (tools/r05/sweep_study.py builds the layout), so a wave's work in
// block b is one contiguous run of column ids lay[seg_beg[wave, b] ...]
// holding its rows' block-b slots back to back (counts[row, b] each). The
// gathers stream through it in batches of UNROLL across row boundaries; the
// running sum switches rows (LDS store + load) where a row's run ends. Exact
// for source-monotone chains (each row's block-b slots contiguous in slot
// order), which the layout builder checks.
// MODE 0 sum, 1 mean, 2 sum continuing every row's chain from its value in
// out (the pipelined multi-GPU segments' SUM_ACCUM).
// RR (r06): the wave's last RR rows keep their running sums in registers
// (two floats per lane per row: a pair of RR-wide register vectors indexed
// by the wave-uniform row, GPR indexing mode, no scratch) and the first
// RPW - RR in LDS, so a CU holds RPW rows per wave instead of the LDS's
// share: fewer launches (row generations) re-sweep the source blocks.
template <int RR>
struct RegRows {
  typedef float T __attribute__((ext_vector_type(RR)));
  T x, y;
};
template <>
struct RegRows<0> {};

template <int VEC, int RPW, int UNROLL, int MODE, int RR = 0>
__global__ __launch_bounds__(256) void gspmm_sweep_stream_kernel(
    int64_t num_rows, int64_t waves_total, int64_t wave_base,
    const int32_t* __restrict__ row_order, const int32_t* __restrict__ counts, int nblocks,
    const int64_t* __restrict__ seg_beg, const int32_t* __restrict__ lay,
    const int64_t* __restrict__ indptr, const float* __restrict__ ufeat,
    float* __restrict__ out, int* __restrict__ arrive, int lag, int max_spin) {
  typedef typename Vec<VEC>::T V;
  constexpr int F = 64 * VEC;
  constexpr int RL = RPW - RR;  // rows whose sums live in LDS
  static_assert(RR == 0 || VEC == 2, "register rows hold two floats per lane");
  static_assert(RPW <= 64 && RL >= 1, "a lane describes each row of the wave");
  __shared__ float sums[kSweepWaves * RL * F];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int64_t wv = wave_base + int64_t(blockIdx.x) * kSweepWaves + w;
  const int64_t f0 = int64_t(lane) * VEC;
  // Soft barrier (lag > 0): a wave starts block b once every workgroup of
  // the launch has finished block b - lag, or after max_spin polls (the
  // results never depend on it, only the L2 locality). The last wave of a
  // workgroup to finish a block (an LDS counter per block) adds 1 to one of 8
  // device-scope counters of that block (sharded by workgroup, each on its
  // own 128-B line); a waiting wave polls the 8 with device-scope loads.
  __shared__ int wg_done[kMaxLagBlocks];
  const bool sync = lag > 0 && nblocks <= kMaxLagBlocks;
  // the launch's workgroups that have begun: after the nblocks blocks' counters
  int* started = sync ? arrive + int64_t(nblocks) * kShards * kStride : nullptr;
  if (sync) {
    for (int i = threadIdx.x; i < kMaxLagBlocks; i += blockDim.x) wg_done[i] = 0;
    if (threadIdx.x == 0)
      __hip_atomic_fetch_add(started, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
  }
  auto arrive_at = [&](int b) {
    if (sync) sweep_arrive(wg_done, arrive, b);
  };
  bool waiting = true;
  auto wait_for = [&](int b) {
    if (sync && waiting && b >= lag) {
      waiting = sweep_wait(arrive, started, b - lag, max_spin);
      if (!waiting && lane == 0)
        __hip_atomic_fetch_add(&g_sweep_expired, 1ull, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  int32_t row = -1, deg = 0;
  if (lane < RPW && wv < waves_total) {
    const int64_t pos = (lane & 1) ? (waves_total - 1 - wv) : wv;
    const int64_t i = int64_t(lane) * waves_total + pos;
    if (i < num_rows) {
      row = row_order ? row_order[i] : static_cast<int32_t>(i);
      if (MODE == 1) deg = static_cast<int32_t>(indptr[row + 1] - indptr[row]);
    }
  }
  const int nrows = __builtin_popcountll(__ballot(row >= 0));
  if (nrows == 0) {
    for (int b = 0; b < nblocks; ++b) arrive_at(b);
    return;
  }
  float* my = sums + w * RL * F;
  RegRows<RR> reg;
  if constexpr (RR > 0) reg.x = reg.y = 0.0f;
  // row j's running sum: LDS for j < RL, registers past it (j is wave-uniform)
  auto get = [&](int j) -> V {
    if constexpr (RR > 0) {
      if (j >= RL) {
        V v;
        v.x = reg.x[j - RL];
        v.y = reg.y[j - RL];
        return v;
      }
    }
    return ldv<VEC>(my + j * F + f0);
  };
  auto put = [&](int j, V v) {
    if constexpr (RR > 0) {
      if (j >= RL) {
        reg.x[j - RL] = v.x;
        reg.y[j - RL] = v.y;
        return;
      }
    }
    stv<VEC>(my + j * F + f0, v);
  };
  for (int j = 0; j < nrows; ++j)
    put(j, MODE == 2 ? ldv<VEC>(out + int64_t(lane_of(row, j)) * F + f0) : Vec<VEC>::zero());
  int32_t cnt_next = row >= 0 ? counts[int64_t(row) * nblocks] : 0;
  int64_t base_next = seg_beg[wv * nblocks];
  for (int b = 0; b < nblocks; ++b) {
    // the previous block's arrival, at one site for both of its exits (two
    // sites cost the gather loop 30 VGPRs: 88 -> 58)
    if (b > 0) arrive_at(b - 1);
    const int32_t cnt = cnt_next;
    // uniform by construction; said so, the column ids load through SGPRs
    const int32_t* run = lay + ((int64_t(__builtin_amdgcn_readfirstlane(
                                     static_cast<int32_t>(base_next >> 32))) << 32) |
                                static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(
                                    static_cast<int32_t>(base_next))));
    if (b + 1 < nblocks) {
      cnt_next = row >= 0 ? counts[int64_t(row) * nblocks + b + 1] : 0;
      base_next = seg_beg[wv * nblocks + b + 1];
    }
    int32_t incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int32_t v = __shfl_up(incl, d);
      if (lane >= d) incl += v;
    }
    const int32_t total = lane_of(incl, 63);
    wait_for(b);
    if (total == 0) continue;
    const uint64_t live = __ballot(cnt > 0);
    int j = __builtin_ctzll(live);
    int32_t rend = lane_of(incl, j);
    V acc = get(j);
    for (int32_t t = 0; t < total; t += UNROLL) {
      const int rem = min(UNROLL, total - t);
      V s[UNROLL];
      if (rem == UNROLL) {
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
          s[u] = gather_row_buf<VEC>(ufeat + int64_t(run[t + u]) * F, F, f0);
      } else {
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
          if (u < rem) s[u] = gather_row_buf<VEC>(ufeat + int64_t(run[t + u]) * F, F, f0);
      }
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        if (u < rem) {
          if (t + u == rend) {
            put(j, acc);
            j = __builtin_ctzll(live & (~0ull << (j + 1)));
            rend = lane_of(incl, j);
            acc = get(j);
          }
          acc += s[u];
        }
      }
    }
    put(j, acc);
  }
  arrive_at(nblocks - 1);
  for (int j = 0; j < nrows; ++j) {
    const int32_t r = lane_of(row, j);
    V acc = get(j);
    if (MODE == 1) {
      const int32_t d = lane_of(deg, j);
      if (d > 1) acc = acc / Vec<VEC>::splat(static_cast<float>(d));
    }
    stv<VEC>(out + int64_t(r) * F + f0, acc);
  }
}

int g_sweep_per_cu = 0;  // study knob: workgroups per CU of a launch (0: occupancy)
// rows per wave the plan lays the streamed sweep out for (19: all in LDS;
// 35 / 51: 16 / 32 more in registers, 124 VGPRs at 51, still 4 waves per
// SIMD: emulated N = 8 rank 7.15 -> 6.90 ms); DGLHIP_SWEEP_ROWS
int g_sweep_rows = [] {
  const char* e = std::getenv("DGLHIP_SWEEP_ROWS");
  const int v = e ? std::atoi(e) : 0;
  return (v == 10 || v == 19 || v == 35 || v == 51) ? v : 51;
}();
int g_sweep_unroll = 16;  // study knob: row gathers in flight per wave (16 or 32)

template <typename K>
int64_t sweep_waves_per_launch(K kern, int cap = 0) {
  int dev = 0, cus = 0, per_cu = 0;
  HIP_CALL(hipGetDevice(&dev));
  HIP_CALL(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  HIP_CALL(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * kSweepWaves, 0));
  if (cap <= 0) cap = g_sweep_per_cu;
  if (cap > 0) per_cu = std::min(per_cu, cap);
  DGLHIP_CHECK(cus > 0 && per_cu > 0, "sweep kernel does not fit a CU");
  return int64_t(cus) * per_cu * kSweepWaves;
}

template <int RPW, int U, int RR>
auto stream_kernel_u(int mode) {
  return mode == 2 ? gspmm_sweep_stream_kernel<2, RPW, U, 2, RR>
         : mode == 1 ? gspmm_sweep_stream_kernel<2, RPW, U, 1, RR>
                     : gspmm_sweep_stream_kernel<2, RPW, U, 0, RR>;
}

template <int RPW, int RR = 0>
auto stream_kernel(int mode) {
  return g_sweep_unroll == 32 ? stream_kernel_u<RPW, 32, RR>(mode)
                              : stream_kernel_u<RPW, 16, RR>(mode);
}

// rows per wave of the streamed kernel: 10 or 19 in LDS; 19 in LDS plus 16
// or 32 in registers (35, 51)
bool stream_rows_ok(int rows_per_wave) {
  return rows_per_wave == 10 || rows_per_wave == 19 || rows_per_wave == 35 ||
         rows_per_wave == 51;
}

template <typename Fn>
auto with_stream_kernel(int rows_per_wave, int mode, Fn fn) {
  switch (rows_per_wave) {
    case 10: return fn(stream_kernel<10>(mode));
    case 35: return fn(stream_kernel<35, 16>(mode));
    case 51: return fn(stream_kernel<51, 32>(mode));
    default: return fn(stream_kernel<19>(mode));
  }
}

template <int VEC, int RPW, bool MEAN>
void launch_sweep(int64_t num_rows, const int64_t* indptr, const int32_t* indices,
                  const float* ufeat, float* out, const int32_t* row_order, int64_t lo,
                  int64_t bs, int nblocks, hipStream_t stream) {
  constexpr int UNROLL = 16;
  auto kern = gspmm_sweep_kernel<VEC, RPW, UNROLL, MEAN>;
  int dev = 0, cus = 0, per_cu = 0;
  HIP_CALL(hipGetDevice(&dev));
  HIP_CALL(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  HIP_CALL(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * kSweepWaves, 0));
  DGLHIP_CHECK(cus > 0 && per_cu > 0, "sweep kernel does not fit a CU");
  // one launch = every workgroup resident at once, so its waves sweep the
  // source blocks together
  const int64_t wgs = int64_t(cus) * per_cu;
  const int64_t rows_per_launch = wgs * kSweepWaves * RPW;
  const int64_t launches = (num_rows + rows_per_launch - 1) / rows_per_launch;
  const int64_t waves_total = launches * wgs * kSweepWaves;
  for (int64_t l = 0; l < launches; ++l) {
    timed_launch(stream, [&] {
      hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(wgs)), dim3(64 * kSweepWaves), 0, stream,
                         num_rows, waves_total, l * wgs * kSweepWaves, indptr, indices, ufeat,
                         out, row_order, lo, bs, nblocks);
    });
  }
}

}  // namespace
}  // namespace dglhip

using namespace dglhip;

extern "C" {

int dglhip_gspmm_sweep_device(int64_t num_rows, int64_t feat_len, const int64_t* indptr,
                              const int32_t* indices, const float* ufeat, float* out,
                              const int32_t* row_order, int64_t col_lo, int64_t block_cols,
                              int num_blocks, int mean, int rows_per_wave, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows >= 0 && num_rows < (int64_t(1) << 31), "row count " << num_rows);
  DGLHIP_CHECK(num_blocks >= 1 && block_cols >= 1 && col_lo >= 0,
               "blocks " << num_blocks << " of " << block_cols << " columns from " << col_lo);
  DGLHIP_CHECK(feat_len == 64 || feat_len == 128 || feat_len == 256,
               "sweep rows are 64, 128 or 256 floats, not " << feat_len);
  if (num_rows == 0) return 0;
  DGLHIP_CHECK(indptr && out && (ufeat || indices == nullptr), "null indptr/ufeat/out");
  const int rpw = rows_per_wave > 0 ? rows_per_wave : 20;
  const bool m = mean != 0;
#define DGLHIP_SWEEP(VEC, R)                                                                 \
  do {                                                                                       \
    if (m) launch_sweep<VEC, R, true>(num_rows, indptr, indices, ufeat, out, row_order,      \
                                      col_lo, block_cols, num_blocks, stream);               \
    else launch_sweep<VEC, R, false>(num_rows, indptr, indices, ufeat, out, row_order,       \
                                     col_lo, block_cols, num_blocks, stream);                \
  } while (0)
  if (feat_len == 128) {
    DGLHIP_CHECK(rpw == 10 || rpw == 20, "rows per wave " << rpw << " at 128 floats: 10 or 20");
    if (rpw == 10) DGLHIP_SWEEP(2, 10);
    else DGLHIP_SWEEP(2, 20);
  } else if (feat_len == 64) {
    DGLHIP_CHECK(rpw == 20 || rpw == 40, "rows per wave " << rpw << " at 64 floats: 20 or 40");
    if (rpw == 20) DGLHIP_SWEEP(1, 20);
    else DGLHIP_SWEEP(1, 40);
  } else {
    DGLHIP_CHECK(rpw == 5 || rpw == 10, "rows per wave " << rpw << " at 256 floats: 5 or 10");
    if (rpw == 5) DGLHIP_SWEEP(4, 5);
    else DGLHIP_SWEEP(4, 10);
  }
#undef DGLHIP_SWEEP
  API_END();
}

int dglhip_set_sweep_per_cu(int per_cu) {
  API_BEGIN();
  DGLHIP_CHECK(per_cu >= 0, "workgroups per CU " << per_cu);
  g_sweep_per_cu = per_cu;
  API_END();
}

int dglhip_set_sweep_rows(int rows_per_wave) {
  API_BEGIN();
  DGLHIP_CHECK(stream_rows_ok(rows_per_wave), "rows per wave " << rows_per_wave);
  g_sweep_rows = rows_per_wave;
  API_END();
}

int dglhip_get_sweep_rows(int* rows_per_wave) {
  API_BEGIN();
  DGLHIP_CHECK(rows_per_wave, "null output");
  *rows_per_wave = g_sweep_rows;
  API_END();
}

int dglhip_set_sweep_unroll(int unroll) {
  API_BEGIN();
  DGLHIP_CHECK(unroll == 16 || unroll == 32, "gathers in flight " << unroll);
  g_sweep_unroll = unroll;
  API_END();
}

int dglhip_sweep_barrier_expiries(int reset, int64_t* out) {
  API_BEGIN();
  DGLHIP_CHECK(out, "null output");
  unsigned long long v = 0;
  HIP_CALL(hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_sweep_expired), sizeof(v), 0,
                               hipMemcpyDeviceToHost));
  *out = static_cast<int64_t>(v);
  if (reset) {
    const unsigned long long zero = 0;
    HIP_CALL(hipMemcpyToSymbol(HIP_SYMBOL(g_sweep_expired), &zero, sizeof(zero), 0,
                               hipMemcpyHostToDevice));
  }
  API_END();
}

int dglhip_gspmm_sweep_stream_geometry_mode(int rows_per_wave, int per_cu, int mode,
                                            int64_t* waves_per_launch) {
  API_BEGIN();
  DGLHIP_CHECK(stream_rows_ok(rows_per_wave), "rows per wave " << rows_per_wave);
  DGLHIP_CHECK(per_cu >= 0, "workgroups per CU " << per_cu);
  DGLHIP_CHECK(mode >= 0 && mode <= 2, "mode " << mode);
  DGLHIP_CHECK(waves_per_launch, "null output");
  // the kernel dglhip_gspmm_sweep_stream_device launches for this mode at the
  // current gathers-in-flight knob
  *waves_per_launch = with_stream_kernel(
      rows_per_wave, mode, [&](auto kern) { return sweep_waves_per_launch(kern, per_cu); });
  API_END();
}

int dglhip_gspmm_sweep_stream_geometry(int rows_per_wave, int per_cu,
                                       int64_t* waves_per_launch) {
  return dglhip_gspmm_sweep_stream_geometry_mode(rows_per_wave, per_cu, 0, waves_per_launch);
}

int dglhip_gspmm_sweep_stream_device(int64_t num_rows, int64_t waves_total,
                                     const int32_t* row_order, const int32_t* counts,
                                     int num_blocks, const int64_t* seg_beg, const int32_t* lay,
                                     const int64_t* indptr, const float* ufeat, float* out,
                                     int mode, int rows_per_wave, int per_cu, int* arrive,
                                     int64_t arrive_len, int lag, int max_spin, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(stream_rows_ok(rows_per_wave), "rows per wave " << rows_per_wave);
  DGLHIP_CHECK(num_rows >= 0 && num_rows < (int64_t(1) << 31) && num_blocks >= 1, "sizes");
  DGLHIP_CHECK(mode >= 0 && mode <= 2 && per_cu >= 0, "mode " << mode << ", per_cu " << per_cu);
  if (num_rows == 0) return 0;
  with_stream_kernel(rows_per_wave, mode, [&](auto kern) {
  const int64_t wpl = sweep_waves_per_launch(kern, per_cu);
  DGLHIP_CHECK(waves_total % wpl == 0 && waves_total * rows_per_wave >= num_rows,
               "layout for " << waves_total << " waves, launches hold " << wpl);
  DGLHIP_CHECK(lag <= 0 || arrive, "the soft barrier needs its counters");
  const int64_t launches = waves_total / wpl;
  // per launch and block 8 counters on 128-B lines of their own, then the
  // launch's count of workgroups begun
  const int64_t per_launch = (int64_t(num_blocks) * 8 + 1) * 32;
  DGLHIP_CHECK(lag <= 0 || arrive_len >= launches * per_launch,
               "the barrier needs " << launches * per_launch << " counters, got " << arrive_len);
  if (lag > 0)
    HIP_CALL(hipMemsetAsync(arrive, 0, sizeof(int) * launches * per_launch, stream));
  for (int64_t l = 0; l < launches; ++l) {
    timed_launch(stream, [&] {
      hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(wpl / kSweepWaves)),
                         dim3(64 * kSweepWaves), 0, stream, num_rows, waves_total, l * wpl,
                         row_order, counts, num_blocks, seg_beg, lay, indptr, ufeat, out,
                         lag > 0 ? arrive + l * per_launch : nullptr, lag, max_spin);
    });
  }
  return 0;
  });
  API_END();
}

}  // extern "C"
