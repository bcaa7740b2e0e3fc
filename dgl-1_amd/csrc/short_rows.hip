// g-SpMM over rows with few slots (copy_u, sum / mean / sum_accum): the tail
// of the degree-descending schedule of a power-law graph.
//
// The main kernel (gspmm_impl.h) gives every row a wave. A row of d slots
// then has only d gathers in flight and one 512-B store (F = 128), and an
// empty row a wave that only stores zeros. On RMAT-26 (tools/rmat_tail_study.py)
// the 15.5M rows of 1..4 slots ran at 3.1 TB/s and the 40M empty rows at
// 2.1 TB/s of their bytes, 17 of the 85 ms of the light-row launch.
//
// Here the short rows come as a compacted CSR of their own, built once per
// schedule (kernel.CSR.tiers): item i is output row rows[i], its column ids
// slot_cols[slot_ptr[i] .. slot_ptr[i+1]) in slot order. A wave takes R
// consecutive items — their row ids, slot ranges and column ids are
// sequential loads, not gathers through indptr — and issues the gathers of all
// of them before any add (R * MAXD in flight: 32), then runs each row's chain
// in slot order and stores the rows. Rows longer than MAXD
// are handled in batches of MAXD slots (correct for any length; the caller
// routes only short rows here). The chain per output element is the main
// kernel's (0 + x_0 + x_1 + ..., or continued from out for sum_accum), so
// the results are bit-identical. MAXD = 0: rows without slots, R of them per
// wave, stored as zeros.

#include "gspmm_impl.h"

namespace dglhip {

template <int VEC, int MAXD, int R, int MSG, int POL>
__global__ __launch_bounds__(256) void gspmm_short_rows_kernel(
    int64_t num_items, int64_t F, const int32_t* __restrict__ rows,
    const int64_t* __restrict__ slot_ptr, const int32_t* __restrict__ slot_cols,
    const float* __restrict__ ufeat, float* __restrict__ out, int mean, int accum, int64_t ldu) {
  typedef typename Vec<VEC>::T V;
  const int64_t wave = block_linear() * (blockDim.x >> 6) +
                       __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int64_t first = wave * R;
  if (first >= num_items) return;
  const int lane = threadIdx.x & 63;
  // the wave's R items are consecutive: their row ids and slot ranges are
  // sequential loads, and the items' column ids one contiguous run
  int64_t row[R], beg[R], deg[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const bool ok = first + r < num_items;
    row[r] = ok ? int64_t(rows[first + r]) : -1;
    if (MAXD > 0) {
      beg[r] = ok ? slot_ptr[first + r] : 0;
      deg[r] = ok ? slot_ptr[first + r + 1] - beg[r] : 0;
    } else {
      beg[r] = deg[r] = 0;
    }
  }
  int64_t dmax = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) dmax = deg[r] > dmax ? deg[r] : dmax;
  for (int64_t f0 = int64_t(lane) * VEC; f0 < F; f0 += 64 * VEC) {
    V acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r)
      acc[r] = (accum && !mean && row[r] >= 0) ? ldv<VEC>(out + row[r] * F + f0)
                                               : Vec<VEC>::zero();
    if (MAXD > 0) {
      for (int64_t b = 0; b < dmax; b += MAXD) {  // one batch unless a row is long
        V v[R][MAXD > 0 ? MAXD : 1];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
          for (int j = 0; j < MAXD; ++j)
            if (b + j < deg[r]) {
              const int32_t c = slot_cols[beg[r] + b + j];
              if (MSG == DGLHIP_MSG_COPY_U_BF16) v[r][j] = gather_bf16<VEC>(ufeat, c, ldu, f0);
              else v[r][j] = gather_row<VEC, POL_DEFAULT>(ufeat, c, ldu, f0);
            }
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
          for (int j = 0; j < MAXD; ++j)
            if (b + j < deg[r]) acc[r] += v[r][j];
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (row[r] < 0) continue;
      V a = acc[r];
      if (mean && deg[r] > 1) a = a / Vec<VEC>::splat(static_cast<float>(deg[r]));
      if (mean && accum) a = ldv<VEC>(out + row[r] * F + f0) + a;  // out + mean
      store_row<VEC, POL>(out + row[r] * F + f0, a);
    }
  }
}

template <int VEC, int MAXD, int R, int MSG>
static void launch_short(int64_t n, int64_t F, int64_t ldu, const int32_t* rows,
                         const int64_t* slot_ptr, const int32_t* slot_cols, const float* ufeat,
                         float* out, bool mean, bool accum, bool nt, hipStream_t stream) {
  const int64_t waves = (n + R - 1) / R;
  const int64_t blocks = (waves + 3) / 4;
  timed_launch(stream, [&] {
    if (nt)
      hipLaunchKernelGGL((gspmm_short_rows_kernel<VEC, MAXD, R, MSG, POL_NT_OUT>),
                         grid_1d(blocks), dim3(256), 0, stream, n, F, rows, slot_ptr,
                         slot_cols, ufeat, out, mean ? 1 : 0, accum ? 1 : 0, ldu);
    else
      hipLaunchKernelGGL((gspmm_short_rows_kernel<VEC, MAXD, R, MSG, POL_DEFAULT>),
                         grid_1d(blocks), dim3(256), 0, stream, n, F, rows, slot_ptr,
                         slot_cols, ufeat, out, mean ? 1 : 0, accum ? 1 : 0, ldu);
  });
}

template <int VEC, int MSG>
static void dispatch_short(int64_t max_deg, int64_t n, int64_t F, int64_t ldu, const int32_t* rows,
                           const int64_t* slot_ptr, const int32_t* slot_cols,
                           const float* ufeat, float* out, bool mean, bool accum, bool nt,
                           hipStream_t stream) {
  // R * MAXD = 32 gathers in flight per wave (the main kernel keeps 16)
  if (max_deg == 0)
    launch_short<VEC, 0, 16, MSG>(n, F, ldu, rows, slot_ptr, slot_cols, ufeat, out, mean, accum,
                                  nt, stream);
  else if (max_deg <= 4)
    launch_short<VEC, 4, 8, MSG>(n, F, ldu, rows, slot_ptr, slot_cols, ufeat, out, mean, accum,
                                 nt, stream);
  else
    launch_short<VEC, 8, 4, MSG>(n, F, ldu, rows, slot_ptr, slot_cols, ufeat, out, mean, accum,
                                 nt, stream);
}

}  // namespace dglhip

using namespace dglhip;

extern "C" int dglhip_gspmm_short_rows_device(int msg_op, int reduce_op, int64_t num_items,
                                              int64_t feat_len, int64_t max_deg,
                                              int64_t total_rows, const int32_t* rows,
                                              const int64_t* slot_ptr,
                                              const int32_t* slot_cols, const float* ufeat,
                                              float* out, int64_t ufeat_ld, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(copies_u(msg_op), "short-row g-SpMM: copy_u messages only, got " << msg_op);
  DGLHIP_CHECK(reduce_op == DGLHIP_REDUCE_SUM || reduce_op == DGLHIP_REDUCE_MEAN ||
                   reduce_op == DGLHIP_REDUCE_SUM_ACCUM || reduce_op == DGLHIP_REDUCE_MEAN_ACCUM,
               "short-row g-SpMM: sum / mean / sum_accum / mean_accum only");
  DGLHIP_CHECK(num_items >= 0 && feat_len >= 0 && max_deg >= 0, "negative size");
  if (num_items == 0 || feat_len == 0) return 0;
  DGLHIP_CHECK(out && rows && (max_deg == 0 || (slot_ptr && slot_cols && ufeat)),
               "null pointer argument");
  DGLHIP_CHECK(ufeat_ld == 0 || ufeat_ld == feat_len || (ufeat_ld > feat_len && ufeat_ld % 2 == 0),
               "ufeat_ld " << ufeat_ld << ": 0, feat_len, or an even width > feat_len");
  const int64_t ldu = ufeat_ld ? ufeat_ld : feat_len;
  const bool mean = reduce_op == DGLHIP_REDUCE_MEAN || reduce_op == DGLHIP_REDUCE_MEAN_ACCUM;
  const bool accum = reduce_op == DGLHIP_REDUCE_SUM_ACCUM || reduce_op == DGLHIP_REDUCE_MEAN_ACCUM;
  // non-temporal output once the whole launch's output is past twice the
  // Infinity Cache (the main kernel's rule, decided on the full row count)
  const bool nt = stream_output(std::max(total_rows, num_items), feat_len);
  const bool v2 = feat_len % 2 == 0 && feat_len >= 4 &&
                  reinterpret_cast<uintptr_t>(out) % 8 == 0 &&
                  (max_deg == 0 || reinterpret_cast<uintptr_t>(ufeat) % 8 == 0);
#define DGLHIP_SHORT(V, M)                                                                  \
  dispatch_short<V, M>(max_deg, num_items, feat_len, ldu, rows, slot_ptr, slot_cols, ufeat, out, \
                       mean, accum, nt, stream)
  if (msg_op == DGLHIP_MSG_COPY_U_BF16) {
    if (v2) DGLHIP_SHORT(2, DGLHIP_MSG_COPY_U_BF16);
    else DGLHIP_SHORT(1, DGLHIP_MSG_COPY_U_BF16);
  } else {
    if (v2) DGLHIP_SHORT(2, DGLHIP_MSG_COPY_U);
    else DGLHIP_SHORT(1, DGLHIP_MSG_COPY_U);
  }
#undef DGLHIP_SHORT
  API_END();
}
