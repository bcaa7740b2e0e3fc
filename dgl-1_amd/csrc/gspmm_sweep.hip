// Source-swept g-SpMM (copy_u over fp32 or bf16 rows; sum, sum_accum, mean,
// mean_accum): one launch that walks the source columns in slices.
//
// The source-blocked schedule (kernel._block_plan) makes the
// eight XCDs gather from one L2-sized slice of H at a time by running one
// launch per slice; every launch then reads and rewrites the partial rows of
// every row with slots in the slice. That output pass is what limits it: per
// call 19 x (read + write) of most of the 119 MB output on the Reddit-shaped
// graph, and with the N-fold larger source tables of a weak-scaled partition
// (N x 119 MB) the slices hold ~3 slots per row, so the pass costs more than
// the gathers it localises.
//
// Here a wave owns R output rows for the whole launch and keeps their partial
// sums in registers. It sweeps the column slices in order; in slice s each
// row consumes its next slots while their column is below the slice's end
// (up to U per row per step, the gathers of all R rows in flight before any
// add), so every resident wave gathers from about the same slice at the same
// time and the partial rows never leave the CU. A row's slots are consumed
// strictly in slot order — a slot is taken only after every earlier one — so
// each output element is the one sequential chain of the one-launch kernel
// (0 + x_0 + x_1 + ...; continued from out for sum_accum), bit for bit, for
// ANY slot order: a row whose columns are not ascending merely waits for the
// slice of its next slot (the last slice takes everything left).
//
// Rows come dealt in a snake over the degree-descending order (kernel
// _sweep_plan), so the waves carry similar slot totals and move through the
// slices at similar speed. Rows of at least `heavy` slots get a wave each with
// a deeper batch (RH = 1, UH = 32), launched first.
#include "gspmm_impl.h"

namespace dglhip {

enum { SW_SUM = 0, SW_SUM_ACCUM = 1, SW_MEAN = 2, SW_MEAN_ACCUM = 3 };

template <int MSG>
__device__ __forceinline__ f32x2 sweep_gather(const float* __restrict__ ufeat, int32_t col,
                                              int64_t ldu, int64_t f0) {
  if (MSG == DGLHIP_MSG_COPY_U_BF16) return gather_bf16<2>(ufeat, col, ldu, f0);
  return ldv<2>(ufeat + int64_t(col) * ldu + f0);
}

// The wave's R rows (wr[0..R), -1 = none) over every slice; lanes hold two
// consecutive features each (VEC 2), 128 features per pass.
template <int R, int U, int MODE, int MSG>
__device__ __forceinline__ void sweep_rows(const int32_t* __restrict__ wr, int64_t F,
                                           int64_t ldu, const int64_t* __restrict__ indptr,
                                           const int32_t* __restrict__ indices,
                                           const float* __restrict__ ufeat,
                                           float* __restrict__ out, int64_t col_lo,
                                           int64_t slice_cols, int64_t num_slices, int lane) {
  typedef f32x2 V;
  int32_t row[R];
  int64_t beg[R], end[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    row[r] = __builtin_amdgcn_readfirstlane(wr[r]);
    beg[r] = row[r] >= 0 ? indptr[row[r]] : 0;
    end[r] = row[r] >= 0 ? indptr[row[r] + 1] : 0;
  }
  const int64_t passes = (F + 127) / 128;
  for (int64_t pass = 0; pass < passes; ++pass) {
    const int64_t f0 = pass * 128 + int64_t(lane) * 2;
    const bool act = f0 < F;
    int64_t k[R];
    V acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      k[r] = beg[r];
      acc[r] = (MODE == SW_SUM_ACCUM && act && row[r] >= 0)
                   ? ldv<2>(out + int64_t(row[r]) * F + f0)
                   : Vec<2>::zero();
    }
    for (int64_t s = 0; s < num_slices; ++s) {
      const int64_t hi = s + 1 == num_slices ? INT64_MAX : col_lo + (s + 1) * slice_cols;
      bool live[R];  // rows that may still have slots in this slice
#pragma unroll
      for (int r = 0; r < R; ++r) live[r] = k[r] < end[r];
      for (;;) {
        int n[R];
        int32_t c[R][U];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          n[r] = 0;
          if (live[r]) {
            // U independent loads (clamped to the row's last slot), then the
            // run of leading slots below the slice's end
#pragma unroll
            for (int j = 0; j < U; ++j)
              c[r][j] = indices[k[r] + j < end[r] ? k[r] + j : end[r] - 1];
#pragma unroll
            for (int j = 0; j < U; ++j)
              if (n[r] == j && k[r] + j < end[r] && int64_t(c[r][j]) < hi) n[r] = j + 1;
          }
        }
        V v[R][U];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
          for (int j = 0; j < U; ++j)
            if (j < n[r] && act) v[r][j] = sweep_gather<MSG>(ufeat, c[r][j], ldu, f0);
        bool more = false;
#pragma unroll
        for (int r = 0; r < R; ++r) {
#pragma unroll
          for (int j = 0; j < U; ++j)
            if (j < n[r]) acc[r] += v[r][j];
          k[r] += n[r];
          live[r] = n[r] == U && k[r] < end[r];
          more |= live[r];
        }
        if (!more) break;
      }
    }
    if (act) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (row[r] < 0) continue;
        V a = acc[r];
        const int64_t deg = end[r] - beg[r];
        if ((MODE == SW_MEAN || MODE == SW_MEAN_ACCUM) && deg > 1)
          a = a / Vec<2>::splat(static_cast<float>(deg));
        float* o = out + int64_t(row[r]) * F + f0;
        if (MODE == SW_MEAN_ACCUM) a = ldv<2>(o) + a;
        stv<2>(o, a);
      }
    }
  }
}

template <int R, int U, int MODE, int MSG>
__global__ __launch_bounds__(256) void gspmm_sweep_kernel(
    int64_t num_heavy, int64_t num_waves, const int32_t* __restrict__ heavy_rows,
    const int32_t* __restrict__ wave_rows, int64_t F, int64_t ldu,
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const float* __restrict__ ufeat, float* __restrict__ out, int64_t col_lo,
    int64_t slice_cols, int64_t num_slices) {
  const int64_t wave = block_linear() * (blockDim.x >> 6) +
                       __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  if (wave < num_heavy)
    sweep_rows<1, 32, MODE, MSG>(heavy_rows + wave, F, ldu, indptr, indices, ufeat, out, col_lo,
                                 slice_cols, num_slices, lane);
  else if (wave < num_heavy + num_waves)
    sweep_rows<R, U, MODE, MSG>(wave_rows + (wave - num_heavy) * R, F, ldu, indptr, indices,
                                ufeat, out, col_lo, slice_cols, num_slices, lane);
}

template <int R, int U, int MSG>
static void launch_sweep(int mode, int64_t num_heavy, int64_t num_waves,
                         const int32_t* heavy_rows, const int32_t* wave_rows, int64_t F,
                         int64_t ldu, const int64_t* indptr, const int32_t* indices,
                         const float* ufeat, float* out, int64_t col_lo, int64_t slice_cols,
                         int64_t num_slices, hipStream_t stream) {
  const int64_t blocks = (num_heavy + num_waves + 3) / 4;
#define DGLHIP_SWEEP_LAUNCH(M)                                                               \
  hipLaunchKernelGGL((gspmm_sweep_kernel<R, U, M, MSG>), grid_1d(blocks), dim3(256), 0,       \
                     stream, num_heavy, num_waves, heavy_rows, wave_rows, F, ldu, indptr,     \
                     indices, ufeat, out, col_lo, slice_cols, num_slices)
  timed_launch(stream, [&] {
    switch (mode) {
      case SW_SUM: DGLHIP_SWEEP_LAUNCH(SW_SUM); break;
      case SW_SUM_ACCUM: DGLHIP_SWEEP_LAUNCH(SW_SUM_ACCUM); break;
      case SW_MEAN: DGLHIP_SWEEP_LAUNCH(SW_MEAN); break;
      default: DGLHIP_SWEEP_LAUNCH(SW_MEAN_ACCUM); break;
    }
  });
#undef DGLHIP_SWEEP_LAUNCH
}

}  // namespace dglhip

using namespace dglhip;

extern "C" {

int dglhip_gspmm_sweep_device(int msg_op, int reduce_op, int64_t feat_len, int64_t num_heavy,
                              const int32_t* heavy_rows, int64_t num_waves,
                              const int32_t* wave_rows, int rows_per_wave,
                              const int64_t* indptr, const int32_t* indices, const float* ufeat,
                              int64_t ufeat_ld, float* out, int64_t col_lo, int64_t slice_cols,
                              int64_t num_slices, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(msg_op == DGLHIP_MSG_COPY_U || msg_op == DGLHIP_MSG_COPY_U_BF16,
               "the swept schedule covers copy_u (fp32 or bf16 rows), got msg op " << msg_op);
  int mode;
  switch (reduce_op) {
    case DGLHIP_REDUCE_SUM: mode = SW_SUM; break;
    case DGLHIP_REDUCE_SUM_ACCUM: mode = SW_SUM_ACCUM; break;
    case DGLHIP_REDUCE_MEAN: mode = SW_MEAN; break;
    case DGLHIP_REDUCE_MEAN_ACCUM: mode = SW_MEAN_ACCUM; break;
    default: DGLHIP_CHECK(false, "the swept schedule covers sum / mean, got reduce op " << reduce_op);
  }
  DGLHIP_CHECK(feat_len >= 0 && num_heavy >= 0 && num_waves >= 0, "negative size");
  if (feat_len == 0 || num_heavy + num_waves == 0) return 0;
  DGLHIP_CHECK(feat_len % 2 == 0, "the swept schedule needs an even feat_len, got " << feat_len);
  const int64_t ldu = ufeat_ld ? ufeat_ld : feat_len;
  DGLHIP_CHECK(ldu >= feat_len && ldu % 2 == 0, "ufeat_ld " << ufeat_ld << ": 0 or an even width >= feat_len");
  DGLHIP_CHECK(indptr && indices && ufeat && out, "null indptr/indices/ufeat/out");
  DGLHIP_CHECK(num_heavy == 0 || heavy_rows, "null heavy_rows");
  DGLHIP_CHECK(num_waves == 0 || wave_rows, "null wave_rows");
  DGLHIP_CHECK(num_slices >= 1 && slice_cols >= 1, "num_slices and slice_cols must be >= 1");
  DGLHIP_CHECK(reinterpret_cast<uintptr_t>(ufeat) % (msg_op == DGLHIP_MSG_COPY_U ? 8 : 4) == 0 &&
                   reinterpret_cast<uintptr_t>(out) % 8 == 0,
               "ufeat / out not aligned for two-feature lanes");
  const bool bf16 = msg_op == DGLHIP_MSG_COPY_U_BF16;
  if (bf16) {
    DGLHIP_CHECK(rows_per_wave == 8, "bf16 rows: rows_per_wave 8, got " << rows_per_wave);
    launch_sweep<8, 4, DGLHIP_MSG_COPY_U_BF16>(mode, num_heavy, num_waves, heavy_rows, wave_rows,
                                               feat_len, ldu, indptr, indices, ufeat, out, col_lo,
                                               slice_cols, num_slices, stream);
    return 0;
  }
  switch (rows_per_wave) {
    case 4:
      launch_sweep<4, 8, DGLHIP_MSG_COPY_U>(mode, num_heavy, num_waves, heavy_rows, wave_rows,
                                            feat_len, ldu, indptr, indices, ufeat, out, col_lo,
                                            slice_cols, num_slices, stream);
      break;
    case 8:
      launch_sweep<8, 4, DGLHIP_MSG_COPY_U>(mode, num_heavy, num_waves, heavy_rows, wave_rows,
                                            feat_len, ldu, indptr, indices, ufeat, out, col_lo,
                                            slice_cols, num_slices, stream);
      break;
    case 16:
      launch_sweep<16, 2, DGLHIP_MSG_COPY_U>(mode, num_heavy, num_waves, heavy_rows, wave_rows,
                                             feat_len, ldu, indptr, indices, ufeat, out, col_lo,
                                             slice_cols, num_slices, stream);
      break;
    default:
      DGLHIP_CHECK(false, "rows_per_wave must be 4, 8 or 16, got " << rows_per_wave);
  }
  API_END();
}

}  // extern "C"
