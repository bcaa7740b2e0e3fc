// Row-wise element passes of the g-SpMM's autograd, written where the next
// kernel reads them.
//
// dglhip_div_rows_device: out[r, :F] = x[r, :F] / d[r] (packed input and
// aligned padded output rows: their pad columns are written with zeros). The backward of the
// mean reducer divides the output gradient by the in-degree before the
// transposed product (dH = Aᵀ (dC / deg)); the quotient is stored straight
// into the row-padded buffer that product gathers (F = 41 at a 48-float
// stride), one pass instead of a division and a padding copy, and one pass at
// the byte rate where PyTorch's strided-output division ran at 3.5 TB/s
// (RMAT-26: 6.8 ms). IEEE division, correctly rounded: the same bits as
// torch.div.
#include "common.h"
#include "launch.h"

#include <hip/hip_runtime.h>

namespace dglhip {

namespace {

constexpr int kThreads = 256;
constexpr int kTileRows = 256;  // rows per workgroup iteration
constexpr int kBatch = 8;

// tiles of kTileRows rows; element i of a tile is row i / F, column i % F
// (exact with the 32-bit reciprocal M = ceil(2^32 / F) for i < 2^32 / F)
__global__ __launch_bounds__(kThreads) void div_rows_kernel(int64_t n, int F, uint32_t M,
                                                            const float* __restrict__ x,
                                                            int64_t ldx,
                                                            const float* __restrict__ d,
                                                            float* __restrict__ out,
                                                            int64_t ldo) {
  const int64_t ntiles = (n + kTileRows - 1) / kTileRows;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t r0 = t * kTileRows;
    const int rows = static_cast<int>(n - r0 < kTileRows ? n - r0 : kTileRows);
    const int total = rows * F;
    // kBatch elements per lane in flight at once (the loads of a batch are
    // all issued before its first division)
    for (int i0 = threadIdx.x; i0 < total; i0 += kBatch * kThreads) {
      float xv[kBatch], dv[kBatch];
      int64_t o[kBatch];
#pragma unroll
      for (int b = 0; b < kBatch; ++b) {
        const int i = i0 + b * kThreads;
        o[b] = -1;
        if (i < total) {
          const int r = static_cast<int>(__umulhi(static_cast<uint32_t>(i), M));
          const int c = i - r * F;
          const int64_t row = r0 + r;
          xv[b] = x[row * ldx + c];
          dv[b] = d[row];
          o[b] = row * ldo + c;
        }
      }
#pragma unroll
      for (int b = 0; b < kBatch; ++b)
        if (o[b] >= 0) out[o[b]] = xv[b] / dv[b];
    }
  }
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Packed input (ldx == F), 16-byte aligned output rows (ldo % 4 == 0): a tile
// of kTileRows rows comes in as one float4 run into LDS and leaves as one
// float4 run of whole padded rows (the pad columns get zeros), so both sides
// are plain 16-B streams. F <= kMaxTiledF; the tile's first input float
// (r0 * F, r0 a multiple of kTiledRows) keeps the runs 16-byte aligned.
constexpr int kMaxTiledF = 64;
constexpr int kTiledRows = 128;  // 32 KB of LDS per workgroup

__global__ __launch_bounds__(kThreads) void div_rows_tiled_kernel(
    int64_t n, int F, int ldo, uint32_t Mo, const float* __restrict__ x,
    const float* __restrict__ d, float* __restrict__ out) {
  __shared__ float tile[kTiledRows * kMaxTiledF];
  __shared__ float dv[kTiledRows];
  const int64_t ntiles = (n + kTiledRows - 1) / kTiledRows;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t r0 = t * kTiledRows;
    const int rows = static_cast<int>(n - r0 < kTiledRows ? n - r0 : kTiledRows);
    const int total = rows * F;
    const f32x4* in4 = reinterpret_cast<const f32x4*>(x + r0 * F);
    __syncthreads();  // the previous tile has left LDS
    const int n4 = total >> 2;
    for (int i = threadIdx.x; i < n4; i += kThreads) reinterpret_cast<f32x4*>(tile)[i] = in4[i];
    for (int i = (n4 << 2) + threadIdx.x; i < total; i += kThreads) tile[i] = x[r0 * F + i];
    if (threadIdx.x < rows) dv[threadIdx.x] = d[r0 + threadIdx.x];
    __syncthreads();
    f32x4* o4 = reinterpret_cast<f32x4*>(out + r0 * ldo);
    const int m4 = rows * ldo / 4;
    for (int j = threadIdx.x; j < m4; j += kThreads) {
      const int e = 4 * j;
      const int r = static_cast<int>(__umulhi(static_cast<uint32_t>(e), Mo));
      const int c = e - r * ldo;  // 4 consecutive columns of row r (ldo % 4 == 0)
      const float q = dv[r];
      f32x4 v;
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = c + k < F ? tile[r * F + c + k] / q : 0.0f;
      o4[j] = v;
    }
  }
}

// The node-row epilogue of a GCN layer after its aggregation (r06):
//   out = act(x * row_scale[r] + bias), act = ReLU or none,
// the value of torch's `x * norm`, `+ bias`, `relu` (each rounding once, in
// that order; ReLU as torch's clamp_min: NaN kept, max(v, 0) otherwise), in
// one pass instead of three. Its backward, one pass: d_pre = out <= 0 ? 0 :
// dout (torch's threshold_backward on the ReLU's result) or dout, dx = d_pre *
// row_scale[r], and each workgroup's column sums of d_pre over its rows (in
// row order) for the bias gradient.
__global__ __launch_bounds__(kThreads) void node_epilogue_fwd_kernel(
    int64_t total, int64_t F, const float* __restrict__ x, const float* __restrict__ row_scale,
    const float* __restrict__ bias, int relu, float* __restrict__ out) {
#pragma clang fp contract(off)
  for (int64_t i = block_linear() * kThreads + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * gridDim.y * kThreads) {
    const int64_t r = i / F, f = i - r * F;
    float v = x[i];
    if (row_scale) v = v * row_scale[r];
    if (bias) v = v + bias[f];
    if (relu) v = __builtin_isnan(v) ? v : fmaxf(v, 0.0f);
    out[i] = v;
  }
}

constexpr int kEpiRows = 128;  // rows per workgroup of the backward (one column sum each)

template <int CPT>
__global__ __launch_bounds__(kThreads) void node_epilogue_bwd_kernel(
    int64_t n, int64_t F, const float* __restrict__ dout, const float* __restrict__ out,
    const float* __restrict__ row_scale, int relu, float* __restrict__ dx,
    float* __restrict__ col_partial) {
#pragma clang fp contract(off)
  const int64_t part = block_linear();
  const int64_t r0 = part * kEpiRows;
  if (r0 >= n) return;
  const int64_t r1 = r0 + kEpiRows < n ? r0 + kEpiRows : n;
  float acc[CPT];
  int64_t col[CPT];
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    acc[c] = 0.0f;
    col[c] = threadIdx.x + int64_t(c) * blockDim.x;
  }
#pragma unroll 8
  for (int64_t r = r0; r < r1; ++r) {
    const float sc = row_scale ? row_scale[r] : 1.0f;
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      if (col[c] < F) {
        const int64_t i = r * F + col[c];
        float d = dout[i];
        if (relu) d = out[i] <= 0.0f ? 0.0f : d;
        acc[c] = acc[c] + d;
        dx[i] = row_scale ? d * sc : d;
      }
    }
  }
  if (col_partial) {
#pragma unroll
    for (int c = 0; c < CPT; ++c)
      if (col[c] < F) col_partial[part * F + col[c]] = acc[c];
  }
}

}  // namespace

}  // namespace dglhip

using namespace dglhip;

extern "C" {

int dglhip_div_rows_device(int64_t num_rows, int64_t feat_len, const float* x, int64_t ldx,
                           const float* divisor, float* out, int64_t ldo, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows >= 0 && feat_len >= 1 && feat_len <= 4096,
               "rows >= 0 and 1..4096 columns, got " << num_rows << " x " << feat_len);
  if (num_rows == 0) return 0;
  DGLHIP_CHECK(ldx >= feat_len && ldo >= feat_len, "row stride below the row width");
  DGLHIP_CHECK(x && divisor && out, "null pointer argument");
  const int F = static_cast<int>(feat_len);
  // M = ceil(2^32 / F): floor(i * M / 2^32) = i / F for i < 2^32 / F >= kTileRows * F
  const uint32_t M = static_cast<uint32_t>(((uint64_t(1) << 32) + F - 1) / F);
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  const int64_t tiles = (num_rows + kTileRows - 1) / kTileRows;
  const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(tiles, int64_t(cus) * 8));
  if (ldx == feat_len && feat_len <= kMaxTiledF && ldo % 4 == 0 && ldo <= 4 * kMaxTiledF &&
      (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
    const uint32_t Mo = static_cast<uint32_t>(((uint64_t(1) << 32) + ldo - 1) / ldo);
    const int64_t ttiles = (num_rows + kTiledRows - 1) / kTiledRows;
    hipLaunchKernelGGL(div_rows_tiled_kernel, dim3(std::min<int64_t>(ttiles, int64_t(cus) * 4)),
                       dim3(kThreads), 0, stream, num_rows, F, static_cast<int>(ldo), Mo, x,
                       divisor, out);
  } else {
    hipLaunchKernelGGL(div_rows_kernel, dim3(grid), dim3(kThreads), 0, stream, num_rows, F, M, x,
                       ldx, divisor, out, ldo);
  }
  DGLHIP_CHECK(hipGetLastError() == hipSuccess, "row division launch failed");
  API_END();
}

int64_t dglhip_node_epilogue_parts(int64_t num_rows) {
  return num_rows > 0 ? (num_rows + kEpiRows - 1) / kEpiRows : 0;
}

int dglhip_node_epilogue_fwd_device(int64_t num_rows, int64_t feat_len, const float* x,
                                    const float* row_scale, const float* bias, int relu,
                                    float* out, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows >= 0 && feat_len >= 1, "bad sizes");
  if (num_rows == 0) return 0;
  DGLHIP_CHECK(x && out, "null pointer argument");
  const int64_t total = num_rows * feat_len;
  const int64_t blocks = std::min<int64_t>((total + kThreads - 1) / kThreads, int64_t(1) << 20);
  hipLaunchKernelGGL(node_epilogue_fwd_kernel, grid_1d(blocks), dim3(kThreads), 0, stream,
                     total, feat_len, x, row_scale, bias, relu, out);
  DGLHIP_CHECK(hipGetLastError() == hipSuccess, "node epilogue launch failed");
  API_END();
}

int dglhip_node_epilogue_bwd_device(int64_t num_rows, int64_t feat_len, const float* dout,
                                    const float* out, const float* row_scale, int relu,
                                    float* dx, float* col_partial, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows >= 0 && feat_len >= 1 && feat_len <= 4 * kThreads,
               "1.." << 4 * kThreads << " columns, got " << feat_len);
  if (num_rows == 0) return 0;
  DGLHIP_CHECK(dout && dx && (!relu || out), "null pointer argument");
  const int64_t parts = dglhip_node_epilogue_parts(num_rows);
  const int cpt = feat_len <= kThreads ? 1 : (feat_len <= 2 * kThreads ? 2 : 4);
#define DGLHIP_EPI(C)                                                                        \
  hipLaunchKernelGGL(node_epilogue_bwd_kernel<C>, grid_1d(parts), dim3(kThreads), 0, stream, \
                     num_rows, feat_len, dout, out, row_scale, relu, dx, col_partial)
  if (cpt == 1) DGLHIP_EPI(1);
  else if (cpt == 2) DGLHIP_EPI(2);
  else DGLHIP_EPI(4);
#undef DGLHIP_EPI
  DGLHIP_CHECK(hipGetLastError() == hipSuccess, "node epilogue backward launch failed");
  API_END();
}

}  // extern "C"
