// Weighted softmax cross-entropy over node rows: the loss of a full-graph node
// classifier (GraphSAGE / GCN output layer, BASELINE configs[1], configs[3]),
//   loss = sum_i w_i (logsumexp(z_i) - z_i[y_i]),
// and its gradient dz_ij = g w_i (softmax(z_i)_j - [j == y_i]) for the
// upstream scalar g. The same value as PyTorch's
// (F.cross_entropy(z, y, reduction="none") * w).sum(), which at 10^7-10^8 rows
// of a few dozen classes runs as five passes over the logits forward and
// backward (log-softmax, the nll gather, a zero fill, the nll scatter, the
// log-softmax backward: 28 ms per RMAT-26 epoch); here one read forward and one
// read + one write backward.
//
// Layout: a workgroup stages a tile of kRows rows into LDS with coalesced
// 16-B loads (rows at an odd LDS stride SC, so the one-row-per-lane pass that
// follows is free of bank conflicts), each lane reduces its row (max, sum of
// exponentials, log) and the backward writes its gradient row back into the
// tile, which then leaves with coalesced stores. The loss sum is per-lane,
// then per workgroup in a fixed tree, then over the workgroups in index order
// (deterministic). Rows labelled -100 (PyTorch's ignore_index) contribute
// nothing; any other label outside [0, C) is an error in PyTorch (an
// exception, a device-side assert on the GPU): here it makes the loss NaN and
// that row's gradient NaN, so a bad label set can never train silently.
#include "../../include/dgl_hip.h"
#include "common.h"
#include "launch.h"

#include <hip/hip_runtime.h>

namespace dglhip {

namespace {

constexpr int kRows = 256;         // rows per tile = lanes per workgroup
constexpr int64_t kIgnore = -100;  // PyTorch's default ignore_index
constexpr int kMaxClasses = 64;
constexpr int kMaxBlocks = 1024;   // workspace floats of the forward

// Staging of one tile's rows, tile[r * SC + c] = z[(r0 + r) * ld + c].
//
// NS > 0 (rows packed back to back at an odd width C = SC from a 16-byte
// aligned start, so a tile is one float4 run of nrows * C floats, at most NS
// float4 per lane): the run is loaded into registers one tile AHEAD and copied
// into LDS when its turn comes, so the next tile's loads are in flight while
// this tile's rows are reduced. NS = 0: loaded element by element straight
// into LDS (padded strides, even widths).
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NS>
struct Ahead {
  f32x4 v[NS > 0 ? NS : 1];
  float tail;
};

// e0: the tile's first element (a multiple of 4: kRows * C floats per tile)
template <int NS>
__device__ inline void fetch_ahead(Ahead<NS>& a, const float* __restrict__ z, int64_t e0,
                                   int total) {
  const int n4 = total >> 2;
  const f32x4* b4 = reinterpret_cast<const f32x4*>(z) + (e0 >> 2);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int i = threadIdx.x + s * kRows;
    if (i < n4) a.v[s] = b4[i];
  }
  const int t = (n4 << 2) + threadIdx.x;
  if (t < total) a.tail = z[e0 + t];
}

template <int NS>
__device__ inline void commit_ahead(const Ahead<NS>& a, int total, float* tile) {
  const int n4 = total >> 2;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int i = threadIdx.x + s * kRows;
    if (i < n4) reinterpret_cast<f32x4*>(tile)[i] = a.v[s];
  }
  const int t = (n4 << 2) + threadIdx.x;
  if (t < total) tile[t] = a.tail;
}

__device__ inline void load_tile(const float* __restrict__ z, int64_t ld, int64_t r0, int nrows,
                                 int C, int SC, float* tile) {
  const int total = nrows * C;
  for (int i = threadIdx.x; i < total; i += blockDim.x) {
    const int r = i / C, c = i - r * C;
    tile[r * SC + c] = z[(r0 + r) * ld + c];
  }
}

__device__ inline void store_tile(float* __restrict__ out, int64_t ld, int64_t r0, int nrows,
                                  int C, int SC, const float* tile) {
  const int total = nrows * C;
  if (ld == C && SC == C && (reinterpret_cast<uintptr_t>(out + r0 * C) & 15) == 0) {
    float* base = out + r0 * C;
    const int n4 = total >> 2;
    for (int i = threadIdx.x; i < n4; i += blockDim.x)
      reinterpret_cast<float4*>(base)[i] = reinterpret_cast<const float4*>(tile)[i];
    for (int i = (n4 << 2) + threadIdx.x; i < total; i += blockDim.x) base[i] = tile[i];
    return;
  }
  for (int i = threadIdx.x; i < total; i += blockDim.x) {
    const int r = i / C, c = i - r * C;
    out[(r0 + r) * ld + c] = tile[r * SC + c];
  }
}

// max and log(sum exp(z - max)) of one staged row
__device__ inline void row_lse(const float* row, int C, float& m, float& lse) {
  m = row[0];
  for (int c = 1; c < C; ++c) m = fmaxf(m, row[c]);
  float s = 0.0f;
  for (int c = 0; c < C; ++c) s += expf(row[c] - m);
  lse = logf(s);
}

__device__ inline int tile_rows(int64_t n, int64_t r0) {
  return static_cast<int>(n - r0 < kRows ? n - r0 : kRows);
}

template <int NS>
__global__ __launch_bounds__(kRows) void xent_fwd_kernel(int64_t n, int C, int SC,
                                                         const float* __restrict__ z, int64_t ld,
                                                         const int64_t* __restrict__ labels,
                                                         const float* __restrict__ w,
                                                         float* __restrict__ partial) {
  extern __shared__ float tile[];
  float acc = 0.0f;
  const int64_t ntiles = (n + kRows - 1) / kRows;
  Ahead<NS> ahead;
  int64_t t = blockIdx.x;
  if (NS > 0 && t < ntiles) fetch_ahead(ahead, z, t * kRows * C, tile_rows(n, t * kRows) * C);
  for (; t < ntiles; t += gridDim.x) {
    const int64_t r0 = t * kRows;
    const int nrows = tile_rows(n, r0);
    const int r = threadIdx.x;
    const int64_t y = r < nrows ? labels[r0 + r] : -1;
    const float wr = (r < nrows && w != nullptr) ? w[r0 + r] : 1.0f;
    __syncthreads();  // the previous tile's rows are consumed
    if (NS > 0) commit_ahead(ahead, nrows * C, tile);
    else load_tile(z, ld, r0, nrows, C, SC, tile);
    __syncthreads();
    const int64_t tn = t + gridDim.x;  // the next tile's loads overlap this one's rows
    if (NS > 0 && tn < ntiles) fetch_ahead(ahead, z, tn * kRows * C, tile_rows(n, tn * kRows) * C);
    if (r < nrows && y >= 0 && y < C) {
      const float* row = tile + r * SC;
      float m, lse;
      row_lse(row, C, m, lse);
      const float nll = -((row[y] - m) - lse);
      acc += w != nullptr ? nll * wr : nll;
    } else if (r < nrows && y != kIgnore) {
      acc = __builtin_nanf("");  // out-of-range label: poison the loss
    }
  }
  // workgroup sum in a fixed tree
  __syncthreads();
  tile[threadIdx.x] = acc;
  __syncthreads();
  for (int s = kRows / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) tile[threadIdx.x] += tile[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = tile[0];
}

// loss = the workgroups' partial sums, in index order
__global__ void xent_sum_kernel(int nparts, const float* __restrict__ partial,
                                float* __restrict__ loss) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    float s = 0.0f;
    for (int i = 0; i < nparts; ++i) s += partial[i];
    loss[0] = s;
  }
}

template <int NS>
__global__ __launch_bounds__(kRows) void xent_bwd_kernel(int64_t n, int C, int SC,
                                                         const float* __restrict__ z, int64_t ld,
                                                         const int64_t* __restrict__ labels,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ grad_loss,
                                                         float* __restrict__ dz, int64_t ldd,
                                                         float* __restrict__ colpart,
                                                         const float* __restrict__ divisor,
                                                         float* __restrict__ dzs, int64_t ldds) {
  extern __shared__ float tile[];
  const float g = grad_loss[0];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float col = 0.0f;  // colpart: this wave's running sum of column `lane`
  const int64_t ntiles = (n + kRows - 1) / kRows;
  Ahead<NS> ahead;
  int64_t t = blockIdx.x;
  if (NS > 0 && t < ntiles) fetch_ahead(ahead, z, t * kRows * C, tile_rows(n, t * kRows) * C);
  for (; t < ntiles; t += gridDim.x) {
    const int64_t r0 = t * kRows;
    const int nrows = tile_rows(n, r0);
    const int r = threadIdx.x;
    const int64_t y = r < nrows ? labels[r0 + r] : -1;
    const float wr = (r < nrows && w != nullptr) ? w[r0 + r] : 1.0f;
    __syncthreads();  // the previous tile has left LDS
    if (NS > 0) commit_ahead(ahead, nrows * C, tile);
    else load_tile(z, ld, r0, nrows, C, SC, tile);
    __syncthreads();
    const int64_t tn = t + gridDim.x;
    if (NS > 0 && tn < ntiles) fetch_ahead(ahead, z, tn * kRows * C, tile_rows(n, tn * kRows) * C);
    if (r < nrows) {
      float* row = tile + r * SC;
      if (y >= 0 && y < C) {
        // one exp per element: e_c = exp(z_c - max) kept in the row, then
        // gw * softmax = e_c * (gw / sum e)
        float m = row[0];
        for (int c = 1; c < C; ++c) m = fmaxf(m, row[c]);
        float s = 0.0f;
        for (int c = 0; c < C; ++c) {
          const float e = expf(row[c] - m);
          row[c] = e;
          s += e;
        }
        const float gw = w != nullptr ? g * wr : g;
        const float k = gw / s;
        for (int c = 0; c < C; ++c) {
          const float gp = row[c] * k;
          row[c] = c == y ? gp - gw : gp;
        }
      } else {
        const float v = y == kIgnore ? 0.0f : __builtin_nanf("");
        for (int c = 0; c < C; ++c) row[c] = v;
      }
    }
    __syncthreads();
    store_tile(dz, ldd, r0, nrows, C, SC, tile);
    if (dzs != nullptr) {
      // dz / divisor[row] at row stride ldds (a multiple of 4, pad columns
      // zeroed): the mean aggregation's backward operand, written from the
      // same tile as whole 16-byte groups (IEEE division: torch.div's bits)
      float* base = dzs + r0 * ldds;
      const int m = nrows * static_cast<int>(ldds);
      // e / ldds as a multiply-high (exact for e < 2^16 <= 2^32 / ldds)
      const uint32_t mo = static_cast<uint32_t>(((uint64_t(1) << 32) + ldds - 1) / ldds);
      for (int e = 4 * threadIdx.x; e < m; e += 4 * kRows) {
        const int rr = static_cast<int>(__umulhi(static_cast<uint32_t>(e), mo));
        const int c = e - rr * static_cast<int>(ldds);
        const float q = divisor[r0 + rr];
        f32x4 v;
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = c + k < C ? tile[rr * SC + c + k] / q : 0.0f;
        *reinterpret_cast<f32x4*>(base + e) = v;
      }
    }
    if (colpart != nullptr && lane < C) {
      // the gradient rows' column sums, read back from the tile: wave w sums
      // rows [64 w, 64 w + 64) of column `lane` in row order (lanes read
      // consecutive LDS words: no bank conflict); the next tile waits on the
      // __syncthreads at the loop's head
      const int rb = wv * 64, re = nrows < rb + 64 ? nrows : rb + 64;
      const float* tc = tile + lane;
      float s = 0.0f;
      if (re - rb == 64) {  // full tiles: the reads issue ahead of the adds
#pragma unroll 16
        for (int rr = rb; rr < rb + 64; ++rr) s += tc[rr * SC];
      } else {
        for (int rr = rb; rr < re; ++rr) s += tc[rr * SC];
      }
      col += s;
    }
  }
  if (colpart != nullptr) {
    // the workgroup's partial: its four waves in order
    __syncthreads();
    if (lane < C) tile[wv * C + lane] = col;
    __syncthreads();
    if (threadIdx.x < C) {
      float s = tile[threadIdx.x];
      for (int w = 1; w < kRows / 64; ++w) s += tile[w * C + threadIdx.x];
      colpart[int64_t(blockIdx.x) * C + threadIdx.x] = s;
    }
  }
}

// colsum[c] = the workgroups' partial column sums: kSegs contiguous runs of
// partials, each summed in index order by one thread, then the runs in order
// (a fixed association: deterministic; kSegs loads in flight per column)
constexpr int kSegs = 16;
__global__ __launch_bounds__(kSegs * 64) void xent_colsum_kernel(
    int nparts, int C, const float* __restrict__ colpart, float* __restrict__ colsum) {
  __shared__ float seg_sum[kSegs * 64];
  const int c = threadIdx.x & 63, seg = threadIdx.x >> 6;
  const int per = (nparts + kSegs - 1) / kSegs;
  const int i0 = seg * per, i1 = nparts < i0 + per ? nparts : i0 + per;
  float s = 0.0f;
  if (c < C)
    for (int i = i0; i < i1; ++i) s += colpart[int64_t(i) * C + c];
  seg_sum[threadIdx.x] = s;
  __syncthreads();
  if (seg == 0 && c < C) {
    float t = seg_sum[c];
    for (int k = 1; k < kSegs; ++k) t += seg_sum[k * 64 + c];
    colsum[c] = t;
  }
}

inline int xent_grid(int64_t n, int SC) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  const int lds = kRows * SC * 4;
  const int per_cu = std::max(1, std::min(8, (160 * 1024) / lds));
  const int64_t tiles = (n + kRows - 1) / kRows;
  return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>({tiles, int64_t(cus) * per_cu,
                                                                    int64_t(kMaxBlocks)})));
}

inline int lds_stride(int C) { return C | 1; }

// rows packed back to back at an odd width, from a 16-byte aligned start: each
// tile is one float4 run (a tile's offset, kRows * C floats, is a multiple of 4)
inline bool flat(const float* z, int64_t ld, int C, int SC) {
  return ld == C && SC == C && (reinterpret_cast<uintptr_t>(z) & 15) == 0;
}

// float4 registers per lane that hold one tile of C-float rows (C / 4 rounded
// up to a compiled count)
inline int ahead_slots(int C) {
  const int s = (C + 3) / 4;
  return s <= 4 ? 4 : s <= 8 ? 8 : s <= 12 ? 12 : 16;
}

}  // namespace

}  // namespace dglhip

using namespace dglhip;

extern "C" {

int dglhip_xent_workspace_floats() { return kMaxBlocks; }

int dglhip_xent_fwd_device(int64_t num_rows, int64_t num_classes, const float* logits,
                           int64_t ld, const int64_t* labels, const float* weight, float* loss,
                           float* workspace, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows >= 0, "negative row count");
  DGLHIP_CHECK(num_classes >= 1 && num_classes <= kMaxClasses,
               "cross-entropy rows: 1.." << kMaxClasses << " classes, got " << num_classes);
  DGLHIP_CHECK(loss && workspace, "null pointer argument");
  const int C = static_cast<int>(num_classes), SC = lds_stride(C);
  if (num_rows == 0) {
    hipLaunchKernelGGL(xent_sum_kernel, dim3(1), dim3(64), 0, stream, 0, workspace, loss);
  } else {
    DGLHIP_CHECK(ld >= num_classes, "row stride " << ld << " below the class count");
    DGLHIP_CHECK(logits && labels, "null pointer argument");
    const int grid = xent_grid(num_rows, SC);
    const int ns = flat(logits, ld, C, SC) ? ahead_slots(C) : 0;
    auto fwd = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(grid), dim3(kRows), kRows * SC * 4, stream, num_rows, C, SC,
                         logits, ld, labels, weight, workspace);
    };
    switch (ns) {
      case 4: fwd(xent_fwd_kernel<4>); break;
      case 8: fwd(xent_fwd_kernel<8>); break;
      case 12: fwd(xent_fwd_kernel<12>); break;
      case 16: fwd(xent_fwd_kernel<16>); break;
      default: fwd(xent_fwd_kernel<0>); break;
    }
    hipLaunchKernelGGL(xent_sum_kernel, dim3(1), dim3(64), 0, stream, grid, workspace, loss);
  }
  DGLHIP_CHECK(hipGetLastError() == hipSuccess, "cross-entropy launch failed");
  API_END();
}

int dglhip_xent_bwd_device(int64_t num_rows, int64_t num_classes, const float* logits,
                           int64_t ld, const int64_t* labels, const float* weight,
                           const float* grad_loss, float* dlogits, int64_t ldd, void* stream_) {
  return dglhip_xent_bwd_ex_device(num_rows, num_classes, logits, ld, labels, weight, grad_loss,
                                   dlogits, ldd, nullptr, nullptr, nullptr, nullptr, 0, stream_);
}

int dglhip_xent_colsum_workspace_floats(int64_t num_classes) {
  return static_cast<int>(kMaxBlocks * std::max<int64_t>(1, num_classes));
}

int dglhip_xent_bwd_ex_device(int64_t num_rows, int64_t num_classes, const float* logits,
                              int64_t ld, const int64_t* labels, const float* weight,
                              const float* grad_loss, float* dlogits, int64_t ldd, float* colsum,
                              float* workspace, const float* divisor, float* dlogits_scaled,
                              int64_t ld_scaled, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows >= 0, "negative row count");
  DGLHIP_CHECK(num_classes >= 1 && num_classes <= kMaxClasses,
               "cross-entropy rows: 1.." << kMaxClasses << " classes, got " << num_classes);
  DGLHIP_CHECK(colsum == nullptr || workspace != nullptr, "column sums need the workspace");
  DGLHIP_CHECK(dlogits_scaled == nullptr ||
                   (divisor != nullptr && ld_scaled >= num_classes && ld_scaled % 4 == 0 &&
                    ld_scaled <= 4 * kMaxClasses &&
                    (reinterpret_cast<uintptr_t>(dlogits_scaled) & 15) == 0),
               "scaled rows: a divisor, a 16-byte aligned output and a row stride >= the "
               "class count that is a multiple of 4");
  if (num_rows == 0) {
    if (colsum != nullptr)
      DGLHIP_CHECK(hipMemsetAsync(colsum, 0, num_classes * 4, stream) == hipSuccess,
                   "column-sum fill failed");
    return 0;
  }
  DGLHIP_CHECK(ld >= num_classes && ldd >= num_classes, "row stride below the class count");
  DGLHIP_CHECK(logits && labels && grad_loss && dlogits, "null pointer argument");
  const int C = static_cast<int>(num_classes), SC = lds_stride(C);
  const int grid = xent_grid(num_rows, SC);
  const int ns = flat(logits, ld, C, SC) ? ahead_slots(C) : 0;
  float* colpart = colsum != nullptr ? workspace : nullptr;
  auto bwd = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kRows), kRows * SC * 4, stream, num_rows, C, SC,
                       logits, ld, labels, weight, grad_loss, dlogits, ldd, colpart, divisor,
                       dlogits_scaled, ld_scaled);
  };
  switch (ns) {
    case 4: bwd(xent_bwd_kernel<4>); break;
    case 8: bwd(xent_bwd_kernel<8>); break;
    case 12: bwd(xent_bwd_kernel<12>); break;
    case 16: bwd(xent_bwd_kernel<16>); break;
    default: bwd(xent_bwd_kernel<0>); break;
  }
  if (colsum != nullptr)
    hipLaunchKernelGGL(xent_colsum_kernel, dim3(1), dim3(kSegs * 64), 0, stream, grid, C, colpart,
                       colsum);
  DGLHIP_CHECK(hipGetLastError() == hipSuccess, "cross-entropy backward launch failed");
  API_END();
}

}  // extern "C"
