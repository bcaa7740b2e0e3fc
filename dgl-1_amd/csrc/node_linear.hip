// Dense per-node Linear on the f32 MFMA (v_mfma_f32_16x16x4_f32), shaped for
// the narrow layers that follow a g-SpMM over 10^7-10^8 nodes: K <= 256 input
// features, at most 64 outputs per product.
//
// hipBLASLt runs such products (67M x 128 by 128 x 41 in GraphSAGE's output
// layer on RMAT-26) with 16x256 tiles at about 2 TB/s, a third of the rate
// the bytes allow; a workgroup here keeps the (transposed) weights in LDS for
// its lifetime and streams 16-row blocks of the input through registers, so
// the input is read once, straight into MFMA operands, and each output row is
// written once.
//
// Forward: up to two products of the same input rows in one pass,
//   y1 = x W1^T (+ b1),  y2 = x W2^T (+ b2),
// each written at its own row stride (y1 may be a row-padded buffer, which
// the next g-SpMM gathers without straddling cache lines).
// Backward (input gradient): dx = dy1 W1 + dy2 W2, one pass over both.
//
// Operand maps of v_mfma_f32_16x16x4_f32 (cdna_hip_programming.md §3): lane l
// supplies A[row l&15][k l>>4] and B[k l>>4][col l&15]; D[row 4(l>>4)+i][col
// l&15] is register i. A block's k runs in the order the lanes load the input
// (lane group h = l>>4 holds input columns 64p + 16j + 4h + c in float4 j of
// pass p, so MFMA step (p, j, c) covers k = 64p + 16j + 4h + c over the four
// lane groups); the weights are read from LDS in the same k order. Each output
// element is one f32 fma chain over k (exact f32, no wider accumulation), the
// association of an ordinary GEMM's.
#include "common.h"
#include "launch.h"

#include <hip/hip_runtime.h>


namespace dglhip {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct LinOut {
  const float* w;   // [m][k1] row-major (nn.Linear weight) for the columns of x1
  const float* wb;  // [m][k2] for the columns of x2 (second input), or null
  const float* b;   // [m] or null
  float* y;         // rows at stride ldy
  int64_t ldy;
  int m;
  int relu;         // store max(y, 0) (the activation fused into the store)
};

// y_o = [x1 | x2] [W_o | Wb_o]^T + b_o for T1 (T2) 16-column tiles of output
// 1 (2); x1 has 64 * KB1 columns, x2 64 * KB2 (0: no second input).
template <int KB1, int KB2, int T1, int T2>
__global__ __launch_bounds__(512) void node_linear_fwd_kernel(
    int64_t n, const float* __restrict__ x1, int64_t ldx1, const float* __restrict__ x2,
    int64_t ldx2, LinOut o1, LinOut o2) {
  constexpr int KB = KB1 + KB2;
  constexpr int K1 = 64 * KB1, K2 = 64 * KB2, K = K1 + K2;
  constexpr int T = T1 + T2;
  // LDS row stride: the four k rows one MFMA reads (4 apart) land 16 banks apart
  constexpr int SW = 16 * T + 4;
  __shared__ float wt[K * SW];
  for (int idx = threadIdx.x; idx < K * 16 * T; idx += blockDim.x) {
    const int k = idx % K, col = idx / K;  // W rows read contiguously
    const bool first = col < 16 * T1;
    const LinOut& o = first ? o1 : o2;
    const int c = first ? col : col - 16 * T1;
    float v = 0.0f;
    if (c < o.m) v = k < K1 ? o.w[int64_t(c) * K1 + k] : o.wb[int64_t(c) * K2 + (k - K1)];
    wt[k * SW + col] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, r = lane & 15, h = lane >> 4;
  const int64_t nwaves = int64_t(gridDim.x) * (blockDim.x >> 6);
  const int64_t nblk = (n + 15) / 16;
  float bias[T];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const LinOut& o = t < T1 ? o1 : o2;
    const int c = 16 * (t < T1 ? t : t - T1) + r;
    bias[t] = (o.b != nullptr && c < o.m) ? o.b[c] : 0.0f;
  }
  // pass p (64 input columns) of the 16 rows of x a block needs, as MFMA
  // operands (zero past the end)
  auto load_pass = [&](int64_t blk, int p, f32x4 (&ap)[4]) {
    const int64_t row = blk * 16 + r;
    if (row < n) {
      const float* xr = p < KB1 ? x1 + row * ldx1 + 64 * p + 4 * h
                                : x2 + row * ldx2 + 64 * (p - KB1) + 4 * h;
#pragma unroll
      for (int j = 0; j < 4; ++j) ap[j] = *reinterpret_cast<const f32x4*>(xr + 16 * j);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) ap[j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    }
  };
  int64_t blk = int64_t(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  f32x4 a[KB][4];
  if (blk < nblk) {
#pragma unroll
    for (int p = 0; p < KB; ++p) load_pass(blk, p, a[p]);
  }
  for (; blk < nblk; blk += nwaves) {
    // the weight operands are loop-invariant: without this the compiler keeps
    // all of them in registers across blocks (K/4 x T values) and spills
    asm volatile("" ::: "memory");
    const int64_t r0 = blk * 16;
    const int64_t next = blk + nwaves;
    f32x4 acc[T];
#pragma unroll
    for (int t = 0; t < T; ++t) acc[t] = f32x4{bias[t], bias[t], bias[t], bias[t]};
    // weight operands of one float4 group (4 k-steps x T tiles) come from LDS
    // one group ahead of the MFMAs that use them: the LDS latency overlaps
    // the previous group's MFMAs instead of stalling each one
    float bw[2][4][T];
    auto load_w = [&](int g, float (&b)[4][T]) {
      const int p = g >> 2, j = g & 3;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float* wk = wt + (64 * p + 16 * j + 4 * h + c) * SW + r;
#pragma unroll
        for (int t = 0; t < T; ++t) b[c][t] = wk[16 * t];
      }
    };
    load_w(0, bw[0]);
#pragma unroll
    for (int g = 0; g < 4 * KB; ++g) {
      if (g + 1 < 4 * KB) load_w(g + 1, bw[(g + 1) & 1]);
      // keep the scheduler from sinking those reads back next to their MFMAs
      __builtin_amdgcn_sched_barrier(0);
      const int p = g >> 2, j = g & 3;
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int t = 0; t < T; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[p][j][c], bw[g & 1][c][t], acc[t], 0,
                                                        0, 0);
      // the pass's operands are consumed: the next block's pass p loads into
      // the same registers, in flight during this block's remaining passes
      if (j == 3 && next < nblk) load_pass(next, p, a[p]);
    }
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const LinOut& o = t < T1 ? o1 : o2;
      const int c = 16 * (t < T1 ? t : t - T1) + r;
      if (c >= o.m) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t orow = r0 + 4 * h + i;
        if (orow < n) o.y[orow * o.ldy + c] = o.relu ? fmaxf(acc[t][i], 0.0f) : acc[t][i];
      }
    }
  }
}

struct GradIn {
  const float* dy;  // rows at stride lddy, m columns
  int64_t lddy;
  const float* w;   // [m][k]
  int m;
};

// dx = dy1 W1 + dy2 W2 over S1 (S2) 4-wide steps of output 1's (2's) columns;
// KT 16-column tiles of dx. Computed transposed, dxᵀ = Wᵀ dyᵀ: the weights
// are the MFMA's A operand and the gradient rows its B operand, so a lane's
// four accumulator registers are four consecutive columns of ONE dx row (D
// row 4(l>>4)+i = dx column, D column l&15 = dx row): each tile leaves as one
// 16-byte store per lane (and the gate arrives as one 16-byte load) instead
// of four scalar ones. With a gate (the ReLU output that x is), the store is
// ReLU's backward rule: 0 where gate <= 0 (torch threshold_backward, NaN
// gates pass the gradient), so the mask costs no pass of its own.
template <int KT, int S1, int S2>
__global__ __launch_bounds__(512) void node_linear_bwd_kernel(int64_t n, GradIn g1, GradIn g2,
                                                              float* __restrict__ dx,
                                                              int64_t lddx,
                                                              const float* __restrict__ gate,
                                                              int64_t ldg,
                                                              float* __restrict__ part) {
  constexpr int K = 16 * KT;
  constexpr int S = S1 + S2;
  constexpr int SK = K + 16;  // rows 4s + h of one MFMA land 16 banks apart
  __shared__ float wl[4 * S * SK];
  for (int idx = threadIdx.x; idx < 4 * S * K; idx += blockDim.x) {
    const int q = idx / K, k = idx % K;
    float v = 0.0f;
    if (q < 4 * S1) {
      if (q < g1.m) v = g1.w[int64_t(q) * K + k];
    } else if (q - 4 * S1 < g2.m) {
      v = g2.w[int64_t(q - 4 * S1) * K + k];
    }
    wl[q * SK + k] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, r = lane & 15, h = lane >> 4;
  const int64_t nwaves = int64_t(gridDim.x) * (blockDim.x >> 6);
  const int64_t nblk = (n + 15) / 16;
  // step s of the gradient rows a block needs: row r, column 4s + h
  auto load_step = [&](int64_t blk, int s) -> float {
    const int64_t row = blk * 16 + r;
    const bool first = s < S1;
    const GradIn& g = first ? g1 : g2;
    const int col = 4 * (first ? s : s - S1) + h;
    return (row < n && col < g.m) ? g.dy[row * g.lddy + col] : 0.0f;
  };
  const int64_t wave = int64_t(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  int64_t blk = wave;
  float a[S];
  if (blk < nblk) {
#pragma unroll
    for (int s = 0; s < S; ++s) a[s] = load_step(blk, s);
  }
  // column sums of the stored dx over this lane's rows (part != null)
  f32x4 cs[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t) cs[t] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  for (; blk < nblk; blk += nwaves) {
    asm volatile("" ::: "memory");  // weight operands re-read from LDS per block
    const int64_t row = blk * 16 + r;  // this lane's dx row
    const int64_t next = blk + nwaves;
    // this row's gate values (4 consecutive columns per tile), in flight
    // during the MFMAs
    f32x4 gv[KT];
    if (gate != nullptr && row < n) {
#pragma unroll
      for (int t = 0; t < KT; ++t)
        gv[t] = *reinterpret_cast<const f32x4*>(gate + row * ldg + 16 * t + 4 * h);
    }
    f32x4 acc[KT];
#pragma unroll
    for (int t = 0; t < KT; ++t) acc[t] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    // weight operands one step ahead of their MFMAs (see the forward kernel)
    float bw[2][KT];
    auto load_w = [&](int s, float (&b)[KT]) {
      const float* ws = wl + (4 * s + h) * SK + r;
#pragma unroll
      for (int t = 0; t < KT; ++t) b[t] = ws[16 * t];
    };
    load_w(0, bw[0]);
#pragma unroll
    for (int s = 0; s < S; ++s) {
      if (s + 1 < S) load_w(s + 1, bw[(s + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < KT; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(bw[s & 1][t], a[s], acc[t], 0, 0, 0);
      // step s's operand is consumed: the next block's loads into its register
      if (next < nblk) a[s] = load_step(next, s);
    }
    if (row < n) {
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        f32x4 v = acc[t];
        if (gate != nullptr) {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = gv[t][i] <= 0.0f ? 0.0f : v[i];
        }
        *reinterpret_cast<f32x4*>(dx + row * lddx + 16 * t + 4 * h) = v;
        if (part != nullptr) cs[t] += v;
      }
    }
  }
  if (part != nullptr) {
    // this wave's column sums: the 16 lanes of a column group (same h) summed
    // in a fixed butterfly, one row of K partials per wave
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = cs[t][i];
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) v += __shfl_xor(v, off, 64);
        if (r == 0) part[wave * K + 16 * t + 4 * h + i] = v;
      }
  }
}

// colsum[c] = the waves' partial column sums: one workgroup per column, lane
// j summing waves j, j + 256, ... in order, then a fixed tree over the lanes
__global__ __launch_bounds__(256) void colsum_partials_kernel(int64_t nparts, int K,
                                                              const float* __restrict__ part,
                                                              float* __restrict__ colsum) {
  __shared__ float red[256];
  const int c = blockIdx.x;
  float s = 0.0f;
  for (int64_t w = threadIdx.x; w < nparts; w += 256) s += part[w * K + c];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) colsum[c] = red[0];
}

// Persistent grid: the weights are staged in LDS once per workgroup and the
// 16-row blocks are strided over its waves; 512-lane workgroups so that even a
// workgroup whose weights fill most of the LDS keeps two waves per SIMD.
// Launch shape (dglhip_set_node_linear_variant; 0 = automatic): lanes per
// workgroup and workgroups per CU.
int g_nl_threads = 0, g_nl_per_cu = 0;

inline int nl_threads() { return g_nl_threads ? g_nl_threads : 512; }

inline int64_t persistent_blocks(int64_t n, int lds_bytes) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  const int per_cu = g_nl_per_cu ? g_nl_per_cu
                                 : std::max(1, std::min(4, (160 * 1024) / std::max(lds_bytes, 1)));
  const int64_t want = int64_t(cus) * per_cu;
  const int waves = nl_threads() / 64;
  const int64_t need = ((n + 15) / 16 + waves - 1) / waves;
  return std::max<int64_t>(1, std::min(want, need));
}

template <int KB1, int KB2, int T1, int T2>
void launch_fwd(int64_t n, const float* x1, int64_t ldx1, const float* x2, int64_t ldx2,
                const LinOut& o1, const LinOut& o2, hipStream_t stream) {
  constexpr int lds = 64 * (KB1 + KB2) * (16 * (T1 + T2) + 4) * 4;
  hipLaunchKernelGGL((node_linear_fwd_kernel<KB1, KB2, T1, T2>),
                     dim3(persistent_blocks(n, lds)), dim3(nl_threads()), 0, stream, n, x1, ldx1, x2,
                     ldx2, o1, o2);
}

// 65..128 outputs of two 128-column inputs in ONE pass over the inputs (8
// tiles; the weights take 135 KB of LDS, one 512-lane workgroup per CU, 256
// registers a lane): 38.4 ms at 67M rows against 41.4 for one pass per 64
// outputs and 43 for hipBLASLt (tools/node_linear_bench.py)
void launch_fwd_wide(int64_t n, const float* x1, int64_t ldx1, const float* x2, int64_t ldx2,
                     const LinOut& o, hipStream_t stream) {
  constexpr int lds = 64 * 4 * (16 * 8 + 4) * 4;
  hipLaunchKernelGGL((node_linear_fwd_kernel<2, 2, 8, 0>), dim3(persistent_blocks(n, lds)),
                     dim3(nl_threads()), 0, stream, n, x1, ldx1, x2, ldx2, o, o);
}

template <int KB, int T1>
void dispatch_fwd_t2(int t2, int64_t n, const float* x, int64_t ldx, const LinOut& o1,
                     const LinOut& o2, hipStream_t s) {
  switch (t2) {
    case 0: return launch_fwd<KB, 0, T1, 0>(n, x, ldx, x, ldx, o1, o2, s);
    case 1: return launch_fwd<KB, 0, T1, 1>(n, x, ldx, x, ldx, o1, o2, s);
    case 2: return launch_fwd<KB, 0, T1, 2>(n, x, ldx, x, ldx, o1, o2, s);
    case 3: return launch_fwd<KB, 0, T1, 3>(n, x, ldx, x, ldx, o1, o2, s);
    default: return launch_fwd<KB, 0, T1, 4>(n, x, ldx, x, ldx, o1, o2, s);
  }
}

template <int KB>
void dispatch_fwd(int t1, int t2, int64_t n, const float* x, int64_t ldx, const LinOut& o1,
                  const LinOut& o2, hipStream_t s) {
  switch (t1) {
    case 1: return dispatch_fwd_t2<KB, 1>(t2, n, x, ldx, o1, o2, s);
    case 2: return dispatch_fwd_t2<KB, 2>(t2, n, x, ldx, o1, o2, s);
    case 3: return dispatch_fwd_t2<KB, 3>(t2, n, x, ldx, o1, o2, s);
    default: return dispatch_fwd_t2<KB, 4>(t2, n, x, ldx, o1, o2, s);
  }
}

// what the input-gradient store does besides storing: the ReLU gate, and the
// per-wave column-sum partials (with the grid it used, for the final sum)
struct Gate {
  const float* p;
  int64_t ld;
  float* part;
  int64_t nparts;  // set by the launch: waves of the grid
};

inline int64_t max_bwd_waves();

template <int KT, int S1, int S2>
void launch_bwd(int64_t n, const GradIn& g1, const GradIn& g2, float* dx, int64_t lddx,
                Gate& gate, hipStream_t stream) {
  constexpr int lds = 4 * (S1 + S2) * (16 * KT + 16) * 4;
  const int64_t grid = persistent_blocks(n, lds);
  gate.nparts = grid * (nl_threads() / 64);
  // every wave writes its column-sum partials: the grid must fit the
  // workspace (sized by dglhip_node_linear_dgrad_workspace_floats) BEFORE the
  // launch, whatever launch shape a tuning knob has set since the query
  DGLHIP_CHECK(gate.part == nullptr || gate.nparts <= max_bwd_waves(),
               "column-sum workspace too small for " << gate.nparts << " waves");
  hipLaunchKernelGGL((node_linear_bwd_kernel<KT, S1, S2>), dim3(grid), dim3(nl_threads()), 0,
                     stream, n, g1, g2, dx, lddx, gate.p, gate.ld, gate.part);
}

// upper bound of launch_bwd's waves: 4 workgroups per CU of up to 512 lanes
// (persistent_blocks) or the tuning knob's count
inline int64_t max_bwd_waves() {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  return int64_t(cus) * 8 * 8;
}

// reduction widths up to 64 per input: S = ceil(m / 4) rounded up to a listed
// step count (11 = the 41 classes of GraphSAGE's output layer); padded steps
// multiply zero operands.
constexpr int kSteps[] = {2, 4, 8, 11, 16};

inline int round_steps(int m) {
  const int s = (m + 3) / 4;
  for (int v : kSteps)
    if (s <= v) return v;
  return -1;
}

template <int KT, int S1>
void dispatch_bwd_s2(int s2, int64_t n, const GradIn& g1, const GradIn& g2, float* dx,
                     int64_t lddx, Gate& gt, hipStream_t st) {
  switch (s2) {
    case 0: return launch_bwd<KT, S1, 0>(n, g1, g2, dx, lddx, gt, st);
    case 2: return launch_bwd<KT, S1, 2>(n, g1, g2, dx, lddx, gt, st);
    case 4: return launch_bwd<KT, S1, 4>(n, g1, g2, dx, lddx, gt, st);
    case 8: return launch_bwd<KT, S1, 8>(n, g1, g2, dx, lddx, gt, st);
    case 11: return launch_bwd<KT, S1, 11>(n, g1, g2, dx, lddx, gt, st);
    default: return launch_bwd<KT, S1, 16>(n, g1, g2, dx, lddx, gt, st);
  }
}

template <int KT>
void dispatch_bwd(int s1, int s2, int64_t n, const GradIn& g1, const GradIn& g2, float* dx,
                  int64_t lddx, Gate& gt, hipStream_t st) {
  switch (s1) {
    case 2: return dispatch_bwd_s2<KT, 2>(s2, n, g1, g2, dx, lddx, gt, st);
    case 4: return dispatch_bwd_s2<KT, 4>(s2, n, g1, g2, dx, lddx, gt, st);
    case 8: return dispatch_bwd_s2<KT, 8>(s2, n, g1, g2, dx, lddx, gt, st);
    case 11: return dispatch_bwd_s2<KT, 11>(s2, n, g1, g2, dx, lddx, gt, st);
    default: return dispatch_bwd_s2<KT, 16>(s2, n, g1, g2, dx, lddx, gt, st);
  }
}

}  // namespace

}  // namespace dglhip

using namespace dglhip;

extern "C" {

int dglhip_node_linear_device(int64_t num_rows, int64_t in_feats, const float* x, int64_t ldx,
                              int64_t m1, const float* w1, const float* b1, float* y1,
                              int64_t ldy1, int64_t m2, const float* w2, const float* b2,
                              float* y2, int64_t ldy2, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows >= 0, "negative row count");
  DGLHIP_CHECK(in_feats == 64 || in_feats == 128 || in_feats == 256,
               "node Linear on the MFMA: in_feats must be 64, 128 or 256, got " << in_feats);
  DGLHIP_CHECK(m1 >= 1 && m1 <= 64 && m2 >= 0 && m2 <= 64,
               "node Linear on the MFMA: 1..64 (+ 0..64) outputs, got " << m1 << ", " << m2);
  if (num_rows == 0) return 0;  // empty tensors may carry any strides and null pointers
  DGLHIP_CHECK(ldx >= in_feats && ldx % 4 == 0, "ldx " << ldx << ": >= in_feats, multiple of 4");
  DGLHIP_CHECK(ldy1 >= m1 && (m2 == 0 || ldy2 >= m2), "output row stride below its width");
  DGLHIP_CHECK(x && w1 && y1 && (m2 == 0 || (w2 && y2)), "null pointer argument");
  DGLHIP_CHECK(reinterpret_cast<uintptr_t>(x) % 16 == 0, "x must be 16-byte aligned");
  LinOut o1{w1, nullptr, b1, y1, ldy1, static_cast<int>(m1), 0};
  LinOut o2{w2, nullptr, b2, y2, ldy2, static_cast<int>(m2), 0};
  const int t1 = static_cast<int>((m1 + 15) / 16), t2 = static_cast<int>((m2 + 15) / 16);
  switch (in_feats / 64) {
    case 1: dispatch_fwd<1>(t1, t2, num_rows, x, ldx, o1, o2, stream); break;
    case 2: dispatch_fwd<2>(t1, t2, num_rows, x, ldx, o1, o2, stream); break;
    default: dispatch_fwd<4>(t1, t2, num_rows, x, ldx, o1, o2, stream); break;
  }
  DGLHIP_CHECK(hipGetLastError() == hipSuccess, "node Linear launch failed");
  API_END();
}

int64_t dglhip_node_linear_dgrad_workspace_floats(int64_t in_feats) {
  return max_bwd_waves() * in_feats;
}

int dglhip_set_node_linear_variant(int threads, int wgs_per_cu) {
  API_BEGIN();
  DGLHIP_CHECK(threads == 0 || threads == 256 || threads == 512, "threads: 0, 256 or 512");
  DGLHIP_CHECK(wgs_per_cu >= 0 && wgs_per_cu <= 8, "workgroups per CU: 0..8");
  g_nl_threads = threads;
  g_nl_per_cu = wgs_per_cu;
  API_END();
}

int dglhip_node_linear_cat_device(int64_t num_rows, int64_t in_feats, const float* x1,
                                  int64_t ldx1, const float* x2, int64_t ldx2, int64_t m,
                                  const float* w1, const float* w2, const float* b, float* y,
                                  int64_t ldy, int relu, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows >= 0, "negative row count");
  DGLHIP_CHECK(in_feats == 64 || in_feats == 128,
               "two-input node Linear on the MFMA: in_feats 64 or 128, got " << in_feats);
  DGLHIP_CHECK(m >= 1 && m <= 128, "two-input node Linear on the MFMA: 1..128 outputs, got " << m);
  if (num_rows == 0) return 0;
  DGLHIP_CHECK(ldx1 >= in_feats && ldx2 >= in_feats && ldx1 % 4 == 0 && ldx2 % 4 == 0,
               "input row strides: >= in_feats, multiples of 4");
  DGLHIP_CHECK(ldy >= m, "output row stride below its width");
  DGLHIP_CHECK(x1 && x2 && w1 && w2 && y, "null pointer argument");
  DGLHIP_CHECK(reinterpret_cast<uintptr_t>(x1) % 16 == 0 && reinterpret_cast<uintptr_t>(x2) % 16 == 0,
               "inputs must be 16-byte aligned");
  // otherwise at most 64 outputs per pass (4 tiles), one pass per 64 columns
  if (in_feats == 128 && m > 64) {
    LinOut o{w1, w2, b, y, ldy, static_cast<int>(m), relu ? 1 : 0};
    launch_fwd_wide(num_rows, x1, ldx1, x2, ldx2, o, stream);
    DGLHIP_CHECK(hipGetLastError() == hipSuccess, "two-input node Linear launch failed");
    return 0;
  }
  for (int64_t c0 = 0; c0 < m; c0 += 64) {
    LinOut o{w1 + c0 * in_feats, w2 + c0 * in_feats, b ? b + c0 : nullptr, y + c0, ldy,
             static_cast<int>(std::min<int64_t>(64, m - c0)), relu ? 1 : 0};
    if (in_feats == 64) launch_fwd<1, 1, 4, 0>(num_rows, x1, ldx1, x2, ldx2, o, o, stream);
    else launch_fwd<2, 2, 4, 0>(num_rows, x1, ldx1, x2, ldx2, o, o, stream);
  }
  DGLHIP_CHECK(hipGetLastError() == hipSuccess, "two-input node Linear launch failed");
  API_END();
}

int dglhip_node_linear_dgrad_device(int64_t num_rows, int64_t in_feats, int64_t m1,
                                    const float* dy1, int64_t lddy1, const float* w1, int64_t m2,
                                    const float* dy2, int64_t lddy2, const float* w2, float* dx,
                                    int64_t lddx, const float* gate, int64_t ldg, float* colsum,
                                    float* workspace, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows >= 0, "negative row count");
  DGLHIP_CHECK(in_feats == 64 || in_feats == 128, "input gradient on the MFMA: in_feats 64 or 128, got "
                                                      << in_feats);
  const int s1 = round_steps(static_cast<int>(m1)), s2 = m2 == 0 ? 0 : round_steps(static_cast<int>(m2));
  DGLHIP_CHECK(m1 >= 1 && m1 <= 64 && m2 >= 0 && m2 <= 64 && s1 > 0 && s2 >= 0,
               "input gradient on the MFMA: 1..64 (+ 0..64) outputs, got " << m1 << ", " << m2);
  if (num_rows == 0) {
    if (colsum != nullptr) DGLHIP_CHECK(hipMemsetAsync(colsum, 0, in_feats * 4, stream) == hipSuccess,
                                        "column-sum clear failed");
    return 0;
  }
  DGLHIP_CHECK(lddy1 >= m1 && (m2 == 0 || lddy2 >= m2) && lddx >= in_feats,
               "row stride below the row width");
  DGLHIP_CHECK(dy1 && w1 && dx && (m2 == 0 || (dy2 && w2)), "null pointer argument");
  DGLHIP_CHECK(gate == nullptr || ldg >= in_feats, "gate row stride below in_feats");
  // dx and the gate move as 16-byte vectors
  DGLHIP_CHECK(lddx % 4 == 0 && reinterpret_cast<uintptr_t>(dx) % 16 == 0,
               "dx: 16-byte aligned rows (row stride a multiple of 4)");
  DGLHIP_CHECK(gate == nullptr || (ldg % 4 == 0 && reinterpret_cast<uintptr_t>(gate) % 16 == 0),
               "gate: 16-byte aligned rows (row stride a multiple of 4)");
  GradIn g1{dy1, lddy1, w1, static_cast<int>(m1)};
  GradIn g2{dy2, lddy2, w2, static_cast<int>(m2)};
  DGLHIP_CHECK(colsum == nullptr || workspace != nullptr, "column sums need the workspace");
  Gate gt{gate, ldg, colsum != nullptr ? workspace : nullptr, 0};
  if (in_feats == 64) dispatch_bwd<4>(s1, s2, num_rows, g1, g2, dx, lddx, gt, stream);
  else dispatch_bwd<8>(s1, s2, num_rows, g1, g2, dx, lddx, gt, stream);
  if (colsum != nullptr) {
    const int K = static_cast<int>(in_feats);
    hipLaunchKernelGGL(colsum_partials_kernel, dim3(K), dim3(256), 0, stream, gt.nparts, K,
                       workspace, colsum);
  }
  DGLHIP_CHECK(hipGetLastError() == hipSuccess, "node Linear input-gradient launch failed");
  API_END();
}

}  // extern "C"
