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

#include <cstdlib>

#include "gspmm_impl.h"

namespace dglhip {

// GAT attention-gradient epilogue of the SDDMM dot (EPI = true): the dot
// d_w[k, h] = <dC[row, h, :], ft[u, h, :]> becomes the gradient of the
// attention's pre-activation, stored in slot order:
//   t = d_w; t = keep ? t * scale : 0 (dropout: keep from the forward's hash
//   of (seed, k * H + h) with hash_keep, else w[k, h] != 0);
//   t = t + dz[row, h] (the normaliser's gradient);
//   g = (t * a) * s (exp; else t * s), s = alpha where the logit x <= 0, else 1
//       (torch's leaky_relu backward). With the logits given (el, er: x =
//       el[u, h] + er[row, h], the forward's sum) s comes from x itself;
//       without them from a (a <= 1 with exp, a <= 0 without), which differs
//       from x's sign only for 0 < x < 2^-24, where exp(x) rounds to 1 (r04
//       ADVICE: the fused backward and the engine's three-pass path take the
//       logits, so every path follows torch there too);
//   g = lo < a < hi ? g : 0
// the float operations, and their order, of kernel._GATAggregate's torch
// backward, so both give the same bits.
struct GatEpi {
  const float* a;     // attention, [nnz, H] slot order
  const float* w;     // its dropped copy (NULL: no dropout)
  const float* dz;    // normaliser gradient, [rows, H] (NULL: zero)
  float alpha, lo, hi, scale;
  int apply_exp;
  // optional: each row's per-head sum of the values stored, added in slot
  // order to what rsum holds ([rows, H]; GAT's er gradient, the copy_e sum
  // of the stored values over the row's slots, fused; sliced kernel only)
  float* rsum = nullptr;
  // dropout keep bits from the forward's hash (seed + *seed_off, threshold
  // thr) instead of w != 0: a kept pair whose attention is exactly 0 keeps
  // its gradient (r03 ADVICE); w is then not read
  int hash_keep = 0;
  uint64_t seed = 0;
  const int64_t* seed_off = nullptr;
  uint32_t thr = 0;
  // the attention's logits (the slope from x's sign; NULL: from a)
  const float* el = nullptr;  // [num_src, H]
  const float* er = nullptr;  // [rows, H]
};

// The leaky_relu slope of a pair: from the logit's sign when it is known
// (xpos >= 0), else from the attention value (see GatEpi).
__device__ __forceinline__ float gat_slope(const GatEpi& e, float a, int xpos) {
  if (xpos >= 0) return xpos ? 1.0f : e.alpha;
  return e.apply_exp ? (a <= 1.0f ? e.alpha : 1.0f) : (a <= 0.0f ? e.alpha : 1.0f);
}

__device__ __forceinline__ uint64_t gat_epi_seed(const GatEpi& e) {
  return e.seed + (e.seed_off ? static_cast<uint64_t>(*e.seed_off) : 0);
}

__device__ __forceinline__ float gat_epi(const GatEpi& e, float t, int64_t k, int64_t H,
                                         int64_t h, int64_t row, int64_t u) {
  const float a = e.a[k * H + h];
  if (e.hash_keep) t = gat_keep(gat_epi_seed(e), k * H + h, e.thr) ? t * e.scale : 0.0f;
  else if (e.w) t = e.w[k * H + h] != 0.0f ? t * e.scale : 0.0f;
  if (e.dz) t = t + e.dz[row * H + h];
  const int xpos = e.el ? ((e.el[u * H + h] + e.er[row * H + h]) > 0.0f ? 1 : 0) : -1;
  const float g = e.apply_exp ? (t * a) * gat_slope(e, a, xpos) : t * gat_slope(e, a, xpos);
  return (a > e.lo && a < e.hi) ? g : 0.0f;
}

// gat_epi on operands loaded ahead (the slot's attention a and keep bit,
// the row's normaliser gradient dz): the same arithmetic.
__device__ __forceinline__ float gat_epi_pre(const GatEpi& e, float t, float a, bool keep,
                                             float dz, int xpos) {
  if (e.w || e.hash_keep) t = keep ? t * e.scale : 0.0f;
  if (e.dz) t = t + dz;
  const float g = e.apply_exp ? (t * a) * gat_slope(e, a, xpos) : t * gat_slope(e, a, xpos);
  return (a > e.lo && a < e.hi) ? g : 0.0f;
}

// SDDMM dot: one wave per row. One head (H == 1): per slot a wave-wide fma
// dot product of two feature rows reduced in a fixed butterfly order. Several
// heads: lane h computes head h's dot over its D = F / H features as one
// sequential fma chain. Both orders are fixed, so results are deterministic.
template <bool EPI = false>
__global__ __launch_bounds__(256) void gsddmm_dot_kernel(
    int64_t num_rows, int64_t F, int64_t H, const int64_t* __restrict__ row_beg,
    const int64_t* __restrict__ row_end, const int32_t* __restrict__ row_order,
    const int32_t* __restrict__ indices, const int64_t* __restrict__ eid,
    const float* __restrict__ lhs, const float* __restrict__ rhs,
    float* __restrict__ out, GatEpi epi) {
  const int64_t it = block_linear() * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (it >= num_rows) return;
  const int64_t wave = row_order ? row_order[it] : it;
  const int lane = threadIdx.x & 63;
  const float* a = lhs + wave * F;
  const int64_t D = F / H;
  const int64_t kb = row_beg[wave], ke = row_end[wave];
  if (H == 1) {
    for (int64_t k = kb; k < ke; ++k) {
      const int64_t col = indices[k];
      const float* c = rhs + col * F;
      float acc = 0.0f;
      for (int64_t f = lane; f < F; f += 64) acc = __builtin_fmaf(a[f], c[f], acc);
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
      if (lane == 0) out[eid ? eid[k] : k] = EPI ? gat_epi(epi, acc, k, 1, 0, wave, col) : acc;
    }
  } else if (H <= 64) {
    // 64 / H slots at a time, lane (sub, h) taking head h of slot k0 + sub:
    // the same per-head chain, 64 / H times the slots in flight (r05: the
    // GAT output layer's 8 heads x 3 ran one slot per step on 8 lanes)
    const int64_t S = 64 / H;
    const int64_t sub = lane / H, h = lane - sub * H;
    for (int64_t k0 = kb; k0 < ke; k0 += S) {
      const int64_t k = k0 + sub;
      if (sub < S && k < ke) {
        const int64_t col = indices[k];
        const float* c = rhs + col * F;
        float acc = 0.0f;
        for (int64_t d = 0; d < D; ++d) acc = __builtin_fmaf(a[h * D + d], c[h * D + d], acc);
        out[(eid ? eid[k] : k) * H + h] = EPI ? gat_epi(epi, acc, k, H, h, wave, col) : acc;
      }
    }
  } else {
    for (int64_t k = kb; k < ke; ++k) {
      const int64_t col = indices[k];
      const float* c = rhs + col * F;
      for (int64_t h = lane; h < H; h += 64) {
        float acc = 0.0f;
        for (int64_t d = 0; d < D; ++d) acc = __builtin_fmaf(a[h * D + d], c[h * D + d], acc);
        out[(eid ? eid[k] : k) * H + h] = EPI ? gat_epi(epi, acc, k, H, h, wave, col) : acc;
      }
    }
  }
}

// Quad butterflies through DPP (a VALU operand modifier) instead of
// ds_bpermute: lane i reads lane i ^ 1 / i ^ 2 of its quad, the same pairing
// as __shfl_xor(v, 1 / 2), so the sums keep their bits.
__device__ __forceinline__ float quad_xor1(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float quad_xor2(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
}

// One xor-exchange across the lanes of a slot (M = 4: __shfl_xor; 2, 1: DPP).
template <int M>
__device__ __forceinline__ float slot_xchg(float v) {
  if (M == 4) return __shfl_xor(v, 4, 64);
  if (M == 2) return quad_xor2(v);
  return quad_xor1(v);
}

// One reduce-scatter stage over lane pairs (j, j ^ M) on Q per-lane values:
// the lane with bit M set keeps the upper half, its partner the lower half;
// each sends the half it drops and adds what it receives to what it keeps
// (own + partner, the butterfly's operand order, so both lanes that end up
// holding a value hold the same bits). Q == 1 is a plain butterfly step.
// The exchanges move only the half that is kept elsewhere: for Q values over
// 8 lanes, Q/2 + Q/4 + Q/8 shuffles instead of the butterfly's 3 Q.
template <int Q, int M>
__device__ __forceinline__ void rs_step(float* q, int j) {
  if (Q == 1) {
    q[0] = q[0] + slot_xchg<M>(q[0]);
    return;
  }
  const bool up = (j & M) != 0;
#pragma unroll
  for (int i = 0; i < Q / 2; ++i) {
    const float keep = up ? q[i + Q / 2] : q[i];
    const float send = up ? q[i] : q[i + Q / 2];
    q[i] = keep + slot_xchg<M>(send);
  }
}

// Reduce-scatter of Q values across L lanes (xor L/2, ..., 1: the pairing
// order of the full butterfly, so every total carries the same bits). Lane r
// of the group (r = j % L) ends with values r * Q/L .. (r+1) * Q/L - 1 of the
// group's totals in q[0..Q/L) when Q >= L; else with value r / (L/Q) in q[0].
template <int Q, int L>
__device__ __forceinline__ void slot_reduce_scatter(float* q, int j) {
  if (L >= 8) rs_step<Q, 4>(q, j);
  constexpr int Q2 = (L >= 8 && Q > 1) ? Q / 2 : Q;
  if (L >= 4) rs_step<Q2, 2>(q, j);
  constexpr int Q3 = (L >= 4 && Q2 > 1) ? Q2 / 2 : Q2;
  if (L >= 2) rs_step<Q3, 1>(q, j);
}

// SDDMM dot for rows of NB x 32 floats (F = 32 * NB) and H heads of
// D = F / H features, one wave per row: the wave takes 8 slots at a time,
// 8 lanes per slot; lane j of a slot reads the 16 B at 32 i + 4 j of every
// 32-float column block i (one instruction = 8 whole 128-B lines), UNROLL
// groups of 8 slots in flight. Per lane and block the partial is an fma chain
// over its 4 features (x, y, z, w).
//   D >= 32 (LPH = 8 lanes per head): a head's lane partial sums its D / 32
//     blocks in block order; the H partials are reduce-scattered over the 8
//     lanes, and lane j stores heads j * H/8 .. (H >= 8), or lane j with
//     j % (8/H) == 0 stores head j / (8/H): one store instruction per slot,
//     the slot's H values contiguous.
//   D < 32 (LPH = D / 4 lanes per head, HPB = 8 / LPH heads per block): the
//     NB block partials are reduce-scattered within each LPH-lane group g;
//     lane (g, r) then holds blocks r * NB/LPH + t, i.e. heads
//     (r * NB/LPH + t) * HPB + g: each t is one store instruction covering 8
//     of the slot's heads (8 heads at D = 16: one 32-B run per slot).
// The pairing of lanes is the full xor butterfly's (4, 2, 1 / 2, 1 / 1), so
// results are deterministic and equal the butterfly's bits.
template <int NB, int UNROLL, int H, bool EPI = false, bool PRE = true>
__global__ __launch_bounds__(256) void gsddmm_dot_sliced_kernel(
    int64_t num_rows, const int64_t* __restrict__ row_beg, const int64_t* __restrict__ row_end,
    const int32_t* __restrict__ row_order, const int32_t* __restrict__ indices, const int64_t* __restrict__ eid,
    const float* __restrict__ lhs, const float* __restrict__ rhs, float* __restrict__ out,
    GatEpi epi) {
  constexpr int F = NB * 32;
  constexpr int D = F / H;
  constexpr int LPH = D >= 32 ? 8 : D / 4;  // lanes sharing a head
  constexpr int DBLK = D >= 32 ? D / 32 : 1;  // blocks per head (D >= 32)
  static_assert(D >= 32 ? D % 32 == 0 : (D == 4 || D == 8 || D == 16), "head width");
  const int64_t it = block_linear() * (blockDim.x >> 6) +
                     __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  if (it >= num_rows) return;
  // rows in the given schedule (degree-descending: the longest rows first)
  const int64_t row = row_order ? __builtin_amdgcn_readfirstlane(row_order[it]) : it;
  const int lane = threadIdx.x & 63;
  const int s = lane >> 3, j = lane & 7;
  const int64_t beg = row_beg[row], end = row_end[row];
  if (beg == end) return;
  // the heads this lane stores per slot (the branches below): T of them
  constexpr int T = LPH == 8 ? (H >= 8 ? H / 8 : 1) : (NB >= LPH ? NB / LPH : 1);
  auto lane_head = [&](int t) -> int {
    if (LPH == 8) return H >= 8 ? j * (H / 8) + t : j / (H >= 8 ? 1 : 8 / H);
    constexpr int HPB = 8 / LPH;
    const int g = j / LPH, r = j % LPH;
    return NB >= LPH ? (r * (NB / LPH) + t) * HPB + g : (r / (NB >= LPH ? 1 : LPH / NB)) * HPB + g;
  };
  // the GAT epilogue's per-row operand, loaded once; the dropout hash's seed
  const uint64_t hseed = (EPI && epi.hash_keep) ? gat_epi_seed(epi) : 0;
  auto keep_of = [&](int64_t k, int hh, float w) -> bool {
    return (EPI && epi.hash_keep) ? gat_keep(hseed, k * H + hh, epi.thr) : w != 0.0f;
  };
  float dzv[T], erv[T];
  const bool xl = EPI && epi.el != nullptr;  // the slope from the logits (wave-uniform)
#pragma unroll
  for (int t = 0; t < T; ++t) {
    dzv[t] = (EPI && PRE && epi.dz) ? epi.dz[row * H + lane_head(t)] : 0.0f;
    erv[t] = xl ? epi.er[row * H + lane_head(t)] : 0.0f;
  }
  // the fused row sums: lanes of slot group s each chain the values of every
  // slot of the row in slot order (s = 0 stores them)
  const bool rs = EPI && epi.rsum != nullptr;  // wave-uniform
  float racc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) racc[t] = rs ? epi.rsum[row * H + lane_head(t)] : 0.0f;
  f32x4 a[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) a[i] = ldv<4>(lhs + row * F + 32 * i + 4 * j);
  for (int64_t k0 = beg; k0 < end; k0 += 8 * UNROLL) {
    f32x4 c[UNROLL][NB];
    float ea[UNROLL][T], ew[UNROLL][T], ex[UNROLL][T];
    int64_t ucol[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      int64_t k = k0 + 8 * u + s;
      k = k < end ? k : end - 1;  // idle slot lanes re-read the row's last slot
      ucol[u] = indices[k];
      const float* r = rhs + ucol[u] * F + 4 * j;
#pragma unroll
      for (int i = 0; i < NB; ++i) c[u][i] = ldv<4>(r + 32 * i);
      // the epilogue's per-slot operands in flight with the gathers, not
      // behind the dot product (attention gradient: fewer serial latencies)
#pragma unroll
      for (int t = 0; t < T; ++t) {
        ea[u][t] = (EPI && PRE) ? epi.a[k * H + lane_head(t)] : 0.0f;
        ew[u][t] = (EPI && PRE && epi.w) ? epi.w[k * H + lane_head(t)] : 0.0f;
        ex[u][t] = (EPI && PRE && xl) ? epi.el[ucol[u] * H + lane_head(t)] : 0.0f;
      }
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
      const int64_t obase = (k < end ? (eid ? eid[k] : k) : 0) * H;
      float sv[T];  // the values this lane's slot stores, by lane_head(t)
      if (LPH == 8) {
        float q[H];
#pragma unroll
        for (int h = 0; h < H; ++h) {  // a head's blocks in order
          q[h] = p[h * DBLK];
#pragma unroll
          for (int b = 1; b < DBLK; ++b) q[h] = q[h] + p[h * DBLK + b];
        }
        slot_reduce_scatter<H, 8>(q, j);
        if (H >= 8) {
#pragma unroll
          for (int t = 0; t < (H >= 8 ? H / 8 : 1); ++t) {
            const int hh = j * (H / 8) + t;
            sv[t] = EPI ? (PRE ? gat_epi_pre(epi, q[t], ea[u][t], keep_of(k, hh, ew[u][t]), dzv[t], xl ? ((ex[u][t] + erv[t]) > 0.0f ? 1 : 0) : -1) : gat_epi(epi, q[t], k, H, hh, row, ucol[u])) : q[t];
            if (k < end) out[obase + hh] = sv[t];
          }
        } else {
          constexpr int DUP = H >= 8 ? 1 : 8 / H;  // lanes holding the same head
          const int hh = j / DUP;
          sv[0] = EPI ? (PRE ? gat_epi_pre(epi, q[0], ea[u][0], keep_of(k, hh, ew[u][0]), dzv[0], xl ? ((ex[u][0] + erv[0]) > 0.0f ? 1 : 0) : -1) : gat_epi(epi, q[0], k, H, hh, row, ucol[u])) : q[0];
          if (k < end && j % DUP == 0) out[obase + hh] = sv[0];
        }
      } else {
        constexpr int HPB = 8 / LPH;
        const int g = j / LPH, r = j % LPH;
        slot_reduce_scatter<NB, LPH>(p, j);
        if (NB >= LPH) {
#pragma unroll
          for (int t = 0; t < (NB >= LPH ? NB / LPH : 1); ++t) {
            const int hh = (r * (NB / LPH) + t) * HPB + g;
            sv[t] = EPI ? (PRE ? gat_epi_pre(epi, p[t], ea[u][t], keep_of(k, hh, ew[u][t]), dzv[t], xl ? ((ex[u][t] + erv[t]) > 0.0f ? 1 : 0) : -1) : gat_epi(epi, p[t], k, H, hh, row, ucol[u])) : p[t];
            if (k < end) out[obase + hh] = sv[t];
          }
        } else {
          constexpr int DUP = NB >= LPH ? 1 : LPH / NB;
          const int hh = (r / DUP) * HPB + g;
          sv[0] = EPI ? (PRE ? gat_epi_pre(epi, p[0], ea[u][0], keep_of(k, hh, ew[u][0]), dzv[0], xl ? ((ex[u][0] + erv[0]) > 0.0f ? 1 : 0) : -1) : gat_epi(epi, p[0], k, H, hh, row, ucol[u])) : p[0];
          if (k < end && r % DUP == 0) out[obase + hh] = sv[0];
        }
      }
      if (rs) {
        // the 8 slots of group u in slot order: lane (s, j) adds slot s2's
        // value of its head from lane (s2, j) (same j, same head)
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2) {
#pragma unroll
          for (int t = 0; t < T; ++t) {
            const float v = __shfl(sv[t], s2 * 8 + j, 64);
            if (k0 + 8 * u + s2 < end) racc[t] = racc[t] + v;
          }
        }
      }
    }
  }
  if (rs && s == 0) {
#pragma unroll
    for (int t = 0; t < T; ++t) epi.rsum[row * H + lane_head(t)] = racc[t];
  }
}

// GAT edge attention, one wave per destination row v (gat/train.py:90-96):
//   out[eid[k], h] = clamp(exp(leaky_relu(lhs[u, h] + rhs[v, h], alpha)), lo, hi)
// with u = indices[k]; lanes run over the row's (slot, head) pairs. Generic
// head count; the common ones take gsddmm_attention_vec_kernel.
__global__ __launch_bounds__(256) void gsddmm_attention_kernel(
    int64_t num_rows, int64_t H, const int64_t* __restrict__ indptr,
    const int32_t* __restrict__ indices, const int64_t* __restrict__ eid,
    const float* __restrict__ lhs, const float* __restrict__ rhs, float alpha, float lo,
    float hi, int apply_exp, float* __restrict__ out) {
  const int64_t row = block_linear() * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= num_rows) return;
  const int lane = threadIdx.x & 63;
  const int64_t beg = indptr[row], n = (indptr[row + 1] - beg) * H;
  for (int64_t idx = lane; idx < n; idx += 64) {
    const int64_t k = beg + idx / H, h = idx - (idx / H) * H;
    float x = lhs[int64_t(indices[k]) * H + h] + rhs[row * H + h];
    x = x > 0.0f ? x : alpha * x;
    if (apply_exp) x = __expf(x);
    out[(eid ? eid[k] : k) * H + h] = fminf(fmaxf(x, lo), hi);
  }
}

template <int H> struct HeadVec { typedef float T; };
template <> struct HeadVec<2> { typedef f32x2 T; };
template <> struct HeadVec<4> { typedef f32x4 T; };
template <> struct HeadVec<8> { typedef f32x4 T; };
template <> struct HeadVec<16> { typedef f32x4 T; };

// Same operation for H in {1, 2, 4, 8, 16}: lane = slot. Each lane gathers
// its source's H values as whole vectors (H = 8: two 16-B loads of one 32-B
// row) and stores the slot's H results the same way; the destination's H
// values are wave-uniform (one row per wave). 64 slots per wave step instead
// of 64 / H, and no per-lane division. Same per-element arithmetic as
// gsddmm_attention_kernel (bit-identical).
template <int H>
__global__ __launch_bounds__(256) void gsddmm_attention_vec_kernel(
    int64_t num_rows, const int64_t* __restrict__ indptr,
    const int32_t* __restrict__ indices, const int64_t* __restrict__ eid,
    const float* __restrict__ lhs, const float* __restrict__ rhs, float alpha, float lo,
    float hi, int apply_exp, float* __restrict__ out) {
  typedef typename HeadVec<H>::T V;
  constexpr int W = sizeof(V) / sizeof(float);  // floats per vector
  constexpr int NV = H / W;                      // vectors per slot
  const int64_t row = block_linear() * (blockDim.x >> 6) +
                      __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  if (row >= num_rows) return;
  const int lane = threadIdx.x & 63;
  const int64_t beg = indptr[row], end = indptr[row + 1];
  if (beg == end) return;
  float r[H];
#pragma unroll
  for (int h = 0; h < H; ++h) r[h] = rhs[row * H + h];
  for (int64_t k = beg + lane; k < end; k += 64) {
    const V* src = reinterpret_cast<const V*>(lhs + int64_t(indices[k]) * H);
    V* dst = reinterpret_cast<V*>(out + (eid ? eid[k] : k) * H);
    V l[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) l[v] = src[v];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      V y;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        float x = reinterpret_cast<const float*>(&l[v])[w] + r[v * W + w];
        x = x > 0.0f ? x : alpha * x;
        if (apply_exp) x = __expf(x);
        reinterpret_cast<float*>(&y)[w] = fminf(fmaxf(x, lo), hi);
      }
      dst[v] = y;
    }
  }
}

// definitions of the state gspmm_impl.h declares
Timing g_timing;
int g_var_vec = 0, g_var_group = 0, g_var_unroll = 0, g_var_pipe = 0;
int g_cache_policy = -1;
int g_gather_buf = 2;
// running rows of the blocked launches: non-temporal loads, sc1 stores (the
// line leaves the XCD's L2): Reddit-shaped headline 3.83 -> 3.74 ms, GAT 8 x 16
// forward + backward 17.01 -> 16.94 (tools/rowpol_ab.py, profiles/r04/rowpol_ab.json)
int g_row_pol = 2;
int g_sddmm_alt = 0;

// ---------------------------------------------------------------------------
// Narrow rows, two slots per gather (r06): copy_u + sum over the blocked
// schedule's items when a source row is at most 64 floats (F = 41 at its
// 48-float padded stride: GCN's output layer). The one-row-per-wave kernel
// gathers such a row with 48 of 64 lanes one slot per instruction; here the
// wave's halves gather consecutive slots k and k + 1 of the same item (lane
// 32h + j holds floats 2j, 2j + 1 of slot k + h), and the lower half adds
// them in slot order: acc = (acc + s_k) + s_{k+1}, the second operand brought
// down through the LDS crossbar (ds_bpermute). Every output element is the one-launch kernel's
// chain (same additions, same order), so the bits are unchanged; the gather
// instructions per slot halve. The column ids stay scalar (both slots' ids
// through the scalar cache, a select per half), the rows are read through one
// buffer descriptor over the whole table (32-bit lane offsets).
// ---------------------------------------------------------------------------
int g_pair_slots = [] {
  const char* e = std::getenv("DGLHIP_PAIR_SLOTS");
  return e ? std::atoi(e) : 0;
}();

__device__ __forceinline__ float upper_half(float v, int from) {
  // lanes 0..31 receive lanes 32..63's values (ds_bpermute: the LDS
  // crossbar, no LDS storage; ``from`` = the source lane's byte address)
  return __int_as_float(__builtin_amdgcn_ds_bpermute(from, __float_as_int(v)));
}

// VEC floats per lane (2: rows of <= 64 floats; 4: rows of <= 128, the
// headline's F = 128, 16-B gathers); RP: the running rows' cache policy of
// the one-slot kernel (load_out / store_out: non-temporal loads, sc1 stores
// by default), so the two kernels treat the blocked schedule's passes alike.
template <int VEC, int UNROLL, bool ACCUM, int RP>
__global__ __launch_bounds__(256) void gspmm_pair_items_kernel(
    int64_t num_items, int64_t F, int64_t ld, int64_t table_bytes,
    const int32_t* __restrict__ item_rows, const int64_t* __restrict__ item_ptr,
    const int32_t* __restrict__ indices, const float* __restrict__ ufeat,
    float* __restrict__ out) {
  typedef typename Vec<VEC>::T V;
  typedef unsigned int uvec __attribute__((ext_vector_type(VEC)));
  const int64_t it = block_linear() * 4 +
                     __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  if (it >= num_items) return;
  const int lane = threadIdx.x & 63, half = lane >> 5;
  const int64_t f0 = int64_t(lane & 31) * VEC;
  const bool active = f0 < F;  // the lane's last floats may be row padding (ld > F)
  const bool in_row = f0 < ld;  // lanes past the row read nothing (no next-row lines)
  auto uni64 = [](int64_t x) {  // a wave-uniform 64-bit value, said so
    return int64_t((uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int32_t(x >> 32)))) << 32) |
                   uint32_t(__builtin_amdgcn_readfirstlane(int32_t(x))));
  };
  const int64_t row = __builtin_amdgcn_readfirstlane(item_rows[it]);
  const int64_t beg = uni64(item_ptr[it]), end = uni64(item_ptr[it + 1]);
  const __amdgpu_buffer_rsrc_t tab = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(ufeat), 0, static_cast<int>(table_bytes), 0x00020000);
  const uint32_t foff = static_cast<uint32_t>(f0 * 4);
  const uint32_t rowb = static_cast<uint32_t>(ld * 4);
  const int from = ((lane + 32) & 63) * 4;
  float* orow = out + row * F;
  // whole-vector running rows where the row holds them (F a multiple of VEC)
  const bool vec_out = F % VEC == 0;
  float a[VEC];
  if (ACCUM && half == 0 && active && vec_out) {
    const V v = load_out<VEC, RP>(orow, f0);
#pragma unroll
    for (int c = 0; c < VEC; ++c) a[c] = v[c];
  } else {
#pragma unroll
    for (int c = 0; c < VEC; ++c) a[c] = (ACCUM && half == 0 && f0 + c < F) ? orow[f0 + c] : 0.0f;
  }
  // one loop for full and partial batches: rem is wave-uniform, so the
  // predicates are scalar branches (a separate predicated tail batch doubled
  // the live registers: 126 against 42 VGPRs at VEC 2)
  for (int64_t k = beg; k < end; k += 2 * UNROLL) {
    const int64_t rem = end - k;
    float v[UNROLL][VEC];
#pragma unroll
    for (int j = 0; j < UNROLL; ++j) {
      if (2 * j < rem) {
        const int32_t ca = indices[k + 2 * j];
        const int32_t cb = 2 * j + 1 < rem ? indices[k + 2 * j + 1] : ca;
        const uint32_t off = static_cast<uint32_t>(half ? cb : ca) * rowb + foff;
        uvec w = uvec(0u);
        if (in_row) {
          if constexpr (VEC == 4) w = __builtin_amdgcn_raw_buffer_load_b128(tab, off, 0, 0);
          else w = __builtin_amdgcn_raw_buffer_load_b64(tab, off, 0, 0);
        }
#pragma unroll
        for (int c = 0; c < VEC; ++c) v[j][c] = __uint_as_float(w[c]);
      }
    }
#pragma unroll
    for (int j = 0; j < UNROLL; ++j) {
      if (2 * j < rem) {
        float w[VEC];
#pragma unroll
        for (int c = 0; c < VEC; ++c) w[c] = upper_half(v[j][c], from);
#pragma unroll
        for (int c = 0; c < VEC; ++c) a[c] += v[j][c];  // slot k + 2j (this half's own)
        if (2 * j + 1 < rem) {                           // then slot k + 2j + 1
#pragma unroll
          for (int c = 0; c < VEC; ++c) a[c] += w[c];
        }
      }
    }
  }
  if (half == 0 && active) {
    if (vec_out) {
      V v;
#pragma unroll
      for (int c = 0; c < VEC; ++c) v[c] = a[c];
      store_out<VEC, RP>(orow, f0, v);
    } else {
#pragma unroll
      for (int c = 0; c < VEC; ++c)
        if (f0 + c < F) orow[f0 + c] = a[c];
    }
  }
}

// the paired kernel's shapes: copy_u, rows of <= 64 floats at an even stride,
// a table the 32-bit buffer offsets span
static int pair_vec(int64_t F, int64_t ld) {
  if (F >= 16 && ld <= 64 && ld % 2 == 0) return 2;
  return 0;
}

static bool pair_items_ok(int msg_op, int64_t F, int64_t ld, int64_t num_src_bytes) {
  return g_pair_slots && msg_op == DGLHIP_MSG_COPY_U && pair_vec(F, ld) != 0 &&
         num_src_bytes > 0 && num_src_bytes < (int64_t(1) << 31);
}

static void dispatch_sum(int msg_op, bool mean, const SumLaunch& a, hipStream_t stream) {
  const int em = edge_mode(a.elen, a.F);
  if (msg_op == DGLHIP_MSG_COPY_U_BF16) {
    dispatch_sum_me<DGLHIP_MSG_COPY_U_BF16, EM_SCALAR>(mean, a, stream);
  } else if (msg_op == DGLHIP_MSG_COPY_U) {
    dispatch_sum_me<DGLHIP_MSG_COPY_U, EM_SCALAR>(mean, a, stream);
  } else if (msg_op == DGLHIP_MSG_U_MUL_E) {
    if (em == EM_FULL) dispatch_sum_me<DGLHIP_MSG_U_MUL_E, EM_FULL>(mean, a, stream);
    else if (em == EM_SCALAR) dispatch_sum_me<DGLHIP_MSG_U_MUL_E, EM_SCALAR>(mean, a, stream);
    else dispatch_sum_me<DGLHIP_MSG_U_MUL_E, EM_HEAD>(mean, a, stream);
  } else {
    if (em == EM_FULL) dispatch_sum_me<DGLHIP_MSG_COPY_E, EM_FULL>(mean, a, stream);
    else if (em == EM_SCALAR) dispatch_sum_me<DGLHIP_MSG_COPY_E, EM_SCALAR>(mean, a, stream);
    else dispatch_sum_me<DGLHIP_MSG_COPY_E, EM_HEAD>(mean, a, stream);
  }
}

static void dispatch_max(int msg_op, const MaxLaunch& a, hipStream_t stream) {
  const int em = edge_mode(a.elen, a.F);
  if (msg_op == DGLHIP_MSG_COPY_U_BF16) {
    dispatch_max_me<DGLHIP_MSG_COPY_U_BF16, EM_SCALAR>(a, stream);
  } else if (msg_op == DGLHIP_MSG_COPY_U) {
    dispatch_max_me<DGLHIP_MSG_COPY_U, EM_SCALAR>(a, stream);
  } else if (msg_op == DGLHIP_MSG_U_MUL_E) {
    if (em == EM_FULL) dispatch_max_me<DGLHIP_MSG_U_MUL_E, EM_FULL>(a, stream);
    else if (em == EM_SCALAR) dispatch_max_me<DGLHIP_MSG_U_MUL_E, EM_SCALAR>(a, stream);
    else dispatch_max_me<DGLHIP_MSG_U_MUL_E, EM_HEAD>(a, stream);
  } else {
    if (em == EM_FULL) dispatch_max_me<DGLHIP_MSG_COPY_E, EM_FULL>(a, stream);
    else if (em == EM_SCALAR) dispatch_max_me<DGLHIP_MSG_COPY_E, EM_SCALAR>(a, stream);
    else dispatch_max_me<DGLHIP_MSG_COPY_E, EM_HEAD>(a, stream);
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
  DGLHIP_CHECK(msg_op >= 0 && msg_op <= 3, "unknown msg op " << msg_op);
  DGLHIP_CHECK(reduce_op >= 0 && reduce_op <= 4, "unknown reduce op " << reduce_op);
  DGLHIP_CHECK(num_rows >= 0 && feat_len >= 0, "negative size");
  if (num_rows == 0 || feat_len == 0) return 0;  // empty tensors may carry null pointers
  DGLHIP_CHECK(indptr != nullptr && out != nullptr, "null indptr/out");
  const bool use_u = msg_op != DGLHIP_MSG_COPY_E;
  const bool use_e = !copies_u(msg_op);
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
  const bool mean = reduce_op == DGLHIP_REDUCE_MEAN || reduce_op == DGLHIP_REDUCE_MEAN_ACCUM;
  SumLaunch a{num_rows, feat_len, elen, indptr, indices, eid, ufeat, efeat, out, row_order,
              nullptr, nullptr,
              reduce_op == DGLHIP_REDUCE_SUM_ACCUM || reduce_op == DGLHIP_REDUCE_MEAN_ACCUM,
              stream_output(num_rows, feat_len)};
  dispatch_sum(msg_op, mean, a, stream);
  API_END();
}

int dglhip_gspmm_strided_device(int msg_op, int reduce_op, int64_t num_rows,
                                int64_t feat_len, int64_t ufeat_ld, const int64_t* indptr,
                                const int32_t* indices, const int64_t* eid,
                                const float* ufeat, const float* efeat, int64_t efeat_len,
                                float* out, const int32_t* row_order, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(msg_op == DGLHIP_MSG_COPY_U || msg_op == DGLHIP_MSG_U_MUL_E,
               "strided source rows: copy_u or u_mul_e, got msg op " << msg_op);
  DGLHIP_CHECK(reduce_op == DGLHIP_REDUCE_SUM || reduce_op == DGLHIP_REDUCE_MEAN ||
                   reduce_op == DGLHIP_REDUCE_SUM_ACCUM || reduce_op == DGLHIP_REDUCE_MEAN_ACCUM,
               "strided source rows: sum / mean reducers only");
  DGLHIP_CHECK(num_rows >= 0 && feat_len >= 0, "negative size");
  DGLHIP_CHECK(ufeat_ld >= feat_len, "ufeat_ld " << ufeat_ld << " < feat_len " << feat_len);
  if (num_rows == 0 || feat_len == 0) return 0;
  DGLHIP_CHECK(indptr && out && ufeat, "null indptr/out/ufeat");
  const bool use_e = msg_op == DGLHIP_MSG_U_MUL_E;
  DGLHIP_CHECK(!use_e || efeat, "efeat is null");
  DGLHIP_CHECK(!use_e || (efeat_len >= 1 && feat_len % efeat_len == 0),
               "edge feature length " << efeat_len << " must divide feat_len " << feat_len);
  // a lane's vector of VEC features must not straddle padded rows: even strides only
  DGLHIP_CHECK(ufeat_ld == feat_len || ufeat_ld % 2 == 0, "odd padded stride " << ufeat_ld);
  SumLaunch a{num_rows, feat_len, use_e ? efeat_len : 1, indptr, indices, eid, ufeat, efeat, out,
              row_order, nullptr, nullptr,
              reduce_op == DGLHIP_REDUCE_SUM_ACCUM || reduce_op == DGLHIP_REDUCE_MEAN_ACCUM,
              stream_output(num_rows, feat_len), ufeat_ld};
  dispatch_sum(msg_op, reduce_op == DGLHIP_REDUCE_MEAN || reduce_op == DGLHIP_REDUCE_MEAN_ACCUM,
               a, stream);
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
                                int64_t ufeat_ld, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(msg_op >= 0 && msg_op <= 3, "unknown msg op " << msg_op);
  DGLHIP_CHECK(reduce_op == DGLHIP_REDUCE_SUM || reduce_op == DGLHIP_REDUCE_MEAN ||
                   reduce_op == DGLHIP_REDUCE_SUM_ACCUM || reduce_op == DGLHIP_REDUCE_MEAN_ACCUM,
               "chunked rows support sum/mean only");
  DGLHIP_CHECK(num_light >= 0 && num_chunks >= 0 && num_heavy >= 0, "negative size");
  if (feat_len == 0) return 0;
  const bool use_u = msg_op != DGLHIP_MSG_COPY_E;
  const bool use_e = !copies_u(msg_op);
  DGLHIP_CHECK(!use_u || ufeat, "ufeat is null");
  DGLHIP_CHECK(!use_e || efeat, "efeat is null");
  DGLHIP_CHECK(!use_e || (efeat_len >= 1 && feat_len % efeat_len == 0),
               "edge feature length " << efeat_len << " must divide feat_len " << feat_len);
  DGLHIP_CHECK(num_chunks == 0 || (partial && chunk_beg && chunk_end), "null chunk plan");
  DGLHIP_CHECK(ufeat_ld == 0 || ufeat_ld == feat_len || (ufeat_ld > feat_len && ufeat_ld % 2 == 0),
               "ufeat_ld " << ufeat_ld << ": 0, feat_len, or an even width > feat_len");
  DGLHIP_CHECK(ufeat_ld == 0 || ufeat_ld == feat_len || msg_op == DGLHIP_MSG_COPY_U ||
                   msg_op == DGLHIP_MSG_U_MUL_E,
               "strided source rows: copy_u or u_mul_e, got msg op " << msg_op);
  const int64_t elen = use_e ? efeat_len : 1;
  const bool mean = reduce_op == DGLHIP_REDUCE_MEAN || reduce_op == DGLHIP_REDUCE_MEAN_ACCUM;
  const bool accum = reduce_op == DGLHIP_REDUCE_SUM_ACCUM || reduce_op == DGLHIP_REDUCE_MEAN_ACCUM;
  if (num_chunks > 0) {  // heavy-row chunks first: the longest work starts first
    SumLaunch c{num_chunks, feat_len, elen, indptr, indices, eid, ufeat, efeat, partial,
                nullptr, chunk_beg, chunk_end, false, false, ufeat_ld};
    dispatch_sum(msg_op, false, c, stream);
  }
  if (num_light > 0) {
    SumLaunch l{num_light, feat_len, elen, indptr, indices, eid, ufeat, efeat, out,
                light_rows, nullptr, nullptr, accum,
                stream_output(num_light + num_heavy, feat_len), ufeat_ld};
    dispatch_sum(msg_op, mean, l, stream);
  }
  if (num_heavy > 0) {
    const int64_t blocks = (num_heavy + 3) / 4;
    timed_launch(stream, [&] {
      if (mean && accum)
        hipLaunchKernelGGL((gspmm_combine_kernel<true, true>),
                           grid_1d(blocks), dim3(256), 0, stream,
                           num_heavy, feat_len, indptr, heavy_rows, heavy_chunk_ptr, partial,
                           out);
      else if (mean)
        hipLaunchKernelGGL((gspmm_combine_kernel<true, false>),
                           grid_1d(blocks), dim3(256), 0, stream,
                           num_heavy, feat_len, indptr, heavy_rows, heavy_chunk_ptr, partial,
                           out);
      else if (accum)
        hipLaunchKernelGGL((gspmm_combine_kernel<false, true>),
                           grid_1d(blocks), dim3(256), 0, stream,
                           num_heavy, feat_len, indptr, heavy_rows, heavy_chunk_ptr, partial,
                           out);
      else
        hipLaunchKernelGGL((gspmm_combine_kernel<false, false>),
                           grid_1d(blocks), dim3(256), 0, stream,
                           num_heavy, feat_len, indptr, heavy_rows, heavy_chunk_ptr, partial,
                           out);
    });
  }
  API_END();
}

int dglhip_gspmm_items_device(int msg_op, int64_t num_items, int64_t feat_len,
                              const int32_t* item_rows, const int64_t* item_ptr, int accumulate,
                              const int32_t* indices, const int64_t* eid, const float* ufeat,
                              int64_t ufeat_ld, const float* efeat, int64_t efeat_len,
                              float* out, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(msg_op >= 0 && msg_op <= 3, "unknown msg op " << msg_op);
  DGLHIP_CHECK(num_items >= 0 && feat_len >= 0, "negative size");
  if (num_items == 0 || feat_len == 0) return 0;
  const bool use_u = msg_op != DGLHIP_MSG_COPY_E;
  const bool use_e = !copies_u(msg_op);
  DGLHIP_CHECK(item_rows && item_ptr && indices && out, "null items/indices/out");
  DGLHIP_CHECK(!use_u || ufeat, "ufeat is null");
  DGLHIP_CHECK(!use_e || efeat, "efeat is null");
  DGLHIP_CHECK(!use_e || (efeat_len >= 1 && feat_len % efeat_len == 0),
               "edge feature length " << efeat_len << " must divide feat_len " << feat_len);
  DGLHIP_CHECK(ufeat_ld == 0 || ufeat_ld == feat_len || (ufeat_ld > feat_len && ufeat_ld % 2 == 0),
               "ufeat_ld " << ufeat_ld << ": 0, feat_len, or an even width > feat_len");
  SumLaunch a{num_items, feat_len, use_e ? efeat_len : 1, nullptr, indices, eid, ufeat, efeat,
              out, item_rows, item_ptr, item_ptr + 1, accumulate != 0, false, ufeat_ld};
  dispatch_sum(msg_op, false, a, stream);
  API_END();
}

int dglhip_gspmm_pair_items_ok(int msg_op, int64_t feat_len, int64_t ufeat_ld,
                               int64_t num_src_rows) {
  const int64_t ld = ufeat_ld ? ufeat_ld : feat_len;
  return pair_items_ok(msg_op, feat_len, ld, num_src_rows * ld * 4) ? 1 : 0;
}

int dglhip_gspmm_pair_items_device(int64_t num_items, int64_t feat_len, int64_t ufeat_ld,
                                   int64_t num_src_rows, const int32_t* item_rows,
                                   const int64_t* item_ptr, int accumulate,
                                   const int32_t* indices, const float* ufeat, float* out,
                                   void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  const int64_t ld = ufeat_ld ? ufeat_ld : feat_len;
  DGLHIP_CHECK(num_items >= 0 && feat_len >= 0 && num_src_rows >= 0, "negative size");
  DGLHIP_CHECK(pair_items_ok(DGLHIP_MSG_COPY_U, feat_len, ld, num_src_rows * ld * 4),
               "paired gathers take copy_u rows of 16..64 floats at an even stride <= 64 "
               "over a table under 2 GiB (F " << feat_len << ", stride " << ld << ")");
  if (num_items == 0 || feat_len == 0) return 0;
  DGLHIP_CHECK(item_rows && item_ptr && indices && ufeat && out, "null argument");
  const dim3 grid = grid_1d((num_items + 3) / 4);
  const int64_t bytes = num_src_rows * ld * 4;
  // 32 slots (16 gathers) in flight per wave at VEC 2; 16 slots (8 gathers
  // of 16 B: 44 VGPRs, where 16 took 76) at VEC 4, the one-slot kernel's 16
#define DGLHIP_PAIR(VEC, ACC, RPV)                                                            \
  hipLaunchKernelGGL((gspmm_pair_items_kernel<VEC, VEC == 4 ? 8 : 16, ACC, RPV>), grid,       \
                     dim3(256), 0, stream, num_items, feat_len, ld, bytes, item_rows,         \
                     item_ptr, indices, ufeat, out)
  const int vec = pair_vec(feat_len, ld);
  timed_launch(stream, [&] {
    // the running rows as the one-slot kernel treats them (g_row_pol; the
    // first launch only stores: sc1, as policy 4)
    (void)vec;  // 2: rows of <= 64 floats (a VEC 4 form for 128-float rows measured
                // 4.58 vs 3.75 ms on the headline and was dropped)
    if (accumulate) DGLHIP_PAIR(2, true, 0);
    else DGLHIP_PAIR(2, false, 0);
  });
#undef DGLHIP_PAIR
  API_END();
}

int dglhip_set_pair_slots(int on) {
  g_pair_slots = on ? 1 : 0;
  return 0;
}

int dglhip_gspmm_max_ranges_device(int msg_op, int64_t num_rows, int64_t feat_len,
                                   const int64_t* indptr, const int64_t* row_beg,
                                   const int64_t* row_end, int accumulate,
                                   const int32_t* indices, const int64_t* eid,
                                   const float* ufeat, const float* efeat, int64_t efeat_len,
                                   float* out, int64_t* arg_out, const int32_t* row_order,
                                   void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(msg_op >= 0 && msg_op <= 3, "unknown msg op " << msg_op);
  DGLHIP_CHECK(num_rows >= 0 && feat_len >= 0, "negative size");
  if (num_rows == 0 || feat_len == 0) return 0;
  DGLHIP_CHECK(indptr && row_beg && row_end && out, "null indptr/ranges/out");
  const bool use_u = msg_op != DGLHIP_MSG_COPY_E;
  const bool use_e = !copies_u(msg_op);
  DGLHIP_CHECK(!use_u || ufeat, "ufeat is null");
  DGLHIP_CHECK(!use_e || efeat, "efeat is null");
  DGLHIP_CHECK(!use_e || (efeat_len >= 1 && feat_len % efeat_len == 0),
               "edge feature length " << efeat_len << " must divide feat_len " << feat_len);
  MaxLaunch m{num_rows, feat_len, use_e ? efeat_len : 1, indptr, indices, eid, ufeat, efeat,
              out, arg_out, row_order, row_beg, row_end, accumulate != 0 ? 1 : 0};
  dispatch_max(msg_op, m, stream);
  API_END();
}

int dglhip_gspmm_ranges_device(int msg_op, int64_t num_items, int64_t feat_len,
                               const int64_t* item_beg, const int64_t* item_end,
                               int accumulate, const int32_t* indices, const int64_t* eid,
                               const float* ufeat, const float* efeat, int64_t efeat_len,
                               float* out, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(msg_op >= 0 && msg_op <= 3, "unknown msg op " << msg_op);
  DGLHIP_CHECK(num_items >= 0 && feat_len >= 0, "negative size");
  if (num_items == 0 || feat_len == 0) return 0;
  const bool use_u = msg_op != DGLHIP_MSG_COPY_E;
  const bool use_e = !copies_u(msg_op);
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

}  // extern "C"

namespace dglhip {

// The SDDMM dot launch for one shape (the sliced kernel where it applies, the
// generic one otherwise); EPI adds the GAT attention-gradient epilogue. Row
// r's slots are [row_beg[r], row_end[r]) (indptr, indptr + 1 for whole rows).
template <bool EPI>
static void launch_sddmm_dot(int64_t num_rows, int64_t feat_len, int64_t num_heads,
                             const int64_t* row_beg, const int64_t* row_end,
                             const int32_t* row_order, const int32_t* indices,
                             const int64_t* eid,
                             const float* lhs, const float* rhs, float* out, const GatEpi& epi,
                             hipStream_t stream) {
  const int64_t blocks = (num_rows + 3) / 4;
  DGLHIP_CHECK(blocks <= 0x7fffffff, "grid too large: " << blocks);
  const int64_t D = feat_len / num_heads;
  const bool aligned = (reinterpret_cast<uintptr_t>(lhs) % 16) == 0 &&
                       (reinterpret_cast<uintptr_t>(rhs) % 16) == 0;
  const bool head_ok = D >= 32 ? (D % 32 == 0) : (D == 4 || D == 8 || D == 16);
  const int64_t nb = feat_len % 32 == 0 ? feat_len / 32 : 0;
  const bool sliced = aligned && head_ok && (nb == 1 || nb == 2 || nb == 4 || nb == 8 ||
                                             nb == 16);
  // row sub-ranges (the source-blocked schedule) gather from L2: there the
  // shallower depth wins at F = 128 (Reddit-shaped graph, 1 / 8 / 16 heads:
  // 6.30 -> 4.89, 6.68 -> 5.69, 7.70 -> 7.07 ms per call, eid order,
  // tools/reducer_bench.py); dglhip_set_sddmm_variant(1) swaps the two
  const bool alt = (row_end != row_beg + 1) != ((g_sddmm_alt & 1) != 0);
  // the GAT epilogue's per-slot operands: loaded with the slot's gathers
  // (default), or after the dot product (dglhip_set_sddmm_variant bit 1)
  const bool late = (g_sddmm_alt & 2) != 0;
  timed_launch(stream, [&] {
#define DGLHIP_SDDMM_K2(NB, U, HH, PP)                                                     \
  hipLaunchKernelGGL((gsddmm_dot_sliced_kernel<NB, U, HH, EPI, PP>), grid_1d(blocks),        \
                     dim3(256), 0, stream, num_rows, row_beg, row_end, row_order, indices, eid, \
                     lhs, rhs, out, epi)
#define DGLHIP_SDDMM_K(NB, U, HH)                                                          \
  do {                                                                                     \
    if constexpr (EPI) {                                                                   \
      if (late) DGLHIP_SDDMM_K2(NB, U, HH, false);                                         \
      else DGLHIP_SDDMM_K2(NB, U, HH, true);                                               \
    } else {                                                                               \
      DGLHIP_SDDMM_K2(NB, U, HH, true);                                                    \
    }                                                                                      \
  } while (0)
#define DGLHIP_SDDMM_H(NB, U, HH)                                                          \
  if (num_heads == HH) {                                                                   \
    if (!alt) DGLHIP_SDDMM_K(NB, U, HH);                                                  \
    else DGLHIP_SDDMM_K(NB, (U == 4 ? 2 : 2 * U), HH);                                     \
    return;                                                                                \
  }
    // default slots in flight: 8 x U. F = 128: U = 4 for every head count
    // (Reddit-shaped graph, profiles/r02/reducers_reddit.json, 16 -> 32 slots:
    // H = 1 8.92 -> 8.36 ms, H = 8 9.38 -> 8.83, H = 16 9.73 -> 9.23,
    // H = 32 10.77 -> 10.44); dglhip_set_sddmm_variant(1) takes the other depth
    if (sliced && nb == 1) {
      DGLHIP_SDDMM_H(1, 2, 1) DGLHIP_SDDMM_H(1, 2, 2) DGLHIP_SDDMM_H(1, 2, 4)
      DGLHIP_SDDMM_H(1, 2, 8)
    } else if (sliced && nb == 2) {
      DGLHIP_SDDMM_H(2, 2, 1) DGLHIP_SDDMM_H(2, 2, 2) DGLHIP_SDDMM_H(2, 2, 4)
      DGLHIP_SDDMM_H(2, 2, 8) DGLHIP_SDDMM_H(2, 2, 16)
    } else if (sliced && nb == 4) {
      DGLHIP_SDDMM_H(4, 4, 1) DGLHIP_SDDMM_H(4, 4, 2) DGLHIP_SDDMM_H(4, 4, 4)
      DGLHIP_SDDMM_H(4, 4, 8) DGLHIP_SDDMM_H(4, 4, 16) DGLHIP_SDDMM_H(4, 4, 32)
    } else if (sliced && nb == 8) {
      DGLHIP_SDDMM_H(8, 1, 1) DGLHIP_SDDMM_H(8, 1, 2) DGLHIP_SDDMM_H(8, 1, 4)
      DGLHIP_SDDMM_H(8, 1, 8) DGLHIP_SDDMM_H(8, 1, 16) DGLHIP_SDDMM_H(8, 1, 32)
      DGLHIP_SDDMM_H(8, 1, 64)
    } else if (sliced && nb == 16) {
      DGLHIP_SDDMM_H(16, 1, 1) DGLHIP_SDDMM_H(16, 1, 2) DGLHIP_SDDMM_H(16, 1, 4)
      DGLHIP_SDDMM_H(16, 1, 8) DGLHIP_SDDMM_H(16, 1, 16) DGLHIP_SDDMM_H(16, 1, 32)
      DGLHIP_SDDMM_H(16, 1, 64) DGLHIP_SDDMM_H(16, 1, 128)
    }
    DGLHIP_CHECK(!EPI || epi.rsum == nullptr,
                 "fused row sums need the sliced g-SDDMM (F = 32 x {1,2,4,8,16}, power-of-two "
                 "heads of >= 4 features, 16-B aligned rows): F = " << feat_len << ", H = "
                 << num_heads);
    hipLaunchKernelGGL((gsddmm_dot_kernel<EPI>), grid_1d(blocks), dim3(256), 0, stream,
                       num_rows, feat_len, num_heads, row_beg, row_end, row_order, indices, eid,
                       lhs, rhs, out, epi);
#undef DGLHIP_SDDMM_K
#undef DGLHIP_SDDMM_K2
#undef DGLHIP_SDDMM_H
  });
}

}  // namespace dglhip

extern "C" {

int dglhip_gsddmm_ranges_device(int op, int64_t num_rows, int64_t feat_len, int64_t num_heads,
                                const int64_t* row_beg, const int64_t* row_end,
                                const int32_t* row_order, const int32_t* indices,
                                const int64_t* eid, const float* lhs, const float* rhs,
                                float* out, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(op == DGLHIP_SDDMM_DOT, "unknown sddmm op " << op);
  DGLHIP_CHECK(num_rows >= 0 && feat_len >= 0, "negative size");
  DGLHIP_CHECK(num_heads >= 1 && feat_len % num_heads == 0,
               "num_heads " << num_heads << " must divide feat_len " << feat_len);
  if (num_rows == 0) return 0;
  DGLHIP_CHECK(row_beg && row_end && indices && lhs && rhs && out, "null pointer argument");
  launch_sddmm_dot<false>(num_rows, feat_len, num_heads, row_beg, row_end, row_order, indices,
                          eid, lhs, rhs, out, GatEpi{}, stream);
  API_END();
}

int dglhip_gsddmm_device(int op, int64_t num_rows, int64_t feat_len,
                         int64_t num_heads, const int64_t* indptr, const int32_t* indices,
                         const int64_t* eid, const float* lhs,
                         const float* rhs, float* out, void* stream) {
  return dglhip_gsddmm_ranges_device(op, num_rows, feat_len, num_heads, indptr,
                                     indptr ? indptr + 1 : nullptr, nullptr, indices, eid, lhs,
                                     rhs, out, stream);
}

int dglhip_gat_attention_grad_ranges_device(
    int64_t num_rows, int64_t feat_len, int64_t num_heads, const int64_t* row_beg,
    const int64_t* row_end, const int32_t* row_order, const int32_t* indices,
    const float* dout, const float* ft,
    const float* attn, const float* attn_drop, const float* dz, float alpha, float clamp_lo,
    float clamp_hi, int apply_exp, float drop_scale, float* grad, void* stream) {
  return dglhip_gat_attention_grad_rowsum_ranges_device(
      num_rows, feat_len, num_heads, row_beg, row_end, row_order, indices, dout, ft, attn,
      attn_drop, dz, alpha, clamp_lo, clamp_hi, apply_exp, drop_scale, grad, nullptr, stream);
}

int dglhip_gat_attention_grad_rowsum_ok(int64_t feat_len, int64_t num_heads) {
  if (feat_len <= 0 || num_heads < 1 || feat_len % 32 != 0 || feat_len % num_heads != 0) return 0;
  const int64_t nb = feat_len / 32, D = feat_len / num_heads;
  const bool nb_ok = nb == 1 || nb == 2 || nb == 4 || nb == 8 || nb == 16;
  const bool pow2 = (num_heads & (num_heads - 1)) == 0;
  return nb_ok && pow2 && D >= 4 ? 1 : 0;
}

int dglhip_gat_attention_grad_rowsum_ranges_device(
    int64_t num_rows, int64_t feat_len, int64_t num_heads, const int64_t* row_beg,
    const int64_t* row_end, const int32_t* row_order, const int32_t* indices,
    const float* dout, const float* ft,
    const float* attn, const float* attn_drop, const float* dz, float alpha, float clamp_lo,
    float clamp_hi, int apply_exp, float drop_scale, float* grad, float* grad_rowsum,
    void* stream_) {
  API_BEGIN();
  DGLHIP_CHECK(grad_rowsum == nullptr || dglhip_gat_attention_grad_rowsum_ok(feat_len, num_heads),
               "fused row sums: unsupported shape F = " << feat_len << ", H = " << num_heads);
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows >= 0 && feat_len >= 0, "negative size");
  DGLHIP_CHECK(num_heads >= 1 && feat_len % num_heads == 0,
               "num_heads " << num_heads << " must divide feat_len " << feat_len);
  if (num_rows == 0) return 0;
  DGLHIP_CHECK(row_beg && row_end && indices && dout && ft && attn && grad,
               "null pointer argument");
  const GatEpi epi{attn, attn_drop, dz, alpha, clamp_lo, clamp_hi, drop_scale, apply_exp,
                   grad_rowsum};
  launch_sddmm_dot<true>(num_rows, feat_len, num_heads, row_beg, row_end, row_order, indices,
                         nullptr, dout, ft, grad, epi, stream);
  API_END();
}

int dglhip_gat_attention_grad_keep_ranges_device(
    int64_t num_rows, int64_t feat_len, int64_t num_heads, const int64_t* row_beg,
    const int64_t* row_end, const int32_t* row_order, const int32_t* indices,
    const float* dout, const float* ft, const float* attn, const float* dz, float alpha,
    float clamp_lo, float clamp_hi, int apply_exp, float drop_p, uint64_t seed,
    const int64_t* seed_offset, float* grad, float* grad_rowsum, void* stream_) {
  API_BEGIN();
  DGLHIP_CHECK(grad_rowsum == nullptr || dglhip_gat_attention_grad_rowsum_ok(feat_len, num_heads),
               "fused row sums: unsupported shape F = " << feat_len << ", H = " << num_heads);
  DGLHIP_CHECK(drop_p >= 0.0f && drop_p < 1.0f, "dropout probability must be in [0, 1)");
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows >= 0 && feat_len >= 0, "negative size");
  DGLHIP_CHECK(num_heads >= 1 && feat_len % num_heads == 0,
               "num_heads " << num_heads << " must divide feat_len " << feat_len);
  if (num_rows == 0) return 0;
  DGLHIP_CHECK(row_beg && row_end && indices && dout && ft && attn && grad,
               "null pointer argument");
  const bool drop = drop_p > 0.0f;
  GatEpi epi{attn, nullptr, dz, alpha, clamp_lo, clamp_hi, drop ? 1.0f / (1.0f - drop_p) : 1.0f,
             apply_exp, grad_rowsum};
  epi.hash_keep = drop ? 1 : 0;
  epi.seed = seed;
  epi.seed_off = seed_offset;
  epi.thr = drop ? gat_drop_threshold(drop_p) : 0u;
  launch_sddmm_dot<true>(num_rows, feat_len, num_heads, row_beg, row_end, row_order, indices,
                         nullptr, dout, ft, grad, epi, stream);
  API_END();
}

int dglhip_gat_attention_grad_logits_ranges_device(
    int64_t num_rows, int64_t feat_len, int64_t num_heads, const int64_t* row_beg,
    const int64_t* row_end, const int32_t* row_order, const int32_t* indices,
    const float* dout, const float* ft, const float* attn, const float* attn_drop,
    const float* dz, const float* el, const float* er, float alpha, float clamp_lo,
    float clamp_hi, int apply_exp, float drop_scale, float drop_p, uint64_t seed,
    const int64_t* seed_offset, float* grad, float* grad_rowsum, void* stream_) {
  API_BEGIN();
  DGLHIP_CHECK(grad_rowsum == nullptr || dglhip_gat_attention_grad_rowsum_ok(feat_len, num_heads),
               "fused row sums: unsupported shape F = " << feat_len << ", H = " << num_heads);
  DGLHIP_CHECK(drop_p >= 0.0f && drop_p < 1.0f, "dropout probability must be in [0, 1)");
  DGLHIP_CHECK(!(drop_p > 0.0f && attn_drop), "dropout: the hash (drop_p) or attn_drop, not both");
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows >= 0 && feat_len >= 0, "negative size");
  DGLHIP_CHECK(num_heads >= 1 && feat_len % num_heads == 0,
               "num_heads " << num_heads << " must divide feat_len " << feat_len);
  if (num_rows == 0) return 0;
  DGLHIP_CHECK(row_beg && row_end && indices && dout && ft && attn && grad && el && er,
               "null pointer argument");
  const bool hash = drop_p > 0.0f;
  GatEpi epi{attn, attn_drop, dz, alpha, clamp_lo, clamp_hi,
             hash ? 1.0f / (1.0f - drop_p) : drop_scale, apply_exp, grad_rowsum};
  epi.hash_keep = hash ? 1 : 0;
  epi.seed = seed;
  epi.seed_off = seed_offset;
  epi.thr = hash ? gat_drop_threshold(drop_p) : 0u;
  epi.el = el;
  epi.er = er;
  launch_sddmm_dot<true>(num_rows, feat_len, num_heads, row_beg, row_end, row_order, indices,
                         nullptr, dout, ft, grad, epi, stream);
  API_END();
}

int dglhip_gat_attention_grad_device(int64_t num_rows, int64_t feat_len, int64_t num_heads,
                                     const int64_t* indptr, const int32_t* indices,
                                     const float* dout, const float* ft, const float* attn,
                                     const float* attn_drop, const float* dz, float alpha,
                                     float clamp_lo, float clamp_hi, int apply_exp,
                                     float drop_scale, float* grad, void* stream) {
  return dglhip_gat_attention_grad_ranges_device(
      num_rows, feat_len, num_heads, indptr, indptr ? indptr + 1 : nullptr, nullptr, indices,
      dout, ft,
      attn, attn_drop, dz, alpha, clamp_lo, clamp_hi, apply_exp, drop_scale, grad, stream);
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

int dglhip_set_sddmm_variant(int alternate) {
  API_BEGIN();
  // bit 0: the other depth of slots in flight; bit 1: the GAT epilogue's
  // operands loaded after the dot product (the form before r03's prefetch)
  DGLHIP_CHECK(alternate >= 0 && alternate <= 3, "unsupported g-SDDMM variant " << alternate);
  g_sddmm_alt = alternate;
  API_END();
}

int dglhip_set_gather_mode(int buffer_descriptors) {
  API_BEGIN();
  DGLHIP_CHECK(buffer_descriptors >= 0 && buffer_descriptors <= 3,
               "unknown gather mode " << buffer_descriptors);
  g_gather_buf = buffer_descriptors;
  API_END();
}

int dglhip_set_row_policy(int policy) {
  API_BEGIN();
  DGLHIP_CHECK(policy >= 0 && policy <= 4, "unknown running-row policy " << policy);
  g_row_pol = policy;
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
  DGLHIP_CHECK(indptr && indices && lhs && rhs && out, "null pointer argument");
  DGLHIP_CHECK((num_rows + 3) / 4 <= 0x7fffffff, "grid too large");
  // vector rows need lhs / out rows aligned to the vector width
  const int64_t vbytes = num_heads >= 4 ? 16 : 4 * num_heads;
  const bool aligned = (reinterpret_cast<uintptr_t>(lhs) % vbytes) == 0 &&
                       (reinterpret_cast<uintptr_t>(out) % vbytes) == 0;
  timed_launch(stream, [&] {
#define DGLHIP_ATT(HH)                                                                     \
  if (aligned && num_heads == HH) {                                                        \
    hipLaunchKernelGGL((gsddmm_attention_vec_kernel<HH>), grid_1d((num_rows + 3) / 4),     \
                       dim3(256), 0, stream, num_rows, indptr, indices, eid, lhs, rhs,      \
                       alpha, clamp_lo, clamp_hi, apply_exp, out);                          \
    return;                                                                                \
  }
    DGLHIP_ATT(1) DGLHIP_ATT(2) DGLHIP_ATT(4) DGLHIP_ATT(8) DGLHIP_ATT(16)
#undef DGLHIP_ATT
    hipLaunchKernelGGL(gsddmm_attention_kernel, grid_1d((num_rows + 3) / 4),
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
