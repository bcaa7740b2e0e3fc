// Fused GAT layer aggregation for gfx950: attention, attention dropout,
// normaliser and head-broadcast aggregation in one pass over the CSR.
//
// The reference's GAT layer (examples/pytorch/gat/train.py:74-96) runs it as
//   apply_edges(edge_attention)   a = clamp(exp(leaky_relu(a1[u] + a2[v])))
//   attn_drop                     a_drop = dropout(a)
//   update_all([src_mul_edge(ft, a_drop), copy_edge(a)], [sum -> ft, sum -> z])
// i.e. an E x H attention tensor written, then read by an incidence SPMV over
// E x H x D materialised messages and again by the normaliser's. Here one wave
// owns one destination row v and, slot by slot in CSR order (u = indices[k]):
//   a[k, h]            = clamp(exp(leaky_relu(el[u, h] + er[v, h], alpha)), lo, hi)
//   w[k, h]            = keep(k, h) ? a[k, h] * scale : 0     (dropout; else a)
//   ft_out[v, hD + d]  = fma chain over k of w[k, h] * ft[u, hD + d]
//   z[v, h]            = add chain over k of a[k, h]
// The per-edge expression is gsddmm_attention_vec_kernel's and the two chains
// are gspmm_sum_kernel's (u_mul_e with per-head weights, copy_e), in the same
// slot order, so the outputs equal the three-kernel path's bit for bit. The
// E x H attention (and its dropped copy) are written, in CSR slot order, only
// when the caller passes buffers for them (autograd needs them); the gathered
// el row of a slot is one 4-B load per lane, shared by the D lanes of a head.
//
// Lane map: VEC consecutive features per lane (VEC divides D), a 64-lane pass
// covers 64 * VEC features; the first lane of each head in a pass keeps and
// stores that head's z and attention values. UNROLL slots are in flight.
//
// Row ranges: a row's slots are [row_beg[row], row_end[row]) of the CSR
// (row_beg = indptr, row_end = indptr + 1 for the whole row). The
// source-blocked schedule (kernel.py _block_cuts) runs one launch per source
// block over the sub-range of each row whose sources lie in it, with
// ``accumulate`` continuing both chains from out_ft / out_z: when the blocks
// never decrease along a row's slots this is the row's own chain, and slot
// indices (dropout hash, attention positions) stay the CSR's.
//
// Dropout mask: keep(k, h) = hash(seed, k * H + h) >= threshold, a stateless
// counter hash (gat_keep, gspmm_impl.h: host and device), so the backward and the host
// path reproduce it from (seed, slot, head) alone.

#include <type_traits>

#include "gspmm_impl.h"

namespace dglhip {

// study knob (dglhip_set_gat_variant): 0 automatic, 1 the per-lane kernel,
// 2 the LDS-shared attention kernel (head counts 1, 2, 4, 8, 16) with each
// batch's feature rows gathered after its attention, 3 the same kernel with
// them gathered before it
int g_gat_variant = 0;
int g_gat_fwd_waves = 0;  // study knob: minimum waves per SIMD of the 8 x 16 forward (0, 5, 6)
// study knob of the transposed backward (dglhip_set_gat_bwd_variant): bits 0-1
// the g store (0 default, 1 non-temporal, 2 none: d_er is then not valid,
// 3 16-B write-through stores regrouped through LDS);
// bit 2 the kernel built for 5 waves per SIMD (96 VGPRs) instead of 4 (97)
int g_gat_bwd_variant = 0;
// study knob (dglhip_set_gat_logit_recompute): 1 lets
// dglhip_gat_aggregate_logits_ranges_device recompute the sources' logits
// from their gathered rows. Off by default: on the Reddit-shaped 8 x 16 layer
// the forward ran 5.93 ms against 5.12 with the logits gathered (r05) — the
// attention then waits for the rows instead of being computed while they
// are in flight, which costs more than the fifth line per slot saves.
int g_gat_logit_on = 0;

// One row of VEC floats per lane through a buffer descriptor built from the
// wave-uniform row address: a 32-bit per-lane byte offset instead of a 64-bit
// address per gather (16 gathers in flight share one offset register).
template <int VEC>
__device__ __forceinline__ typename Vec<VEC>::T gather_rsrc(const float* row, int64_t F,
                                                            uint32_t voff) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(row), 0, static_cast<int>(F * sizeof(float)), 0x00020000);
  if (VEC == 2) {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 w = __builtin_amdgcn_raw_buffer_load_b64(r, voff, 0, 0);
    return *reinterpret_cast<const typename Vec<VEC>::T*>(&w);
  }
  const unsigned int w = __builtin_amdgcn_raw_buffer_load_b32(r, voff, 0, 0);
  return *reinterpret_cast<const typename Vec<VEC>::T*>(&w);
}

// Tables under 2 GB: one descriptor over the whole table, the row's byte
// offset as the (wave-uniform, SGPR) soffset and the lane's as voffset: no
// per-gather descriptor (4 SGPRs each, 16 in flight) and no per-gather VGPR.
struct GatTable {
  __amdgpu_buffer_rsrc_t r;
};

__device__ __forceinline__ GatTable gat_table(const float* ft, int64_t bytes) {
  return GatTable{__builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ft), 0,
                                                    static_cast<int>(bytes), 0x00020000)};
}

template <int VEC>
__device__ __forceinline__ typename Vec<VEC>::T gather_soff(const GatTable& t, int64_t src,
                                                            int64_t F, uint32_t voff) {
  const uint32_t soff = static_cast<uint32_t>(src * F * int64_t(sizeof(float)));
  if (VEC == 2) {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 w = __builtin_amdgcn_raw_buffer_load_b64(t.r, voff, soff, 0);
    return *reinterpret_cast<const typename Vec<VEC>::T*>(&w);
  }
  const unsigned int w = __builtin_amdgcn_raw_buffer_load_b32(t.r, voff, soff, 0);
  return *reinterpret_cast<const typename Vec<VEC>::T*>(&w);
}

template <int VEC, bool SMALL>
__device__ __forceinline__ typename Vec<VEC>::T gat_gather(const float* ft, const GatTable& t,
                                                           int64_t src, int64_t F,
                                                           uint32_t voff) {
  if (SMALL) return gather_soff<VEC>(t, src, F, voff);
  return gather_rsrc<VEC>(ft + src * F, F, voff);
}

template <int VEC, int UNROLL, bool DROP, bool SMALL>
__global__ __launch_bounds__(256) void gat_aggregate_kernel(
    int64_t num_rows, int64_t H, int64_t D, const int64_t* __restrict__ row_beg,
    const int64_t* __restrict__ row_end, int accumulate, const int32_t* __restrict__ indices, const int32_t* __restrict__ row_order,
    const float* __restrict__ el, const float* __restrict__ er, const float* __restrict__ ft,
    float alpha, float lo, float hi, int apply_exp, uint64_t seed0,
    const int64_t* __restrict__ seed_off, uint32_t thr, float scale, float* __restrict__ out_ft,
    float* __restrict__ out_z, float* __restrict__ a_out, float* __restrict__ w_out,
    int64_t table_bytes) {
  typedef typename Vec<VEC>::T V;
  const int lane = threadIdx.x & 63;
  const int64_t it = block_linear() * (blockDim.x >> 6) +
                     __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  if (it >= num_rows) return;
  int64_t row = row_order ? row_order[it] : it;
  row = __builtin_amdgcn_readfirstlane(static_cast<int>(row));
  const int64_t beg = row_beg[row], end = row_end[row];
  if (accumulate && beg == end) return;  // nothing to add: the row keeps its value
  const int64_t F = H * D;
  const uint64_t seed = DROP ? seed0 + (seed_off ? static_cast<uint64_t>(*seed_off) : 0) : 0;
  const GatTable tab = gat_table(ft, SMALL ? table_bytes : 0);
  for (int64_t f0 = int64_t(lane) * VEC; f0 < F; f0 += 64 * VEC) {
    const int64_t h = f0 / D;
    const bool head_lane = f0 - h * D == 0;  // first lane of head h in this pass
    const uint32_t voff = static_cast<uint32_t>(f0 * int64_t(sizeof(float)));
    const float r = er[row * H + h];
    V acc = accumulate ? ldv<VEC>(out_ft + row * F + f0) : Vec<VEC>::zero();
    float zacc = accumulate ? out_z[row * H + h] : 0.0f;
    auto attend = [&](float x) {
      x = x + r;
      x = x > 0.0f ? x : alpha * x;
      if (apply_exp) x = __expf(x);
      return fminf(fmaxf(x, lo), hi);
    };
    auto consume = [&](int64_t k, float l, V u) {
      const float a = attend(l);
      float w = a;
      if (DROP) w = gat_keep(seed, k * H + h, thr) ? a * scale : 0.0f;
      acc = Vec<VEC>::fma(Vec<VEC>::splat(w), u, acc);
      zacc += a;
      if (head_lane && a_out) {
        a_out[k * H + h] = a;
        if (DROP) w_out[k * H + h] = w;
      }
    };
    int64_t k = beg;
    for (; k + UNROLL <= end; k += UNROLL) {
      float l[UNROLL];
      V u[UNROLL];
#pragma unroll
      for (int j = 0; j < UNROLL; ++j) {
        const int64_t src = indices[k + j];
        l[j] = el[src * H + h];
        u[j] = gat_gather<VEC, SMALL>(ft, tab, src, F, voff);
      }
#pragma unroll
      for (int j = 0; j < UNROLL; ++j) consume(k + j, l[j], u[j]);
    }
    const int64_t rem = end - k;  // one predicated batch, as reduce_range's tail
    if (rem > 0) {
      float l[UNROLL];
      V u[UNROLL];
#pragma unroll
      for (int j = 0; j < UNROLL - 1; ++j) {
        if (j < rem) {
          const int64_t src = indices[k + j];
          l[j] = el[src * H + h];
          u[j] = gat_gather<VEC, SMALL>(ft, tab, src, F, voff);
        }
      }
#pragma unroll
      for (int j = 0; j < UNROLL - 1; ++j)
        if (j < rem) consume(k + j, l[j], u[j]);
    }
    stv<VEC>(out_ft + row * F + f0, acc);
    if (head_lane) out_z[row * H + h] = zacc;
  }
}

// The same operation for H in {1, 2, 4, 8, 16}, with each (slot, head)
// attention computed ONCE per batch instead of once per lane: a batch is U
// slots; its U x H (slot, head) pairs are spread over the wave (lane l takes
// head l % H of slots l / H, l / H + 64 / H, ...), each computed value goes to
// the wave's LDS row of its head, and every lane then reads the U values of
// its own head back (lanes of a head read the same words: broadcast). The
// gathers of the batch's feature rows are issued before the attention is
// computed, so the exp work overlaps their latency. gat_aggregate_kernel ran
// the exp, the clamp and a 4-B logit gather per lane and slot (8x redundant
// at 8 heads of 16 features). Same per-element arithmetic and chain order.
// One batch of the LDS kernel: slots [k, k + nb) of the row (FULL: nb == U,
// no predication; the row's last partial batch runs with FULL = false, as
// reduce_range's predicated tail).
// LDS row stride of a head's U = 16 batch values: 20 words, so the pairs'
// writes (lane jc * H + hc at hc * 20 + jc) spread over the banks and a
// head's 16-B reads stay aligned
#define GAT_LDS_STRIDE 20

// The quad and half-row butterflies of gat_logit_tree (DPP: the same
// pairings as __shfl_xor 1, 2 and a mirror of the 8 lanes).
__device__ __forceinline__ float gat_dpp_xor1(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float gat_dpp_xor2(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
}
__device__ __forceinline__ float gat_dpp_half_mirror(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
}

// LOGIT (8 heads x 16, two-float lanes): the source's logit el[u, h] is not
// gathered but recomputed from the gathered feature row and the head's
// attention vector attn_l (alv: this lane's two entries), in
// dglhip_gat_logits_device's association, so the value is el's bit for bit
// and the slot needs 4 lines instead of 5.
template <int H, int VEC, bool DROP, bool SMALL, bool FULL, bool EARLY, bool LOGIT = false>
__device__ __forceinline__ void gat_batch(
    int64_t k, int nb, int64_t F, uint32_t voff, int64_t h, int hc, int jc, float rc,
    const int32_t* __restrict__ indices, const float* __restrict__ el,
    const float* __restrict__ ft, const GatTable& tab, float alpha, float lo, float hi, int apply_exp,
    uint64_t seed, uint32_t thr, float scale, float* la, float* lw, float* __restrict__ a_out,
    float* __restrict__ w_out, typename Vec<VEC>::T& acc, float& zacc,
    typename Vec<VEC>::T alv = typename Vec<VEC>::T()) {
#pragma clang fp contract(off)
  typedef typename Vec<VEC>::T V;
  constexpr int U = 16;
  static_assert(!LOGIT || (H == 8 && VEC == 2 && EARLY), "LOGIT: 8 heads x 16, early gathers");
  constexpr int LA = GAT_LDS_STRIDE;
  constexpr int SPP = 64 / H;               // slots covered per pass of the wave
  constexpr int PPL = (U + SPP - 1) / SPP;  // attention values per lane per batch
  V u[U];
  float lg[PPL];  // EARLY: the pairs' logits, loaded ahead of the row gathers
  if (EARLY) {
    // the batch's column ids through the scalar cache (one wide load when
    // FULL); each lane's pair columns selected from them, so the pairs' logit
    // loads go out first and the 16 feature-row gathers right behind them:
    // the attention is computed while the rows are in flight
    int cj[U];
#pragma unroll
    for (int j = 0; j < U; ++j) cj[j] = indices[k + (FULL || j < nb ? j : 0)];
#pragma unroll
    for (int i = 0; i < PPL; ++i) {
      const int j = jc + SPP * i;
      int c = cj[SPP * i < U ? SPP * i : 0];
#pragma unroll
      for (int t = 1; t < SPP; ++t)
        if (SPP * i + t < U) c = jc == t ? cj[SPP * i + t] : c;
      if (!((SPP * PPL == U || j < U) && (FULL || j < nb))) c = cj[0];
      if (!LOGIT) lg[i] = el[int64_t(c) * H + hc];
    }
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (FULL || j < nb) u[j] = gat_gather<VEC, SMALL>(ft, tab, cj[j], F, voff);
  }
  if constexpr (LOGIT) {
    // lane 8 h + t holds features 2t, 2t + 1 of head h: its pair product,
    // then the head's 8 lanes summed ((p0 + p1) + (p2 + p3)) + ((p4 + p5) +
    // (p6 + p7)) in every lane of the head; lane t keeps slot t's (and
    // t + 8's) and the pair lane (hc, jc) reads slot jc of head hc from lane
    // 8 hc + jc
    const int t = static_cast<int>(threadIdx.x & 7);
    float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (FULL || j < nb) {
        float p = __builtin_fmaf(u[j].y, alv.y, u[j].x * alv.x);
        p = p + gat_dpp_xor1(p);
        p = p + gat_dpp_xor2(p);
        p = p + gat_dpp_half_mirror(p);
        if (j < 8) s0 = t == j ? p : s0;
        else s1 = t == j - 8 ? p : s1;
      }
    }
    const int src = 8 * hc + jc;
    lg[0] = __shfl(s0, src, 64);
    lg[1] = __shfl(s1, src, 64);
  }
#pragma unroll
  for (int i = 0; i < PPL; ++i) {
    const int j = jc + SPP * i;
    if ((SPP * PPL == U || j < U) && (FULL || j < nb)) {
      float x = (EARLY ? lg[i] : el[int64_t(indices[k + j]) * H + hc]) + rc;
      x = x > 0.0f ? x : alpha * x;
      if (apply_exp) x = __expf(x);
      const float a = fminf(fmaxf(x, lo), hi);
      la[hc * LA + j] = a;
      if (a_out) a_out[(k + j) * H + hc] = a;
      if (DROP) {
        const float w = gat_keep(seed, (k + j) * H + hc, thr) ? a * scale : 0.0f;
        lw[hc * LA + j] = w;
        if (a_out) w_out[(k + j) * H + hc] = w;
      }
    }
  }
  // the batch's feature-row gathers (column ids through the scalar cache),
  // after the attention unless EARLY: then they are in flight during the
  // logit gathers and the attention (84 instead of 92 VGPRs at 8 x 16, five
  // waves per SIMD either way; the default on two-float lanes)
  // row base from the scalar slot stream (SGPRs) + the lane's 32-bit byte
  // offset: the saddr load form, one offset VGPR for all 16 gathers instead
  // of a 64-bit address per gather (80 -> fewer VGPRs, more waves per SIMD)
  if (!EARLY) {
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (FULL || j < nb) u[j] = gat_gather<VEC, SMALL>(ft, tab, indices[k + j], F, voff);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // the head's values four at a time (one 16-B LDS read), consumed in slot order
#pragma unroll
  for (int q = 0; q < U / 4; ++q) {
    // with dropout, keep the two 16-B LDS reads of each quad next to their
    // use (hoisted, the eight reads held 32 VGPRs: 109 -> 4 waves per SIMD)
    if (q > 0) __builtin_amdgcn_sched_barrier(0);
    const f32x4 t = *reinterpret_cast<const f32x4*>(la + h * LA + 4 * q);
    const float av[4] = {t.x, t.y, t.z, t.w};
    f32x4 t2 = t;
    if (DROP) t2 = *reinterpret_cast<const f32x4*>(lw + h * LA + 4 * q);
    const float wv[4] = {t2.x, t2.y, t2.z, t2.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = 4 * q + i;
      if (FULL || j < nb) {
        acc = Vec<VEC>::fma(Vec<VEC>::splat(wv[i]), u[j], acc);
        zacc += av[i];
      }
    }
  }
  // the next batch overwrites the rows only after every lane has read them
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// el[n, h] = the logit of node n's head h, sum_d ft[n, h, d] * attn[h, d]: at
// 16 features per head the tree ((p0 + p1) + (p2 + p3)) + ((p4 + p5) + (p6 +
// p7)), p_l = fma(x[2l+1], a[2l+1], x[2l] * a[2l]) (the association LOGIT
// recomputes in gat_batch), else one fma chain over d. One thread per (n, h).
__device__ __forceinline__ float gat_logit(const float* __restrict__ x,
                                           const float* __restrict__ a, int64_t D) {
#pragma clang fp contract(off)
  if (D == 16) {
    float p[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) p[l] = __builtin_fmaf(x[2 * l + 1], a[2 * l + 1], x[2 * l] * a[2 * l]);
    return ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
  }
  float acc = 0.0f;
  for (int64_t d = 0; d < D; ++d) acc = __builtin_fmaf(x[d], a[d], acc);
  return acc;
}

__global__ __launch_bounds__(256) void gat_logits_kernel(
    int64_t total, int64_t H, int64_t D, const float* __restrict__ ft,
    const float* __restrict__ attn_l, const float* __restrict__ attn_r, float* __restrict__ el,
    float* __restrict__ er) {
  const int64_t i = block_linear() * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int64_t h = i % H;
  const float* x = ft + i * D;  // row n, head h: (n * H + h) * D
  el[i] = gat_logit(x, attn_l + h * D, D);
  if (er) er[i] = gat_logit(x, attn_r + h * D, D);
}

template <int H, int VEC, bool DROP, bool SMALL, bool EARLY = false, int RP = 0,
          bool LOGIT = false, int WPE = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
void gat_aggregate_lds_kernel(
    int64_t num_rows, int64_t D, const int64_t* __restrict__ row_beg,
    const int64_t* __restrict__ row_end, int accumulate, const int32_t* __restrict__ indices, const int32_t* __restrict__ row_order,
    const float* __restrict__ el, const float* __restrict__ er, const float* __restrict__ ft,
    float alpha, float lo, float hi, int apply_exp, uint64_t seed0,
    const int64_t* __restrict__ seed_off, uint32_t thr, float scale, float* __restrict__ out_ft,
    float* __restrict__ out_z, float* __restrict__ a_out, float* __restrict__ w_out,
    int64_t table_bytes, const float* __restrict__ attn_l = nullptr) {
  typedef typename Vec<VEC>::T V;
  constexpr int U = 16;
  constexpr int LA = GAT_LDS_STRIDE;
  const GatTable tab = gat_table(ft, SMALL ? table_bytes : 0);
  __shared__ float s_a[4][H * LA];
  __shared__ float s_w[4][DROP ? H * LA : 1];
  const int lane = threadIdx.x & 63;
  const int wi = threadIdx.x >> 6;
  const int64_t it = block_linear() * (blockDim.x >> 6) +
                     __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  if (it >= num_rows) return;
  int64_t row = row_order ? row_order[it] : it;
  row = __builtin_amdgcn_readfirstlane(static_cast<int>(row));
  const int64_t beg = row_beg[row], end = row_end[row];
  if (accumulate && beg == end) return;  // nothing to add: the row keeps its value
  const int64_t F = H * D;
  const uint64_t seed = DROP ? seed0 + (seed_off ? static_cast<uint64_t>(*seed_off) : 0) : 0;
  // the pairs this lane computes: head hc of slots jc + (64 / H) * i
  const int hc = lane % H, jc = lane / H;
  const float rc = er[row * H + hc];
  for (int64_t base = 0; base < F; base += 64 * VEC) {
    // every lane takes part in the attention of each pass; lanes past F
    // gather a valid row (feature 0) and store nothing
    const int64_t f0 = base + int64_t(lane) * VEC;
    const bool active = f0 < F;
    const int64_t fa = active ? f0 : 0;
    const int64_t h = fa / D;
    const uint32_t voff = static_cast<uint32_t>(fa * int64_t(sizeof(float)));
    V acc = Vec<VEC>::zero();
    float zacc = 0.0f;
    if (accumulate && active) {
      acc = load_out<VEC, RP>(out_ft + row * F, f0);
      if (f0 - h * D == 0) zacc = out_z[row * H + h];
    }
    V alv = Vec<VEC>::zero();
    if (LOGIT) alv = ldv<VEC>(attn_l + fa);  // attn_l [H, D]: this lane's two entries
    int64_t k = beg;
    for (; k + U <= end; k += U)
      gat_batch<H, VEC, DROP, SMALL, true, EARLY, LOGIT>(
          k, U, F, voff, h, hc, jc, rc, indices, el, ft, tab, alpha, lo, hi, apply_exp, seed, thr,
          scale, s_a[wi], s_w[wi], a_out, w_out, acc, zacc, alv);
    if (k < end)
      gat_batch<H, VEC, DROP, SMALL, false, EARLY, LOGIT>(
          k, static_cast<int>(end - k), F, voff, h, hc, jc, rc, indices, el, ft, tab, alpha, lo,
          hi, apply_exp, seed, thr, scale, s_a[wi], s_w[wi], a_out, w_out, acc, zacc, alv);
    if (active) {
      store_out<VEC, RP>(out_ft + row * F, f0, acc);
      if (f0 - h * D == 0) out_z[row * H + h] = zacc;
    }
  }
}

// ---------------------------------------------------------------------------
// Fused GAT backward over the transpose (r04), 8 heads x 16 features.
//
// The backward of gat_aggregate needs, per edge u -> v (a forward slot kf of
// row v, a transposed slot of row u):
//   a  = clamp(exp(leaky_relu(el[u] + er[v])))        (the forward's attention)
//   w  = keep(kf) ? a * scale : 0                      (its dropped copy)
//   d_ft[u] += w * dout[v]                            (u_mul_e over the transpose)
//   t  = <dout[v, h], ft[u, h]>                        (the g-SDDMM dot)
//   g  = epilogue(t, a, keep, dz[v])                   (gat_epi_pre's operations)
//   d_el[u] += g  (copy_e over the transpose)    d_er[v] += g  (copy_e over the CSR)
// r03 ran it as three passes: the attention gradient over the CSR (storing g),
// d_ft over the transpose (reading w through the slot map: a 128-B line per
// 32-B value) and d_el over the transpose (g through the slot map), with a
// and w stored by the forward. Here ONE pass over the transpose, one wave per
// row u, computes d_ft and d_el (their chains in the transpose's slot order,
// as before) and every g, stored at its forward slot for d_er's sum (a
// sequential copy_e pass over the CSR). a and w are recomputed from el, er
// and the dropout hash of the forward slot (the forward's expressions, so
// the same bits), so the forward stores no E x H tensor.
//
// The dot keeps the sliced g-SDDMM's association (gsddmm_dot_sliced_kernel,
// D = 16: four lanes of 4 features per head, partials p_r = fma chains over
// features 4r..4r+3 starting with a product, total (p0 + p2) + (p1 + p3)):
// here lane 2m holds features 4m, 4m+1 and lane 2m+1 features 4m+2, 4m+3; the
// even lane's half chain continues on the odd lane (DPP), and the partials of
// lanes 8h+1, 8h+3, 8h+5, 8h+7 combine by xor 4 then xor 2. The per-(slot,
// head) attention and keep bit are computed once per batch of 16 slots (two
// pairs per lane) and shared through LDS, as the forward's LDS kernel does.
//
// Items: as dglhip_gspmm_items_device (the transposed CSR's source-blocked
// plan: item i = row item_row[i], slots [item_beg[i], item_end[i]) of cols /
// fslot, accumulate continuing both chains), or whole rows (by_row: item i is
// row item_row[i] with slots [item_beg[row], item_end[row])).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float dpp_even_to_odd(float v) {
  // quad_perm [0, 0, 2, 2]: lane 2m+1 reads lane 2m
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xA0, 0xF, 0xF, false));
}

// row_shl:N (within a 16-lane row): lane i reads lane i + N
template <int N>
__device__ __forceinline__ float dpp_shl(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x100 + N, 0xF, 0xF,
                                                    false));
}

// PACK: er and dz arrive as one [rows, 2H] table (er then dz per row, the
// caller's packing): the pair's two operands sit in one 64-B run, one line
// per slot instead of two (r05: 230M of the backward's 873M L2 requests per
// call were these two 32-B reads)
template <bool DROP, bool SMALL, int RP = 0, int WPE = 4, bool PACK = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void gat_backward_t_kernel(
    int64_t num_items, const int32_t* __restrict__ item_row, const int64_t* __restrict__ item_beg,
    const int64_t* __restrict__ item_end, int by_row, int accumulate,
    const int32_t* __restrict__ cols, const int64_t* __restrict__ fslot,
    const float* __restrict__ ft, const float* __restrict__ el, const float* __restrict__ er,
    const float* __restrict__ dz, const float* __restrict__ dout, float alpha, float lo,
    float hi, int apply_exp, uint64_t seed0, const int64_t* __restrict__ seed_off, uint32_t thr,
    float scale, float* __restrict__ d_ft, float* __restrict__ d_el, float* __restrict__ g_out,
    int64_t table_bytes, int gpol) {
  constexpr int H = 8, F = 128, U = 16;
  constexpr int LU = U + 4;  // LDS row stride by head: the pairs' writes (lane
                             // 8 jc + hc at hc * LU + jc) hit distinct banks
  typedef Vec<2>::T V;
  __shared__ float s_w[4][H * LU];  // the batch's dropped attention, by head
  __shared__ float s_d[4][H * LU];  // its dots, then its attention gradients
  const int lane = threadIdx.x & 63;
  const int wi = threadIdx.x >> 6;
  const int64_t it = block_linear() * (blockDim.x >> 6) +
                     __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  if (it >= num_items) return;
  int64_t row = item_row ? item_row[it] : it;
  row = __builtin_amdgcn_readfirstlane(static_cast<int>(row));
  const int64_t ix = by_row ? row : it;
  const int64_t beg = item_beg[ix], end = item_end[ix];
  if (accumulate && beg == end) return;
  const uint64_t seed = DROP ? seed0 + (seed_off ? static_cast<uint64_t>(*seed_off) : 0) : 0;
  const GatTable tab = gat_table(dout, SMALL ? table_bytes : 0);
  const int64_t f0 = int64_t(lane) * 2;
  const int h = lane >> 3;                 // this lane's head (16 features = 8 lanes)
  const bool head_lane = (lane & 7) == 1;  // holds the head's dot: lane 8h + 1
  const uint32_t voff = static_cast<uint32_t>(f0 * int64_t(sizeof(float)));
  // the (slot, head) pairs this lane computes: head hc of slots jc and jc + 8
  const int hc = lane & 7, jc = lane >> 3;
  const float elc = el[row * H + hc];
  const V ftv = ldv<2>(ft + row * F + f0);
  V acc = accumulate ? load_out<2, RP>(d_ft + row * F, f0) : Vec<2>::zero();
  float elacc = (accumulate && head_lane) ? d_el[row * H + h] : 0.0f;
  float* lw = s_w[wi];
  float* ld = s_d[wi];
  const int rbytes = SMALL ? static_cast<int>(table_bytes / (F / H)) * (PACK ? 2 : 1) : 0;
  constexpr uint32_t ERS = PACK ? 2 * H : H;  // er / dz row stride (floats)
  const __amdgpu_buffer_rsrc_t er_r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(er), 0, rbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t dz_r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dz ? dz : er), 0, rbytes, 0x00020000);
  // One batch of U slots [k, k + nb) (FULL: nb == U, no predication). The
  // column ids come through the scalar cache first; the pairs' operands
  // (er, dz, the forward slot) are loaded before the 16 row gathers, so the
  // attention is computed while the rows are in flight; the attention
  // gradients are stored at the end of the batch, so no wait on their
  // write acknowledgements sits inside it.
  auto batch = [&](int64_t k, int nb, auto full_tag) {
    constexpr bool FULL = decltype(full_tag)::value;
    int cj[U];
#pragma unroll
    for (int j = 0; j < U; ++j) cj[j] = cols[k + (FULL || j < nb ? j : 0)];
    // this lane's pairs: slots jc and jc + 8 (clamped into the batch when
    // partial; the values of slots past nb are never used)
    int pc[2];
    int64_t pj[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int c = cj[8 * i];
#pragma unroll
      for (int t = 1; t < 8; ++t) c = jc == t ? cj[8 * i + t] : c;
      const int j = jc + 8 * i;
      pj[i] = FULL || j < nb ? j : 0;
      pc[i] = FULL || j < nb ? c : cj[0];
    }
    float per[2], pz[2];
    int64_t pf[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (SMALL) {  // er and dz are 32 B per row of dout's: 32-bit offsets
        const uint32_t o = static_cast<uint32_t>(pc[i]) * (ERS * 4u) + hc * 4u;
        per[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(er_r, o, 0, 0));
        if (PACK)
          pz[i] = __builtin_bit_cast(float,
                                     __builtin_amdgcn_raw_buffer_load_b32(er_r, o + H * 4u, 0, 0));
        else
          pz[i] = dz ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dz_r, o, 0, 0))
                     : 0.0f;
      } else {
        per[i] = er[int64_t(pc[i]) * ERS + hc];
        pz[i] = PACK ? er[int64_t(pc[i]) * ERS + H + hc] : (dz ? dz[int64_t(pc[i]) * H + hc] : 0.0f);
      }
      pf[i] = fslot[k + pj[i]];
    }
    V u[U];
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (FULL || j < nb) u[j] = gat_gather<2, SMALL>(dout, tab, cj[j], F, voff);
    // the pairs: attention, keep bit, dropped weight (the forward's
    // expressions)
    float pa[2];
    bool pk[2], px[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int j = jc + 8 * i;
      float x = elc + per[i];
      px[i] = x > 0.0f;  // the slope from the logit's sign (torch's backward)
      x = px[i] ? x : alpha * x;
      if (apply_exp) x = __expf(x);
      const float a = fminf(fmaxf(x, lo), hi);
      float w = a;
      pk[i] = true;
      if (DROP) {
        pk[i] = gat_keep(seed, pf[i] * H + hc, thr);
        w = pk[i] ? a * scale : 0.0f;
      }
      pa[i] = a;
      lw[hc * LU + j] = w;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // per slot: d_ft's chain and the head's dot (as below)
#pragma unroll
    for (int q = 0; q < U / 4; ++q) {
      // each quad's LDS read next to its use (here and in d_el's sum below:
      // hoisted, they held the one-pass kernel at 103 VGPRs, 4 waves per SIMD;
      // kept in place 95, 5 waves)
      if (q > 0) __builtin_amdgcn_sched_barrier(0);
      const f32x4 w4 = *reinterpret_cast<const f32x4*>(lw + h * LU + 4 * q);
      const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = 4 * q + i;
        if (FULL || j < nb) {
          acc = Vec<2>::fma(Vec<2>::splat(wv[i]), u[j], acc);
          float t = u[j].x * ftv.x;
          t = __builtin_fmaf(u[j].y, ftv.y, t);
          float p = __builtin_fmaf(u[j].x, ftv.x, dpp_even_to_odd(t));
          p = __builtin_fmaf(u[j].y, ftv.y, p);
          const float s2 = p + dpp_shl<4>(p);
          const float dot = s2 + dpp_shl<2>(s2);
          if (head_lane) ld[h * LU + j] = dot;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the epilogue per pair (gat_epi_pre's operations), g back into the
    // LDS row by head for d_el's chain
    float pg[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int j = jc + 8 * i;
      const float a = pa[i];
      float tt = ld[hc * LU + j];
      if (DROP) tt = pk[i] ? tt * scale : 0.0f;
      if (PACK || dz) tt = tt + pz[i];
      const float sl = px[i] ? 1.0f : alpha;
      float g = apply_exp ? (tt * a) * sl : tt * sl;
      g = (a > lo && a < hi) ? g : 0.0f;
      pg[i] = g;
      ld[hc * LU + j] = g;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (head_lane) {
#pragma unroll
      for (int q = 0; q < U / 4; ++q) {
        if (q > 0) __builtin_amdgcn_sched_barrier(0);
        const f32x4 g4 = *reinterpret_cast<const f32x4*>(ld + h * LU + 4 * q);
        const float gv[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (FULL || 4 * q + i < nb) elacc = elacc + gv[i];
      }
    }
    // g at its forward slot, for d_er's sum over the CSR
    if (gpol == 3) {
      // 16-B write-through stores that drop the line from the XCD's L2
      // (sc1): lane 2j + half takes heads 4 half .. 4 half + 3 of slot j
      // from the LDS rows (already holding g by head), so the scattered
      // partial lines stop evicting the block's dout rows
      const int j = lane >> 1, half = lane & 1;
      const int64_t p0 = __shfl(pf[0], 8 * (j & 7), 64), p1 = __shfl(pf[1], 8 * (j & 7), 64);
      if (j < U && (FULL || j < nb)) {
        const int64_t pj = j < 8 ? p0 : p1;
        f32x4 gv;
        gv.x = ld[(4 * half + 0) * LU + j];
        gv.y = ld[(4 * half + 1) * LU + j];
        gv.z = ld[(4 * half + 2) * LU + j];
        gv.w = ld[(4 * half + 3) * LU + j];
        float* dst = g_out + pj * H + 4 * half;
        asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(dst), "v"(gv) : "memory");
      }
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (FULL || jc + 8 * i < nb) {
          if (gpol == 0) g_out[pf[i] * H + hc] = pg[i];
          else if (gpol == 1) __builtin_nontemporal_store(pg[i], g_out + pf[i] * H + hc);
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  int64_t k = beg;
  for (; k + U <= end; k += U) batch(k, U, std::true_type());
  if (k < end) batch(k, static_cast<int>(end - k), std::false_type());
  store_out<2, RP>(d_ft + row * F, f0, acc);
  if (head_lane) d_el[row * H + h] = elacc;
}

// Per row and head, the sum of an [nnz, 8] slot-ordered tensor over the row's
// slots, as the copy_e sum's chain ((0 + v0) + v1) + ... in slot order (GAT's
// d_er from the attention gradient). gspmm_sum_kernel gives each row 4 lanes
// and walks it slot by slot, so a hub row of ~20,000 slots (Reddit-shaped
// graph) is ~1,300 serial load latencies (1.32 ms per call). Here a wave owns
// a row: 64 slots per step arrive as 8 coalesced 256-B loads (lane = slot %
// 8 x 8 + head), pass through LDS transposed to head-major, and the head's
// lane adds its 64 values in slot order.
__global__ __launch_bounds__(256) void rowsum_heads8_kernel(
    int64_t num_rows, const int64_t* __restrict__ indptr, const int32_t* __restrict__ row_order,
    const float* __restrict__ vals, float* __restrict__ out) {
  constexpr int H = 8, S = 64;
  constexpr int LS = S + 4;  // head-row stride: the transposing writes and the
                             // head lanes' 16-B reads hit distinct banks
  __shared__ float s_v[4][H * LS];
  const int lane = threadIdx.x & 63;
  const int wi = threadIdx.x >> 6;
  const int64_t it = block_linear() * (blockDim.x >> 6) +
                     __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  if (it >= num_rows) return;
  int64_t row = row_order ? row_order[it] : it;
  row = __builtin_amdgcn_readfirstlane(static_cast<int>(row));
  const int64_t beg = indptr[row], end = indptr[row + 1];
  const int s = lane >> 3, hh = lane & 7;
  float* lv = s_v[wi];
  float acc = 0.0f;
  // the step's 8 loads per lane; the next step's are issued before this
  // step's serial sum, so their latency overlaps it
  auto load = [&](int64_t k, float* v) {
    const int nb = end - k < S ? static_cast<int>(end - k) : S;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int j = 8 * q + s;
      v[q] = j < nb ? vals[(k + j) * H + hh] : 0.0f;
    }
  };
  float v[8];
  if (beg < end) load(beg, v);
  for (int64_t k = beg; k < end; k += S) {
    const int nb = end - k < S ? static_cast<int>(end - k) : S;
#pragma unroll
    for (int q = 0; q < 8; ++q) lv[hh * LS + 8 * q + s] = v[q];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (k + S < end) load(k + S, v);
    if (lane < H) {
      if (nb == S) {
#pragma unroll
        for (int q = 0; q < S / 4; ++q) {
          const f32x4 t = *reinterpret_cast<const f32x4*>(lv + lane * LS + 4 * q);
          acc = acc + t.x;
          acc = acc + t.y;
          acc = acc + t.z;
          acc = acc + t.w;
        }
      } else {
#pragma unroll
        for (int q = 0; q < S / 4; ++q) {
          const f32x4 t = *reinterpret_cast<const f32x4*>(lv + lane * LS + 4 * q);
          const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (4 * q + i < nb) acc = acc + tv[i];
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (lane < H) out[row * H + lane] = acc;
}

}  // namespace dglhip

using namespace dglhip;

extern "C" {

int dglhip_gat_aggregate_ranges_device(
    int64_t num_rows, int64_t num_src, int64_t num_heads, int64_t head_dim,
    const int64_t* row_beg, const int64_t* row_end, int accumulate, const int32_t* indices,
    const int32_t* row_order, const float* el, const float* er, const float* ft, float alpha,
    float clamp_lo, float clamp_hi, int apply_exp, float drop_p, uint64_t seed,
    const int64_t* seed_offset, float* out_ft, float* out_z, float* attn_out,
    float* attn_drop_out, void* stream_) {
  return dglhip_gat_aggregate_logits_ranges_device(
      num_rows, num_src, num_heads, head_dim, row_beg, row_end, accumulate, indices, row_order,
      el, er, ft, nullptr, alpha, clamp_lo, clamp_hi, apply_exp, drop_p, seed, seed_offset,
      out_ft, out_z, attn_out, attn_drop_out, stream_);
}

int dglhip_gat_aggregate_logits_ranges_device(
    int64_t num_rows, int64_t num_src, int64_t num_heads, int64_t head_dim,
    const int64_t* row_beg, const int64_t* row_end, int accumulate, const int32_t* indices,
    const int32_t* row_order, const float* el, const float* er, const float* ft,
    const float* attn_l, float alpha, float clamp_lo, float clamp_hi, int apply_exp,
    float drop_p, uint64_t seed, const int64_t* seed_offset, float* out_ft, float* out_z,
    float* attn_out, float* attn_drop_out, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows >= 0 && num_src >= 0 && num_heads >= 1 && head_dim >= 1, "bad sizes");
  DGLHIP_CHECK(drop_p >= 0.0f && drop_p < 1.0f, "dropout probability must be in [0, 1)");
  if (num_rows == 0) return 0;
  DGLHIP_CHECK(row_beg && row_end && indices && el && er && ft && out_ft && out_z,
               "null pointer argument");
  const bool drop = drop_p > 0.0f;
  DGLHIP_CHECK(!drop || (attn_out == nullptr) == (attn_drop_out == nullptr),
               "with dropout, the attention and its dropped copy are written together");
  const int64_t blocks = (num_rows + 3) / 4;
  DGLHIP_CHECK(blocks <= 0x7fffffff, "grid too large");
  const uint32_t thr = drop ? gat_drop_threshold(drop_p) : 0u;
  const float scale = drop ? 1.0f / (1.0f - drop_p) : 1.0f;
  const int64_t F = num_heads * head_dim;
  // the source table in bytes: under 4 GB one descriptor spans it (row
  // offsets as soffset), else one descriptor per gathered row
  const int64_t tbytes = num_src * F * int64_t(sizeof(float));
  const bool small = tbytes < (int64_t(1) << 31);
  // VEC 2 when a lane's two features stay in one head and rows are 8-B aligned
  const bool v2 = head_dim % 2 == 0 && F >= 128 &&
                  reinterpret_cast<uintptr_t>(ft) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(out_ft) % 8 == 0;
  // per-(slot, head) attention through LDS for the common head counts on
  // one-float lanes (rows of <= 64 floats or odd head widths: Pubmed's 8 x 8
  // and 8 x 3, 0.015 vs 0.023 ms); two-float lanes (8 x 16 on the
  // Reddit-shaped graph) run the per-lane kernel, 9.37 vs 9.87 ms
  // (tools/gat_bench.py). Both are bound by the line rate: per slot the
  // feature row's lines plus one line for the source's H logits.
  // Under the source-blocked schedule (row sub-ranges, not whole rows) the
  // gathers come from L2 and the per-lane attention's exp and hash work
  // becomes the bound: the LDS kernel there for every width (Reddit-shaped
  // 8 x 16: 7.39 vs 11.37 ms, with dropout 9.44 vs 17.04).
  const bool whole_rows = row_end == row_beg + 1;
  const bool lds_heads = num_heads == 1 || num_heads == 2 || num_heads == 4 ||
                         num_heads == 8 || num_heads == 16;
  if (lds_heads && (g_gat_variant == 2 || (g_gat_variant != 1 && (!v2 || !whole_rows)))) {
    // the batch's feature rows issued before its attention on two-float lanes
    // (Reddit-shaped 8 x 16, blocked: 6.25 -> 6.07 ms, with dropout 7.05 ->
    // 6.49; one-float lanes level: Pubmed's 8 x 8 and 8 x 3;
    // tools/gat_early_ab.py); variant 2 keeps them after it, 3 before it
    const bool early = g_gat_variant == 3 || (g_gat_variant == 0 && v2);
    if (num_heads == 8 && v2 && early && (g_row_pol == 2 || g_row_pol == 4)) {
      // the running rows' cache policy (dglhip_set_row_policy) on the 8-head
      // two-float shape (the Reddit-shaped 8 x 16 layer); with attn_l the
      // sources' logits recomputed from their gathered rows (LOGIT)
      const bool logit = attn_l != nullptr && head_dim == 16 && g_gat_logit_on;
      timed_launch(stream, [&] {
#define DGLHIP_GATRP(DD, SM, RPV)                                                              \
  do {                                                                                         \
    if (logit)                                                                                 \
      hipLaunchKernelGGL((gat_aggregate_lds_kernel<8, 2, DD, SM, true, RPV, true>),             \
                         grid_1d(blocks), dim3(256), 0, stream, num_rows, head_dim, row_beg,    \
                         row_end, accumulate, indices, row_order, el, er, ft, alpha, clamp_lo,  \
                         clamp_hi, apply_exp, seed, seed_offset, thr, scale, out_ft, out_z,     \
                         attn_out, attn_drop_out, tbytes, attn_l);                              \
    else                                                                                       \
      hipLaunchKernelGGL((gat_aggregate_lds_kernel<8, 2, DD, SM, true, RPV>), grid_1d(blocks),  \
                         dim3(256), 0, stream, num_rows, head_dim, row_beg, row_end,           \
                         accumulate, indices, row_order, el, er, ft, alpha, clamp_lo,          \
                         clamp_hi, apply_exp, seed, seed_offset, thr, scale, out_ft, out_z,    \
                         attn_out, attn_drop_out, tbytes, nullptr);                            \
  } while (0)
#define DGLHIP_GATW(DD, SM, W)                                                                 \
  hipLaunchKernelGGL((gat_aggregate_lds_kernel<8, 2, DD, SM, true, 2, false, W>),              \
                     grid_1d(blocks), dim3(256), 0, stream, num_rows, head_dim, row_beg, row_end, \
                     accumulate, indices, row_order, el, er, ft, alpha, clamp_lo, clamp_hi,      \
                     apply_exp, seed, seed_offset, thr, scale, out_ft, out_z, attn_out,          \
                     attn_drop_out, tbytes, nullptr)
        if (g_row_pol == 2 && !logit && g_gat_fwd_waves == 6) {
          // study knob: at least 6 waves per SIMD (the no-dropout kernel is 81
          // VGPRs, one over the 80 that 6 waves allow)
          if (drop) { if (small) DGLHIP_GATW(true, true, 6); else DGLHIP_GATW(true, false, 6); }
          else { if (small) DGLHIP_GATW(false, true, 6); else DGLHIP_GATW(false, false, 6); }
        } else if (g_row_pol == 2 && !logit && g_gat_fwd_waves == 5) {
          if (drop) { if (small) DGLHIP_GATW(true, true, 5); else DGLHIP_GATW(true, false, 5); }
          else { if (small) DGLHIP_GATW(false, true, 5); else DGLHIP_GATW(false, false, 5); }
        } else if (g_row_pol == 2) {
          if (drop) { if (small) DGLHIP_GATRP(true, true, 2); else DGLHIP_GATRP(true, false, 2); }
          else { if (small) DGLHIP_GATRP(false, true, 2); else DGLHIP_GATRP(false, false, 2); }
        } else {
          if (drop) { if (small) DGLHIP_GATRP(true, true, 4); else DGLHIP_GATRP(true, false, 4); }
          else { if (small) DGLHIP_GATRP(false, true, 4); else DGLHIP_GATRP(false, false, 4); }
        }
#undef DGLHIP_GATRP
#undef DGLHIP_GATW
      });
      return 0;
    }
    timed_launch(stream, [&] {
#define DGLHIP_GATL_E(HH, VV, DD, SM, EE)                                                    \
  hipLaunchKernelGGL((gat_aggregate_lds_kernel<HH, VV, DD, SM, EE>), grid_1d(blocks),        \
                     dim3(256), 0, stream, num_rows, head_dim, row_beg, row_end, accumulate, \
                     indices, row_order, el, er, ft,                                         \
                     alpha, clamp_lo, clamp_hi, apply_exp, seed, seed_offset, thr, scale,    \
                     out_ft, out_z, attn_out, attn_drop_out, tbytes)
#define DGLHIP_GATL(HH, VV, DD, SM)                                                          \
  do {                                                                                       \
    if (early) DGLHIP_GATL_E(HH, VV, DD, SM, true);                                          \
    else DGLHIP_GATL_E(HH, VV, DD, SM, false);                                               \
  } while (0)
#define DGLHIP_GATS(HH, VV, DD) \
  if (small) DGLHIP_GATL(HH, VV, DD, true); else DGLHIP_GATL(HH, VV, DD, false);
#define DGLHIP_GATH(HH)                                                                    \
  if (num_heads == HH) {                                                                   \
    if (v2) { if (drop) { DGLHIP_GATS(HH, 2, true) } else { DGLHIP_GATS(HH, 2, false) } }   \
    else { if (drop) { DGLHIP_GATS(HH, 1, true) } else { DGLHIP_GATS(HH, 1, false) } }      \
    return;                                                                                \
  }
      DGLHIP_GATH(1) DGLHIP_GATH(2) DGLHIP_GATH(4) DGLHIP_GATH(8) DGLHIP_GATH(16)
#undef DGLHIP_GATH
#undef DGLHIP_GATS
#undef DGLHIP_GATL
#undef DGLHIP_GATL_E
    });
    return 0;
  }
  timed_launch(stream, [&] {
#define DGLHIP_GAT(VV, DD, SM)                                                             \
  hipLaunchKernelGGL((gat_aggregate_kernel<VV, 16, DD, SM>), grid_1d(blocks), dim3(256), 0, \
                     stream, num_rows, num_heads, head_dim, row_beg, row_end, accumulate,   \
                     indices, row_order, el,                                                 \
                     er, ft, alpha, clamp_lo, clamp_hi, apply_exp, seed, seed_offset, thr, scale, \
                     out_ft, out_z, attn_out, attn_drop_out, tbytes)
#define DGLHIP_GATS(VV, DD) if (small) DGLHIP_GAT(VV, DD, true); else DGLHIP_GAT(VV, DD, false);
    if (v2) {
      if (drop) { DGLHIP_GATS(2, true) } else { DGLHIP_GATS(2, false) }
    } else {
      if (drop) { DGLHIP_GATS(1, true) } else { DGLHIP_GATS(1, false) }
    }
#undef DGLHIP_GATS
#undef DGLHIP_GAT
  });
  API_END();
}

int dglhip_gat_aggregate_device(int64_t num_rows, int64_t num_src, int64_t num_heads,
                                int64_t head_dim, const int64_t* indptr, const int32_t* indices,
                                const int32_t* row_order, const float* el, const float* er,
                                const float* ft, float alpha, float clamp_lo, float clamp_hi,
                                int apply_exp, float drop_p, uint64_t seed,
                                const int64_t* seed_offset, float* out_ft, float* out_z,
                                float* attn_out, float* attn_drop_out, void* stream) {
  return dglhip_gat_aggregate_ranges_device(
      num_rows, num_src, num_heads, head_dim, indptr, indptr ? indptr + 1 : nullptr, 0, indices,
      row_order, el, er, ft, alpha, clamp_lo, clamp_hi, apply_exp, drop_p, seed, seed_offset,
      out_ft, out_z, attn_out, attn_drop_out, stream);
}

int dglhip_gat_backward_t_ok(int64_t num_heads, int64_t head_dim) {
  return num_heads == 8 && head_dim == 16 ? 1 : 0;
}

static int gat_backward_t_impl(
    bool packed, int64_t num_items, const int32_t* item_row, const int64_t* item_beg, const int64_t* item_end,
    int by_row, int accumulate, int64_t num_rows, int64_t num_src, int64_t num_heads,
    int64_t head_dim, const int32_t* cols, const int64_t* fslot, const float* ft, const float* el,
    const float* er, const float* dz, const float* dout, float alpha, float clamp_lo,
    float clamp_hi, int apply_exp, float drop_p, uint64_t seed, const int64_t* seed_offset,
    float* d_ft, float* d_el, float* grad, void* stream_) {
  API_BEGIN();
  DGLHIP_CHECK(!packed || er != nullptr, "the packed form takes er and dz as one table");
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(dglhip_gat_backward_t_ok(num_heads, head_dim) == 1,
               "the transposed GAT backward runs 8 heads x 16 features, got " << num_heads
               << " x " << head_dim);
  DGLHIP_CHECK(num_items >= 0 && num_rows >= 0 && num_src >= 0, "bad sizes");
  DGLHIP_CHECK(drop_p >= 0.0f && drop_p < 1.0f, "dropout probability must be in [0, 1)");
  if (num_items == 0) return 0;
  DGLHIP_CHECK(item_beg && item_end && cols && fslot && ft && el && er && dout && d_ft && d_el,
               "null pointer argument");
  DGLHIP_CHECK(reinterpret_cast<uintptr_t>(ft) % 8 == 0 &&
               reinterpret_cast<uintptr_t>(dout) % 8 == 0 &&
               reinterpret_cast<uintptr_t>(d_ft) % 8 == 0, "rows must be 8-B aligned");
  const int64_t blocks = (num_items + 3) / 4;
  DGLHIP_CHECK(blocks <= 0x7fffffff, "grid too large");
  const bool drop = drop_p > 0.0f;
  const uint32_t thr = drop ? gat_drop_threshold(drop_p) : 0u;
  const float scale = drop ? 1.0f / (1.0f - drop_p) : 1.0f;
  // dout is gathered by destination v: num_rows rows of the forward CSR
  const int64_t tbytes = num_rows * num_heads * head_dim * int64_t(sizeof(float));
  const bool small = tbytes < (int64_t(1) << 31);
  const int gpol = grad ? (g_gat_bwd_variant & 3) : 2;  // no grad buffer: nothing stored
  const bool w5 = (g_gat_bwd_variant & 4) != 0;
  timed_launch(stream, [&] {
#define DGLHIP_GBT_W(DD, SM, RPV, W, PK)                                                      \
  hipLaunchKernelGGL((gat_backward_t_kernel<DD, SM, RPV, W, PK>), grid_1d(blocks), dim3(256),  \
                     0, stream, num_items, item_row, item_beg, item_end, by_row, accumulate,    \
                     cols, fslot, ft, el, er, dz, dout, alpha, clamp_lo, clamp_hi, apply_exp,   \
                     seed, seed_offset, thr, scale, d_ft, d_el, grad, tbytes, gpol)
#define DGLHIP_GBT_R(DD, SM, RPV)                                                             \
  do {                                                                                        \
    if (packed) DGLHIP_GBT_W(DD, SM, RPV, 4, true);                                           \
    else if (w5) DGLHIP_GBT_W(DD, SM, RPV, 5, false);                                         \
    else DGLHIP_GBT_W(DD, SM, RPV, 4, false);                                                 \
  } while (0)
#define DGLHIP_GBT(DD, SM)                                                                    \
  do {                                                                                        \
    if (g_row_pol == 2) DGLHIP_GBT_R(DD, SM, 2);                                              \
    else if (g_row_pol == 4) DGLHIP_GBT_R(DD, SM, 4);                                         \
    else DGLHIP_GBT_R(DD, SM, 0);                                                             \
  } while (0)
    if (drop) {
      if (small) DGLHIP_GBT(true, true); else DGLHIP_GBT(true, false);
    } else {
      if (small) DGLHIP_GBT(false, true); else DGLHIP_GBT(false, false);
    }
#undef DGLHIP_GBT
#undef DGLHIP_GBT_R
#undef DGLHIP_GBT_W
  });
  API_END();
}

int dglhip_gat_backward_t_device(
    int64_t num_items, const int32_t* item_row, const int64_t* item_beg, const int64_t* item_end,
    int by_row, int accumulate, int64_t num_rows, int64_t num_src, int64_t num_heads,
    int64_t head_dim, const int32_t* cols, const int64_t* fslot, const float* ft, const float* el,
    const float* er, const float* dz, const float* dout, float alpha, float clamp_lo,
    float clamp_hi, int apply_exp, float drop_p, uint64_t seed, const int64_t* seed_offset,
    float* d_ft, float* d_el, float* grad, void* stream) {
  return gat_backward_t_impl(false, num_items, item_row, item_beg, item_end, by_row, accumulate,
                             num_rows, num_src, num_heads, head_dim, cols, fslot, ft, el, er, dz,
                             dout, alpha, clamp_lo, clamp_hi, apply_exp, drop_p, seed, seed_offset,
                             d_ft, d_el, grad, stream);
}

int dglhip_gat_backward_t_packed_device(
    int64_t num_items, const int32_t* item_row, const int64_t* item_beg, const int64_t* item_end,
    int by_row, int accumulate, int64_t num_rows, int64_t num_src, int64_t num_heads,
    int64_t head_dim, const int32_t* cols, const int64_t* fslot, const float* ft, const float* el,
    const float* erdz, const float* dout, float alpha, float clamp_lo, float clamp_hi,
    int apply_exp, float drop_p, uint64_t seed, const int64_t* seed_offset, float* d_ft,
    float* d_el, float* grad, void* stream) {
  return gat_backward_t_impl(true, num_items, item_row, item_beg, item_end, by_row, accumulate,
                             num_rows, num_src, num_heads, head_dim, cols, fslot, ft, el, erdz,
                             nullptr, dout, alpha, clamp_lo, clamp_hi, apply_exp, drop_p, seed,
                             seed_offset, d_ft, d_el, grad, stream);
}

int dglhip_rowsum_heads8_device(int64_t num_rows, const int64_t* indptr,
                                const int32_t* row_order, const float* vals, float* out,
                                void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows >= 0, "bad sizes");
  if (num_rows == 0) return 0;
  DGLHIP_CHECK(indptr && vals && out, "null pointer argument");
  const int64_t blocks = (num_rows + 3) / 4;
  DGLHIP_CHECK(blocks <= 0x7fffffff, "grid too large");
  timed_launch(stream, [&] {
    hipLaunchKernelGGL(rowsum_heads8_kernel, grid_1d(blocks), dim3(256), 0, stream, num_rows,
                       indptr, row_order, vals, out);
  });
  API_END();
}

int dglhip_set_gat_variant(int variant) {
  API_BEGIN();
  DGLHIP_CHECK(variant >= 0 && variant <= 3, "unknown GAT kernel variant " << variant);
  g_gat_variant = variant;
  API_END();
}

int dglhip_set_gat_fwd_waves(int waves) {
  API_BEGIN();
  DGLHIP_CHECK(waves == 0 || waves == 5 || waves == 6, "forward waves per SIMD " << waves);
  g_gat_fwd_waves = waves;
  API_END();
}

int dglhip_set_gat_logit_recompute(int on) {
  API_BEGIN();
  g_gat_logit_on = on ? 1 : 0;
  API_END();
}

int dglhip_gat_logits_device(int64_t num_nodes, int64_t num_heads, int64_t head_dim,
                             const float* ft, const float* attn_l, const float* attn_r, float* el,
                             float* er, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_nodes >= 0 && num_heads >= 1 && head_dim >= 1, "bad sizes");
  const int64_t total = num_nodes * num_heads;
  if (total == 0) return 0;
  DGLHIP_CHECK(ft && attn_l && el && (attn_r == nullptr) == (er == nullptr),
               "null pointer argument");
  timed_launch(stream, [&] {
    hipLaunchKernelGGL(gat_logits_kernel, grid_1d((total + 255) / 256), dim3(256), 0, stream,
                       total, num_heads, head_dim, ft, attn_l, attn_r, el, er);
  });
  API_END();
}

int dglhip_set_gat_bwd_variant(int variant) {
  API_BEGIN();
  DGLHIP_CHECK(variant >= 0 && variant <= 7, "unknown GAT backward variant " << variant);
  g_gat_bwd_variant = variant;
  API_END();
}

int dglhip_gat_dropout_mask_host(int64_t num_slots, int64_t num_heads, float drop_p,
                                 uint64_t seed, uint8_t* keep) {
  API_BEGIN();
  DGLHIP_CHECK(num_slots >= 0 && num_heads >= 1, "bad sizes");
  DGLHIP_CHECK(drop_p >= 0.0f && drop_p < 1.0f, "dropout probability must be in [0, 1)");
  if (num_slots == 0) return 0;
  DGLHIP_CHECK(keep != nullptr, "null pointer argument");
  const uint32_t thr = drop_p > 0.0f ? gat_drop_threshold(drop_p) : 0u;
  const int64_t n = num_slots * num_heads;
  parallel_for(n, default_num_threads(), [&](int64_t b, int64_t e, int) {
    for (int64_t i = b; i < e; ++i) keep[i] = gat_keep(seed, i, thr) ? 1 : 0;
  }, 1 << 16);
  API_END();
}

}  // extern "C"
