// Typed-edge block-diagonal g-SpMM for R-GCN.
//
// Replaces the reference's R-GCN block layer message path
// (examples/pytorch/rgcn/layers.py:121-132): per edge, gather h[src] and the
// relation's block-diagonal weight W[type] (num_blocks blocks of
// in_block x out_block), multiply with torch.bmm into an E x out message
// tensor, then reduce by destination (builtin sum -> incidence SPMV /
// degree bucketing). Here the three steps are one kernel over the
// destination-major CSR and no E x out message tensor is materialised:
//   out[v, b*so + j] = sum over v's slots of norm_e * sum_i h[u, b*si + i] * W[r, b, i, j]
//
// Work items (r04). A row is cut into chunks of DGLHIP_TYPED_CHUNK slots;
// each chunk is one item whose wave(s) run the chain over its slots from
// zero, and a row of several chunks gets out = ((p0 + p1) + p2) ... in chunk
// order (typed_block_combine_kernel). R-GCN's sampled graphs have hub
// entities of ~1,000 in-edges; walked by one wave (r03) such a row set the
// kernel time (0.43 ms per call for a 30,000-edge sample, rocprof,
// profiles/r04/rgcn_step_kernel_stats.csv). A row of at most one chunk is
// the plain slot-order chain, as before. The relation and norm of every slot
// come in slot order (typed_block_spmm gathers them per call), so a slot's
// loads are one dependent step (column id, relation, norm), then the row and
// the weight column; a wave keeps kEdges of them in flight, predicated
// (no serial tail).
//
// The backward runs the same kernel over the transposed CSR with the blocks
// transposed (dH), and dW the same way over the relation-major grouping:
// every weight element a chain over a chunk of its relation's edges
// (relation-major, forward-slot order), the chunks' partials added in order.
// Deterministic, no atomics; the host entry points run the same chains.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_scan.hpp>

#include <cstdlib>
#include <type_traits>

#include "../../include/dgl_hip.h"
#include "common.h"
#include "launch.h"
#include "timing.h"

namespace dglhip {

namespace {

constexpr int64_t kChunk = DGLHIP_TYPED_CHUNK;

// most output slices per wave of the typed-block g-SpMM: 1 by default (one
// wave per 64 outputs); 8 — one wave per item at R-GCN's 500 — ran the
// configs[4] forward at 0.20 ms against 0.12 (r05, fewer waves in flight)
int g_typed_t = 1;

// slots in flight per wave at block width SI (their row and weight values
// in VGPRs: 2 * SI * kEdges of them)
template <int SI>
struct EdgesInFlight {
  static constexpr int value = SI == 0 ? 4 : (SI <= 5 ? 8 : (SI <= 8 ? 4 : 2));
};

// The slot range of item `it` of the chunked rows (item_ptr: a row's first
// item; a row of deg slots has max(1, ceil(deg / kChunk)) items) and where
// its chain goes: the row itself when the row is one item, else the item's
// partial row.
// Items past the last row's (item_row[it] >= num_rows: the caller sized the
// item list by its bound num_rows + nnz / kChunk, no host sync) do nothing.
__device__ __forceinline__ bool item_range(int64_t it, int64_t num_rows,
                                           const int64_t* __restrict__ ptr,
                                           const int64_t* __restrict__ item_ptr,
                                           const int32_t* __restrict__ item_row, int64_t* row,
                                           int64_t* beg, int64_t* end, bool* single) {
  const int64_t r = item_row[it];
  if (r >= num_rows) return false;
  const int64_t first = item_ptr[r], nit = item_ptr[r + 1] - first;
  const int64_t b = ptr[r] + (it - first) * kChunk;
  *row = r;
  *beg = b;
  *end = nit == 1 ? ptr[r + 1] : (b + kChunk < ptr[r + 1] ? b + kChunk : ptr[r + 1]);
  *single = nit == 1;
  return true;
}

// One wave per (item, slice of 64 * T output features): lane l of pass p
// takes outputs p * 64 * T + 64 t + l, t < T (R-GCN's 500 features: T = 8, one
// wave per item; r05 — eight waves per item had each resolved the same slots'
// column, relation and norm, 95k waves of two dependent round trips for a
// 30,000-edge sample). For every output element:
//   m_e = fma chain over i of h[u, b*si+i] * W[r, b, i, j];
//   acc = fma(norm_e, m_e, acc) over the item's slots in slot order
// (the same per-element arithmetic at every T). SI > 0: the block width as a
// compile-time constant; SI == 0: runtime width (T = 1 only).
template <int SI, int T>
__global__ __launch_bounds__(256) void typed_block_spmm_kernel(
    int64_t num_items, int64_t num_rows, int64_t npass, int64_t nb, int64_t si_rt, int64_t so,
    const int64_t* __restrict__ indptr, const int64_t* __restrict__ item_ptr,
    const int32_t* __restrict__ item_row, const int32_t* __restrict__ indices,
    const int32_t* __restrict__ slot_rel, const float* __restrict__ slot_norm,
    const float* __restrict__ ufeat, const float* __restrict__ weight,
    float* __restrict__ out, float* __restrict__ partial) {
  // slots in flight: the T = 1 depths; at T > 1 every slot's T rows and
  // weight columns are loaded per t, so fewer slots per batch
  constexpr int G1 = EdgesInFlight<SI>::value;
  constexpr int G = T == 1 ? G1 : (G1 >= 4 ? 4 : G1);
  const int64_t si = SI > 0 ? SI : si_rt;
  const int64_t wave = block_linear() * (blockDim.x >> 6) +
                       __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int64_t it = wave / npass, pass = wave - it * npass;
  if (it >= num_items) return;
  int64_t row, beg, end;
  bool single;
  if (!item_range(it, num_rows, indptr, item_ptr, item_row, &row, &beg, &end, &single)) return;
  const int lane = threadIdx.x & 63;
  const int64_t Fi = nb * si, Fo = nb * so, wr = nb * si * so;
  int64_t hoff[T], woff[T];
  bool active[T];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int64_t jg = pass * 64 * T + 64 * t + lane;
    active[t] = jg < Fo;
    // idle lanes of the last slice read block 0 (valid addresses) and never store
    const int64_t b = active[t] ? jg / so : 0, j = active[t] ? jg - b * so : 0;
    hoff[t] = b * si;
    woff[t] = b * si * so + j;
  }
  float acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = 0.0f;
  // one batch of up to GB slots from k (slots q >= cnt predicated off: their
  // loads read a valid slot, their products are dropped)
  auto batch = [&](int64_t k, auto gb_tag) {
    constexpr int GB = decltype(gb_tag)::value;
    const int64_t cnt = end - k;  // wave-uniform
    const float* hb[GB];
    const float* wb[GB];
    float nrm[GB];
#pragma unroll
    for (int q = 0; q < GB; ++q) {
      const int64_t kk = q < cnt ? k + q : end - 1;  // a valid slot for idle q
      hb[q] = ufeat + int64_t(indices[kk]) * Fi;
      wb[q] = weight + int64_t(slot_rel[kk]) * wr;
      nrm[q] = slot_norm ? slot_norm[kk] : 1.0f;
    }
#pragma unroll
    for (int t = 0; t < T; ++t) {
      if (SI > 0) {
        float hv[GB][SI > 0 ? SI : 1], wv[GB][SI > 0 ? SI : 1];
#pragma unroll
        for (int q = 0; q < GB; ++q) {
#pragma unroll
          for (int i = 0; i < SI; ++i) {
            hv[q][i] = hb[q][hoff[t] + i];
            wv[q][i] = wb[q][woff[t] + i * so];
          }
        }
#pragma unroll
        for (int q = 0; q < GB; ++q) {
          float m = 0.0f;
#pragma unroll
          for (int i = 0; i < SI; ++i) m = __builtin_fmaf(hv[q][i], wv[q][i], m);
          if (q < cnt) acc[t] = __builtin_fmaf(nrm[q], m, acc[t]);
        }
      } else {
        float m[GB];
#pragma unroll
        for (int q = 0; q < GB; ++q) m[q] = 0.0f;
        for (int64_t i = 0; i < si; ++i) {
#pragma unroll
          for (int q = 0; q < GB; ++q)
            m[q] = __builtin_fmaf(hb[q][hoff[t] + i], wb[q][woff[t] + i * so], m[q]);
        }
#pragma unroll
        for (int q = 0; q < GB; ++q)
          if (q < cnt) acc[t] = __builtin_fmaf(nrm[q], m[q], acc[t]);
      }
    }
  };
  // short batches (most items of a sampled KG hold 1-4 slots) at a quarter
  // or half of the width: a G-wide batch issues its loads for every q, idle
  // or not
  constexpr int G4 = G >= 8 ? G / 4 : (G >= 4 ? G / 2 : G), G2 = G >= 4 ? G / 2 : G;
  for (int64_t k = beg; k < end; k += G) {
    if (end - k <= G4) {
      batch(k, std::integral_constant<int, G4>());
      break;
    }
    if (end - k <= G2) {
      batch(k, std::integral_constant<int, G2>());
      break;
    }
    batch(k, std::integral_constant<int, G>());
  }
  float* dst = single ? out + row * Fo : partial + it * Fo;
#pragma unroll
  for (int t = 0; t < T; ++t)
    if (active[t]) dst[pass * 64 * T + 64 * t + lane] = acc[t];
}

// out[row] = ((p0 + p1) + p2) ... over the row's items in order, for the
// rows (or relations) of several items: one thread per (row, element).
// heavy_row NULL: every row, those of one item skipped.
// row_scale (optional): out[row] = that sum * row_scale[row] (the R-GCN
// layer's 1 / in-degree, one rounding as `agg * norm` has it)
__global__ __launch_bounds__(256) void typed_block_combine_kernel(
    int64_t num_heavy, int64_t F, const int32_t* __restrict__ heavy_row,
    const int64_t* __restrict__ item_ptr, const float* __restrict__ partial,
    float* __restrict__ out, const float* __restrict__ row_scale = nullptr) {
  const int64_t idx = block_linear() * blockDim.x + threadIdx.x;
  if (idx >= num_heavy * F) return;
  const int64_t h = idx / F, f = idx - h * F;
  const int64_t r = heavy_row ? heavy_row[h] : h;
  const int64_t i0 = item_ptr[r], i1 = item_ptr[r + 1];
  if (i1 - i0 <= 1) return;
  float s = partial[i0 * F + f];
  for (int64_t i = i0 + 1; i < i1; ++i) s = s + partial[i * F + f];
  out[r * F + f] = row_scale ? s * row_scale[r] : s;
}

// dW[r, b, i, j] over item `it` (a chunk of relation r's edges, relation-major
// order): sum of norm_e * h[src_e, b*si + i] * dout[dst_e, b*so + j]. One
// thread per (item, weight element of the relation); kEdges edges in flight.
__global__ __launch_bounds__(256) void typed_block_wgrad_kernel(
    int64_t num_items, int64_t num_rels, int64_t nb, int64_t si, int64_t so,
    const int64_t* __restrict__ rel_ptr,
    const int64_t* __restrict__ item_ptr, const int32_t* __restrict__ item_rel,
    const int32_t* __restrict__ rel_src, const int32_t* __restrict__ rel_dst,
    const float* __restrict__ rel_norm, const float* __restrict__ ufeat,
    const float* __restrict__ dout, float* __restrict__ dw, float* __restrict__ partial) {
  constexpr int G = 8;
  const int64_t wr = nb * si * so;
  const int64_t idx = block_linear() * blockDim.x + threadIdx.x;
  if (idx >= num_items * wr) return;
  const int64_t it = idx / wr, rem = idx - it * wr;
  int64_t r, beg, end;
  bool single;
  if (!item_range(it, num_rels, rel_ptr, item_ptr, item_rel, &r, &beg, &end, &single)) return;
  const int64_t b = rem / (si * so), i = (rem / so) % si, j = rem % so;
  const int64_t Fi = nb * si, Fo = nb * so;
  const int64_t xoff = b * si + i, goff = b * so + j;
  float acc = 0.0f;
  for (int64_t k = beg; k < end; k += G) {
    const int64_t cnt = end - k;
    float x[G], g[G], nrm[G];
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const int64_t kk = q < cnt ? k + q : end - 1;
      x[q] = ufeat[int64_t(rel_src[kk]) * Fi + xoff];
      g[q] = dout[int64_t(rel_dst[kk]) * Fo + goff];
      nrm[q] = rel_norm ? rel_norm[kk] : 1.0f;
    }
#pragma unroll
    for (int q = 0; q < G; ++q)
      if (q < cnt) acc = __builtin_fmaf(rel_norm ? nrm[q] * x[q] : x[q], g[q], acc);
  }
  (single ? dw + r * wr : partial + it * wr)[rem] = acc;
}

// ---- Relation-major messages (r06) -----------------------------------------
// The destination-major kernel above loads, per slot and per 64 outputs, the
// source row's si values and the relation's si weight columns: ten 4-byte
// gathers per lane for every slot at R-GCN's 5 x 5 blocks, each weight gather
// spanning ~11 cache lines, and every wave resolves its item and slots before
// the first of them (0.10 ms per call for a 30,000-edge sample against a few
// MB of data). Split in two, with the same per-element arithmetic:
//   messages: one workgroup per item of the relation-major grouping (a chunk
//     of one relation's edges); the relation's weight columns are loaded once
//     into registers (thread t: outputs t + 256 q), PB source rows at a time
//     are staged whole in LDS, and m_e[j] = fma chain over i of
//     row[b*si+i] * W[r, b, i, j] (the chain above, from 0) is stored at the
//     edge's forward slot: msg[slot * Fo + j];
//   sum: the destination-major items as above, but a slot's contribution is
//     one coalesced read of its message row: acc = fma(norm_e, m_e, acc) in
//     slot order, chunked rows' partials combined in chunk order.
// Bits: the same m_e and the same accumulation order as
// typed_block_spmm_kernel, so the same outputs (test_typed_block.py).
constexpr int kMsgRows = 8;  // source rows staged per step of a message workgroup

template <int SI, int QO, int RI>
__global__ __launch_bounds__(256) void typed_block_msg_kernel(
    int64_t num_items, int64_t num_rels, int64_t nb, int64_t so,
    const int64_t* __restrict__ rel_ptr, const int64_t* __restrict__ item_ptr,
    const int32_t* __restrict__ item_rel, const int32_t* __restrict__ pos_row,
    const int64_t* __restrict__ pos_slot, const float* __restrict__ ufeat,
    const float* __restrict__ row_scale, const float* __restrict__ weight, int wtrans,
    float* __restrict__ msg) {
  extern __shared__ float rows[];  // kMsgRows x Fi
  const int64_t it = block_linear();
  if (it >= num_items) return;  // the whole workgroup
  int64_t r, beg, end;
  bool single;
  if (!item_range(it, num_rels, rel_ptr, item_ptr, item_rel, &r, &beg, &end, &single)) return;
  const int t = threadIdx.x;
  const int64_t Fi = nb * SI, Fo = nb * so, wr = nb * SI * so;
  float w[QO][SI];
  int xo[QO];
  bool act[QO];
#pragma unroll
  for (int q = 0; q < QO; ++q) {
    const int64_t j = t + 256 * q;
    act[q] = j < Fo;
    const int64_t b = act[q] ? j / so : 0, jj = act[q] ? j - b * so : 0;
    xo[q] = static_cast<int>(b * SI);
#pragma unroll
    for (int i = 0; i < SI; ++i)  // wtrans: weight is (R, nb, so, SI), read as its transpose
      w[q][i] = weight[r * wr + b * SI * so + (wtrans ? jj * SI + i : i * so + jj)];
  }
  for (int64_t k = beg; k < end; k += kMsgRows) {
    const int64_t cnt = end - k;  // uniform
    float v[kMsgRows][RI];
#pragma unroll
    for (int p = 0; p < kMsgRows; ++p) {
      const int64_t row = pos_row[p < cnt ? k + p : k];  // idle p re-read a valid row
      // a scaled operand row (the backward's dout * norm[dst]) as torch's
      // product rounds it
      const float sc = row_scale ? row_scale[row] : 1.0f;
#pragma unroll
      for (int ri = 0; ri < RI; ++ri) {
        const int64_t f = t + 256 * ri;
        const float x = f < Fi ? ufeat[row * Fi + f] : 0.0f;
        v[p][ri] = row_scale ? x * sc : x;
      }
    }
#pragma unroll
    for (int p = 0; p < kMsgRows; ++p)
#pragma unroll
      for (int ri = 0; ri < RI; ++ri) {
        const int64_t f = t + 256 * ri;
        if (f < Fi) rows[p * Fi + f] = v[p][ri];
      }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < kMsgRows; ++p) {
      if (p < cnt) {
        const int64_t slot = pos_slot[k + p];
        const float* rp = rows + p * Fi;
#pragma unroll
        for (int q = 0; q < QO; ++q) {
          float m = 0.0f;
#pragma unroll
          for (int i = 0; i < SI; ++i) m = __builtin_fmaf(rp[xo[q] + i], w[q][i], m);
          if (act[q]) msg[slot * Fo + t + 256 * q] = m;
        }
      }
    }
    __syncthreads();
  }
}

// out[row] (or the item's partial) = fma(norm_e, msg[mrow(e)], acc) over the
// item's slots in slot order, mrow = slot_map[slot] or the slot itself. One
// wave per (item, 64 * T outputs); G slots' message rows in flight.
template <int T>
__global__ __launch_bounds__(256) void typed_msg_sum_kernel(
    int64_t num_items, int64_t num_rows, int64_t npass, int64_t Fo,
    const int64_t* __restrict__ indptr, const int64_t* __restrict__ item_ptr,
    const int32_t* __restrict__ item_row, const int64_t* __restrict__ slot_map,
    const float* __restrict__ slot_norm, const float* __restrict__ msg,
    const float* __restrict__ row_scale, float* __restrict__ out,
    float* __restrict__ partial) {
  constexpr int G = T >= 4 ? 4 : 8;
  const int64_t wave = block_linear() * (blockDim.x >> 6) +
                       __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int64_t it = wave / npass, pass = wave - it * npass;
  if (it >= num_items) return;
  int64_t row, beg, end;
  bool single;
  if (!item_range(it, num_rows, indptr, item_ptr, item_row, &row, &beg, &end, &single)) return;
  const int lane = threadIdx.x & 63;
  const int64_t f0 = pass * 64 * T + lane;
  float acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = 0.0f;
  auto batch = [&](int64_t k, auto gb_tag) {
    constexpr int GB = decltype(gb_tag)::value;
    const int64_t cnt = end - k;  // wave-uniform
    float mv[GB][T], nrm[GB];
#pragma unroll
    for (int q = 0; q < GB; ++q) {
      const int64_t kk = q < cnt ? k + q : end - 1;  // a valid slot for idle q
      const int64_t mr = slot_map ? slot_map[kk] : kk;
      nrm[q] = slot_norm ? slot_norm[kk] : 1.0f;
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const int64_t f = f0 + 64 * t;
        mv[q][t] = f < Fo ? msg[mr * Fo + f] : 0.0f;
      }
    }
#pragma unroll
    for (int q = 0; q < GB; ++q)
      if (q < cnt)
#pragma unroll
        for (int t = 0; t < T; ++t) acc[t] = __builtin_fmaf(nrm[q], mv[q][t], acc[t]);
  };
  constexpr int G2 = G / 2, G4 = G / 4;
  for (int64_t k = beg; k < end; k += G) {
    if (end - k <= G4) {
      batch(k, std::integral_constant<int, G4>());
      break;
    }
    if (end - k <= G2) {
      batch(k, std::integral_constant<int, G2>());
      break;
    }
    batch(k, std::integral_constant<int, G>());
  }
  float* dst = single ? out + row * Fo : partial + it * Fo;
  const float sc = row_scale && single ? row_scale[row] : 1.0f;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int64_t f = f0 + 64 * t;
    if (f < Fo) dst[f] = row_scale && single ? acc[t] * sc : acc[t];
  }
}

// dW over item `it` as typed_block_wgrad_kernel computes it (the same chain
// per weight element, acc = fma(norm * x, g, acc) in position order), with
// the positions' source and gradient rows staged whole in LDS, kMsgRows at a
// time, instead of two 4-byte gathers per (position, weight element): one
// workgroup per item, thread t owning weight elements t + 256 q.
template <int QW, int RI, int RO>
__global__ __launch_bounds__(256) void typed_block_wgrad_lds_kernel(
    int64_t num_items, int64_t num_rels, int64_t nb, int64_t si, int64_t so,
    const int64_t* __restrict__ rel_ptr, const int64_t* __restrict__ item_ptr,
    const int32_t* __restrict__ item_rel, const int32_t* __restrict__ rel_src,
    const int32_t* __restrict__ rel_dst, const float* __restrict__ rel_norm,
    const float* __restrict__ ufeat, const float* __restrict__ dout,
    const float* __restrict__ dout_scale, float* __restrict__ dw,
    float* __restrict__ partial) {
  extern __shared__ float stage[];  // kMsgRows x Fi source rows, kMsgRows x Fo, kMsgRows norms
  const int64_t it = block_linear();
  if (it >= num_items) return;
  int64_t r, beg, end;
  bool single;
  if (!item_range(it, num_rels, rel_ptr, item_ptr, item_rel, &r, &beg, &end, &single)) return;
  const int t = threadIdx.x;
  const int64_t wr = nb * si * so, Fi = nb * si, Fo = nb * so;
  float* xs = stage;
  float* gs = stage + kMsgRows * Fi;
  float* ns = gs + kMsgRows * Fo;
  int xo[QW], go[QW];
  float acc[QW];
#pragma unroll
  for (int q = 0; q < QW; ++q) {
    const int64_t e = t + 256 * q;
    const int64_t ec = e < wr ? e : 0;
    const int64_t b = ec / (si * so), i = (ec / so) % si, j = ec % so;
    xo[q] = static_cast<int>(b * si + i);
    go[q] = static_cast<int>(b * so + j);
    acc[q] = 0.0f;
  }
  for (int64_t k = beg; k < end; k += kMsgRows) {
    const int64_t cnt = end - k;
    float xv[kMsgRows][RI], gv[kMsgRows][RO];
#pragma unroll
    for (int p = 0; p < kMsgRows; ++p) {
      const int64_t kk = p < cnt ? k + p : k;
      const int64_t s = rel_src[kk], d = rel_dst[kk];
#pragma unroll
      for (int ri = 0; ri < RI; ++ri) {
        const int64_t f = t + 256 * ri;
        xv[p][ri] = f < Fi ? ufeat[s * Fi + f] : 0.0f;
      }
      const float dsc = dout_scale ? dout_scale[d] : 1.0f;
#pragma unroll
      for (int ro = 0; ro < RO; ++ro) {
        const int64_t f = t + 256 * ro;
        const float g = f < Fo ? dout[d * Fo + f] : 0.0f;
        gv[p][ro] = dout_scale ? g * dsc : g;
      }
    }
#pragma unroll
    for (int p = 0; p < kMsgRows; ++p) {
#pragma unroll
      for (int ri = 0; ri < RI; ++ri) {
        const int64_t f = t + 256 * ri;
        if (f < Fi) xs[p * Fi + f] = xv[p][ri];
      }
#pragma unroll
      for (int ro = 0; ro < RO; ++ro) {
        const int64_t f = t + 256 * ro;
        if (f < Fo) gs[p * Fo + f] = gv[p][ro];
      }
    }
    // the batch's norms staged too (read per position below, not one global
    // round trip each)
    if (t < kMsgRows) ns[t] = rel_norm && t < cnt ? rel_norm[k + t] : 1.0f;
    __syncthreads();
    // one position at a time: its 2 * QW LDS reads (unrolled over positions
    // the compiler hoists all of them, 256 VGPRs at QW = 12)
    const int pc = cnt < kMsgRows ? static_cast<int>(cnt) : kMsgRows;
#pragma unroll 1
    for (int p = 0; p < pc; ++p) {
      {
        const float nrm = ns[p];
#pragma unroll
        for (int q = 0; q < QW; ++q) {
          const float x = xs[p * Fi + xo[q]];
          acc[q] = __builtin_fmaf(rel_norm ? nrm * x : x, gs[p * Fo + go[q]], acc[q]);
        }
      }
    }
    __syncthreads();
  }
  float* dst = single ? dw + r * wr : partial + it * wr;
#pragma unroll
  for (int q = 0; q < QW; ++q) {
    const int64_t e = t + 256 * q;
    if (e < wr) dst[e] = acc[q];
  }
}

// 0: the one-kernel forms above; 1 (default): messages + sum, and the
// LDS-staged dW (DGLHIP_TYPED_MESSAGES; dglhip_set_typed_block_messages).
// configs[4] step, r06: forward 0.116 -> 0.078 ms, dH 0.122 -> 0.079, dW
// 0.110 -> 0.063 per layer (gpurun_out rgcn_leg0/1).
int g_typed_msg = -1;

int typed_msg_level() {
  if (g_typed_msg < 0) {
    const char* s = std::getenv("DGLHIP_TYPED_MESSAGES");
    g_typed_msg = s && *s ? std::atoi(s) : 1;
  }
  return g_typed_msg;
}

int round_up_q(int64_t n) {  // 1, 2, 4, 8, 12 or 16 (0: too wide)
  if (n <= 1) return 1;
  if (n <= 2) return 2;
  if (n <= 4) return 4;
  if (n <= 8) return 8;
  if (n <= 12) return 12;
  if (n <= 16) return 16;
  return 0;
}

// DistMult decoder (R-GCN link prediction, the reference's calc_score:
// examples/pytorch/rgcn/link_predict.py:50-55, s = h[s] * w_rel[r] * h[o],
// score = s.sum(1)). One wave per sample: lane l takes features l, l + 64, ...
// (acc + (a * b) * c in feature order), then a xor butterfly over the 64
// lanes. The host entry emulates exactly that association. Indices out of
// range give a NaN score (no host sync to check them; no read out of bounds).
__global__ __launch_bounds__(256) void distmult_score_kernel(
    int64_t n, int64_t F, int64_t num_nodes, int64_t num_rels, const int64_t* __restrict__ s,
    const int64_t* __restrict__ r, const int64_t* __restrict__ o, const float* __restrict__ h,
    const float* __restrict__ w, float* __restrict__ score) {
#pragma clang fp contract(off)
  const int64_t i = block_linear() * 4 +
                    __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  if (i >= n) return;
  const int lane = threadIdx.x & 63;
  const int64_t si = s[i], ri = r[i], oi = o[i];
  if (si < 0 || si >= num_nodes || oi < 0 || oi >= num_nodes || ri < 0 || ri >= num_rels) {
    if (lane == 0) score[i] = __builtin_nanf("");
    return;
  }
  const float* a = h + si * F;
  const float* b = w + ri * F;
  const float* c = h + oi * F;
  float acc = 0.0f;
  for (int64_t f = lane; f < F; f += 64) acc = acc + (a[f] * b[f]) * c[f];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc = acc + __shfl_xor(acc, off, 64);
  if (lane == 0) score[i] = acc;
}

// The decoder's gradients as chains over positions grouped by target row
// (kernel._DistMult: a stable grouping of the index array, rows cut into
// DGLHIP_TYPED_CHUNK-slot items, partials combined in order), each position's
// term computed as torch's autograd of (h[s] * w[r]) * h[o] computes it:
//   task 0 (dh, positions p in [0, 2n)): p < n, subject of sample p:
//            (ds * h[o]) * w[r];  p >= n, object of sample p - n: ds * (h[s] * w[r])
//   task 1 (dw, positions p in [0, n)): (ds * h[o]) * h[s]
// chained acc + term in position order: the bits of kernel.gather_rows'
// backward over those terms (the decoder before r05).
// One wave per (item, slice of 64 * T features). An item holds at most 64
// positions (DGLHIP_TYPED_CHUNK), so lane q first resolves position q — its
// sample, both operand rows, ds — in two dependent round trips for the whole
// item; the batches then only gather rows, at row bases read from lane q
// (wave-uniform), G positions in flight.
static_assert(kChunk == 64, "one position per lane");

// The fused loss's gradient inputs (all null / 0: ds given): ds_i =
// (sigmoid(score_i) - label_i) * (g * inv_n), the BCE-with-logits mean's
// gradient, and the regulariser's term reg_coef * g * base[row] added to
// every output row (base = h for dh, w for dw).
constexpr int64_t kLossChunks = 512;  // blocks summing h^2 (and w^2) in the fused loss

struct LossGrad {
  const float* score;
  const float* labels;
  const float* g;
  float inv_n;
  float reg_coef;
  __device__ __forceinline__ float dscore(int64_t i) const {
    const float x = score[i];
    return (1.0f / (1.0f + expf(-x)) - labels[i]) * (g[0] * inv_n);
  }
  __device__ __forceinline__ float reg_scale() const { return g ? g[0] * reg_coef : 0.0f; }
};
template <int T>
__global__ __launch_bounds__(256) void distmult_grad_kernel(
    int task, int64_t num_items, int64_t num_rows, int64_t npass, int64_t F, int64_t n,
    int64_t num_nodes, int64_t num_rels, const int64_t* __restrict__ ptr,
    const int64_t* __restrict__ item_ptr, const int32_t* __restrict__ item_row,
    const int32_t* __restrict__ order, const int64_t* __restrict__ s,
    const int64_t* __restrict__ r, const int64_t* __restrict__ o,
    const float* __restrict__ ds, const float* __restrict__ h, const float* __restrict__ w,
    float* __restrict__ out, float* __restrict__ partial, const LossGrad lg) {
#pragma clang fp contract(off)
  constexpr int G = 4;
  const int64_t wave = block_linear() * 4 +
                       __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int64_t it = wave / npass, pass = wave - it * npass;
  if (it >= num_items) return;
  int64_t row, beg, end;
  bool single;
  if (!item_range(it, num_rows, ptr, item_ptr, item_row, &row, &beg, &end, &single)) return;
  const int lane = threadIdx.x & 63;
  const int cnt = static_cast<int>(end - beg);  // <= 64, wave-uniform
  // lane q: position beg + q resolved (operand rows as element offsets)
  int64_t xoff = 0, yoff = 0;
  float dq = 0.0f;
  int objq = 0;
  // positions grouped by row: 2n (subjects, then objects) for dh, n for dw;
  // a grouping that points past them (a malformed ptr / order) reads nothing
  // and gives NaN, as an out-of-range id does
  const int64_t m = task == 0 ? 2 * n : n;
  if (lane < cnt) {
    const int64_t k = beg + lane;
    const int64_t p = k >= 0 && k < m ? order[k] : -1;
    const bool inside = p >= 0 && p < m;
    const bool obj = task == 0 && p >= n;
    const int64_t i = obj ? p - n : p;
    const int64_t si = inside ? s[i] : -1, ri = inside ? r[i] : -1, oi = inside ? o[i] : -1;
    const bool ok = inside && si >= 0 && si < num_nodes && oi >= 0 && oi < num_nodes &&
                    ri >= 0 && ri < num_rels;
    dq = ok ? (lg.labels ? lg.dscore(i) : ds[i]) : __builtin_nanf("");
    objq = obj ? 1 : 0;
    xoff = ok ? (obj ? si : oi) * F : 0;
    yoff = ok ? (task == 1 ? si * F : ri * F) : 0;
  }
  const float* ybase = task == 1 ? h : w;
  const int64_t f0 = pass * 64 * T + lane;
  float acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = 0.0f;
  for (int q0 = 0; q0 < cnt; q0 += G) {
    float x[G][T], y[G][T], d[G];
    bool ob[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int q = q0 + g < cnt ? q0 + g : cnt - 1;  // idle slots re-read a valid one
      const int64_t xo = __shfl(xoff, q, 64), yo = __shfl(yoff, q, 64);
      d[g] = __shfl(dq, q, 64);
      ob[g] = __shfl(objq, q, 64) != 0;
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const int64_t f = f0 + 64 * t;
        const int64_t fc = f < F ? f : 0;
        x[g][t] = h[xo + fc];
        y[g][t] = ybase[yo + fc];
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (q0 + g < cnt) {
#pragma unroll
        for (int t = 0; t < T; ++t)
          acc[t] = acc[t] + (ob[g] ? d[g] * (x[g][t] * y[g][t]) : (d[g] * x[g][t]) * y[g][t]);
      }
    }
  }
  float* dst = single ? out + row * F : partial + it * F;
  // the regulariser's term on rows of one item (chunked rows: at the combine)
  const float rc = single ? lg.reg_scale() : 0.0f;
  const float* base = task == 0 ? h : w;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int64_t f = f0 + 64 * t;
    if (f < F) dst[f] = lg.reg_coef != 0.0f && single ? acc[t] + rc * base[row * F + f] : acc[t];
  }
}

// out[row] = ((p0 + p1) + ...) over the row's items, + the regulariser's term
// (DistMult loss gradient, rows of several items)
__global__ __launch_bounds__(256) void distmult_combine_kernel(
    int64_t num_rows, int64_t F, const int64_t* __restrict__ item_ptr,
    const float* __restrict__ partial, const float* __restrict__ base, const LossGrad lg,
    float* __restrict__ out) {
  const int64_t idx = block_linear() * blockDim.x + threadIdx.x;
  if (idx >= num_rows * F) return;
  const int64_t r = idx / F, f = idx - r * F;
  const int64_t i0 = item_ptr[r], i1 = item_ptr[r + 1];
  if (i1 - i0 <= 1) return;
  float s = partial[i0 * F + f];
  for (int64_t i = i0 + 1; i < i1; ++i) s = s + partial[i * F + f];
  out[r * F + f] = lg.reg_coef != 0.0f ? s + lg.reg_scale() * base[r * F + f] : s;
}

// The link-prediction loss of the R-GCN example in two launches
// (examples/pytorch/rgcn/link_predict.py get_loss: BCE-with-logits of the
// DistMult scores, mean over the samples, + reg * (mean(h^2) + mean(w^2))):
// partials — blocks [0, nb_s): 4 samples each, a wave per sample scoring it
// as distmult_score_kernel does (the same bits) and its BCE term; blocks
// [nb_s, nb_s + nb_h): sums of h^2 over contiguous chunks; then the w^2
// chunks — then one block adding each kind's partials in block order.
__device__ __forceinline__ float bce_with_logits(float x, float y) {
  // (1 - y) * x + log(1 + exp(-x)), stably: max(x, 0) - x * y + log1p(exp(-|x|))
  return fmaxf(x, 0.0f) - x * y + log1pf(expf(-fabsf(x)));
}

__device__ __forceinline__ float block_sum_256(float v, float* red) {
  // a fixed tree: the same order at every call
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = v + __shfl_xor(v, off, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  const float s = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return s;
}

__global__ __launch_bounds__(256) void distmult_loss_partials_kernel(
    int64_t n, int64_t F, int64_t num_nodes, int64_t num_rels, const int64_t* __restrict__ s,
    const int64_t* __restrict__ r, const int64_t* __restrict__ o, const float* __restrict__ h,
    const float* __restrict__ w, const float* __restrict__ labels, int64_t nb_s, int64_t nb_h,
    int64_t nb_w, float* __restrict__ score, float* __restrict__ partial) {
  __shared__ float red[4];
  const int64_t b = block_linear();
  const int lane = threadIdx.x & 63;
  float v = 0.0f;
  if (b < nb_s) {
    const int64_t i = b * 4 + (threadIdx.x >> 6);
    if (i < n) {
      const int64_t si = s[i], ri = r[i], oi = o[i];
      float sc;
      if (si < 0 || si >= num_nodes || oi < 0 || oi >= num_nodes || ri < 0 || ri >= num_rels) {
        sc = __builtin_nanf("");
      } else {
#pragma clang fp contract(off)
        const float* a = h + si * F;
        const float* bb = w + ri * F;
        const float* c = h + oi * F;
        float acc = 0.0f;
        for (int64_t f = lane; f < F; f += 64) acc = acc + (a[f] * bb[f]) * c[f];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) acc = acc + __shfl_xor(acc, off, 64);
        sc = acc;
      }
      if (lane == 0) {
        score[i] = sc;
        v = bce_with_logits(sc, labels[i]);
      }
    }
  } else {
    const bool hb = b < nb_s + nb_h;
    const float* x = hb ? h : w;
    const int64_t elems = hb ? num_nodes * F : num_rels * F;
    const int64_t nbk = hb ? nb_h : nb_w, k = hb ? b - nb_s : b - nb_s - nb_h;
    const int64_t chunk = (elems + nbk - 1) / nbk;
    const int64_t e0 = k * chunk, e1 = e0 + chunk < elems ? e0 + chunk : elems;
    for (int64_t e = e0 + threadIdx.x; e < e1; e += 256) v = __builtin_fmaf(x[e], x[e], v);
  }
  const float tot = block_sum_256(v, red);
  if (threadIdx.x == 0) partial[b] = tot;
}

__global__ __launch_bounds__(256) void distmult_loss_final_kernel(
    int64_t n, int64_t h_elems, int64_t w_elems, int64_t nb_s, int64_t nb_h, int64_t nb_w,
    float reg, const float* __restrict__ partial, float* __restrict__ loss) {
  __shared__ float red[4];
  float sums[3];
  const int64_t beg[3] = {0, nb_s, nb_s + nb_h}, cnt[3] = {nb_s, nb_h, nb_w};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float v = 0.0f;
    for (int64_t j = threadIdx.x; j < cnt[k]; j += 256) v = v + partial[beg[k] + j];
    sums[k] = block_sum_256(v, red);
  }
  if (threadIdx.x == 0)
    loss[0] = sums[0] / float(n) +
              reg * (sums[1] / float(h_elems > 0 ? h_elems : 1) +
                     sums[2] / float(w_elems > 0 ? w_elems : 1));
}

// The chunked item list (kernel._typed_items): items per row, scanned by
// rocPRIM, then every item index's row by a binary search of item_ptr.
__global__ __launch_bounds__(256) void typed_nitems_kernel(int64_t num_rows,
                                                           const int64_t* __restrict__ ptr,
                                                           int64_t* __restrict__ nit) {
  const int64_t r = block_linear() * blockDim.x + threadIdx.x;
  if (r >= num_rows) return;
  const int64_t deg = ptr[r + 1] - ptr[r];
  const int64_t c = (deg + kChunk - 1) / kChunk;
  nit[r] = c > 1 ? c : 1;
}

__global__ __launch_bounds__(256) void typed_item_rows_kernel(
    int64_t num_rows, int64_t bound, const int64_t* __restrict__ item_ptr,
    int32_t* __restrict__ item_row) {
  const int64_t j = block_linear() * blockDim.x + threadIdx.x;
  if (j >= bound) return;
  // the row r with item_ptr[r] <= j < item_ptr[r + 1]; num_rows past the last
  int64_t lo = 0, hi = num_rows;  // answer in [lo, hi]
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (item_ptr[mid] <= j) lo = mid;
    else hi = mid - 1;
  }
  item_row[j] = static_cast<int32_t>(lo);
}

size_t typed_items_scan_bytes(int64_t num_rows) {
  size_t bytes = 0;
  HIP_CALL(rocprim::inclusive_scan(nullptr, bytes, static_cast<const int64_t*>(nullptr),
                                   static_cast<int64_t*>(nullptr), size_t(num_rows),
                                   rocprim::plus<int64_t>()));
  return bytes;
}

}  // namespace
}  // namespace dglhip

using namespace dglhip;

extern "C" {

int dglhip_typed_block_spmm_device(int64_t num_rows, int64_t num_items, int64_t num_blocks,
                                   int64_t in_block, int64_t out_block, const int64_t* indptr,
                                   const int64_t* item_ptr, const int32_t* item_row,
                                   int64_t num_heavy, const int32_t* heavy_row,
                                   const int32_t* indices, const int32_t* slot_rel,
                                   const float* slot_norm, const float* ufeat,
                                   const float* weight, float* out, float* partial,
                                   void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows >= 0 && num_items >= 0 && num_heavy >= 0 && num_blocks > 0 &&
               in_block > 0 && out_block > 0, "bad sizes");
  const int64_t Fo = num_blocks * out_block;
  if (num_rows == 0) return 0;
  DGLHIP_CHECK(indptr && item_ptr && item_row && indices && slot_rel && ufeat && weight && out,
               "null pointer argument");
  DGLHIP_CHECK(num_heavy == 0 || partial, "chunked rows need their partials");
  // outputs per lane: a wave covers up to 64 * T of them, T capped by
  // g_typed_t (the study knob dglhip_set_typed_block_width; default 1)
  const int64_t n64 = (Fo + 63) / 64;
  int T = n64 >= 8 ? 8 : (n64 >= 4 ? 4 : (n64 >= 2 ? 2 : 1));
  if (T > g_typed_t) T = g_typed_t;
  const bool known = in_block == 1 || in_block == 2 || in_block == 4 || in_block == 5 ||
                     in_block == 8 || in_block == 16;
  if (!known || in_block > 8) T = 1;
  const int64_t npass = (Fo + 64 * T - 1) / (64 * T);
  const int64_t waves = num_items * npass;
  DGLHIP_CHECK((waves + 3) / 4 <= 0x7fffffff, "grid too large");
  const dim3 grid = grid_1d((waves + 3) / 4), block(256);
#define DGLHIP_TB(S, TT)                                                                      \
  hipLaunchKernelGGL((typed_block_spmm_kernel<S, TT>), grid, block, 0, stream, num_items,      \
                     num_rows, npass, num_blocks, in_block, out_block, indptr, item_ptr,       \
                     item_row, indices, slot_rel, slot_norm, ufeat, weight, out, partial)
#define DGLHIP_TBT(S)                       \
  switch (T) {                              \
    case 8: DGLHIP_TB(S, 8); break;         \
    case 4: DGLHIP_TB(S, 4); break;         \
    case 2: DGLHIP_TB(S, 2); break;         \
    default: DGLHIP_TB(S, 1); break;        \
  }
  timed_launch(stream, [&] {
    switch (in_block) {
      case 1: DGLHIP_TBT(1); break;
      case 2: DGLHIP_TBT(2); break;
      case 4: DGLHIP_TBT(4); break;
      case 5: DGLHIP_TBT(5); break;
      case 8: DGLHIP_TBT(8); break;
      case 16: DGLHIP_TB(16, 1); break;
      default: DGLHIP_TB(0, 1); break;
    }
  });
#undef DGLHIP_TBT
#undef DGLHIP_TB
  if (num_heavy > 0) {
    const int64_t total = num_heavy * Fo;
    timed_launch(stream, [&] {
      hipLaunchKernelGGL(typed_block_combine_kernel, grid_1d((total + 255) / 256), dim3(256), 0,
                         stream, num_heavy, Fo, heavy_row, item_ptr, partial, out);
    });
  }
  API_END();
}

int dglhip_typed_block_msg_ok(int64_t num_blocks, int64_t in_block, int64_t out_block) {
  const bool known = in_block == 1 || in_block == 2 || in_block == 4 || in_block == 5 ||
                     in_block == 8 || in_block == 16;
  return typed_msg_level() >= 1 && known && num_blocks > 0 && out_block > 0 &&
                 num_blocks * in_block <= 1024 && num_blocks * out_block <= 1024
             ? 1
             : 0;
}

int dglhip_set_typed_block_messages(int on) {
  g_typed_msg = on ? 1 : 0;
  return 0;
}

int dglhip_typed_block_msg_device(int64_t num_rels, int64_t num_items, int64_t num_blocks,
                                  int64_t in_block, int64_t out_block, const int64_t* rel_ptr,
                                  const int64_t* item_ptr, const int32_t* item_rel,
                                  const int32_t* pos_row, const int64_t* pos_slot,
                                  const float* ufeat, const float* row_scale,
                                  const float* weight, int weight_transposed, float* msg,
                                  void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rels >= 0 && num_items >= 0 && num_blocks > 0 && in_block > 0 &&
                   out_block > 0, "bad sizes");
  const int64_t Fi = num_blocks * in_block, Fo = num_blocks * out_block;
  DGLHIP_CHECK(Fi <= 1024 && Fo <= 1024, "message rows of " << Fi << " -> " << Fo
                                                             << " features: at most 1024");
  if (num_rels == 0 || num_items == 0) return 0;
  DGLHIP_CHECK(rel_ptr && item_ptr && item_rel && pos_row && pos_slot && ufeat && weight && msg,
               "null pointer argument");
  DGLHIP_CHECK(num_items <= 0x7fffffff, "grid too large");
  const int Q = (Fi > 512 || Fo > 512) ? 4 : 2;
  const size_t lds = size_t(kMsgRows) * size_t(Fi) * sizeof(float);
#define DGLHIP_MSG(S, QQ)                                                                     \
  hipLaunchKernelGGL((typed_block_msg_kernel<S, QQ, QQ>), grid_1d(num_items), dim3(256), lds, \
                     stream, num_items, num_rels, num_blocks, out_block, rel_ptr, item_ptr,   \
                     item_rel, pos_row, pos_slot, ufeat, row_scale, weight,                  \
                     weight_transposed, msg)
#define DGLHIP_MSGQ(S)                 \
  if (Q == 4) DGLHIP_MSG(S, 4);        \
  else DGLHIP_MSG(S, 2);
  timed_launch(stream, [&] {
    switch (in_block) {
      case 1: DGLHIP_MSGQ(1); break;
      case 2: DGLHIP_MSGQ(2); break;
      case 4: DGLHIP_MSGQ(4); break;
      case 5: DGLHIP_MSGQ(5); break;
      case 8: DGLHIP_MSGQ(8); break;
      case 16: DGLHIP_MSGQ(16); break;
      default: DGLHIP_CHECK(false, "message kernel for block width " << in_block);
    }
  });
#undef DGLHIP_MSGQ
#undef DGLHIP_MSG
  API_END();
}

int dglhip_typed_msg_sum_device(int64_t num_rows, int64_t num_items, int64_t feat_len,
                                const int64_t* indptr, const int64_t* item_ptr,
                                const int32_t* item_row, int64_t num_heavy,
                                const int32_t* heavy_row, const int64_t* slot_map,
                                const float* slot_norm, const float* msg,
                                const float* row_scale, float* out, float* partial,
                                void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows >= 0 && num_items >= 0 && num_heavy >= 0 && feat_len > 0, "bad sizes");
  if (num_rows == 0) return 0;
  DGLHIP_CHECK(indptr && item_ptr && item_row && msg && out, "null pointer argument");
  DGLHIP_CHECK(num_heavy == 0 || partial, "chunked rows need their partials");
  const int64_t n64 = (feat_len + 63) / 64;
  const int T = n64 >= 8 ? 8 : (n64 >= 4 ? 4 : (n64 >= 2 ? 2 : 1));
  const int64_t npass = (feat_len + 64 * T - 1) / (64 * T);
  const int64_t waves = num_items * npass;
  DGLHIP_CHECK((waves + 3) / 4 <= 0x7fffffff, "grid too large");
#define DGLHIP_MS(TT)                                                                           \
  hipLaunchKernelGGL((typed_msg_sum_kernel<TT>), grid_1d((waves + 3) / 4), dim3(256), 0, stream, \
                     num_items, num_rows, npass, feat_len, indptr, item_ptr, item_row, slot_map,  \
                     slot_norm, msg, row_scale, out, partial)
  timed_launch(stream, [&] {
    switch (T) {
      case 8: DGLHIP_MS(8); break;
      case 4: DGLHIP_MS(4); break;
      case 2: DGLHIP_MS(2); break;
      default: DGLHIP_MS(1); break;
    }
  });
#undef DGLHIP_MS
  if (num_heavy > 0) {
    const int64_t total = num_heavy * feat_len;
    timed_launch(stream, [&] {
      hipLaunchKernelGGL(typed_block_combine_kernel, grid_1d((total + 255) / 256), dim3(256), 0,
                         stream, num_heavy, feat_len, heavy_row, item_ptr, partial, out,
                         row_scale);
    });
  }
  API_END();
}

int dglhip_typed_block_wgrad_scaled_device(int64_t num_rels, int64_t num_items,
                                           int64_t num_blocks, int64_t in_block,
                                           int64_t out_block, const int64_t* rel_ptr,
                                           const int64_t* item_ptr, const int32_t* item_rel,
                                           int64_t num_heavy, const int32_t* heavy_rel,
                                           const int32_t* rel_src, const int32_t* rel_dst,
                                           const float* rel_norm, const float* ufeat,
                                           const float* dout, const float* dout_scale,
                                           float* dweight, float* partial, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rels >= 0 && num_items >= 0 && num_heavy >= 0 && num_blocks >= 0 &&
               in_block >= 0 && out_block >= 0, "bad sizes");
  const int64_t wr = num_blocks * in_block * out_block;
  if (num_rels == 0 || wr == 0) return 0;
  DGLHIP_CHECK(rel_ptr && item_ptr && item_rel && ufeat && dout && dweight,
               "null pointer argument");
  DGLHIP_CHECK(num_heavy == 0 || partial, "chunked relations need their partials");
  const int64_t total = num_items * wr;
  DGLHIP_CHECK((total + 255) / 256 <= 0x7fffffff, "grid too large");
  const int64_t Fi = num_blocks * in_block, Fo = num_blocks * out_block;
  const int qw = round_up_q((wr + 255) / 256);
  if (typed_msg_level() >= 1 && qw > 0 && Fi <= 1024 && Fo <= 1024 && rel_src && rel_dst) {
    // staged rows (r06): one workgroup per item
    const int R = (Fi > 512 || Fo > 512) ? 4 : 2;
    const size_t lds = size_t(kMsgRows) * size_t(Fi + Fo + 1) * sizeof(float);
#define DGLHIP_WG(QQ, RR)                                                                        \
  hipLaunchKernelGGL((typed_block_wgrad_lds_kernel<QQ, RR, RR>), grid_1d(num_items), dim3(256),   \
                     lds, stream, num_items, num_rels, num_blocks, in_block, out_block, rel_ptr, \
                     item_ptr, item_rel, rel_src, rel_dst, rel_norm, ufeat, dout, dout_scale,    \
                     dweight, partial)
#define DGLHIP_WGR(QQ)             \
  if (R == 4) DGLHIP_WG(QQ, 4);    \
  else DGLHIP_WG(QQ, 2);
    timed_launch(stream, [&] {
      switch (qw) {
        case 1: DGLHIP_WGR(1); break;
        case 2: DGLHIP_WGR(2); break;
        case 4: DGLHIP_WGR(4); break;
        case 8: DGLHIP_WGR(8); break;
        case 12: DGLHIP_WGR(12); break;
        default: DGLHIP_WGR(16); break;
      }
    });
#undef DGLHIP_WGR
#undef DGLHIP_WG
  } else {
    DGLHIP_CHECK(dout_scale == nullptr, "a scaled dout needs the staged weight gradient");
    timed_launch(stream, [&] {
      hipLaunchKernelGGL(typed_block_wgrad_kernel, grid_1d((total + 255) / 256), dim3(256), 0,
                         stream, num_items, num_rels, num_blocks, in_block, out_block, rel_ptr,
                         item_ptr, item_rel, rel_src, rel_dst, rel_norm, ufeat, dout, dweight,
                         partial);
    });
  }
  if (num_heavy > 0) {
    const int64_t t2 = num_heavy * wr;
    timed_launch(stream, [&] {
      hipLaunchKernelGGL(typed_block_combine_kernel, grid_1d((t2 + 255) / 256), dim3(256), 0,
                         stream, num_heavy, wr, heavy_rel, item_ptr, partial, dweight);
    });
  }
  API_END();
}

int dglhip_typed_block_wgrad_device(int64_t num_rels, int64_t num_items, int64_t num_blocks,
                                    int64_t in_block, int64_t out_block, const int64_t* rel_ptr,
                                    const int64_t* item_ptr, const int32_t* item_rel,
                                    int64_t num_heavy, const int32_t* heavy_rel,
                                    const int32_t* rel_src, const int32_t* rel_dst,
                                    const float* rel_norm, const float* ufeat, const float* dout,
                                    float* dweight, float* partial, void* stream_) {
  return dglhip_typed_block_wgrad_scaled_device(num_rels, num_items, num_blocks, in_block,
                                                out_block, rel_ptr, item_ptr, item_rel,
                                                num_heavy, heavy_rel, rel_src, rel_dst, rel_norm,
                                                ufeat, dout, nullptr, dweight, partial, stream_);
}

int64_t dglhip_typed_items_workspace_bytes(int64_t num_rows) {
  try {
    if (num_rows <= 0) return 0;
    return ((num_rows * 8 + 255) & ~int64_t(255)) + int64_t(typed_items_scan_bytes(num_rows));
  } catch (const std::exception& e) {
    set_last_error(e.what());
    return -1;
  }
}

int dglhip_typed_items_device(int64_t num_rows, const int64_t* ptr, int64_t bound,
                              int64_t* item_ptr, int32_t* item_row, void* workspace,
                              int64_t workspace_bytes, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_rows >= 0 && bound >= num_rows, "bad sizes");
  DGLHIP_CHECK(item_ptr, "null pointer argument");
  HIP_CALL(hipMemsetAsync(item_ptr, 0, sizeof(int64_t), stream));
  if (num_rows == 0) {
    if (bound > 0) {
      hipLaunchKernelGGL(typed_item_rows_kernel, grid_1d((bound + 255) / 256), dim3(256), 0,
                         stream, num_rows, bound, item_ptr, item_row);
    }
    return 0;
  }
  DGLHIP_CHECK(ptr && item_row && workspace, "null pointer argument");
  const int64_t need = dglhip_typed_items_workspace_bytes(num_rows);
  DGLHIP_CHECK(workspace_bytes >= need, "workspace of " << workspace_bytes << " B, "
                                                        << need << " needed");
  char* ws = static_cast<char*>(workspace);
  int64_t* nit = reinterpret_cast<int64_t*>(ws);
  const int64_t nb = (num_rows * 8 + 255) & ~int64_t(255);
  size_t tmp = size_t(workspace_bytes - nb);
  hipLaunchKernelGGL(typed_nitems_kernel, grid_1d((num_rows + 255) / 256), dim3(256), 0, stream,
                     num_rows, ptr, nit);
  HIP_CALL(hipGetLastError());
  HIP_CALL(rocprim::inclusive_scan(ws + nb, tmp, static_cast<const int64_t*>(nit), item_ptr + 1,
                                   size_t(num_rows), rocprim::plus<int64_t>(), stream));
  hipLaunchKernelGGL(typed_item_rows_kernel, grid_1d((bound + 255) / 256), dim3(256), 0, stream,
                     num_rows, bound, item_ptr, item_row);
  HIP_CALL(hipGetLastError());
  API_END();
}

int dglhip_set_typed_block_width(int slices) {
  API_BEGIN();
  DGLHIP_CHECK(slices == 1 || slices == 2 || slices == 4 || slices == 8,
               "typed-block width must be 1, 2, 4 or 8 slices, got " << slices);
  g_typed_t = slices;
  API_END();
}

int dglhip_distmult_score_device(int64_t num_samples, int64_t feat_len, int64_t num_nodes,
                                 int64_t num_rels, const int64_t* subj, const int64_t* rel,
                                 const int64_t* obj, const float* h, const float* w_rel,
                                 float* score, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_samples >= 0 && feat_len >= 0 && num_nodes >= 0 && num_rels >= 0,
               "bad sizes");
  if (num_samples == 0) return 0;
  DGLHIP_CHECK(subj && rel && obj && h && w_rel && score, "null pointer argument");
  timed_launch(stream, [&] {
    hipLaunchKernelGGL(distmult_score_kernel, grid_1d((num_samples + 3) / 4), dim3(256), 0,
                       stream, num_samples, feat_len, num_nodes, num_rels, subj, rel, obj, h,
                       w_rel, score);
  });
  API_END();
}

}  // extern "C"

namespace dglhip {
namespace {

int distmult_grad_launch(int task, int64_t num_rows, int64_t num_items, int64_t feat_len,
                         int64_t num_samples, int64_t num_nodes, int64_t num_rels,
                         const int64_t* ptr, const int64_t* item_ptr, const int32_t* item_row,
                         const int32_t* order, const int64_t* subj, const int64_t* rel,
                         const int64_t* obj, const float* dscore, const LossGrad& lg,
                         const float* h, const float* w_rel, float* out, float* partial,
                         hipStream_t stream) {
  DGLHIP_CHECK(task == 0 || task == 1, "unknown DistMult gradient task " << task);
  DGLHIP_CHECK(num_rows >= 0 && num_items >= 0 && feat_len >= 0 && num_samples >= 0,
               "bad sizes");
  if (num_rows == 0 || feat_len == 0) return 0;
  DGLHIP_CHECK(ptr && item_ptr && item_row && out && partial, "null pointer argument");
  DGLHIP_CHECK(num_samples == 0 || (order && subj && rel && obj && (dscore || lg.labels) && h &&
                                    w_rel),
               "null pointer argument");
  DGLHIP_CHECK(!lg.labels || (lg.score && lg.g), "loss gradient without scores or its scale");
  // features per lane: up to 8 (F = 500: one wave covers the row)
  const int64_t lanes64 = (feat_len + 63) / 64;
  const int T = lanes64 >= 8 ? 8 : (lanes64 >= 4 ? 4 : (lanes64 >= 2 ? 2 : 1));
  const int64_t npass = (feat_len + 64 * T - 1) / (64 * T);
  const int64_t waves = num_items * npass;
  DGLHIP_CHECK((waves + 3) / 4 <= 0x7fffffff, "grid too large");
#define DGLHIP_DM(TT)                                                                       \
  hipLaunchKernelGGL(distmult_grad_kernel<TT>, grid_1d((waves + 3) / 4), dim3(256), 0, stream, \
                     task, num_items, num_rows, npass, feat_len, num_samples, num_nodes,      \
                     num_rels, ptr, item_ptr, item_row, order, subj, rel, obj, dscore, h,     \
                     w_rel, out, partial, lg)
  timed_launch(stream, [&] {
    switch (T) {
      case 8: DGLHIP_DM(8); break;
      case 4: DGLHIP_DM(4); break;
      case 2: DGLHIP_DM(2); break;
      default: DGLHIP_DM(1); break;
    }
  });
#undef DGLHIP_DM
  const int64_t total = num_rows * feat_len;
  timed_launch(stream, [&] {
    if (lg.reg_coef != 0.0f)
      hipLaunchKernelGGL(distmult_combine_kernel, grid_1d((total + 255) / 256), dim3(256), 0,
                         stream, num_rows, feat_len, item_ptr, partial, task == 0 ? h : w_rel,
                         lg, out);
    else
      hipLaunchKernelGGL(typed_block_combine_kernel, grid_1d((total + 255) / 256), dim3(256), 0,
                         stream, num_rows, feat_len, nullptr, item_ptr, partial, out);
  });
  return 0;
}

}  // namespace
}  // namespace dglhip

extern "C" {

int dglhip_distmult_grad_device(int task, int64_t num_rows, int64_t num_items, int64_t feat_len,
                                int64_t num_samples, int64_t num_nodes, int64_t num_rels,
                                const int64_t* ptr, const int64_t* item_ptr,
                                const int32_t* item_row, const int32_t* order,
                                const int64_t* subj, const int64_t* rel, const int64_t* obj,
                                const float* dscore, const float* h, const float* w_rel,
                                float* out, float* partial, void* stream_) {
  API_BEGIN();
  const LossGrad lg{nullptr, nullptr, nullptr, 0.0f, 0.0f};
  distmult_grad_launch(task, num_rows, num_items, feat_len, num_samples, num_nodes, num_rels,
                       ptr, item_ptr, item_row, order, subj, rel, obj, dscore, lg, h, w_rel, out,
                       partial, static_cast<hipStream_t>(stream_));
  API_END();
}

int64_t dglhip_distmult_loss_workspace_floats(int64_t num_samples, int64_t num_nodes,
                                              int64_t num_rels, int64_t feat_len) {
  (void)num_nodes;
  (void)num_rels;
  (void)feat_len;
  return (num_samples + 3) / 4 + 2 * kLossChunks;
}

int dglhip_distmult_loss_fwd_device(int64_t num_samples, int64_t feat_len, int64_t num_nodes,
                                    int64_t num_rels, const int64_t* subj, const int64_t* rel,
                                    const int64_t* obj, const float* h, const float* w_rel,
                                    const float* labels, float reg, float* score, float* loss,
                                    float* workspace, int64_t workspace_floats, void* stream_) {
  API_BEGIN();
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  DGLHIP_CHECK(num_samples > 0 && feat_len > 0 && num_nodes > 0 && num_rels > 0, "bad sizes");
  DGLHIP_CHECK(subj && rel && obj && h && w_rel && labels && score && loss && workspace,
               "null pointer argument");
  const int64_t nb_s = (num_samples + 3) / 4, nb_h = kLossChunks, nb_w = kLossChunks;
  DGLHIP_CHECK(workspace_floats >= nb_s + nb_h + nb_w, "workspace too small");
  timed_launch(stream, [&] {
    hipLaunchKernelGGL(distmult_loss_partials_kernel, grid_1d(nb_s + nb_h + nb_w), dim3(256), 0,
                       stream, num_samples, feat_len, num_nodes, num_rels, subj, rel, obj, h,
                       w_rel, labels, nb_s, nb_h, nb_w, score, workspace);
  });
  timed_launch(stream, [&] {
    hipLaunchKernelGGL(distmult_loss_final_kernel, dim3(1), dim3(256), 0, stream, num_samples,
                       num_nodes * feat_len, num_rels * feat_len, nb_s, nb_h, nb_w, reg,
                       workspace, loss);
  });
  API_END();
}

int dglhip_distmult_loss_grad_device(int task, int64_t num_rows, int64_t num_items,
                                     int64_t feat_len, int64_t num_samples, int64_t num_nodes,
                                     int64_t num_rels, const int64_t* ptr, const int64_t* item_ptr,
                                     const int32_t* item_row, const int32_t* order,
                                     const int64_t* subj, const int64_t* rel, const int64_t* obj,
                                     const float* score, const float* labels, const float* g,
                                     float reg, const float* h, const float* w_rel, float* out,
                                     float* partial, void* stream_) {
  API_BEGIN();
  DGLHIP_CHECK(score && labels && g, "null pointer argument");
  const int64_t elems = (task == 0 ? num_nodes : num_rels) * feat_len;
  // d/dx of reg * mean(x^2): 2 * reg / elems * x
  const LossGrad lg{score, labels, g, 1.0f / float(num_samples > 0 ? num_samples : 1),
                    elems > 0 ? 2.0f * reg / float(elems) : 0.0f};
  distmult_grad_launch(task, num_rows, num_items, feat_len, num_samples, num_nodes, num_rels,
                       ptr, item_ptr, item_row, order, subj, rel, obj, nullptr, lg, h, w_rel,
                       out, partial, static_cast<hipStream_t>(stream_));
  API_END();
}

}  // extern "C"
