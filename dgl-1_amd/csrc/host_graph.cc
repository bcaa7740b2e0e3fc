// Host-side graph ingestion and the CPU device of the engine.
//
//  * COO -> CSR with the slot order the reference's sparse product consumes
//    (replaces Graph::GetAdj, src/graph/graph.cc:506-554, and the CSR built by
//    ImmutableGraph, src/graph/immutable_graph.cc:206-237).
//  * degree-descending launch schedule.
//  * g-SpMM / g-SDDMM on host memory (same numerics contract as the HIP
//    kernels; this is the CPU device, not the test oracle in oracle/).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>
#include <numeric>

#include "../../include/dgl_hip.h"
#include "common.h"

namespace dglhip {

static thread_local std::string g_last_error;

void set_last_error(const std::string& msg) { g_last_error = msg; }

int default_num_threads() {
  for (const char* var : {"DGL_NUM_THREADS", "OMP_NUM_THREADS"}) {
    if (const char* s = std::getenv(var)) {
      int v = std::atoi(s);
      if (v > 0) return std::min(v, 64);
    }
  }
  unsigned hc = std::thread::hardware_concurrency();
  return static_cast<int>(std::max(1u, std::min(hc, 64u)));
}

// Stable counting sort of edges by row. Parallel version: rows are split into
// contiguous ranges of roughly equal nnz; each thread scans the edge list in
// edge-id order and places only the edges of its own row range, so slot order
// inside each row is ascending edge id regardless of thread count.
static void csr_by_eid(int64_t num_rows, int64_t nnz, const int64_t* row,
                       const int64_t* col, int64_t* indptr, int32_t* indices,
                       int64_t* eid, int nthreads) {
  std::vector<int64_t> deg(num_rows + 1, 0);
  for (int64_t e = 0; e < nnz; ++e) deg[row[e]]++;
  indptr[0] = 0;
  for (int64_t r = 0; r < num_rows; ++r) indptr[r + 1] = indptr[r] + deg[r];
  if (nnz == 0) return;
  if (nthreads > 1 && nnz >= (int64_t(1) << 20)) {
    // row-range boundaries balanced by nnz
    std::vector<int64_t> bounds(nthreads + 1, num_rows);
    bounds[0] = 0;
    for (int t = 1; t < nthreads; ++t) {
      const int64_t target = nnz * t / nthreads;
      bounds[t] = std::upper_bound(indptr, indptr + num_rows + 1, target) -
                  indptr - 1;
      bounds[t] = std::max(bounds[t], bounds[t - 1]);
    }
    parallel_for(nthreads, nthreads, [&](int64_t b, int64_t e, int) {
      for (int64_t t = b; t < e; ++t) {
        const int64_t r0 = bounds[t], r1 = bounds[t + 1];
        if (r0 >= r1) continue;
        std::vector<int64_t> cursor(indptr + r0, indptr + r1);
        for (int64_t i = 0; i < nnz; ++i) {
          const int64_t r = row[i];
          if (r < r0 || r >= r1) continue;
          const int64_t p = cursor[r - r0]++;
          indices[p] = static_cast<int32_t>(col[i]);
          eid[p] = i;
        }
      }
    }, 2);  // one item = one thread's whole row range
  } else {
    std::vector<int64_t> cursor(indptr, indptr + num_rows);
    for (int64_t i = 0; i < nnz; ++i) {
      const int64_t p = cursor[row[i]]++;
      indices[p] = static_cast<int32_t>(col[i]);
      eid[p] = i;
    }
  }
}

}  // namespace dglhip

using namespace dglhip;

extern "C" {

const char* DGLGetLastError(void) { return g_last_error.c_str(); }
void DGLAPISetLastError(const char* msg) { g_last_error = msg ? msg : ""; }
int dglhip_abi_version(void) { return DGLHIP_ABI_VERSION; }
const char* dglhip_build_info(void) {
  return "libdgl_hip abi=1 target=gfx950 built " __DATE__ " " __TIME__;
}

int dglhip_coo_to_csr_host(int64_t num_rows, int64_t num_cols, int64_t nnz,
                           const int64_t* row, const int64_t* col, int order,
                           int64_t* indptr, int32_t* indices, int64_t* eid) {
  API_BEGIN();
  DGLHIP_CHECK(num_rows >= 0 && num_cols >= 0 && nnz >= 0, "negative size");
  DGLHIP_CHECK(num_cols <= std::numeric_limits<int32_t>::max(),
               "num_cols " << num_cols << " exceeds int32 column ids");
  DGLHIP_CHECK(order == DGLHIP_ORDER_EID || order == DGLHIP_ORDER_COL,
               "unknown order " << order);
  DGLHIP_CHECK(indptr != nullptr, "indptr is null");
  DGLHIP_CHECK(nnz == 0 || (row && col && indices && eid), "null array");
  for (int64_t e = 0; e < nnz; ++e) {
    DGLHIP_CHECK(row[e] >= 0 && row[e] < num_rows,
                 "row id " << row[e] << " of edge " << e << " out of range [0,"
                           << num_rows << ")");
    DGLHIP_CHECK(col[e] >= 0 && col[e] < num_cols,
                 "col id " << col[e] << " of edge " << e << " out of range [0,"
                           << num_cols << ")");
  }
  const int nthreads = default_num_threads();
  csr_by_eid(num_rows, nnz, row, col, indptr, indices, eid, nthreads);
  if (order == DGLHIP_ORDER_COL) {
    parallel_for(num_rows, nthreads, [&](int64_t b, int64_t e, int) {
      std::vector<std::pair<int32_t, int64_t>> tmp;
      for (int64_t r = b; r < e; ++r) {
        const int64_t s = indptr[r], t = indptr[r + 1];
        if (t - s < 2) continue;
        tmp.resize(t - s);
        for (int64_t k = s; k < t; ++k) tmp[k - s] = {indices[k], eid[k]};
        std::sort(tmp.begin(), tmp.end());  // (col, eid) lexicographic
        for (int64_t k = s; k < t; ++k) {
          indices[k] = tmp[k - s].first;
          eid[k] = tmp[k - s].second;
        }
      }
    });
  }
  API_END();
}

int dglhip_rows_by_degree_host(int64_t num_rows, const int64_t* indptr,
                               int32_t* row_order) {
  API_BEGIN();
  DGLHIP_CHECK(num_rows >= 0 && num_rows <= std::numeric_limits<int32_t>::max(),
               "num_rows out of int32 range");
  if (num_rows == 0) return 0;
  int64_t maxdeg = 0;
  for (int64_t r = 0; r < num_rows; ++r)
    maxdeg = std::max(maxdeg, indptr[r + 1] - indptr[r]);
  if (maxdeg > 8 * num_rows + 1024) {
    // very skewed: comparison sort is cheaper than a huge histogram
    std::iota(row_order, row_order + num_rows, 0);
    std::stable_sort(row_order, row_order + num_rows, [&](int32_t a, int32_t b) {
      return indptr[a + 1] - indptr[a] > indptr[b + 1] - indptr[b];
    });
    return 0;
  }
  // counting sort on degree, descending, stable in row id
  std::vector<int64_t> cnt(maxdeg + 2, 0);
  for (int64_t r = 0; r < num_rows; ++r) cnt[maxdeg - (indptr[r + 1] - indptr[r])]++;
  int64_t acc = 0;
  for (auto& c : cnt) {
    const int64_t v = c;
    c = acc;
    acc += v;
  }
  for (int64_t r = 0; r < num_rows; ++r)
    row_order[cnt[maxdeg - (indptr[r + 1] - indptr[r])]++] = static_cast<int32_t>(r);
  API_END();
}

// ---------------------------------------------------------------------------
// CPU device: g-SpMM / g-SDDMM on host memory.
// ---------------------------------------------------------------------------

}  // extern "C"

// bf16 source rows (DGLHIP_MSG_COPY_U_BF16) on the host: the rows the slots
// reference are widened to fp32 (exact: bits << 16) and the fp32 kernel runs
// on them, so host and device agree bit for bit.
static std::vector<float> widen_bf16(const float* bits, int64_t n) {
  const uint16_t* b = reinterpret_cast<const uint16_t*>(bits);
  std::vector<float> w(static_cast<size_t>(n));
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t x = uint32_t(b[i]) << 16;
    std::memcpy(&w[i], &x, sizeof(float));
  }
  return w;
}

static int64_t max_index_plus_one(const int64_t* beg, const int64_t* end, int64_t n,
                                  const int32_t* indices) {
  int64_t m = 0;
  for (int64_t i = 0; i < n; ++i)
    for (int64_t k = beg[i]; k < end[i]; ++k) m = std::max<int64_t>(m, int64_t(indices[k]) + 1);
  return m;
}

static int gspmm_host_bf16(int reduce_op, int64_t num_rows, int64_t feat_len,
                           const int64_t* indptr, const int32_t* indices, const float* ufeat,
                           float* out, int64_t* arg_out, int num_threads) {
  DGLHIP_CHECK(ufeat && indptr && indices, "null indptr/indices/ufeat");
  const int64_t cols = max_index_plus_one(indptr, indptr + 1, num_rows, indices);
  std::vector<float> wide = widen_bf16(ufeat, cols * feat_len);
  return dglhip_gspmm_host(DGLHIP_MSG_COPY_U, reduce_op, num_rows, feat_len, indptr, indices,
                           nullptr, wide.data(), nullptr, 0, out, arg_out, num_threads);
}

// The chunked chains of the typed-block kernels (typed_block.hip): a row of
// `ptr` is cut into chunks of DGLHIP_TYPED_CHUNK slots, each chunk's chain
// chain(k0, k1, acc) runs from zero, and the partials are added in order.
template <typename ChainFn>
static void typed_chunked_rows(int64_t num_rows, int64_t F, const int64_t* ptr, float* out,
                               int nt, ChainFn&& chain) {
  const int64_t C = DGLHIP_TYPED_CHUNK;
  dglhip::parallel_for(num_rows, nt, [&](int64_t b0, int64_t b1, int) {
    std::vector<float> part(F);
    for (int64_t r = b0; r < b1; ++r) {
      float* o = out + r * F;
      const int64_t beg = ptr[r], end = ptr[r + 1];
      for (int64_t f = 0; f < F; ++f) o[f] = 0.0f;
      if (end - beg <= C) {
        chain(beg, end, o);
        continue;
      }
      chain(beg, beg + C, o);
      for (int64_t k = beg + C; k < end; k += C) {
        for (int64_t f = 0; f < F; ++f) part[f] = 0.0f;
        chain(k, std::min(k + C, end), part.data());
        for (int64_t f = 0; f < F; ++f) o[f] = o[f] + part[f];
      }
    }
  });
}

extern "C" {

int dglhip_gspmm_host(int msg_op, int reduce_op, int64_t num_rows,
                      int64_t feat_len, const int64_t* indptr,
                      const int32_t* indices, const int64_t* eid,
                      const float* ufeat, const float* efeat,
                      int64_t efeat_len, float* out, int64_t* arg_out,
                      int num_threads) {
  API_BEGIN();
  DGLHIP_CHECK(msg_op >= 0 && msg_op <= 3, "unknown msg op " << msg_op);
  DGLHIP_CHECK(reduce_op >= 0 && reduce_op <= 4, "unknown reduce op " << reduce_op);
  DGLHIP_CHECK(num_rows >= 0 && feat_len >= 0, "negative size");
  if (num_rows == 0 || feat_len == 0) return 0;
  if (msg_op == DGLHIP_MSG_COPY_U_BF16) {  // widen the rows once, then the fp32 path
    return gspmm_host_bf16(reduce_op, num_rows, feat_len, indptr, indices, ufeat, out,
                           arg_out, num_threads);
  }
  const bool use_u = msg_op != DGLHIP_MSG_COPY_E;
  const bool use_e = msg_op != DGLHIP_MSG_COPY_U;
  DGLHIP_CHECK(!use_u || ufeat, "ufeat is null");
  DGLHIP_CHECK(!use_e || (efeat && efeat_len >= 1 && feat_len % efeat_len == 0),
               "edge feature length " << efeat_len << " must divide feat_len " << feat_len);
  const int nt = num_threads > 0 ? num_threads : default_num_threads();
  const int64_t F = feat_len;
  const int64_t dpe = use_e ? F / efeat_len : 1;  // features per edge value
  const bool add_mean = reduce_op == DGLHIP_REDUCE_MEAN_ACCUM;
  parallel_for(num_rows, nt, [&](int64_t b, int64_t e, int) {
    std::vector<float> mean_row(add_mean ? F : 0);  // MEAN_ACCUM: the mean, then out + mean
    for (int64_t r = b; r < e; ++r) {
      float* o = add_mean ? mean_row.data() : out + r * F;
      const int64_t s = indptr[r], t = indptr[r + 1];
      if (reduce_op == DGLHIP_REDUCE_MAX) {
        for (int64_t f = 0; f < F; ++f) {
          float best = -std::numeric_limits<float>::infinity();
          int64_t arg = -1;
          for (int64_t k = s; k < t; ++k) {
            float x;
            const float* er = use_e ? efeat + (eid ? eid[k] : k) * efeat_len : nullptr;
            if (msg_op == DGLHIP_MSG_COPY_U) x = ufeat[int64_t(indices[k]) * F + f];
            else if (msg_op == DGLHIP_MSG_COPY_E) x = er[f / dpe];
            else x = ufeat[int64_t(indices[k]) * F + f] * er[f / dpe];
            if (arg < 0 || x > best) { best = x; arg = k; }
          }
          o[f] = arg < 0 ? 0.0f : best;
          if (arg_out) arg_out[r * F + f] = arg;
        }
        continue;
      }
      if (reduce_op != DGLHIP_REDUCE_SUM_ACCUM)
        for (int64_t f = 0; f < F; ++f) o[f] = 0.0f;
      for (int64_t k = s; k < t; ++k) {
        const float* ur = use_u ? ufeat + int64_t(indices[k]) * F : nullptr;
        const float* er = use_e ? efeat + (eid ? eid[k] : k) * efeat_len : nullptr;
        if (msg_op == DGLHIP_MSG_COPY_U) {
          for (int64_t f = 0; f < F; ++f) o[f] += ur[f];
        } else if (msg_op == DGLHIP_MSG_COPY_E) {
          for (int64_t f = 0; f < F; ++f) o[f] += er[f / dpe];
        } else if (efeat_len == 1) {
          const float w = er[0];
          for (int64_t f = 0; f < F; ++f) o[f] = std::fma(w, ur[f], o[f]);
        } else {
          for (int64_t f = 0; f < F; ++f) o[f] = std::fma(er[f / dpe], ur[f], o[f]);
        }
      }
      if ((reduce_op == DGLHIP_REDUCE_MEAN || add_mean) && t - s > 1) {
        const float inv = static_cast<float>(t - s);
        for (int64_t f = 0; f < F; ++f) o[f] = o[f] / inv;
      }
      if (add_mean && t > s) {
        float* dst = out + r * F;
        for (int64_t f = 0; f < F; ++f) dst[f] = dst[f] + o[f];
      }
    }
  });
  API_END();
}

int dglhip_gspmm_ranges_host(int msg_op, int64_t num_items, int64_t feat_len,
                             const int64_t* item_beg, const int64_t* item_end,
                             int accumulate, const int32_t* indices, const int64_t* eid,
                             const float* ufeat, const float* efeat, int64_t efeat_len,
                             float* out, int num_threads) {
  API_BEGIN();
  DGLHIP_CHECK(msg_op >= 0 && msg_op <= 3, "unknown msg op " << msg_op);
  if (num_items == 0 || feat_len == 0) return 0;
  if (msg_op == DGLHIP_MSG_COPY_U_BF16) {
    DGLHIP_CHECK(ufeat && indices, "ufeat is null");
    const int64_t cols = max_index_plus_one(item_beg, item_end, num_items, indices);
    std::vector<float> wide = widen_bf16(ufeat, cols * feat_len);
    return dglhip_gspmm_ranges_host(DGLHIP_MSG_COPY_U, num_items, feat_len, item_beg, item_end,
                                    accumulate, indices, eid, wide.data(), efeat, efeat_len,
                                    out, num_threads);
  }
  const bool use_e = msg_op != DGLHIP_MSG_COPY_U;
  DGLHIP_CHECK(!use_e || (efeat && efeat_len >= 1 && feat_len % efeat_len == 0),
               "bad edge feature");
  const int nt = num_threads > 0 ? num_threads : default_num_threads();
  const int64_t F = feat_len, dpe = use_e ? F / efeat_len : 1;
  parallel_for(num_items, nt, [&](int64_t b, int64_t e, int) {
    for (int64_t i = b; i < e; ++i) {
      float* o = out + i * F;
      if (!accumulate)
        for (int64_t f = 0; f < F; ++f) o[f] = 0.0f;
      for (int64_t k = item_beg[i]; k < item_end[i]; ++k) {
        const float* ur = msg_op != DGLHIP_MSG_COPY_E ? ufeat + int64_t(indices[k]) * F : nullptr;
        const float* er = use_e ? efeat + (eid ? eid[k] : k) * efeat_len : nullptr;
        for (int64_t f = 0; f < F; ++f) {
          if (msg_op == DGLHIP_MSG_COPY_U) o[f] += ur[f];
          else if (msg_op == DGLHIP_MSG_COPY_E) o[f] += er[f / dpe];
          else o[f] = std::fma(er[f / dpe], ur[f], o[f]);
        }
      }
    }
  });
  API_END();
}

int dglhip_typed_block_spmm_host(int64_t num_rows, int64_t num_blocks, int64_t in_block,
                                 int64_t out_block, const int64_t* indptr,
                                 const int32_t* indices, const int32_t* slot_rel,
                                 const float* slot_norm, const float* ufeat,
                                 const float* weight, float* out, int num_threads) {
  API_BEGIN();
  DGLHIP_CHECK(num_rows >= 0 && num_blocks > 0 && in_block > 0 && out_block > 0, "bad sizes");
  if (num_rows == 0) return 0;
  DGLHIP_CHECK(indptr && indices && slot_rel && ufeat && weight && out, "null pointer argument");
  const int64_t nb = num_blocks, si = in_block, so = out_block;
  const int64_t Fi = nb * si, Fo = nb * so, wr = nb * si * so;
  const int nt = num_threads > 0 ? num_threads : default_num_threads();
  typed_chunked_rows(num_rows, Fo, indptr, out, nt, [&](int64_t k0, int64_t k1, float* o) {
    for (int64_t k = k0; k < k1; ++k) {
      const float* h = ufeat + int64_t(indices[k]) * Fi;
      const float* w = weight + int64_t(slot_rel[k]) * wr;
      const float nrm = slot_norm ? slot_norm[k] : 1.0f;
      for (int64_t jg = 0; jg < Fo; ++jg) {
        const int64_t b = jg / so, j = jg - b * so;
        float m = 0.0f;
        for (int64_t i = 0; i < si; ++i) m = std::fma(h[b * si + i], w[b * si * so + i * so + j], m);
        o[jg] = std::fma(nrm, m, o[jg]);
      }
    }
  });
  API_END();
}

int dglhip_typed_block_wgrad_host(int64_t num_rels, int64_t num_blocks, int64_t in_block,
                                  int64_t out_block, const int64_t* rel_ptr,
                                  const int32_t* rel_src, const int32_t* rel_dst,
                                  const float* rel_norm, const float* ufeat, const float* dout,
                                  float* dweight, int num_threads) {
  API_BEGIN();
  DGLHIP_CHECK(num_rels >= 0 && num_blocks >= 0 && in_block >= 0 && out_block >= 0,
               "bad sizes");
  const int64_t nb = num_blocks, si = in_block, so = out_block;
  const int64_t Fi = nb * si, Fo = nb * so, wr = nb * si * so;
  if (num_rels == 0 || wr == 0) return 0;
  DGLHIP_CHECK(rel_ptr && ufeat && dout && dweight, "null pointer argument");
  const int nt = num_threads > 0 ? num_threads : default_num_threads();
  typed_chunked_rows(num_rels, wr, rel_ptr, dweight, nt, [&](int64_t k0, int64_t k1, float* o) {
    for (int64_t k = k0; k < k1; ++k) {
      const float* x = ufeat + int64_t(rel_src[k]) * Fi;
      const float* g = dout + int64_t(rel_dst[k]) * Fo;
      for (int64_t rem = 0; rem < wr; ++rem) {
        const int64_t b = rem / (si * so), i = (rem / so) % si, j = rem % so;
        const float xv = x[b * si + i];
        o[rem] = std::fma(rel_norm ? rel_norm[k] * xv : xv, g[b * so + j], o[rem]);
      }
    }
  });
  API_END();
}

int dglhip_gat_logits_host(int64_t num_nodes, int64_t num_heads, int64_t head_dim,
                           const float* ft, const float* attn_l, const float* attn_r, float* el,
                           float* er, int num_threads) {
#pragma clang fp contract(off)
  API_BEGIN();
  DGLHIP_CHECK(num_nodes >= 0 && num_heads >= 1 && head_dim >= 1, "bad sizes");
  const int64_t total = num_nodes * num_heads, H = num_heads, D = head_dim;
  if (total == 0) return 0;
  DGLHIP_CHECK(ft && attn_l && el && (attn_r == nullptr) == (er == nullptr),
               "null pointer argument");
  // dglhip_gat_logits_device's association (gat_fused.hip, gat_logit)
  auto logit = [D](const float* x, const float* a) {
    if (D == 16) {
      float p[8];
      for (int l = 0; l < 8; ++l) {
        const float m = x[2 * l] * a[2 * l];
        p[l] = std::fma(x[2 * l + 1], a[2 * l + 1], m);
      }
      const float s01 = p[0] + p[1], s23 = p[2] + p[3], s45 = p[4] + p[5], s67 = p[6] + p[7];
      const float s0123 = s01 + s23, s4567 = s45 + s67;
      return s0123 + s4567;
    }
    float acc = 0.0f;
    for (int64_t d = 0; d < D; ++d) acc = std::fma(x[d], a[d], acc);
    return acc;
  };
  const int nt = num_threads > 0 ? num_threads : default_num_threads();
  parallel_for(total, nt, [&](int64_t b0, int64_t b1, int) {
    for (int64_t i = b0; i < b1; ++i) {
      const int64_t h = i % H;
      el[i] = logit(ft + i * D, attn_l + h * D);
      if (er) er[i] = logit(ft + i * D, attn_r + h * D);
    }
  });
  API_END();
}

int dglhip_distmult_score_host(int64_t num_samples, int64_t feat_len, int64_t num_nodes,
                               int64_t num_rels, const int64_t* subj, const int64_t* rel,
                               const int64_t* obj, const float* h, const float* w_rel,
                               float* score, int num_threads) {
#pragma clang fp contract(off)
  API_BEGIN();
  DGLHIP_CHECK(num_samples >= 0 && feat_len >= 0 && num_nodes >= 0 && num_rels >= 0,
               "bad sizes");
  if (num_samples == 0) return 0;
  DGLHIP_CHECK(subj && rel && obj && h && w_rel && score, "null pointer argument");
  const int64_t F = feat_len;
  const int nt = num_threads > 0 ? num_threads : default_num_threads();
  parallel_for(num_samples, nt, [&](int64_t b0, int64_t b1, int) {
    float lane[64];
    for (int64_t i = b0; i < b1; ++i) {
      const int64_t si = subj[i], ri = rel[i], oi = obj[i];
      if (si < 0 || si >= num_nodes || oi < 0 || oi >= num_nodes || ri < 0 || ri >= num_rels) {
        score[i] = std::nanf("");
        continue;
      }
      const float *a = h + si * F, *b = w_rel + ri * F, *c = h + oi * F;
      // the device kernel's association: 64 lane chains, then a xor butterfly
      for (int l = 0; l < 64; ++l) {
        float acc = 0.0f;
        for (int64_t f = l; f < F; f += 64) {
          const float ab = a[f] * b[f];
          const float t = ab * c[f];
          acc = acc + t;
        }
        lane[l] = acc;
      }
      for (int off = 32; off > 0; off >>= 1) {
        float nxt[64];
        for (int l = 0; l < 64; ++l) nxt[l] = lane[l] + lane[l ^ off];
        for (int l = 0; l < 64; ++l) lane[l] = nxt[l];
      }
      score[i] = lane[0];
    }
  });
  API_END();
}

int dglhip_distmult_grad_host(int task, int64_t num_rows, int64_t feat_len, int64_t num_samples,
                              int64_t num_nodes, int64_t num_rels, const int64_t* ptr,
                              const int32_t* order, const int64_t* subj, const int64_t* rel,
                              const int64_t* obj, const float* dscore, const float* h,
                              const float* w_rel, float* out, int num_threads) {
#pragma clang fp contract(off)
  API_BEGIN();
  DGLHIP_CHECK(task == 0 || task == 1, "unknown DistMult gradient task " << task);
  DGLHIP_CHECK(num_rows >= 0 && feat_len >= 0 && num_samples >= 0, "bad sizes");
  if (num_rows == 0 || feat_len == 0) return 0;
  DGLHIP_CHECK(ptr && out, "null pointer argument");
  DGLHIP_CHECK(num_samples == 0 || (order && subj && rel && obj && dscore && h && w_rel),
               "null pointer argument");
  const int64_t F = feat_len, n = num_samples;
  const int nt = num_threads > 0 ? num_threads : default_num_threads();
  typed_chunked_rows(num_rows, F, ptr, out, nt, [&](int64_t k0, int64_t k1, float* o) {
    for (int64_t k = k0; k < k1; ++k) {
      const int64_t p = order[k];
      const bool objp = task == 0 && p >= n;
      const int64_t i = objp ? p - n : p;
      const int64_t si = subj[i], ri = rel[i], oi = obj[i];
      if (si < 0 || si >= num_nodes || oi < 0 || oi >= num_nodes || ri < 0 || ri >= num_rels) {
        for (int64_t f = 0; f < F; ++f) o[f] = std::nanf("");
        continue;
      }
      const float d = dscore[i];
      const float* x = objp ? h + si * F : h + oi * F;
      const float* y = task == 1 ? h + si * F : w_rel + ri * F;
      for (int64_t f = 0; f < F; ++f) {
        float t;
        if (objp) {
          const float xy = x[f] * y[f];
          t = d * xy;
        } else {
          const float dx = d * x[f];
          t = dx * y[f];
        }
        o[f] = o[f] + t;
      }
    }
  });
  API_END();
}

int dglhip_gsddmm_attention_host(int64_t num_rows, int64_t num_heads, const int64_t* indptr,
                                 const int32_t* indices, const int64_t* eid, const float* lhs,
                                 const float* rhs, float alpha, float clamp_lo,
                                 float clamp_hi, int apply_exp, float* out,
                                 int num_threads) {
  API_BEGIN();
  const int64_t H = num_heads;
  const int nt = num_threads > 0 ? num_threads : default_num_threads();
  parallel_for(num_rows, nt, [&](int64_t b, int64_t e, int) {
    for (int64_t r = b; r < e; ++r)
      for (int64_t k = indptr[r]; k < indptr[r + 1]; ++k)
        for (int64_t h = 0; h < H; ++h) {
          float x = lhs[int64_t(indices[k]) * H + h] + rhs[r * H + h];
          x = x > 0.0f ? x : alpha * x;
          if (apply_exp) x = std::exp(x);
          out[(eid ? eid[k] : k) * H + h] = std::min(std::max(x, clamp_lo), clamp_hi);
        }
  });
  API_END();
}

// Degree-bucketing schedule for UDF reduces (replaces sched::DegreeBucketing,
// src/scheduler/scheduler.cc:13-93). Messages m (0..num_msgs-1) go to
// receiver position msg_recv[m] in [0, num_recv). Buckets are the distinct
// non-zero degrees in ascending order; inside a bucket nodes ascend, and each
// node's messages keep message order. Outputs (caller-allocated, max sizes):
//   bucket_deg[num_recv], bucket_node_ptr[num_recv+1], nodes[num_recv],
//   msg_ids[num_msgs]; *num_buckets = number of buckets. Nodes without
// messages are not listed (the caller fills them with the initializer).
int dglhip_degree_bucketing_host(int64_t num_msgs, const int64_t* msg_recv,
                                 int64_t num_recv, int64_t* num_buckets,
                                 int64_t* bucket_deg, int64_t* bucket_node_ptr,
                                 int64_t* nodes, int64_t* msg_ids) {
  API_BEGIN();
  DGLHIP_CHECK(num_msgs >= 0 && num_recv >= 0, "negative size");
  std::vector<int64_t> deg(num_recv, 0);
  for (int64_t m = 0; m < num_msgs; ++m) {
    DGLHIP_CHECK(msg_recv[m] >= 0 && msg_recv[m] < num_recv, "receiver out of range");
    deg[msg_recv[m]]++;
  }
  // message lists per receiver (stable counting sort)
  std::vector<int64_t> start(num_recv + 1, 0);
  for (int64_t v = 0; v < num_recv; ++v) start[v + 1] = start[v] + deg[v];
  std::vector<int64_t> by_node(num_msgs), cur(start.begin(), start.end() - 1);
  for (int64_t m = 0; m < num_msgs; ++m) by_node[cur[msg_recv[m]]++] = m;
  // nodes ordered by (degree, node id), zero degree dropped
  int64_t maxdeg = 0;
  for (int64_t v = 0; v < num_recv; ++v) maxdeg = std::max(maxdeg, deg[v]);
  std::vector<int64_t> cnt(maxdeg + 2, 0);
  for (int64_t v = 0; v < num_recv; ++v) cnt[deg[v] + 1]++;
  for (int64_t d = 0; d <= maxdeg; ++d) cnt[d + 1] += cnt[d];
  std::vector<int64_t> order(num_recv), pos(cnt.begin(), cnt.end() - 1);
  for (int64_t v = 0; v < num_recv; ++v) order[pos[deg[v]]++] = v;
  int64_t nb = 0, nn = 0, nm = 0;
  bucket_node_ptr[0] = 0;
  for (int64_t d = 1; d <= maxdeg; ++d) {
    const int64_t b = cnt[d], e = cnt[d + 1];
    if (b == e) continue;
    bucket_deg[nb] = d;
    for (int64_t i = b; i < e; ++i) {
      const int64_t v = order[i];
      nodes[nn++] = v;
      for (int64_t k = start[v]; k < start[v + 1]; ++k) msg_ids[nm++] = by_node[k];
    }
    bucket_node_ptr[++nb] = nn;
  }
  *num_buckets = nb;
  API_END();
}

int dglhip_gsddmm_host(int op, int64_t num_rows, int64_t feat_len, int64_t num_heads,
                       const int64_t* indptr, const int32_t* indices,
                       const int64_t* eid, const float* lhs, const float* rhs,
                       float* out, int num_threads) {
  API_BEGIN();
  DGLHIP_CHECK(op == DGLHIP_SDDMM_DOT, "unknown sddmm op " << op);
  DGLHIP_CHECK(num_heads >= 1 && feat_len % num_heads == 0,
               "num_heads " << num_heads << " must divide feat_len " << feat_len);
  const int nt = num_threads > 0 ? num_threads : default_num_threads();
  const int64_t F = feat_len, H = num_heads, D = feat_len / num_heads;
  parallel_for(num_rows, nt, [&](int64_t b, int64_t e, int) {
    for (int64_t r = b; r < e; ++r) {
      const float* a = lhs + r * F;
      for (int64_t k = indptr[r]; k < indptr[r + 1]; ++k) {
        const float* c = rhs + int64_t(indices[k]) * F;
        for (int64_t h = 0; h < H; ++h) {
          float acc = 0.0f;
          for (int64_t d = 0; d < D; ++d) acc = std::fma(a[h * D + d], c[h * D + d], acc);
          out[(eid ? eid[k] : k) * H + h] = acc;
        }
      }
    }
  });
  API_END();
}

}  // extern "C"
