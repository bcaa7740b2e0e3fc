// The g-SpMM launch plan (spmm_plan.h): schedule policy, the plan build and
// the planned run, and its C-ABI (dglhip_spmm_*, include/dgl_hip.h).
//
// This is the engine's equivalent of the adjacency cache the reference builds
// per context (GraphIndex.adjacency_matrix, python/dgl/graph_index.py:537-585)
// together with the product F.spmm runs on it (python/dgl/backend/pytorch/
// tensor.py:145-146, driven by SPMVExecutor.run, runtime/ir/executor.py:
// 452-473): one object per CSR and device that a caller builds once and hands
// to every product over that CSR, through the typed entry points or the
// PackedFunc registry (dglhip._CAPI_GSpMM's plan argument, registry.cc).
#include "spmm_plan.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>

#include "../../include/dgl_hip.h"
#include "common.h"

namespace dglhip {

namespace {

constexpr int64_t kRefWaves = 7168;  // MI355X's; host parts and unknown devices
constexpr int64_t kCriticalMin = 16384;
constexpr int64_t kCutNum = 7168, kCutDen = 12000;
constexpr int64_t kChunkMin = 1024;

void hip_ok(hipError_t e, const char* what) {
  DGLHIP_CHECK(e == hipSuccess, what << ": " << hipGetErrorString(e));
}

std::string env_str(const char* name, const char* dflt) {
  const char* v = std::getenv(name);
  return v ? std::string(v) : std::string(dflt);
}

SpmmPolicy policy_from_env() {
  SpmmPolicy p;
  const std::string rs = env_str("DGLHIP_ROW_SPLIT", "auto");
  if (rs == "auto") p.row_split = -1;
  else if (rs == "off" || rs == "0" || rs.empty() || rs == "none" || rs == "None") p.row_split = 0;
  else p.row_split = std::stoll(rs);
  p.blocked = env_str("DGLHIP_BLOCKED", "auto") != "off";
  p.block_bytes = std::stoll(env_str("DGLHIP_BLOCK_BYTES", "6291456"));
  p.block_min_slots = std::stoll(env_str("DGLHIP_BLOCK_MIN_SLOTS", "12"));
  p.block_max_stretch = std::stod(env_str("DGLHIP_BLOCK_MAX_STRETCH", "3"));
  p.short_rows = env_str("DGLHIP_SHORT_ROWS", "on") != "off";
  p.pad_rows = env_str("DGLHIP_PAD_ROWS", "auto") == "auto";
  return p;
}

std::mutex g_pol_mu;
SpmmPolicy& pol_ref() {
  static SpmmPolicy p = policy_from_env();
  return p;
}

double lines_per_row(int64_t F, int64_t ld) {
  int64_t tot = 0;
  for (int64_t u = 0; u < 32; ++u) {
    const int64_t off = (u * ld * 4) % 128;
    tot += (off + 4 * F + 127) / 128;
  }
  return tot / 32.0;
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

inline bool copies_u(int msg) {
  return msg == DGLHIP_MSG_COPY_U || msg == DGLHIP_MSG_COPY_U_BF16;
}

inline bool accum(int red) {
  return red == DGLHIP_REDUCE_SUM_ACCUM || red == DGLHIP_REDUCE_MEAN_ACCUM;
}

}  // namespace

SpmmPolicy spmm_policy() {
  std::lock_guard<std::mutex> lk(g_pol_mu);
  return pol_ref();
}

namespace {
SweepPolicy& sweep_ref() {
  static SweepPolicy p = [] {
    SweepPolicy q;
    const char* e = std::getenv("DGLHIP_SWEEP");
    if (e && (std::strcmp(e, "0") == 0 || std::strcmp(e, "off") == 0)) q.on = 0;
    const char* pc = std::getenv("DGLHIP_SWEEP_ACCUM_PER_CU");
    if (pc) q.accum_per_cu = std::max(0, std::atoi(pc));
    const char* lg = std::getenv("DGLHIP_SWEEP_LAG");
    if (lg) q.lag = std::max(0, std::atoi(lg));
    const char* tm = std::getenv("DGLHIP_SWEEP_ACCUM_TABLE_MIN");  // bytes
    if (tm) q.accum_table_min = std::max<int64_t>(0, std::atoll(tm));
    const char* ms = std::getenv("DGLHIP_SWEEP_ACCUM_MIN_SLOTS");
    if (ms) q.accum_min_slots = std::max<int64_t>(0, std::atoll(ms));
    const char* bb = std::getenv("DGLHIP_SWEEP_BLOCK_BYTES");  // a study knob
    if (bb && std::atoll(bb) >= (int64_t(1) << 20)) q.block_bytes = std::atoll(bb);
    return q;
  }();
  return p;
}
}  // namespace

SweepPolicy sweep_policy() {
  std::lock_guard<std::mutex> lk(g_pol_mu);
  return sweep_ref();
}

void set_spmm_policy(const SpmmPolicy& p) {
  DGLHIP_CHECK(p.block_bytes > 0 && p.block_min_slots >= 1 && p.block_max_stretch > 0 &&
                   p.block_table_min >= 0 && p.block_table_max >= p.block_table_min &&
                   p.block_max_suffix >= 0 && p.tier_min_rows >= 0 && p.pad_min_bytes >= 0,
               "invalid g-SpMM schedule policy");
  DGLHIP_CHECK(p.row_split >= -1, "row_split: -1 auto, 0 off or a chunk length");
  std::lock_guard<std::mutex> lk(g_pol_mu);
  pol_ref() = p;
}

// kernel.py's _split_threshold before r05 (DESIGN.md §4.1 "Heavy-row policy")
int64_t split_threshold(const SpmmPolicy& p, int64_t nnz, int64_t max_degree, int64_t waves) {
  if (p.row_split == 0) return 0;
  if (p.row_split < 0) {
    const int64_t R = std::max<int64_t>(waves, 2);
    const int64_t t = std::max<int64_t>(4096, nnz * kCutNum / (kCutDen * R));
    return max_degree > std::max<int64_t>(kCriticalMin, nnz / (R / 2)) ? t : 0;
  }
  return max_degree > p.row_split ? p.row_split : 0;
}

// F itself, or F rounded up to 16 / 32 floats when that cuts the 128-B lines
// a gathered row touches by at least 5 % (F = 41: 2.28 -> 2.0 lines at 48)
int64_t padded_width(int64_t F) {
  int64_t best = F;
  double best_lines = lines_per_row(F, F);
  for (int64_t ld : {cdiv(F, 16) * 16, cdiv(F, 32) * 32}) {
    if (ld > F && ld % 2 == 0) {
      const double l = lines_per_row(F, ld);
      if (l < best_lines * 0.95 && l < lines_per_row(F, best) - 1e-9) {
        best = ld;
        best_lines = l;
      }
    }
  }
  return best;
}

// ---------------------------------------------------------------------------
// SpmmPlan
// ---------------------------------------------------------------------------
SpmmPlan::SpmmPlan(int device_type, int device_id, int64_t num_rows, int64_t num_cols,
                   int64_t nnz, const int64_t* indptr, const int32_t* indices,
                   const int64_t* host_indptr, const int32_t* row_order, hipStream_t s)
    : device_type_(device_type), device_id_(device_id), R_(num_rows), C_(num_cols), nnz_(nnz),
      indptr_(indptr), indices_(indices) {
  DGLHIP_CHECK(device_type == rt::kDLCPU || device_type == rt::kDLROCM,
               "unsupported device type " << device_type);
  DGLHIP_CHECK(num_rows >= 0 && num_cols >= 0 && nnz >= 0, "negative size");
  DGLHIP_CHECK(num_rows <= INT32_MAX, "num_rows out of int32 range");
  DGLHIP_CHECK(indptr != nullptr, "null indptr");
  DGLHIP_CHECK(nnz == 0 || indices != nullptr, "null indices");
  if (device_type == rt::kDLCPU) host_indptr = indptr;
  if (host_indptr) {
    host_indptr_ = std::make_shared<std::vector<int64_t>>(host_indptr, host_indptr + R_ + 1);
  } else {
    host_indptr_ = std::make_shared<std::vector<int64_t>>(R_ + 1);
    hip_ok(hipMemcpyAsync(host_indptr_->data(), indptr, (R_ + 1) * sizeof(int64_t),
                          hipMemcpyDeviceToHost, s), "plan indptr copy");
    hip_ok(hipStreamSynchronize(s), "plan indptr copy");
  }
  const int64_t* ip = host_indptr_->data();
  DGLHIP_CHECK(ip[0] == 0 && ip[R_] == nnz, "indptr does not span " << nnz << " slots");
  for (int64_t r = 0; r < R_; ++r) {
    const int64_t d = ip[r + 1] - ip[r];
    DGLHIP_CHECK(d >= 0, "indptr decreases at row " << r);
    max_degree_ = std::max(max_degree_, d);
    num_nonempty_ += d > 0;
  }
  if (row_order) {
    row_order_ = row_order;  // its host copy is made when a split plan or tiers need it
  } else {
    host_order_.resize(R_);
    have_host_order_ = true;
    if (R_) DGLHIP_CHECK(dglhip_rows_by_degree_host(R_, ip, host_order_.data()) == 0,
                         DGLGetLastError());
    if (device_type == rt::kDLCPU) {
      row_order_ = host_order_.data();
    } else {
      order_own_ = upload(host_order_.data(), R_, 0, 32, s);
      row_order_ = order_own_.data<int32_t>();
    }
  }
  waves_ = kRefWaves;
  if (on_device()) {
    // queried once per device (graphs built per training step make plans)
    static std::mutex wmu;
    static std::map<int, int64_t> wcache;
    std::lock_guard<std::mutex> lk(wmu);
    auto hit = wcache.find(device_id_);
    if (hit == wcache.end()) {
      int64_t w = 0;
      DGLHIP_CHECK(dglhip_gspmm_resident_waves(device_id_, &w) == 0, DGLGetLastError());
      hit = wcache.emplace(device_id_, w).first;
    }
    waves_ = hit->second;
  }
}

const std::vector<int32_t>& SpmmPlan::host_order(hipStream_t s) {
  // called with mu_ held
  if (!have_host_order_) {
    host_order_.resize(R_);
    if (R_) {
      if (on_device()) {
        hip_ok(hipMemcpyAsync(host_order_.data(), row_order_, R_ * sizeof(int32_t),
                              hipMemcpyDeviceToHost, s), "plan row order copy");
        hip_ok(hipStreamSynchronize(s), "plan row order copy");
      } else {
        std::memcpy(host_order_.data(), row_order_, R_ * sizeof(int32_t));
      }
    }
    have_host_order_ = true;
  }
  return host_order_;
}

rt::NDArray SpmmPlan::empty(const std::vector<int64_t>& shape, int code, int bits) const {
  return rt::NDArray::Empty(shape, code, bits, device_type_, device_id_);
}

rt::NDArray SpmmPlan::upload(const void* src, int64_t n, int code, int bits,
                             hipStream_t s) const {
  rt::NDArray a = empty({n}, code, bits);
  const size_t bytes = static_cast<size_t>(n) * (bits / 8);
  if (bytes == 0) return a;
  if (on_device()) {
    hip_ok(hipMemcpyAsync(a.data<void>(), src, bytes, hipMemcpyHostToDevice, s), "plan upload");
    // the host buffer may be released right after: complete the copy
    hip_ok(hipStreamSynchronize(s), "plan upload");
  } else {
    std::memcpy(a.data<void>(), src, bytes);
  }
  return a;
}

std::pair<int64_t, int64_t> SpmmPlan::span(hipStream_t s) {
  std::lock_guard<std::mutex> lk(mu_);
  if (lo_ >= 0 || nnz_ == 0) return nnz_ == 0 ? std::make_pair(int64_t(0), int64_t(0))
                                               : std::make_pair(lo_, hi_);
  int32_t lh[2] = {INT_MAX, -1};
  if (on_device()) {
    rt::NDArray d = upload(lh, 2, 0, 32, s);
    plan_span_device(nnz_, indices_, d.data<int32_t>(), s);
    hip_ok(hipMemcpyAsync(lh, d.data<int32_t>(), sizeof(lh), hipMemcpyDeviceToHost, s),
           "plan span");
    hip_ok(hipStreamSynchronize(s), "plan span");
  } else {
    for (int64_t k = 0; k < nnz_; ++k) {
      lh[0] = std::min(lh[0], indices_[k]);
      lh[1] = std::max(lh[1], indices_[k]);
    }
  }
  DGLHIP_CHECK(lh[0] >= 0 && lh[1] < C_, "column ids outside [0, " << C_ << ")");
  lo_ = lh[0];
  hi_ = int64_t(lh[1]) + 1;
  return {lo_, hi_};
}

bool SpmmPlan::eid_identity(const int64_t* eid, hipStream_t s) {
  if (eid == nullptr) return true;
  std::lock_guard<std::mutex> lk(mu_);
  // a CSR's edge ids never change: the answer holds for every copy of them
  if (eid_ident_ >= 0) return eid_ident_ == 1;
  int32_t flag = 0;
  if (on_device()) {
    rt::NDArray d = upload(&flag, 1, 0, 32, s);
    plan_eid_identity_device(nnz_, eid, d.data<int32_t>(), s);
    hip_ok(hipMemcpyAsync(&flag, d.data<int32_t>(), sizeof(flag), hipMemcpyDeviceToHost, s),
           "plan eid check");
    hip_ok(hipStreamSynchronize(s), "plan eid check");
  } else {
    for (int64_t k = 0; k < nnz_ && !flag; ++k) flag = eid[k] != k;
  }
  eid_ident_ = flag ? 0 : 1;
  return eid_ident_ == 1;
}

int SpmmPlan::block_count(int64_t table_bytes, int64_t block_bytes) const {
  const SpmmPolicy p = spmm_policy();
  // a plan holds about 12 B per slot: graphs past 2^31 slots keep one launch
  if (R_ == 0 || nnz_ == 0 || nnz_ >= (int64_t(1) << 31)) return 0;
  if (table_bytes < p.block_table_min || table_bytes > p.block_table_max) return 0;
  const int64_t want = cdiv(table_bytes, block_bytes);
  const int64_t B = std::min<int64_t>(
      want, nnz_ / (p.block_min_slots * std::max<int64_t>(num_nonempty_, 1)));
  // rows too short to cut the table into L2-sized slices: slices stretched
  // past max_stretch x the target gain nothing (tools/segment_block_study.py)
  if (p.block_max_stretch * static_cast<double>(B) < static_cast<double>(want)) return 0;
  return B >= 2 ? static_cast<int>(B) : 0;
}

int64_t SpmmPlan::heavy_threshold() const {
  return split_threshold(spmm_policy(), nnz_, max_degree_, waves_);
}

std::shared_ptr<BlockSplit> SpmmPlan::block_split(int B, hipStream_t s) {
  // called with mu_ held
  auto it = splits_.find(B);
  if (it != splits_.end()) return it->second;
  auto sp = std::make_shared<BlockSplit>();
  sp->B = B;
  sp->lo = lo_;
  sp->bs = std::max<int64_t>(1, cdiv(hi_ - lo_, B));
  const int64_t* ip = host_indptr_->data();
  sp->counts.assign(static_cast<size_t>(R_) * B, 0);
  sp->pend.assign(R_, 0);
  if (on_device()) {
    rt::NDArray cnt = empty({R_ * B}, 0, 32);
    rt::NDArray pend = empty({R_}, 0, 64);
    hip_ok(hipMemsetAsync(cnt.data<int32_t>(), 0, R_ * B * sizeof(int32_t), s), "plan walk");
    plan_block_walk_device(R_, indptr_, indices_, sp->lo, sp->bs, B, cnt.data<int32_t>(),
                           pend.data<int64_t>(), s);
    hip_ok(hipMemcpyAsync(sp->counts.data(), cnt.data<int32_t>(), R_ * B * sizeof(int32_t),
                          hipMemcpyDeviceToHost, s), "plan walk");
    hip_ok(hipMemcpyAsync(sp->pend.data(), pend.data<int64_t>(), R_ * sizeof(int64_t),
                          hipMemcpyDeviceToHost, s), "plan walk");
    hip_ok(hipStreamSynchronize(s), "plan walk");
  } else {
    const int64_t lo = sp->lo, bs = sp->bs;
    parallel_for(R_, default_num_threads(), [&](int64_t b0, int64_t b1, int) {
      for (int64_t r = b0; r < b1; ++r) {
        int32_t* cnt = sp->counts.data() + r * B;
        int64_t prev = -1, pe = ip[r + 1];
        for (int64_t k = ip[r]; k < ip[r + 1]; ++k) {
          const int64_t b = (int64_t(indices_[k]) - lo) / bs;
          if (b < prev) {
            pe = k;
            break;
          }
          cnt[b] += 1;
          prev = b;
        }
        sp->pend[r] = pe;
      }
    });
  }
  int64_t sfx = 0;
  for (int64_t r = 0; r < R_; ++r) sfx += ip[r + 1] - sp->pend[r];
  sp->total_suffix = sfx;
  const SpmmPolicy p = spmm_policy();
  sp->ok = static_cast<double>(sfx) <= static_cast<double>(nnz_) * p.block_max_suffix;
  splits_[B] = sp;
  return sp;
}

std::shared_ptr<BlockedPlan> SpmmPlan::blocked(int64_t row_bytes, int64_t block_bytes,
                                               hipStream_t s) {
  const SpmmPolicy p = spmm_policy();
  if (!p.blocked || nnz_ == 0 || row_bytes <= p.block_min_row_bytes) return nullptr;
  const auto lh = span(s);
  const int B = block_count((lh.second - lh.first) * row_bytes, block_bytes);
  if (!B) return nullptr;
  if (heavy_threshold()) return nullptr;  // a row long enough to need the heavy-row split
  return blocked_for(B, s);
}

std::shared_ptr<BlockedPlan> SpmmPlan::blocked_for(int B, hipStream_t s) {
  DGLHIP_CHECK(B >= 1, "block count " << B);
  span(s);
  std::lock_guard<std::mutex> lk(mu_);
  auto hit = blocked_.find(B);
  if (hit != blocked_.end()) return hit->second;
  auto split = block_split(B, s);
  if (!split->ok) {
    blocked_[B] = nullptr;
    return nullptr;
  }
  const int64_t* ip = host_indptr_->data();
  auto bp = std::make_shared<BlockedPlan>();
  bp->B = B;
  bp->has_suffix = split->total_suffix > 0;
  const int L = B + (bp->has_suffix ? 1 : 0);
  // items of each launch: rows with slots in it, longest first, stable by row
  std::vector<std::vector<std::pair<int64_t, int32_t>>> items(L);
  parallel_for(L, default_num_threads(), [&](int64_t l0, int64_t l1, int) {
    for (int64_t l = l0; l < l1; ++l) {
      auto& v = items[l];
      for (int64_t r = 0; r < R_; ++r) {
        const int64_t c = l < B ? split->counts[r * B + l] : ip[r + 1] - split->pend[r];
        if (c > 0) v.emplace_back(c, static_cast<int32_t>(r));
      }
      std::stable_sort(v.begin(), v.end(), [](const std::pair<int64_t, int32_t>& a,
                                              const std::pair<int64_t, int32_t>& b) {
        return a.first > b.first;
      });
    }
  }, 2);
  std::vector<int64_t> item_start(static_cast<size_t>(R_) * B, -1), sfx_start(R_, -1);
  int64_t off = 0;
  for (int l = 0; l < L; ++l) {
    const auto& v = items[l];
    BlockItems it;
    it.n_items = static_cast<int64_t>(v.size());
    it.off = off;
    it.suffix = l == B;
    std::vector<int32_t> rows(v.size());
    std::vector<int64_t> ptr(v.size() + 1);
    ptr[0] = off;
    for (size_t i = 0; i < v.size(); ++i) {
      rows[i] = v[i].second;
      if (l < B) item_start[int64_t(v[i].second) * B + l] = ptr[i];
      else sfx_start[v[i].second] = ptr[i];
      ptr[i + 1] = ptr[i] + v[i].first;
    }
    it.nnz = ptr.back() - off;
    off = ptr.back();
    it.rows = upload(rows.data(), it.n_items, 0, 32, s);
    it.ptr = upload(ptr.data(), it.n_items + 1, 0, 64, s);
    bp->launches.push_back(std::move(it));
  }
  DGLHIP_CHECK(off == nnz_, "blocked plan covers " << off << " of " << nnz_ << " slots");
  std::vector<int32_t> absent;
  for (int64_t r = 0; r < R_; ++r)
    if (split->counts[r * B] == 0) absent.push_back(static_cast<int32_t>(r));
  bp->n_absent = static_cast<int64_t>(absent.size());
  bp->absent = upload(absent.data(), bp->n_absent, 0, 32, s);
  bp->indices = empty({nnz_}, 0, 32);
  bp->pos = empty({nnz_}, 0, 32);
  int32_t* oi = bp->indices.data<int32_t>();
  int32_t* op = bp->pos.data<int32_t>();
  if (on_device()) {
    rt::NDArray ist = upload(item_start.data(), R_ * B, 0, 64, s);
    rt::NDArray sst = upload(sfx_start.data(), R_, 0, 64, s);
    rt::NDArray pend = upload(split->pend.data(), R_, 0, 64, s);
    plan_block_scatter_device(R_, indptr_, indices_, split->lo, split->bs, B,
                              pend.data<int64_t>(), ist.data<int64_t>(), sst.data<int64_t>(), oi,
                              op, s);
    hip_ok(hipStreamSynchronize(s), "plan scatter");  // the staging arrays go out of scope
  } else {
    const int64_t lo = split->lo, bs = split->bs;
    parallel_for(R_, default_num_threads(), [&](int64_t b0, int64_t b1, int) {
      for (int64_t r = b0; r < b1; ++r) {
        const int64_t pe = split->pend[r];
        int64_t run_s = ip[r], prev = -1;
        for (int64_t k = ip[r]; k < pe; ++k) {
          const int64_t b = (int64_t(indices_[k]) - lo) / bs;
          if (b != prev) run_s = k;
          prev = b;
          const int64_t dst = item_start[r * B + b] + (k - run_s);
          oi[dst] = indices_[k];
          op[dst] = static_cast<int32_t>(k);
        }
        for (int64_t k = pe; k < ip[r + 1]; ++k) {
          const int64_t dst = sfx_start[r] + (k - pe);
          oi[dst] = indices_[k];
          op[dst] = static_cast<int32_t>(k);
        }
      }
    });
  }
  blocked_[B] = bp;
  return bp;
}

std::shared_ptr<Cuts> SpmmPlan::cuts(int64_t row_bytes, int64_t block_bytes, hipStream_t s) {
  const SpmmPolicy p = spmm_policy();
  if (!p.blocked || nnz_ == 0 || row_bytes <= p.block_min_row_bytes) return nullptr;
  const auto lh = span(s);
  const int B = block_count((lh.second - lh.first) * row_bytes, block_bytes);
  if (!B) return nullptr;
  return cuts_for(B, s);
}

std::shared_ptr<Cuts> SpmmPlan::cuts_for(int B, hipStream_t s) {
  DGLHIP_CHECK(B >= 1, "block count " << B);
  span(s);
  std::lock_guard<std::mutex> lk(mu_);
  auto hit = cuts_.find(B);
  if (hit != cuts_.end()) return hit->second;
  auto split = block_split(B, s);
  if (!split->ok) {
    cuts_[B] = nullptr;
    return nullptr;
  }
  auto c = std::make_shared<Cuts>();
  c->B = B;
  c->has_suffix = split->total_suffix > 0;
  c->n = B + 1 + (c->has_suffix ? 1 : 0);
  const int64_t* ip = host_indptr_->data();
  std::vector<int64_t> h(static_cast<size_t>(c->n) * R_);
  parallel_for(R_, default_num_threads(), [&](int64_t r0, int64_t r1, int) {
    for (int64_t r = r0; r < r1; ++r) {
      int64_t acc = ip[r];
      h[r] = acc;
      for (int b = 0; b < B; ++b) {
        acc += split->counts[r * B + b];
        h[(b + 1) * R_ + r] = acc;
      }
      if (c->has_suffix) h[(B + 1) * R_ + r] = ip[r + 1];
    }
  });
  c->data = upload(h.data(), c->n * R_, 0, 64, s);
  c->data.get()->shape = {c->n, R_};
  c->data.get()->dl.ndim = 2;
  c->data.get()->dl.shape = c->data.get()->shape.data();
  cuts_[B] = c;
  return c;
}

std::shared_ptr<SweepPlan> SpmmPlan::sweep(int64_t row_bytes, int mode, hipStream_t s) {
  const bool accum = mode == 2;
  const SweepPolicy sp = sweep_policy();
  int RPW = 19;  // rows per wave of the 128-float sweep kernel (dglhip_set_sweep_rows)
  DGLHIP_CHECK(dglhip_get_sweep_rows(&RPW) == 0, DGLGetLastError());
  if (!sp.on || !on_device() || nnz_ == 0 || nnz_ >= (int64_t(1) << 31) || R_ == 0) return nullptr;
  const auto lh = span(s);
  const int64_t table = (lh.second - lh.first) * row_bytes;
  if (table < (accum ? sp.accum_table_min : sp.table_min)) return nullptr;
  const int64_t want = cdiv(table, sp.block_bytes);
  if (want < 2 || want > 256) return nullptr;  // the barrier covers 256 blocks
  // measured on rows of 108-493 slots: sparser rows switch
  // rows every slot and many generations re-sweep every block, so those keep
  // the other schedules
  if (nnz_ < (accum ? sp.accum_min_slots : 128) * std::max<int64_t>(num_nonempty_, 1))
    return nullptr;
  const int B = static_cast<int>(want);
  // the layout is dealt over the waves one launch of THE kernel that will run
  // holds (its mode and the current gathers-in-flight knob decide its
  // occupancy), so that geometry is part of the key: a knob changed after
  // the plan was built gets a layout of its own instead of a mismatch
  const int per_cu = accum ? sp.accum_per_cu : 0;
  int64_t wpl = 0;
  DGLHIP_CHECK(dglhip_gspmm_sweep_stream_geometry_mode(RPW, per_cu, mode, &wpl) == 0 && wpl > 0,
               DGLGetLastError());
  const std::tuple<int, int, int64_t, int> key(B, mode, wpl, RPW);
  std::lock_guard<std::mutex> lk(mu_);
  auto hit = sweeps_.find(key);
  if (hit != sweeps_.end()) return hit->second;
  auto split = block_split(B, s);
  if (split->total_suffix != 0) {  // a row's blocks go back down: no run layout
    sweeps_[key] = nullptr;
    return nullptr;
  }
  auto sw = std::make_shared<SweepPlan>();
  sw->per_cu = per_cu;
  sw->B = B;
  sw->rows_per_wave = RPW;
  sw->accum = accum;
  // an accumulating run leaves rows without slots as they are: it deals only
  // the schedule's non-empty prefix when the order is degree-descending (a
  // caller's order that is not: every row, the empty ones rewritten as they are)
  const std::vector<int32_t>& ord = host_order(s);
  const int64_t* ip = host_indptr_->data();
  bool prefix = accum;
  for (int64_t i = 0; prefix && i < num_nonempty_; ++i) {
    const int64_t r = ord.empty() ? i : ord[i];
    prefix = ip[r + 1] > ip[r];
  }
  sw->rows_dealt = prefix ? num_nonempty_ : R_;
  sw->launches = cdiv(sw->rows_dealt, wpl * RPW);
  if (sw->launches > 16) {
    sweeps_[key] = nullptr;
    return nullptr;
  }
  const int64_t W = sw->launches * wpl;
  sw->waves_total = W;
  // the kernel's deal: row i of the schedule order -> wave (i / W odd ?
  // W - 1 - i % W : i % W), its row i / W; each wave's run in block b holds
  // its rows' block-b slots in that order; runs ordered (launch, block, wave)
  const std::vector<int32_t>& order = ord;
  const int32_t* cnt = split->counts.data();
  std::vector<int64_t> item_start(static_cast<size_t>(R_) * B, 0);
  std::vector<int64_t> seg(static_cast<size_t>(W) * B, 0);
  int64_t off = 0;
  for (int64_t l = 0; l < sw->launches; ++l) {
    for (int b = 0; b < B; ++b) {
      for (int64_t w = l * wpl; w < (l + 1) * wpl; ++w) {
        seg[w * B + b] = off;
        for (int j = 0; j < RPW; ++j) {
          const int64_t pos = (j & 1) ? (W - 1 - w) : w;
          const int64_t i = int64_t(j) * W + pos;
          if (i >= sw->rows_dealt) break;  // rows of a wave are a prefix of its rounds
          const int64_t r = order.empty() ? i : order[i];
          item_start[r * B + b] = off;
          off += cnt[r * B + b];
        }
      }
    }
  }
  DGLHIP_CHECK(off == nnz_, "sweep layout covers " << off << " of " << nnz_ << " slots");
  sw->lay = empty({nnz_}, 0, 32);
  sw->pos = empty({nnz_}, 0, 32);
  {
    rt::NDArray ist = upload(item_start.data(), R_ * B, 0, 64, s);
    rt::NDArray pend = upload(split->pend.data(), R_, 0, 64, s);
    plan_block_scatter_device(R_, indptr_, indices_, split->lo, split->bs, B,
                              pend.data<int64_t>(), ist.data<int64_t>(), nullptr,
                              sw->lay.data<int32_t>(), sw->pos.data<int32_t>(), s);
    sw->seg = upload(seg.data(), W * B, 0, 64, s);
    sw->counts = upload(cnt, R_ * B, 0, 32, s);
    hip_ok(hipStreamSynchronize(s), "sweep layout");  // the staging arrays go out of scope
  }
  sw->arrive = empty({sw->launches * (int64_t(B) * 8 + 1) * 32}, 0, 32);
  sweeps_[key] = sw;
  return sw;
}

const int64_t* SpmmPlan::plan_pos64(BlockedPlan& bp, hipStream_t s) {
  std::lock_guard<std::mutex> lk(mu_);
  if (!bp.pos64.defined()) {
    bp.pos64 = empty({nnz_}, 0, 64);
    if (on_device()) {
      plan_compose_device(nnz_, bp.pos.data<int32_t>(), nullptr, bp.pos64.data<int64_t>(), s);
    } else {
      const int32_t* p = bp.pos.data<int32_t>();
      int64_t* o = bp.pos64.data<int64_t>();
      for (int64_t j = 0; j < nnz_; ++j) o[j] = p[j];
    }
  }
  return bp.pos64.data<int64_t>();
}

const int64_t* SpmmPlan::plan_eidmap(BlockedPlan& bp, const int64_t* eid, hipStream_t s) {
  std::lock_guard<std::mutex> lk(mu_);
  // the CSR's edge ids have one content whatever copy of them the caller
  // holds (offloaded and brought back, for instance): one composed map
  if (!bp.eidmap.defined()) {
    bp.eidmap = empty({nnz_}, 0, 64);
    if (on_device()) {
      plan_compose_device(nnz_, bp.pos.data<int32_t>(), eid, bp.eidmap.data<int64_t>(), s);
    } else {
      const int32_t* p = bp.pos.data<int32_t>();
      int64_t* o = bp.eidmap.data<int64_t>();
      for (int64_t j = 0; j < nnz_; ++j) o[j] = eid[p[j]];
    }
  }
  return bp.eidmap.data<int64_t>();
}

SplitPlan& SpmmPlan::split_plan(int64_t threshold, bool skip_empty, int64_t chunk,
                                hipStream_t s) {
  std::lock_guard<std::mutex> lk(mu_);
  const auto key = std::make_tuple(threshold, skip_empty, chunk);
  auto hit = split_plans_.find(key);
  if (hit != split_plans_.end()) return hit->second;
  const int64_t* ip = host_indptr_->data();
  const std::vector<int32_t>& order = host_order(s);
  std::vector<int32_t> light, heavy;
  for (int64_t i = 0; i < R_; ++i) {
    const int32_t r = order[i];
    const int64_t d = ip[r + 1] - ip[r];
    if (skip_empty && d == 0) continue;
    (d > threshold ? heavy : light).push_back(r);
  }
  if (chunk <= 0) {
    int64_t heavy_slots = 0;
    for (int32_t r : heavy) heavy_slots += ip[r + 1] - ip[r];
    const int64_t chunk_waves = std::max<int64_t>(1, waves_ * 4 / 7);  // 4,096 on MI355X
    chunk = std::min<int64_t>(threshold, std::max<int64_t>(kChunkMin, cdiv(heavy_slots, chunk_waves)));
  }
  std::vector<int64_t> cptr(heavy.size() + 1, 0), beg, end;
  for (size_t h = 0; h < heavy.size(); ++h) {
    const int64_t b0 = ip[heavy[h]], b1 = ip[heavy[h] + 1];
    for (int64_t b = b0; b < b1; b += chunk) {
      beg.push_back(b);
      end.push_back(std::min(b + chunk, b1));
    }
    cptr[h + 1] = static_cast<int64_t>(beg.size());
  }
  SplitPlan sp;
  sp.n_light = static_cast<int64_t>(light.size());
  sp.n_heavy = static_cast<int64_t>(heavy.size());
  sp.n_chunks = static_cast<int64_t>(beg.size());
  sp.light = upload(light.data(), sp.n_light, 0, 32, s);
  sp.heavy = upload(heavy.data(), sp.n_heavy, 0, 32, s);
  sp.chunk_ptr = upload(cptr.data(), sp.n_heavy + 1, 0, 64, s);
  sp.beg = upload(beg.data(), sp.n_chunks, 0, 64, s);
  sp.end = upload(end.data(), sp.n_chunks, 0, 64, s);
  return split_plans_.emplace(key, std::move(sp)).first->second;
}

Tiers SpmmPlan::build_tiers(const int32_t* rows, const rt::NDArray& /*rows_dev*/, int64_t n,
                            hipStream_t s) {
  // rows: a degree-descending row list; tiers of rows of <= 8, <= 4 and 0 slots
  const int64_t* ip = host_indptr_->data();
  auto deg = [&](int64_t i) { return ip[rows[i] + 1] - ip[rows[i]]; };
  auto first_le = [&](int64_t t) {  // first position whose degree is <= t
    int64_t a = 0, b = n;
    while (a < b) {
      const int64_t m = (a + b) / 2;
      if (deg(m) <= t) b = m;
      else a = m + 1;
    }
    return a;
  };
  const int64_t c0 = first_le(8), c1 = first_le(4), c2 = first_le(0);
  Tiers t;
  t.n_long = c0;
  t.n_tail = n - c0;
  const int64_t bounds[3][3] = {{8, c0, c1}, {4, c1, c2}, {0, c2, n}};
  for (const auto& bd : bounds) {
    const int64_t maxd = bd[0], lo = bd[1], hi = bd[2];
    if (hi <= lo) continue;
    Tier tier;
    tier.maxd = static_cast<int>(maxd);
    tier.n = hi - lo;
    tier.rows = upload(rows + lo, tier.n, 0, 32, s);
    if (maxd > 0) {
      std::vector<int64_t> sp(tier.n + 1, 0);
      for (int64_t i = 0; i < tier.n; ++i) sp[i + 1] = sp[i] + deg(lo + i);
      tier.sp = upload(sp.data(), tier.n + 1, 0, 64, s);
      tier.cols = empty({std::max<int64_t>(sp.back(), 1)}, 0, 32);
      if (on_device()) {
        plan_tier_cols_device(tier.n, tier.rows.data<int32_t>(), indptr_, indices_,
                              tier.sp.data<int64_t>(), tier.cols.data<int32_t>(), s);
      } else {
        int32_t* c = tier.cols.data<int32_t>();
        for (int64_t i = 0; i < tier.n; ++i)
          for (int64_t j = 0; j < sp[i + 1] - sp[i]; ++j) c[sp[i] + j] = indices_[ip[rows[lo + i]] + j];
      }
    }
    t.tiers.push_back(std::move(tier));
  }
  if (on_device()) hip_ok(hipStreamSynchronize(s), "plan tiers");
  return t;
}

Tiers& SpmmPlan::tiers_plain(bool skip, hipStream_t s) {
  std::lock_guard<std::mutex> lk(mu_);
  const int64_t key = skip ? 1 : 0;
  auto hit = tiers_.find(key);
  if (hit != tiers_.end()) return hit->second;
  const int64_t n = skip ? num_nonempty_ : R_;
  const std::vector<int32_t>& order = host_order(s);
  return tiers_.emplace(key, build_tiers(order.data(), rt::NDArray(), n, s)).first->second;
}

Tiers& SpmmPlan::tiers_light(const SplitPlan& sp, int64_t threshold, bool skip, hipStream_t s) {
  std::lock_guard<std::mutex> lk(mu_);
  const int64_t key = 2 + threshold * 2 + (skip ? 1 : 0);
  auto hit = tiers_.find(key);
  if (hit != tiers_.end()) return hit->second;
  // the light list, as split_plan made it: the schedule minus the heavy rows
  const int64_t* ip = host_indptr_->data();
  std::vector<int32_t> light;
  light.reserve(sp.n_light);
  const std::vector<int32_t>& order = host_order(s);
  for (int64_t i = 0; i < R_; ++i) {
    const int32_t r = order[i];
    const int64_t d = ip[r + 1] - ip[r];
    if ((skip && d == 0) || d > threshold) continue;
    light.push_back(r);
  }
  return tiers_.emplace(key, build_tiers(light.data(), rt::NDArray(), sp.n_light, s))
      .first->second;
}

PlanDevice::PlanDevice(const SpmmPlan& p) {
  if (!p.on_device()) return;
  int cur = 0;
  hip_ok(hipGetDevice(&cur), "hipGetDevice");
  if (cur != p.device_id()) {
    hip_ok(hipSetDevice(p.device_id()), "hipSetDevice");
    prev_ = cur;
  }
}

PlanDevice::~PlanDevice() {
  if (prev_ >= 0) (void)hipSetDevice(prev_);
}

// ---------------------------------------------------------------------------
// The planned run
// ---------------------------------------------------------------------------
namespace {

struct RunArgs {
  int msg, red;
  int64_t F;
  const void* ufeat;
  int64_t ldu;    // caller's row stride (0 or F: dense)
  int64_t urows;  // rows of ufeat
  const float* efeat;
  int64_t elen;
  int emode;
  const int64_t* erow;
  float* out;
  int64_t* arg;
};

enum Path { PATH_HOST = 0, PATH_ROWS = 1, PATH_BLOCKED = 2, PATH_MAX_BLOCKED = 3, PATH_SWEEP = 4 };

// mean_add on the blocked schedule (DGLHIP_BLOCKED_MEAN_ADD;
// dglhip_set_blocked_mean_add). On by default since r06's box check: same
// bits as the one-launch schedule, GraphSAGE-mean Reddit-shaped epoch
// 15.4 -> 14.2 ms (profiles/r06/sage_blocked_mean_add/). 0 restores the
// one-launch schedule.
int g_blocked_mean_add = [] {
  const char* e = std::getenv("DGLHIP_BLOCKED_MEAN_ADD");
  return e && *e ? std::atoi(e) : 1;
}();

inline bool blocked_mean_add() { return g_blocked_mean_add != 0; }

struct Decision {
  Path path = PATH_ROWS;
  std::shared_ptr<BlockedPlan> bp;
  std::shared_ptr<Cuts> cuts;
  std::shared_ptr<SweepPlan> sw;
  bool pad = false;     // gather from a padded copy (workspace)
  int64_t ld = 0;       // row stride the kernels read (0: dense)
  int64_t split = 0;
  // workspace pieces (bytes, 256-B aligned offsets)
  int64_t ws_pad = 0, ws_vals = 0, ws_map = 0, ws_partial = 0;
  // mean_add on the blocked schedule: the running sums' own rows (out holds
  // the value the mean is added to)
  int64_t ws_sums = 0;
  int64_t total() const { return ws_pad + ws_vals + ws_map + ws_partial + ws_sums; }
};

inline int64_t align256(int64_t b) { return (b + 255) / 256 * 256; }

bool pad_rows(const SpmmPolicy& p, int msg, int red, int64_t F, int64_t urows) {
  return p.pad_rows && (msg == DGLHIP_MSG_COPY_U || msg == DGLHIP_MSG_U_MUL_E) &&
         (red == DGLHIP_REDUCE_SUM || red == DGLHIP_REDUCE_MEAN || accum(red)) &&
         urows * F * 4 >= p.pad_min_bytes && padded_width(F) != F;
}

void check_args(const SpmmPlan& plan, const RunArgs& a) {
  DGLHIP_CHECK(a.msg >= 0 && a.msg <= 3, "unknown msg op " << a.msg);
  DGLHIP_CHECK(a.red >= 0 && a.red <= 4, "unknown reduce op " << a.red);
  DGLHIP_CHECK(a.F >= 0, "negative feat_len");
  DGLHIP_CHECK(a.emode >= DGLHIP_EDGE_BY_SLOT && a.emode <= DGLHIP_EDGE_BY_MAP,
               "unknown edge layout " << a.emode);
  DGLHIP_CHECK(a.ldu == 0 || a.ldu == a.F || (a.ldu > a.F && a.ldu % 2 == 0),
               "ufeat_ld " << a.ldu << ": 0, feat_len, or an even width > feat_len");
  DGLHIP_CHECK(a.ldu <= a.F || (a.msg == DGLHIP_MSG_COPY_U || a.msg == DGLHIP_MSG_U_MUL_E),
               "row-strided source rows: copy_u or u_mul_e");
  DGLHIP_CHECK(a.ldu <= a.F || a.red != DGLHIP_REDUCE_MAX, "row-strided source rows: not max");
  const bool use_u = a.msg != DGLHIP_MSG_COPY_E;
  const bool use_e = !copies_u(a.msg);
  DGLHIP_CHECK(!use_u || a.ufeat || plan.nnz() == 0, "ufeat is null");
  DGLHIP_CHECK(!use_e || a.efeat || plan.nnz() == 0, "efeat is null");
  DGLHIP_CHECK(!use_e || (a.elen >= 1 && a.F % a.elen == 0),
               "edge feature length " << a.elen << " must divide feat_len " << a.F);
  DGLHIP_CHECK(!use_e || a.emode == DGLHIP_EDGE_BY_SLOT || a.erow != nullptr ||
                   a.emode == DGLHIP_EDGE_BY_EID,
               "edge layout " << a.emode << " needs erow");
  DGLHIP_CHECK(a.out != nullptr || plan.num_rows() == 0 || a.F == 0, "null out");
}

Decision decide(SpmmPlan& plan, const RunArgs& a, hipStream_t s) {
  Decision d;
  if (!plan.on_device()) {
    d.path = PATH_HOST;
    return d;
  }
  const SpmmPolicy p = spmm_policy();
  const bool cu = copies_u(a.msg);
  const bool sumlike = a.red == DGLHIP_REDUCE_SUM || a.red == DGLHIP_REDUCE_MEAN ||
                       a.red == DGLHIP_REDUCE_SUM_ACCUM;
  const int64_t elem = a.msg == DGLHIP_MSG_COPY_U_BF16 ? 2 : 4;
  const bool strided = a.ldu > a.F;
  const int64_t ld_in = strided ? a.ldu : a.F;
  const bool fp32u = a.msg != DGLHIP_MSG_COPY_U_BF16;
  if (a.F == 0 || plan.num_rows() == 0) return d;
  if ((a.red == DGLHIP_REDUCE_SUM || a.red == DGLHIP_REDUCE_MEAN ||
       a.red == DGLHIP_REDUCE_SUM_ACCUM) && a.msg == DGLHIP_MSG_COPY_U &&
      a.ufeat && !a.efeat && !strided && a.F == 128) {
    // tables past the L2-sized blocked schedule's range: the source sweep
    // (running sums in LDS, no per-block pass over out)
    d.sw = plan.sweep(a.F * 4,
                      a.red == DGLHIP_REDUCE_SUM_ACCUM ? 2 : (a.red == DGLHIP_REDUCE_MEAN ? 1 : 0),
                      s);
    if (d.sw) {
      d.path = PATH_SWEEP;
      return d;
    }
  }
  // out + mean (GraphSAGE's narrowing layer, kernel.gspmm_mean_add): the
  // blocked chains run into rows of their own, then one pass adds sum / deg
  // to out (r06: the same bits as the one-launch store, 3.4 -> ~2.1 ms at F = 41
  // on the headline graph)
  const bool mean_add = blocked_mean_add() && a.red == DGLHIP_REDUCE_MEAN_ACCUM &&
                        a.msg == DGLHIP_MSG_COPY_U && !a.efeat;
  if ((sumlike || mean_add) && a.ufeat &&
      ((cu && !a.efeat) || (a.msg == DGLHIP_MSG_U_MUL_E && a.efeat))) {
    d.bp = plan.blocked(ld_in * elem, p.block_bytes, s);
    if (d.bp) {
      d.path = PATH_BLOCKED;
      if (mean_add) d.ws_sums = align256(plan.num_rows() * a.F * 4);
      if (!strided && fp32u && pad_rows(p, a.msg, DGLHIP_REDUCE_SUM, a.F, a.urows)) {
        d.pad = true;
        d.ld = padded_width(a.F);
        d.ws_pad = align256(a.urows * d.ld * 4);
      } else {
        d.ld = strided ? a.ldu : 0;
      }
      if (a.msg == DGLHIP_MSG_U_MUL_E) {
        if (a.elen == 1) d.ws_vals = align256(plan.nnz() * 4);
        if (a.emode == DGLHIP_EDGE_BY_MAP) d.ws_map = align256(plan.nnz() * 8);
      }
      return d;
    }
  }
  if (a.red == DGLHIP_REDUCE_MAX && a.ufeat && !strided && fp32u &&
      (a.msg == DGLHIP_MSG_COPY_U ||
       (a.msg == DGLHIP_MSG_U_MUL_E &&
        (a.emode == DGLHIP_EDGE_BY_SLOT ||
         (a.emode == DGLHIP_EDGE_BY_EID && plan.eid_identity(a.erow, s)))))) {
    // max over the blocks' row ranges, continued block by block: the same
    // values and (strict >, slot order) the same argmax; edge values by edge
    // id stay in one launch (a dependent 4-B load per slot: 8.75 vs 8.50 ms)
    d.cuts = plan.cuts(a.F * 4, p.block_bytes, s);
    if (d.cuts) {
      d.path = PATH_MAX_BLOCKED;
      return d;
    }
  }
  d.path = PATH_ROWS;
  d.split = a.red != DGLHIP_REDUCE_MAX ? plan.heavy_threshold() : 0;
  if (strided) {
    d.ld = a.ldu;
  } else if (fp32u && pad_rows(p, a.msg, a.red, a.F, a.urows)) {
    d.pad = true;
    d.ld = padded_width(a.F);
    d.ws_pad = align256(a.urows * d.ld * 4);
  }
  if (d.split) {
    const bool skip = accum(a.red);
    const int64_t chunk = p.row_split < 0 ? -1 : d.split;
    const SplitPlan& sp = plan.split_plan(d.split, skip, chunk, s);
    d.ws_partial = align256(sp.n_chunks * a.F * 4);
  }
  return d;
}

struct Workspace {
  char* base;
  int64_t bytes;
  char* take(int64_t n) {
    char* p = base;
    base += n;
    return p;
  }
};

void short_rows(SpmmPlan& plan, const RunArgs& a, const Tiers& t, const void* uf, int64_t ld,
                hipStream_t s) {
  for (const Tier& tier : t.tiers) {
    if (tier.maxd == 0 && accum(a.red)) continue;  // nothing to add
    DGLHIP_CHECK(dglhip_gspmm_short_rows_device(
                     a.msg, a.red, tier.n, a.F, tier.maxd, plan.num_rows(),
                     tier.rows.data<int32_t>(),
                     tier.maxd ? tier.sp.data<int64_t>() : nullptr,
                     tier.maxd ? tier.cols.data<int32_t>() : nullptr,
                     static_cast<const float*>(uf), a.out, ld, s) == 0,
                 DGLGetLastError());
  }
}

void run_rows(SpmmPlan& plan, const RunArgs& a, int64_t nrows, const int64_t* eid, const void* uf,
              int64_t ld, hipStream_t s) {
  if (ld) {
    DGLHIP_CHECK(dglhip_gspmm_strided_device(a.msg, a.red, nrows, a.F, ld, plan.indptr(),
                                             plan.indices(), eid, static_cast<const float*>(uf),
                                             a.efeat, a.elen, a.out, plan.row_order(), s) == 0,
                 DGLGetLastError());
  } else {
    DGLHIP_CHECK(dglhip_gspmm_device(a.msg, a.red, nrows, a.F, plan.indptr(), plan.indices(), eid,
                                     static_cast<const float*>(uf), a.efeat, a.elen, a.out,
                                     a.arg, plan.row_order(), s) == 0,
                 DGLGetLastError());
  }
}

void run_planned(SpmmPlan& plan, const RunArgs& a, const Decision& d, void* workspace,
                 int64_t ws_bytes, hipStream_t s) {
  const SpmmPolicy p = spmm_policy();
  DGLHIP_CHECK(ws_bytes >= d.total(), "workspace of " << ws_bytes << " bytes, the run needs "
                                                      << d.total());
  DGLHIP_CHECK(d.total() == 0 || workspace != nullptr, "null workspace");
  Workspace ws{static_cast<char*>(workspace), ws_bytes};
  const int64_t elen = copies_u(a.msg) ? 0 : a.elen;
  const void* uf = a.ufeat;
  if (d.pad) {
    char* up = ws.take(d.ws_pad);
    plan_pad_rows_device(a.urows, a.F, d.ld, static_cast<const float*>(a.ufeat),
                         reinterpret_cast<float*>(up), s);
    uf = up;
  }
  if (d.path == PATH_SWEEP) {
    const SweepPlan& sw = *d.sw;
    const SweepPolicy sp = sweep_policy();
    DGLHIP_CHECK(dglhip_gspmm_sweep_stream_device(
                     sw.rows_dealt, sw.waves_total, plan.row_order(),
                     sw.counts.data<int32_t>(), sw.B, sw.seg.data<int64_t>(),
                     sw.lay.data<int32_t>(), plan.indptr(), static_cast<const float*>(uf), a.out,
                     sw.accum ? 2 : (a.red == DGLHIP_REDUCE_MEAN ? 1 : 0), sw.rows_per_wave,
                     sw.per_cu, sw.arrive.data<int32_t>(), sw.arrive.numel(), sp.lag, sp.max_spin,
                     s) == 0,
                 DGLGetLastError());
    return;
  }
  if (d.path == PATH_BLOCKED) {
    BlockedPlan& bp = *d.bp;
    const bool first_writes = a.red != DGLHIP_REDUCE_SUM_ACCUM;
    // mean_add: the chains in their own rows, added to out at the end
    float* sums = d.ws_sums ? reinterpret_cast<float*>(ws.take(d.ws_sums)) : a.out;
    if (first_writes && bp.n_absent)
      plan_zero_rows_device(bp.n_absent, bp.absent.data<int32_t>(), a.F, sums, s);
    const float* ev = nullptr;     // edge values in plan order (scalar weights)
    const int64_t* erows = nullptr;  // or their rows per plan slot
    if (a.msg == DGLHIP_MSG_U_MUL_E) {
      // the edge-value row of every plan slot: the CSR slot itself, its edge
      // id (cached per plan), or the caller's map composed for this call
      const int64_t* rows = nullptr;
      if (a.emode == DGLHIP_EDGE_BY_SLOT) {
        rows = plan.plan_pos64(bp, s);
      } else if (a.emode == DGLHIP_EDGE_BY_EID) {
        rows = plan.eid_identity(a.erow, s) ? plan.plan_pos64(bp, s)
                                            : plan.plan_eidmap(bp, a.erow, s);
      } else {
        int64_t* m = reinterpret_cast<int64_t*>(ws.take(d.ws_map));
        plan_compose_device(plan.nnz(), bp.pos.data<int32_t>(), a.erow, m, s);
        rows = m;
      }
      if (a.elen == 1) {
        float* v = reinterpret_cast<float*>(ws.take(d.ws_vals));
        plan_gather_vals_device(plan.nnz(), rows, a.efeat, v, s);
        ev = v;
      } else {
        erows = rows;
      }
    }
    const int64_t ldk = d.ld;
    const bool paired = a.msg == DGLHIP_MSG_COPY_U &&
                        dglhip_gspmm_pair_items_ok(a.msg, a.F, ldk, a.urows) == 1;
    for (size_t i = 0; i < bp.launches.size(); ++i) {
      const BlockItems& it = bp.launches[i];
      if (paired) {  // narrow rows: two slots per gather, the same chains
        DGLHIP_CHECK(dglhip_gspmm_pair_items_device(
                         it.n_items, a.F, ldk, a.urows, it.rows.data<int32_t>(),
                         it.ptr.data<int64_t>(), (i == 0 && first_writes) ? 0 : 1,
                         bp.indices.data<int32_t>(), static_cast<const float*>(uf), sums,
                         s) == 0,
                     DGLGetLastError());
        continue;
      }
      DGLHIP_CHECK(dglhip_gspmm_items_device(
                       a.msg, it.n_items, a.F, it.rows.data<int32_t>(), it.ptr.data<int64_t>(),
                       (i == 0 && first_writes) ? 0 : 1, bp.indices.data<int32_t>(),
                       ev ? nullptr : erows, static_cast<const float*>(uf), ldk,
                       ev ? ev : (a.msg == DGLHIP_MSG_U_MUL_E ? a.efeat : nullptr),
                       elen, sums, s) == 0,
                   DGLGetLastError());
    }
    if (a.red == DGLHIP_REDUCE_MEAN) plan_div_degree_device(plan.num_rows(), a.F, plan.indptr(),
                                                            a.out, s);
    if (d.ws_sums) plan_add_mean_device(plan.num_rows(), a.F, plan.indptr(), sums, a.out, s);
    return;
  }
  if (d.path == PATH_MAX_BLOCKED) {
    const Cuts& c = *d.cuts;
    const int64_t* base = c.data.data<int64_t>();
    const int64_t* eid = nullptr;
    for (int64_t b = 0; b + 1 < c.n; ++b) {
      DGLHIP_CHECK(dglhip_gspmm_max_ranges_device(
                       a.msg, plan.num_rows(), a.F, plan.indptr(), base + b * plan.num_rows(),
                       base + (b + 1) * plan.num_rows(), b ? 1 : 0, plan.indices(), eid,
                       static_cast<const float*>(uf), a.efeat, a.elen, a.out, a.arg,
                       plan.row_order(), s) == 0,
                   DGLGetLastError());
    }
    return;
  }
  // one wave per row over the degree-descending schedule; heavy rows chunked
  const int64_t* eid = nullptr;
  if (!copies_u(a.msg) && a.emode != DGLHIP_EDGE_BY_SLOT) {
    if (a.emode == DGLHIP_EDGE_BY_MAP) eid = a.erow;
    else if (!plan.eid_identity(a.erow, s)) eid = a.erow;
  }
  const bool skip = accum(a.red);  // empty rows: nothing to add
  const bool tiered = p.short_rows && copies_u(a.msg) &&
                      (a.red == DGLHIP_REDUCE_SUM || a.red == DGLHIP_REDUCE_MEAN || accum(a.red));
  const int64_t ld = d.ld;
  if (d.split) {
    const int64_t chunk = p.row_split < 0 ? -1 : d.split;
    SplitPlan& sp = plan.split_plan(d.split, skip, chunk, s);
    float* partial = reinterpret_cast<float*>(ws.take(d.ws_partial));
    int64_t n_light = sp.n_light;
    const Tiers* tail = nullptr;
    if (tiered) {
      const Tiers& t = plan.tiers_light(sp, d.split, skip, s);
      if (t.n_tail >= p.tier_min_rows) {
        n_light = t.n_long;
        tail = &t;
      }
    }
    DGLHIP_CHECK(dglhip_gspmm_chunked_device(
                     a.msg, a.red, a.F, plan.indptr(), plan.indices(), eid,
                     static_cast<const float*>(uf), a.efeat, elen ? elen : 1, a.out, n_light,
                     sp.light.data<int32_t>(), sp.n_chunks, sp.beg.data<int64_t>(),
                     sp.end.data<int64_t>(), sp.n_heavy, sp.heavy.data<int32_t>(),
                     sp.chunk_ptr.data<int64_t>(), partial, ld, s) == 0,
                 DGLGetLastError());
    if (tail) short_rows(plan, a, *tail, uf, ld, s);
    return;
  }
  const int64_t nrows = skip ? plan.num_nonempty() : plan.num_rows();
  if (tiered) {
    const Tiers& t = plan.tiers_plain(skip, s);
    if (t.n_tail >= p.tier_min_rows) {
      run_rows(plan, a, t.n_long, eid, uf, ld, s);
      short_rows(plan, a, t, uf, ld, s);
      return;
    }
  }
  run_rows(plan, a, nrows, eid, uf, ld, s);
}

RunArgs make_args(int msg, int red, int64_t F, const void* ufeat, int64_t ldu, int64_t urows,
                  const float* efeat, int64_t elen, int emode, const int64_t* erow, float* out,
                  int64_t* arg) {
  return RunArgs{msg, red, F, ufeat, ldu == F ? 0 : ldu, urows, efeat,
                 copies_u(msg) ? 0 : elen, emode, erow, out, arg};
}

SpmmPlan* as_plan(DGLHipSpmmPlan h) {
  DGLHIP_CHECK(h != nullptr, "null g-SpMM plan");
  return reinterpret_cast<SpmmPlan*>(h);
}

}  // namespace

// Workspace bytes and the run (also used by the registry, registry.cc).
int64_t spmm_plan_workspace(SpmmPlan& plan, int msg, int red, int64_t F, int64_t ldu,
                            int64_t urows, int64_t elen, int emode, const int64_t* erow,
                            hipStream_t s) {
  RunArgs a = make_args(msg, red, F, reinterpret_cast<const void*>(1), ldu, urows,
                        reinterpret_cast<const float*>(copies_u(msg) ? nullptr : (void*)1), elen,
                        emode, erow, nullptr, nullptr);
  if (msg == DGLHIP_MSG_COPY_E) a.ufeat = nullptr;
  return decide(plan, a, s).total();
}

void spmm_plan_run(SpmmPlan& plan, int msg, int red, int64_t F, const void* ufeat, int64_t ldu,
                   int64_t urows, const float* efeat, int64_t elen, int emode,
                   const int64_t* erow, float* out, int64_t* arg, void* workspace,
                   int64_t ws_bytes, hipStream_t s) {
  const RunArgs a = make_args(msg, red, F, ufeat, ldu, urows, efeat, elen, emode, erow, out, arg);
  check_args(plan, a);
  if (plan.num_rows() == 0 || F == 0) return;
  if (!plan.on_device()) {
    DGLHIP_CHECK(a.ldu == 0, "host g-SpMM reads dense rows");
    const int64_t* eid = nullptr;
    if (!copies_u(msg) && emode != DGLHIP_EDGE_BY_SLOT) eid = erow;
    DGLHIP_CHECK(dglhip_gspmm_host(msg, red, plan.num_rows(), F, plan.indptr(), plan.indices(),
                                   eid, static_cast<const float*>(ufeat), efeat,
                                   copies_u(msg) ? 0 : elen, out, arg, 0) == 0,
                 DGLGetLastError());
    return;
  }
  const Decision d = decide(plan, a, s);
  run_planned(plan, a, d, workspace, ws_bytes, s);
}

int spmm_plan_path(SpmmPlan& plan, int msg, int red, int64_t F, int64_t ldu, int64_t urows,
                   int64_t elen, int emode, const int64_t* erow, hipStream_t s,
                   int64_t* launches) {
  RunArgs a = make_args(msg, red, F, reinterpret_cast<const void*>(1), ldu, urows,
                        reinterpret_cast<const float*>(copies_u(msg) ? nullptr : (void*)1), elen,
                        emode, erow, nullptr, nullptr);
  if (msg == DGLHIP_MSG_COPY_E) a.ufeat = nullptr;
  const Decision d = decide(plan, a, s);
  if (launches) {
    *launches = d.path == PATH_BLOCKED ? static_cast<int64_t>(d.bp->launches.size())
                : d.path == PATH_MAX_BLOCKED ? d.cuts->n - 1
                : d.path == PATH_SWEEP ? d.sw->launches : 1;
  }
  return d.path;
}

}  // namespace dglhip

using namespace dglhip;

extern "C" {

int dglhip_set_blocked_mean_add(int on) {
  const int old = g_blocked_mean_add;
  g_blocked_mean_add = on ? 1 : 0;
  return old;
}

int dglhip_set_sweep_schedule(int on, int64_t table_min, int64_t block_bytes, int lag,
                              int max_spin, int64_t accum_table_min, int64_t accum_min_slots,
                              int accum_per_cu) {
  API_BEGIN();
  DGLHIP_CHECK(table_min >= 0 && block_bytes > 0 && lag >= 0 && max_spin >= 0 &&
                   accum_table_min >= 0 && accum_min_slots >= 0 && accum_per_cu >= 0,
               "invalid sweep schedule");
  std::lock_guard<std::mutex> lk(g_pol_mu);
  SweepPolicy& p = sweep_ref();
  p.on = on != 0 ? 1 : 0;
  p.table_min = table_min;
  p.block_bytes = block_bytes;
  p.lag = lag;
  p.max_spin = max_spin;
  p.accum_table_min = accum_table_min;
  p.accum_min_slots = accum_min_slots;
  p.accum_per_cu = accum_per_cu;
  API_END();
}

int dglhip_get_sweep_schedule(int* on, int64_t* table_min, int64_t* block_bytes, int* lag,
                              int* max_spin, int64_t* accum_table_min, int64_t* accum_min_slots,
                              int* accum_per_cu) {
  API_BEGIN();
  DGLHIP_CHECK(on && table_min && block_bytes && lag && max_spin && accum_table_min &&
                   accum_min_slots && accum_per_cu,
               "null pointer argument");
  const SweepPolicy p = sweep_policy();
  *on = p.on;
  *table_min = p.table_min;
  *block_bytes = p.block_bytes;
  *lag = p.lag;
  *max_spin = p.max_spin;
  *accum_table_min = p.accum_table_min;
  *accum_min_slots = p.accum_min_slots;
  *accum_per_cu = p.accum_per_cu;
  API_END();
}

int dglhip_spmm_get_policy(DGLHipSpmmPolicy* out) {
  API_BEGIN();
  DGLHIP_CHECK(out != nullptr, "null pointer argument");
  const SpmmPolicy p = spmm_policy();
  out->row_split = p.row_split;
  out->blocked = p.blocked;
  out->short_rows = p.short_rows;
  out->pad_rows = p.pad_rows;
  out->block_bytes = p.block_bytes;
  out->block_table_min = p.block_table_min;
  out->block_table_max = p.block_table_max;
  out->block_min_slots = p.block_min_slots;
  out->block_max_stretch = p.block_max_stretch;
  out->block_max_suffix = p.block_max_suffix;
  out->block_min_row_bytes = p.block_min_row_bytes;
  out->tier_min_rows = p.tier_min_rows;
  out->pad_min_bytes = p.pad_min_bytes;
  API_END();
}

int dglhip_spmm_set_policy(const DGLHipSpmmPolicy* in) {
  API_BEGIN();
  DGLHIP_CHECK(in != nullptr, "null pointer argument");
  SpmmPolicy p;
  p.row_split = in->row_split;
  p.blocked = in->blocked != 0;
  p.short_rows = in->short_rows != 0;
  p.pad_rows = in->pad_rows != 0;
  p.block_bytes = in->block_bytes;
  p.block_table_min = in->block_table_min;
  p.block_table_max = in->block_table_max;
  p.block_min_slots = in->block_min_slots;
  p.block_max_stretch = in->block_max_stretch;
  p.block_max_suffix = in->block_max_suffix;
  p.block_min_row_bytes = in->block_min_row_bytes;
  p.tier_min_rows = in->tier_min_rows;
  p.pad_min_bytes = in->pad_min_bytes;
  set_spmm_policy(p);
  API_END();
}

int dglhip_spmm_split_threshold(int64_t nnz, int64_t max_degree, int64_t waves, int64_t* out) {
  API_BEGIN();
  DGLHIP_CHECK(out != nullptr, "null pointer argument");
  *out = split_threshold(spmm_policy(), nnz, max_degree, waves > 0 ? waves : kRefWaves);
  API_END();
}

int dglhip_spmm_padded_width(int64_t feat_len, int64_t* out) {
  API_BEGIN();
  DGLHIP_CHECK(out != nullptr && feat_len >= 1, "bad argument");
  *out = padded_width(feat_len);
  API_END();
}

int dglhip_spmm_plan_create(int device_type, int device_id, int64_t num_rows, int64_t num_cols,
                            int64_t nnz, const int64_t* indptr, const int32_t* indices,
                            const int64_t* host_indptr, const int32_t* row_order, void* stream,
                            DGLHipSpmmPlan* out) {
  API_BEGIN();
  DGLHIP_CHECK(out != nullptr, "null pointer argument");
  *out = nullptr;
  int prev = 0;
  const bool dev = device_type == rt::kDLROCM;
  if (dev) {
    hip_ok(hipGetDevice(&prev), "hipGetDevice");
    hip_ok(hipSetDevice(device_id), "hipSetDevice");
  }
  try {
    auto* p = new SpmmPlan(device_type, device_id, num_rows, num_cols, nnz, indptr, indices,
                           host_indptr, row_order, static_cast<hipStream_t>(stream));
    *out = reinterpret_cast<DGLHipSpmmPlan>(p);
  } catch (...) {
    if (dev) (void)hipSetDevice(prev);
    throw;
  }
  if (dev) hip_ok(hipSetDevice(prev), "hipSetDevice");
  API_END();
}

int dglhip_spmm_plan_free(DGLHipSpmmPlan plan) {
  API_BEGIN();
  SpmmPlan* p = reinterpret_cast<SpmmPlan*>(plan);
  if (p) {
    PlanDevice guard(*p);
    delete p;
  }
  API_END();
}

int dglhip_spmm_plan_workspace(DGLHipSpmmPlan plan, int msg_op, int reduce_op, int64_t feat_len,
                               int64_t ufeat_ld, int64_t num_src_rows, int64_t efeat_len,
                               int edge_layout, const int64_t* erow, void* stream,
                               int64_t* bytes) {
  API_BEGIN();
  DGLHIP_CHECK(bytes != nullptr, "null pointer argument");
  PlanDevice guard(*as_plan(plan));
  *bytes = spmm_plan_workspace(*as_plan(plan), msg_op, reduce_op, feat_len, ufeat_ld,
                               num_src_rows, efeat_len, edge_layout, erow,
                               static_cast<hipStream_t>(stream));
  API_END();
}

int dglhip_spmm_plan_run(DGLHipSpmmPlan plan, int msg_op, int reduce_op, int64_t feat_len,
                         const void* ufeat, int64_t ufeat_ld, int64_t num_src_rows,
                         const float* efeat, int64_t efeat_len, int edge_layout,
                         const int64_t* erow, float* out, int64_t* arg_out, void* workspace,
                         int64_t workspace_bytes, void* stream) {
  API_BEGIN();
  PlanDevice guard(*as_plan(plan));
  spmm_plan_run(*as_plan(plan), msg_op, reduce_op, feat_len, ufeat, ufeat_ld, num_src_rows, efeat,
                efeat_len, edge_layout, erow, out, arg_out, workspace, workspace_bytes,
                static_cast<hipStream_t>(stream));
  API_END();
}

int dglhip_spmm_plan_schedule(DGLHipSpmmPlan plan, int msg_op, int reduce_op, int64_t feat_len,
                              int64_t ufeat_ld, int64_t num_src_rows, int64_t efeat_len,
                              int edge_layout, const int64_t* erow, void* stream, int* path,
                              int64_t* launches) {
  API_BEGIN();
  PlanDevice guard(*as_plan(plan));
  const int pth = spmm_plan_path(*as_plan(plan), msg_op, reduce_op, feat_len, ufeat_ld,
                                 num_src_rows, efeat_len, edge_layout, erow,
                                 static_cast<hipStream_t>(stream), launches);
  if (path) *path = pth;
  API_END();
}

int dglhip_spmm_plan_stats(DGLHipSpmmPlan plan, int64_t* stats) {
  API_BEGIN();
  DGLHIP_CHECK(stats != nullptr, "null pointer argument");
  SpmmPlan& p = *as_plan(plan);
  stats[0] = p.num_rows();
  stats[1] = p.num_cols();
  stats[2] = p.nnz();
  stats[3] = p.max_degree();
  stats[4] = p.num_nonempty();
  stats[5] = p.waves();
  stats[6] = p.heavy_threshold();
  API_END();
}

}  // extern "C"
