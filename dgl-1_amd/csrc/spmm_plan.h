// Launch plan of a g-SpMM over one CSR (rows = destinations): the schedule
// choice behind the C-ABI (dglhip_spmm_plan_*, include/dgl_hip.h).
//
// The reference reaches its sparse product through F.spmm
// (python/dgl/backend/pytorch/tensor.py:145-146) on an adjacency that
// GraphIndex.adjacency_matrix builds once and caches per context
// (python/dgl/graph_index.py:537-585). The plan is that cache for this
// engine: built once per CSR and device, it holds every schedule the g-SpMM
// kernels run over it, decided and laid out natively:
//   * the source-blocked schedule: B launches over contiguous
//     source blocks, items = rows with slots in a block, longest first, their
//     slots re-laid in item order; rows whose blocks decrease along their
//     slots keep a monotone prefix and run the rest as a suffix launch; the
//     same split as per-row sub-ranges (cuts) for the kernels that keep the
//     CSR's slot indices (max, g-SDDMM, fused GAT);
//   * the heavy-row split (rows cut into chunks whose partials are added in
//     order) and the short-row tiers of a degree-descending schedule;
//   * the run: which of these a call takes, the padded-stride copy of
//     line-straddling rows, the edge values in plan order, the mean's division.
// Everything E-sized (the walk over the slots, the scatter into item order,
// the tiers' column ids) runs as device kernels on a ROCm CSR and as host
// loops on a host CSR; the R x B-sized bookkeeping (sorting rows by their
// slot counts) runs on the host.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <vector>

#include "runtime.h"

namespace dglhip {

// Schedule policy (process-wide; dglhip_spmm_get_policy / _set_policy).
struct SpmmPolicy {
  int64_t row_split = -1;          // -1 auto, 0 off, > 0 explicit chunk length
  int blocked = 1;                 // source-blocked schedule where exact (0: off)
  int short_rows = 1;              // short-row tiers (0: off)
  int pad_rows = 1;                // padded-stride gathers (0: off)
  int64_t block_bytes = 6 << 20;   // source slice per launch
  int64_t block_table_min = 16 << 20;
  int64_t block_table_max = 256 << 20;
  int64_t block_min_slots = 12;    // slots per row and block, on average
  double block_max_stretch = 3.0;  // how far the slot rule may stretch the slices
  double block_max_suffix = 1.0 / 16;
  int64_t block_min_row_bytes = 128;
  int64_t tier_min_rows = 1 << 16;
  int64_t pad_min_bytes = 4 << 20;
};

SpmmPolicy spmm_policy();
void set_spmm_policy(const SpmmPolicy& p);

// Heavy-row gate (DESIGN.md §4.1 "Heavy-row policy"): rows longer than the
// result are chunked (0: none), for a launch of nnz slots whose longest row
// has max_degree slots on a part with `waves` resident waves.
int64_t split_threshold(const SpmmPolicy& p, int64_t nnz, int64_t max_degree, int64_t waves);

// Row stride (floats) of a padded copy of F-float rows (F itself: none).
int64_t padded_width(int64_t F);

// One launch of the blocked schedule: items [0, n_items), item i = output row
// rows[i] with plan slots [ptr[i], ptr[i+1]) (global offsets into the plan's
// indices / pos).
struct BlockItems {
  rt::NDArray rows;  // int32[n_items]
  rt::NDArray ptr;   // int64[n_items + 1]
  int64_t n_items = 0, nnz = 0, off = 0;
  bool suffix = false;
};

struct BlockedPlan {
  int B = 0;
  bool has_suffix = false;
  std::vector<BlockItems> launches;  // B blocks, then the suffix if any
  rt::NDArray indices;               // int32[nnz]: column ids in plan order
  rt::NDArray pos;                   // int32[nnz]: the CSR slot of each plan slot
  rt::NDArray absent;                // int32 rows the first launch does not list
  int64_t n_absent = 0;
  // lazily, per edge layout: plan slot -> edge-value row (int64[nnz])
  rt::NDArray pos64;  // slot layout
  rt::NDArray eidmap; // edge-id layout (eid[pos])
};

// Per-row slot ranges of the blocked schedule: (B + 1) or (B + 2) arrays of
// num_rows int64, range i of row r = [cuts[i][r], cuts[i + 1][r]).
struct Cuts {
  int B = 0;
  bool has_suffix = false;
  int64_t n = 0;       // arrays
  rt::NDArray data;    // int64[n, num_rows]
};

// The monotone-prefix split of the slots over B source blocks.
struct BlockSplit {
  bool ok = false;                 // suffixes within policy
  int B = 0;
  int64_t lo = 0, bs = 1;
  std::vector<int32_t> counts;     // [num_rows * B]: prefix slots per row and block
  std::vector<int64_t> pend;       // [num_rows]: end of each row's prefix
  int64_t total_suffix = 0;
};

// The source sweep (DESIGN.md §4.1 "Source sweep", csrc/sweep.hip): every
// row's running sum in LDS for a whole launch, the slots laid out per
// (launch, block, wave, row) so a wave's block is one run of column ids;
// one launch per generation of rows, a soft barrier keeping the waves on
// the same source blocks.
struct SweepPlan {
  int B = 0;
  int rows_per_wave = 0;
  int per_cu = 0;         // workgroups per CU of a launch (0: occupancy)
  bool accum = false;     // continues the rows' chains (SUM_ACCUM)
  int64_t rows_dealt = 0; // rows of the schedule order the launches cover
  int64_t waves_total = 0, launches = 0;
  rt::NDArray lay;     // int32[nnz]: column ids in sweep order
  rt::NDArray pos;     // int32[nnz]: the CSR slot of each (the scatter's by-product)
  rt::NDArray seg;     // int64[waves_total * B]: each wave's run per block
  rt::NDArray counts;  // int32[num_rows * B]: each row's slots per block
  rt::NDArray arrive;  // int32[launches * B * 256]: the barrier's counters
};

// Sweep schedule knobs (process-wide; dglhip_set_sweep_schedule): on where
// it applies (copy_u sum / mean of fp32 rows of 128 floats, a source-monotone
// CSR, source tables of table_min bytes or more, at most 256 blocks)
struct SweepPolicy {
  int on = 1;
  int64_t table_min = int64_t(256) << 20;  // past the blocked schedule's range
  int64_t block_bytes = 6 << 20;
  int lag = 4;
  int max_spin = 2000;
  // accumulating runs (the pipelined multi-GPU segments, SUM_ACCUM): their
  // own table and row-length floors, and workgroups per CU (0: occupancy, 4;
  // emulated N = 8 rank: 4 / 3 / 2 per CU 7.16 / 7.75 / 9.19 ms; a workgroup
  // held back by the exchange's kernels is not waited for, so the full grid
  // costs at most its late workgroups' solo time; DGLHIP_SWEEP_ACCUM_PER_CU)
  int64_t accum_table_min = int64_t(160) << 20;
  int64_t accum_min_slots = 64;
  int accum_per_cu = 0;
};
SweepPolicy sweep_policy();

struct SplitPlan {
  rt::NDArray light, heavy, chunk_ptr, beg, end;
  int64_t n_light = 0, n_heavy = 0, n_chunks = 0;
};

struct Tier {
  int maxd = 0;
  int64_t n = 0;
  rt::NDArray rows;  // int32[n]
  rt::NDArray sp;    // int64[n + 1] (none for maxd 0)
  rt::NDArray cols;  // int32[sp[n]]
};

struct Tiers {
  int64_t n_long = 0;
  int64_t n_tail = 0;  // rows in the tiers
  std::vector<Tier> tiers;
};

class SpmmPlan {
 public:
  SpmmPlan(int device_type, int device_id, int64_t num_rows, int64_t num_cols, int64_t nnz,
           const int64_t* indptr, const int32_t* indices, const int64_t* host_indptr,
           const int32_t* row_order, hipStream_t stream);

  bool on_device() const { return device_type_ == rt::kDLROCM; }
  int device_id() const { return device_id_; }
  int64_t num_rows() const { return R_; }
  int64_t num_cols() const { return C_; }
  int64_t nnz() const { return nnz_; }
  int64_t max_degree() const { return max_degree_; }
  int64_t num_nonempty() const { return num_nonempty_; }
  const int64_t* indptr() const { return indptr_; }
  const int32_t* indices() const { return indices_; }
  const int32_t* row_order() const { return row_order_; }
  int64_t waves() const { return waves_; }

  // (lo, hi): the column range the slots reference
  std::pair<int64_t, int64_t> span(hipStream_t s);
  // whether eid is the identity (the slots walk edge-id order); cached
  bool eid_identity(const int64_t* eid, hipStream_t s);

  // blocks for gathered rows of row_bytes in slices of block_bytes (0: none)
  int block_count(int64_t table_bytes, int64_t block_bytes) const;
  // the blocked plan for row_bytes / block_bytes; nullptr when none applies
  // (policy, sizes, a heavy row, or suffixes past the policy's share)
  std::shared_ptr<BlockedPlan> blocked(int64_t row_bytes, int64_t block_bytes, hipStream_t s);
  std::shared_ptr<BlockedPlan> blocked_for(int B, hipStream_t s);
  std::shared_ptr<Cuts> cuts(int64_t row_bytes, int64_t block_bytes, hipStream_t s);
  std::shared_ptr<Cuts> cuts_for(int B, hipStream_t s);
  // plan slot -> edge-value row (int64[nnz]) for the slot / edge-id layouts
  const int64_t* plan_pos64(BlockedPlan& bp, hipStream_t s);
  const int64_t* plan_eidmap(BlockedPlan& bp, const int64_t* eid, hipStream_t s);

  // the sweep plan for row_bytes (nullptr when it does not apply)
  // mode: the stream kernel's (0 sum, 1 mean, 2 sum continuing out)
  std::shared_ptr<SweepPlan> sweep(int64_t row_bytes, int mode, hipStream_t s);

  int64_t heavy_threshold() const;  // split_threshold on this CSR and part
  SplitPlan& split_plan(int64_t threshold, bool skip_empty, int64_t chunk, hipStream_t s);
  // tiers of the first n rows of the degree-descending schedule (key 0), or
  // of a split plan's light rows (key 1 + threshold * 2 + skip)
  Tiers& tiers_plain(bool skip, hipStream_t s);
  Tiers& tiers_light(const SplitPlan& sp, int64_t threshold, bool skip, hipStream_t s);

  const std::vector<int64_t>& host_indptr() const { return *host_indptr_; }

 private:
  std::shared_ptr<BlockSplit> block_split(int B, hipStream_t s);
  Tiers build_tiers(const int32_t* rows_host, const rt::NDArray& rows_dev, int64_t n,
                    hipStream_t s);
  rt::NDArray empty(const std::vector<int64_t>& shape, int code, int bits) const;
  rt::NDArray upload(const void* src, int64_t n, int code, int bits, hipStream_t s) const;

  int device_type_, device_id_;
  int64_t R_, C_, nnz_;
  const int64_t* indptr_;
  const int32_t* indices_;
  std::shared_ptr<std::vector<int64_t>> host_indptr_;
  // the schedule's host copy (split plans, tiers): made on first use
  const std::vector<int32_t>& host_order(hipStream_t s);
  std::vector<int32_t> host_order_;
  bool have_host_order_ = false;
  rt::NDArray order_own_;
  const int32_t* row_order_ = nullptr;
  int64_t max_degree_ = 0, num_nonempty_ = 0, waves_ = 0;
  int64_t lo_ = -1, hi_ = -1;
  int eid_ident_ = -1;

  std::mutex mu_;
  std::map<int, std::shared_ptr<BlockSplit>> splits_;
  std::map<int, std::shared_ptr<BlockedPlan>> blocked_;
  std::map<int, std::shared_ptr<Cuts>> cuts_;
  // (blocks, kernel mode, waves per launch, rows per wave) -> layout
  // (nullptr: none fits)
  std::map<std::tuple<int, int, int64_t, int>, std::shared_ptr<SweepPlan>> sweeps_;
  std::map<std::tuple<int64_t, bool, int64_t>, SplitPlan> split_plans_;
  std::map<int64_t, Tiers> tiers_;
};

// The planned run and its workspace (spmm_plan.cc; the C-ABI and the
// registry's dglhip._CAPI_GSpMM call these). path: DGLHIP_PLAN_PATH_*.
int64_t spmm_plan_workspace(SpmmPlan& plan, int msg, int red, int64_t F, int64_t ldu,
                            int64_t urows, int64_t elen, int emode, const int64_t* erow,
                            hipStream_t s);
void spmm_plan_run(SpmmPlan& plan, int msg, int red, int64_t F, const void* ufeat, int64_t ldu,
                   int64_t urows, const float* efeat, int64_t elen, int emode,
                   const int64_t* erow, float* out, int64_t* arg, void* workspace,
                   int64_t ws_bytes, hipStream_t s);
int spmm_plan_path(SpmmPlan& plan, int msg, int red, int64_t F, int64_t ldu, int64_t urows,
                   int64_t elen, int emode, const int64_t* erow, hipStream_t s,
                   int64_t* launches);

// Makes the plan's device current for a scope (its lazily built structures
// are allocated there and its kernels launched on that device's streams).
class PlanDevice {
 public:
  explicit PlanDevice(const SpmmPlan& p);
  ~PlanDevice();
  PlanDevice(const PlanDevice&) = delete;
  PlanDevice& operator=(const PlanDevice&) = delete;

 private:
  int prev_ = -1;
};

// ---------------------------------------------------------------------------
// Device kernels of the plan build and run (spmm_plan_kernels.hip)
// ---------------------------------------------------------------------------
// lo_hi[0] = min(indices), lo_hi[1] = max(indices) (caller sets INT_MAX, -1)
void plan_span_device(int64_t nnz, const int32_t* indices, int32_t* lo_hi, hipStream_t s);
// *flag = 1 if any eid[k] != k (caller zeroes it)
void plan_eid_identity_device(int64_t nnz, const int64_t* eid, int32_t* flag, hipStream_t s);
// the monotone-prefix walk: counts[r * B + b] (zeroed by the caller) = prefix
// slots of row r in block b; pend[r] = end of row r's prefix
void plan_block_walk_device(int64_t R, const int64_t* indptr, const int32_t* indices, int64_t lo,
                            int64_t bs, int B, int32_t* counts, int64_t* pend, hipStream_t s);
// the scatter into plan order: prefix slot k of row r in block b (run start
// s) goes to item_start[r * B + b] + (k - s); suffix slot k to
// sfx_start[r] + (k - pend[r])
void plan_block_scatter_device(int64_t R, const int64_t* indptr, const int32_t* indices,
                               int64_t lo, int64_t bs, int B, const int64_t* pend,
                               const int64_t* item_start, const int64_t* sfx_start,
                               int32_t* out_indices, int32_t* out_pos, hipStream_t s);
// tier item i: cols[sp[i] + j] = indices[indptr[rows[i]] + j], j < sp[i+1] - sp[i]
void plan_tier_cols_device(int64_t n, const int32_t* rows, const int64_t* indptr,
                           const int32_t* indices, const int64_t* sp, int32_t* cols,
                           hipStream_t s);
// out[j] = map ? map[pos[j]] : pos[j]
void plan_compose_device(int64_t n, const int32_t* pos, const int64_t* map, int64_t* out,
                         hipStream_t s);
// out[j] = vals[rows[j]] (one float per edge)
void plan_gather_vals_device(int64_t n, const int64_t* rows, const float* vals, float* out,
                             hipStream_t s);
// out[rows[i], :] = 0 for i < n
void plan_zero_rows_device(int64_t n, const int32_t* rows, int64_t F, float* out, hipStream_t s);
void plan_pad_rows_device(int64_t n, int64_t F, int64_t ld, const float* src, float* dst,
                          hipStream_t s);
// out[r, f] = out[r, f] / max(deg r, 1) (IEEE division, torch.div's bits)
void plan_div_degree_device(int64_t R, int64_t F, const int64_t* indptr, float* out,
                            hipStream_t s);
// out[r, f] = out[r, f] + sums[r, f] / deg r (division when deg > 1) for rows
// with in-edges: the blocked schedule's mean_add (DGLHIP_REDUCE_MEAN_ACCUM)
void plan_add_mean_device(int64_t R, int64_t F, const int64_t* indptr, const float* sums,
                          float* out, hipStream_t s);

}  // namespace dglhip
