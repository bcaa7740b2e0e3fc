/*
 * dgl_hip.h — C-ABI of the MI355X-native g-SpMM engine (libdgl_hip.so).
 *
 * This is the drop-in boundary for the one hot path this project accelerates:
 * DGLGraph.update_all / send_and_recv / pull / push with the builtin
 * message/reduce pairs (copy_src|src_mul_edge|copy_edge  x  sum|max|mean).
 *
 * In the reference (GaiYu0/dgl-1 = DGL 0.1.3) that path is
 *   SPMVExecutor.run            python/dgl/runtime/ir/executor.py:452-473
 *   SPMVWithDataExecutor.run    python/dgl/runtime/ir/executor.py:535-566
 *   F.spmm = torch.sparse.mm    python/dgl/backend/pytorch/tensor.py:145-146
 * fed by the adjacency index produced natively by
 *   _CAPI_DGLGraphGetAdj        src/graph/graph_apis.cc:474-482
 *   Graph::GetAdj               src/graph/graph.cc:506-554
 *   ImmutableGraph CSR build    src/graph/immutable_graph.cc:206-237,553-574
 * and bound from Python through the ctypes PackedFunc FFI
 *   DGLFuncGetGlobal/DGLFuncCall include/dgl/runtime/c_runtime_api.h:255-260
 *   error convention            src/runtime/runtime_base.h:13-32 (API_BEGIN/END),
 *                               src/runtime/c_runtime_api.cc:130-145 (DGLGetLastError)
 *
 * Conventions (same as the reference's C API):
 *   - every int-returning entry point returns 0 on success and -1 on failure;
 *     the message is then available from DGLGetLastError() (thread-local).
 *   - plain pointers and sizes only; no framework types cross this boundary.
 *   - "device" entry points take device pointers and a hipStream_t passed as
 *     void*; they enqueue work on that stream and never synchronise it.
 *   - "host" entry points take host pointers and run synchronously on the
 *     calling thread (parallelised internally with std::thread).
 *   - CSR layout: indptr int64[num_rows+1], indices int32[nnz] (column ids),
 *     eid int64[nnz] (original edge id of each CSR slot). Within a row the
 *     slots keep the order in which the reference's sparse product consumes
 *     them (see DGLHIP_ORDER_*), which is what makes results bit-exact.
 *   - dense features are row-major contiguous float32 [rows, feat_len].
 */
#ifndef DGL_HIP_H_
#define DGL_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DGLHIP_ABI_VERSION 1

/* ------------------------------------------------------------------------ */
/* Error handling / build info                                               */
/* ------------------------------------------------------------------------ */

/* Replaces DGLGetLastError (src/runtime/c_runtime_api.cc:138-140). */
const char* DGLGetLastError(void);
/* Replaces DGLAPISetLastError (src/runtime/c_runtime_api.cc:142-145). */
void DGLAPISetLastError(const char* msg);
/* ABI version (DGLHIP_ABI_VERSION) and a human-readable build string. */
int dglhip_abi_version(void);
const char* dglhip_build_info(void);

/* ------------------------------------------------------------------------ */
/* Graph ingestion: COO -> CSR (replaces Graph::GetAdj + the uncoalesced COO  */
/* that torch.sparse.mm consumes; graph.cc:506-554, graph_index.py:565-583)  */
/* ------------------------------------------------------------------------ */

/* Slot order inside a CSR row.
 *  EID    : ascending edge id — the nnz order of the mutable graph's COO
 *           (graph.cc:509-524 emits [dst..., src...] in edge-id order).
 *  COL    : ascending (column, edge id) — the order of ImmutableGraph's CSR
 *           (immutable_graph.cc:206-237 sorts by (dst, src)).            */
#define DGLHIP_ORDER_EID 0
#define DGLHIP_ORDER_COL 1

/* Host: build a CSR over `num_rows` rows from COO (row[e], col[e]), e < nnz.
 * Stable: slots of a row follow `order`. All ids are validated. */
int dglhip_coo_to_csr_host(int64_t num_rows, int64_t num_cols, int64_t nnz,
                           const int64_t* row, const int64_t* col, int order,
                           int64_t* indptr, int32_t* indices, int64_t* eid);

/* Host: rows sorted by descending degree (ties: ascending row id). Used as
 * the launch schedule so the longest rows start first. */
int dglhip_rows_by_degree_host(int64_t num_rows, const int64_t* indptr,
                               int32_t* row_order);

/* Device: the same COO -> CSR build on the GPU (stable LSD radix sort on
 * (row[, col]) with edge-id as the final tie-break). `workspace` must be at
 * least dglhip_coo_to_csr_workspace_bytes(...) bytes of device memory. */
int64_t dglhip_coo_to_csr_workspace_bytes(int64_t num_rows, int64_t num_cols,
                                          int64_t nnz, int order);
int dglhip_coo_to_csr_device(int64_t num_rows, int64_t num_cols, int64_t nnz,
                             const int64_t* row, const int64_t* col, int order,
                             int64_t* indptr, int32_t* indices, int64_t* eid,
                             void* workspace, int64_t workspace_bytes,
                             void* stream);

/* Host: degree-bucketing schedule for user-defined reduce functions
 * (replaces sched::DegreeBucketing, src/scheduler/scheduler.cc:13-93, and
 * _CAPI_DGLDegreeBucketing*, src/scheduler/scheduler_apis.cc:16-60). Message
 * m goes to receiver position msg_recv[m]. Buckets = distinct non-zero
 * degrees, ascending; nodes ascend inside a bucket; a node's messages keep
 * message order. Outputs are caller-allocated at their maximum sizes:
 * bucket_deg[num_recv], bucket_node_ptr[num_recv+1], nodes[num_recv],
 * msg_ids[num_msgs]; *num_buckets receives the bucket count. */
int dglhip_degree_bucketing_host(int64_t num_msgs, const int64_t* msg_recv,
                                 int64_t num_recv, int64_t* num_buckets,
                                 int64_t* bucket_deg, int64_t* bucket_node_ptr,
                                 int64_t* nodes, int64_t* msg_ids);

/* ------------------------------------------------------------------------ */
/* g-SpMM: out[r,:] = REDUCE_{slot k of row r} MSG(ufeat[indices[k],:],      */
/*                                                  efeat[eid[k],:])        */
/* Replaces F.spmm / SPMV / SPMV_WITH_DATA (executor.py:452-473,535-566,    */
/* backend/pytorch/tensor.py:145-146) and, for max/mean, the degree-bucketing*/
/* UDF reduce (runtime/degree_bucketing.py:13-190, src/scheduler/scheduler.cc*/
/* :13-93).                                                                  */
/* ------------------------------------------------------------------------ */

#define DGLHIP_MSG_COPY_U  0  /* copy_src(src, out)                 message.py:215-235 */
#define DGLHIP_MSG_U_MUL_E 1  /* src_mul_edge(src, edge, out)       message.py:190-213 */
#define DGLHIP_MSG_COPY_E  2  /* copy_edge(edge, out)               message.py:237-257 */
#define DGLHIP_MSG_COPY_U_BF16 3  /* copy_src over source rows held as bf16: ufeat
                                   * points to uint16 bf16 bits (cast to const float*);
                                   * each value widens exactly to fp32 before the fp32
                                   * chain, so the result equals COPY_U on the widened
                                   * rows bit for bit. New design: a halved exchange of
                                   * remote rows (dgl.distributed halo_dtype=bf16) is
                                   * reduced where it lands, with no fp32 copy. */

#define DGLHIP_REDUCE_SUM  0  /* sum(msg, out)                      reducer.py:52-73   */
#define DGLHIP_REDUCE_MAX  1  /* max(msg, out)                      reducer.py:75-97   */
#define DGLHIP_REDUCE_MEAN 2  /* mean: sum / max(deg, 1) (north-star extension) */
#define DGLHIP_REDUCE_SUM_ACCUM 3  /* out += sum: each row's chain continues from the
                                    * value already in out (segment-by-segment
                                    * evaluation of one product; new design) */
#define DGLHIP_REDUCE_MEAN_ACCUM 4  /* out = out + mean: the row's mean added to the
                                     * value already in out (GraphSAGE's
                                     * fc_self(h) + mean(...) in the aggregation's
                                     * own store; new design) */

/* efeat_len: 0 (no edge feature), 1 (one scalar per edge, broadcast over the
 * feature row; the only case the reference specialises, message.py:37-44),
 * feat_len (one value per edge and feature), or any H dividing feat_len (one
 * value per edge and head, broadcast over the D = feat_len / H consecutive
 * features of that head: GAT's (E, H, 1) attention x (N, H, D) features).
 * eid may be NULL for the g-SpMM entry points: edge features are then
 * indexed by CSR slot (efeat already permuted into slot order).
 * arg_out (int64[num_rows*feat_len], may be NULL): for MAX, the CSR slot that
 * won each element (-1 for empty rows); needed by the backward.
 * row_order (int32[num_rows], may be NULL): launch schedule; rows are launched
 * in this order and results never depend on it. It may list a subset of the
 * CSR's rows (num_rows then counts the listed rows, indptr still spans the
 * CSR): rows not listed are not written, which SUM_ACCUM and MEAN_ACCUM use
 * to skip rows without slots.
 * Numerics: SUM/MEAN accumulate per output element in CSR slot order with
 * one fused multiply-add per slot (acc = fma(w, x, acc); copy: acc += x),
 * starting from +0.0 — the arithmetic of torch's CPU sparse x dense product
 * on the reference's uncoalesced COO. Empty rows produce 0. */
int dglhip_gspmm_device(int msg_op, int reduce_op, int64_t num_rows,
                        int64_t feat_len, const int64_t* indptr,
                        const int32_t* indices, const int64_t* eid,
                        const float* ufeat, const float* efeat,
                        int64_t efeat_len, float* out, int64_t* arg_out,
                        const int32_t* row_order, void* stream);

/* Heavy-row variant (sum / mean): rows are split into a launch plan so that
 * no single sequential chain dominates the kernel on very skewed graphs
 * (RMAT in-degrees reach ~1e6). Light rows (light_rows[num_light]) run as in
 * dglhip_gspmm_device. Each heavy row is cut into consecutive slot ranges
 * [chunk_beg[c], chunk_end[c]); chunk c's sequential partial sum goes to
 * partial[c, :] (float32[num_chunks, feat_len] workspace), and heavy row
 * heavy_rows[h] = ((p[c0] + p[c0+1]) + ...) over its chunks
 * c0 = heavy_chunk_ptr[h] .. heavy_chunk_ptr[h+1]-1. Deterministic; differs
 * from the single chain only by re-association (fp32 tolerance, not bits).
 * ufeat_ld: row stride of ufeat in elements (0 = feat_len; an even padded
 * width >= feat_len for line-aligned gathers, see dglhip_gspmm_strided_device). */
int dglhip_gspmm_chunked_device(int msg_op, int reduce_op, int64_t feat_len,
                                const int64_t* indptr, const int32_t* indices,
                                const int64_t* eid, const float* ufeat,
                                const float* efeat, int64_t efeat_len, float* out,
                                int64_t num_light, const int32_t* light_rows,
                                int64_t num_chunks, const int64_t* chunk_beg,
                                const int64_t* chunk_end, int64_t num_heavy,
                                const int32_t* heavy_rows,
                                const int64_t* heavy_chunk_ptr, float* partial,
                                int64_t ufeat_ld, void* stream);

/* Range-list g-SpMM (sum): for every item i, out[i, :] = (accumulate ?
 * out[i, :] : 0) (+)= chain over slots [item_beg[i], item_end[i]) in slot
 * order. With accumulate the chain of a row can be evaluated segment by
 * segment (e.g. as its source features arrive over the network) and equals
 * the single chain over the concatenated segments bit for bit. */
int dglhip_gspmm_ranges_device(int msg_op, int64_t num_items, int64_t feat_len,
                               const int64_t* item_beg, const int64_t* item_end,
                               int accumulate, const int32_t* indices,
                               const int64_t* eid, const float* ufeat,
                               const float* efeat, int64_t efeat_len, float* out,
                               void* stream);

int dglhip_gspmm_ranges_host(int msg_op, int64_t num_items, int64_t feat_len,
                             const int64_t* item_beg, const int64_t* item_end,
                             int accumulate, const int32_t* indices,
                             const int64_t* eid, const float* ufeat,
                             const float* efeat, int64_t efeat_len, float* out,
                             int num_threads);

/* Device g-SpMM whose source rows have a row stride of ufeat_ld >= feat_len
 * elements (feature f of row u at ufeat[u * ufeat_ld + f]): rows padded so
 * that none straddles more cache lines than its width needs (F = 41: 164-B
 * rows padded to 192 B touch 2 lines instead of 2.3 on average). Messages
 * copy_u / u_mul_e, reducers sum / mean / sum_accum; the per-element chains
 * are those of dglhip_gspmm_device (identical results). ufeat_ld must equal
 * feat_len or be even. */
int dglhip_gspmm_strided_device(int msg_op, int reduce_op, int64_t num_rows,
                                int64_t feat_len, int64_t ufeat_ld, const int64_t* indptr,
                                const int32_t* indices, const int64_t* eid,
                                const float* ufeat, const float* efeat, int64_t efeat_len,
                                float* out, const int32_t* row_order, void* stream);

/* copy_u g-SpMM (sum / mean / sum_accum) over SHORT rows given as a compacted
 * CSR of their own: item i writes output row rows[i] from its column ids
 * slot_cols[slot_ptr[i] .. slot_ptr[i+1]) in slot order, every item having
 * at most max_deg slots (0 = rows without slots: stored as zeros, or left as
 * they are for sum_accum; slot_ptr / slot_cols may then be NULL). Several
 * items per wave with all their gathers in flight together, for the tail of a
 * power-law graph's degree-descending schedule where one wave per row leaves
 * the memory system idle. Longer items are still reduced correctly, in batches
 * of the kernel's depth. Results equal dglhip_gspmm_device's on the same rows
 * bit for bit. total_rows: rows of the whole output (non-temporal store rule).
 * ufeat_ld: row stride of ufeat in elements (0 = feat_len, else even and
 * >= feat_len). */
int dglhip_gspmm_short_rows_device(int msg_op, int reduce_op, int64_t num_items,
                                   int64_t feat_len, int64_t max_deg, int64_t total_rows,
                                   const int32_t* rows, const int64_t* slot_ptr,
                                   const int32_t* slot_cols, const float* ufeat, float* out,
                                   int64_t ufeat_ld, void* stream);

/* ------------------------------------------------------------------------ */
/* Launch plan of a g-SpMM over one CSR (csrc/spmm_plan.{h,cc,hip}).         */
/*                                                                           */
/* Replaces what the reference caches per context and runs per call:         */
/*   GraphIndex.adjacency_matrix (cached per ctx)  python/dgl/graph_index.py:537-585 */
/*   F.spmm on it (SPMVExecutor.run)  backend/pytorch/tensor.py:145-146,    */
/*                                    runtime/ir/executor.py:452-473,535-566 */
/* A plan is built once per CSR and device and holds every schedule the      */
/* g-SpMM runs over it: the source-blocked schedule (items  */
/* per contiguous source block, each row's chain continued block by block,   */
/* taken only where that is the row's own slot order: the same bits), the    */
/* heavy-row split, the short-row tiers, the degree-descending row order.    */
/* dglhip_spmm_plan_run picks among them per call exactly as the engine's    */
/* Python operators do (they call it too), so a C / ctypes / PackedFunc       */
/* caller gets the benchmarked schedule.                                     */
/* ------------------------------------------------------------------------ */
typedef struct DGLHipSpmmPlanObj* DGLHipSpmmPlan;

/* Where the edge value of CSR slot k is (u_mul_e / copy_e):
 *  BY_SLOT: efeat row k (values laid out in the CSR's slot order);
 *  BY_EID : efeat row erow[k], erow = the CSR's edge ids (NULL: identity);
 *           the plan caches what it derives from them (the same CSR's ids);
 *  BY_MAP : efeat row erow[k] for an arbitrary int64 map. */
#define DGLHIP_EDGE_BY_SLOT 0
#define DGLHIP_EDGE_BY_EID 1
#define DGLHIP_EDGE_BY_MAP 2

/* Schedule policy (process-wide). Defaults: row_split -1 (auto: chunk a row
 * only when it is the launch's critical path), blocked 1, short_rows 1,
 * pad_rows 1, block_bytes 6 MiB, block_table_min 16 MiB, block_table_max
 * 256 MiB, block_min_slots 12, block_max_stretch 3, block_max_suffix 1/16,
 * block_min_row_bytes 128, tier_min_rows 65536, pad_min_bytes 4 MiB; the
 * environment variables DGLHIP_ROW_SPLIT / _BLOCKED / _BLOCK_BYTES /
 * _BLOCK_MIN_SLOTS / _BLOCK_MAX_STRETCH / _SHORT_ROWS / _PAD_ROWS set the
 * initial values. Results never depend on it beyond the documented
 * tolerance of the heavy-row split (re-association of a chunked row). */
typedef struct {
  int64_t row_split;      /* -1 auto, 0 off (every row one chain), > 0 chunk length */
  int32_t blocked;        /* source-blocked schedule where exact */
  int32_t short_rows;     /* short-row tiers */
  int32_t pad_rows;       /* padded-stride gathers of line-straddling rows */
  int32_t reserved;
  int64_t block_bytes;    /* source slice per launch */
  int64_t block_table_min, block_table_max;  /* gathered table range that blocks */
  int64_t block_min_slots;                   /* slots per row and block */
  double block_max_stretch;                  /* slices at most this x block_bytes */
  double block_max_suffix;                   /* share of slots after the prefixes */
  int64_t block_min_row_bytes;               /* rows of at most this keep one launch */
  int64_t tier_min_rows;                     /* short rows needed to tier */
  int64_t pad_min_bytes;                     /* tables smaller than this: no padding */
} DGLHipSpmmPolicy;
int dglhip_spmm_get_policy(DGLHipSpmmPolicy* out);
int dglhip_spmm_set_policy(const DGLHipSpmmPolicy* policy);
/* The heavy-row gate under the current policy: rows longer than *out slots
 * are chunked (0: none) in a launch of nnz slots whose longest row has
 * max_degree, on a part with `waves` resident waves (<= 0: MI355X's). */
int dglhip_spmm_split_threshold(int64_t nnz, int64_t max_degree, int64_t waves, int64_t* out);
/* Row stride (floats) the plan gathers F-float rows at (F: unpadded). */
int dglhip_spmm_padded_width(int64_t feat_len, int64_t* out);

/* Build the plan of a CSR on device_type 10 (ROCm, device_id) or 1 (host).
 * indptr int64[num_rows+1] and indices int32[nnz] are borrowed: they must
 * stay allocated and unchanged while the plan lives. host_indptr (optional,
 * borrowed only during the call) spares a device-to-host copy; row_order
 * (optional, borrowed like indptr): the degree-descending launch schedule
 * (built when NULL). The structures of each schedule are built on first
 * use, on the stream of that call (which waits for them); building inside a
 * HIP-graph capture fails, so a captured caller runs once outside first.
 * A plan serves one stream at a time (its lazily built structures). */
int dglhip_spmm_plan_create(int device_type, int device_id, int64_t num_rows, int64_t num_cols,
                            int64_t nnz, const int64_t* indptr, const int32_t* indices,
                            const int64_t* host_indptr, const int32_t* row_order, void* stream,
                            DGLHipSpmmPlan* out);
/* Frees the plan's own memory (arrays handed out through the registry keep
 * theirs until released). Work already enqueued must have finished. */
int dglhip_spmm_plan_free(DGLHipSpmmPlan plan);
/* Bytes of workspace dglhip_spmm_plan_run needs for these arguments (the
 * padded copy of line-straddling rows, edge values in plan order, the
 * heavy-row partials); may build plan structures on `stream`. */
int dglhip_spmm_plan_workspace(DGLHipSpmmPlan plan, int msg_op, int reduce_op, int64_t feat_len,
                               int64_t ufeat_ld, int64_t num_src_rows, int64_t efeat_len,
                               int edge_layout, const int64_t* erow, void* stream, int64_t* bytes);
/* The g-SpMM of dglhip_gspmm_device over the plan's CSR, on the schedule the
 * plan picks: out[r, :] = REDUCE over r's slots of MSG(ufeat[col], efeat[..]).
 * ufeat: num_src_rows rows at stride ufeat_ld (0 or feat_len: dense; else an
 * even padded width, copy_u / u_mul_e sum-like reducers), fp32, or bf16 bits
 * for DGLHIP_MSG_COPY_U_BF16. Edge values per edge_layout. arg_out (MAX,
 * optional). workspace: device memory of dglhip_spmm_plan_workspace bytes.
 * Bit-identical to dglhip_gspmm_device with the same arguments, except rows
 * the heavy-row policy chunks (fp32 re-association, deterministic). A host
 * plan runs dglhip_gspmm_host. Enqueues on `stream`; never synchronises once
 * the plan's structures for these arguments exist. */
int dglhip_spmm_plan_run(DGLHipSpmmPlan plan, int msg_op, int reduce_op, int64_t feat_len,
                         const void* ufeat, int64_t ufeat_ld, int64_t num_src_rows,
                         const float* efeat, int64_t efeat_len, int edge_layout,
                         const int64_t* erow, float* out, int64_t* arg_out, void* workspace,
                         int64_t workspace_bytes, void* stream);
/* The schedule a run with these arguments takes: *path 0 host, 1 one wave per
 * row (heavy-row chunks and short-row tiers included), 2 source-blocked items,
 * 3 source-blocked max ranges, 4 the source sweep; *launches the blocked
 * launches, the sweep's launches (row generations), 1 otherwise. */
#define DGLHIP_PLAN_PATH_HOST 0
#define DGLHIP_PLAN_PATH_ROWS 1
#define DGLHIP_PLAN_PATH_BLOCKED 2
#define DGLHIP_PLAN_PATH_MAX_BLOCKED 3
#define DGLHIP_PLAN_PATH_SWEEP 4
int dglhip_spmm_plan_schedule(DGLHipSpmmPlan plan, int msg_op, int reduce_op, int64_t feat_len,
                              int64_t ufeat_ld, int64_t num_src_rows, int64_t efeat_len,
                              int edge_layout, const int64_t* erow, void* stream, int* path,
                              int64_t* launches);
/* stats[7] = rows, columns, nnz, max degree, rows with slots, resident waves
 * of the part, heavy-row threshold (0: no row chunked). */
int dglhip_spmm_plan_stats(DGLHipSpmmPlan plan, int64_t* stats);

/* ------------------------------------------------------------------------ */
/* Dense per-node Linear on the f32 MFMA (the Linear that follows a g-SpMM;  */
/* csrc/node_linear.hip). No reference counterpart: the reference runs these */
/* products as torch nn.Linear (examples/pytorch/gcn/gcn_spmv.py:45-62).     */
/* ------------------------------------------------------------------------ */
/* y1 = x W1^T (+ b1) and, with m2 > 0, y2 = x W2^T (+ b2) in one pass over
 * the num_rows rows of x (row stride ldx, a multiple of 4; 16-byte aligned).
 * in_feats 64, 128 or 256; 1 <= m1 <= 64, 0 <= m2 <= 64; W row-major [m][in_feats]
 * (nn.Linear's weight); b may be NULL; outputs at their own row strides. Each
 * output element is one f32 fma chain over the inputs (exact f32). */
int dglhip_node_linear_device(int64_t num_rows, int64_t in_feats, const float* x, int64_t ldx,
                              int64_t m1, const float* w1, const float* b1, float* y1,
                              int64_t ldy1, int64_t m2, const float* w2, const float* b2,
                              float* y2, int64_t ldy2, void* stream);

/* y = x1 W1^T + x2 W2^T (+ b), relu != 0: max(that, 0): one output from two
 * inputs of in_feats (64 or 128) columns each (GraphSAGE's fc_self(h) +
 * fc_neigh(agg) and its activation); W1, W2 [m][in_feats], 1 <= m <= 128 (one
 * pass over the inputs; with in_feats 64 and m > 64, one per 64 outputs). */
int dglhip_node_linear_cat_device(int64_t num_rows, int64_t in_feats, const float* x1,
                                  int64_t ldx1, const float* x2, int64_t ldx2, int64_t m,
                                  const float* w1, const float* w2, const float* b, float* y,
                                  int64_t ldy, int relu, void* stream);

/* Tuning knob of the three node-Linear entries: lanes per workgroup (256 or
 * 512) and workgroups per CU; 0 restores the automatic choice. Results do not
 * depend on it. */
int dglhip_set_node_linear_variant(int threads, int wgs_per_cu);

/* Input gradient of the first: dx = dy1 W1 + dy2 W2 (m2 = 0: dy1 W1 only);
 * in_feats 64 or 128; dy rows at their own strides; dx at stride lddx (16-byte aligned rows). gate
 * (optional, rows at stride ldg): x's own values when x is a ReLU output; dx
 * is then 0 where gate <= 0 (ReLU's backward rule, torch threshold_backward),
 * the mask applied in the store instead of a pass of its own. colsum
 * (optional, in_feats floats): the column sums of the stored dx (the bias
 * gradient of the layer whose output x is), per lane, per wave in a fixed
 * butterfly and over the waves in order; workspace holds the per-wave
 * partials (dglhip_node_linear_dgrad_workspace_floats(in_feats) floats). */
int dglhip_node_linear_dgrad_device(int64_t num_rows, int64_t in_feats, int64_t m1,
                                    const float* dy1, int64_t lddy1, const float* w1, int64_t m2,
                                    const float* dy2, int64_t lddy2, const float* w2, float* dx,
                                    int64_t lddx, const float* gate, int64_t ldg, float* colsum,
                                    float* workspace, void* stream);

/* Floats of the input-gradient entry's column-sum workspace. */
int64_t dglhip_node_linear_dgrad_workspace_floats(int64_t in_feats);

/* out[r, :F] = x[r, :F] / divisor[r] (IEEE division: torch.div's bits) over
 * num_rows rows of feat_len (1..4096) floats, x and out at their own row
 * strides: the mean reducer's backward dC / deg written into the row-padded
 * buffer the transposed g-SpMM gathers (csrc/rowops.hip). out's pad columns
 * [feat_len, ldo) may be overwritten (with zeros). */
int dglhip_div_rows_device(int64_t num_rows, int64_t feat_len, const float* x, int64_t ldx,
                           const float* divisor, float* out, int64_t ldo, void* stream);
/* The node-row epilogue of a GCN layer after its aggregation (r06): out =
 * act(x * row_scale[r] + bias[f]) over num_rows x feat_len packed rows,
 * act = ReLU (relu = 1; torch's clamp_min: NaN kept) or none, each operation
 * rounded as torch's separate `*`, `+` and relu; row_scale / bias may be
 * NULL. Backward: d_pre = relu ? (out <= 0 ? 0 : dout) : dout, dx = d_pre *
 * row_scale[r], and col_partial[p, f] = the sum of d_pre over rows [128 p,
 * 128 p + 128) in row order (dglhip_node_epilogue_parts(num_rows) parts; NULL:
 * not wanted): the bias gradient is their sum over p. */
int64_t dglhip_node_epilogue_parts(int64_t num_rows);
int dglhip_node_epilogue_fwd_device(int64_t num_rows, int64_t feat_len, const float* x,
                                    const float* row_scale, const float* bias, int relu,
                                    float* out, void* stream);
int dglhip_node_epilogue_bwd_device(int64_t num_rows, int64_t feat_len, const float* dout,
                                    const float* out, const float* row_scale, int relu,
                                    float* dx, float* col_partial, void* stream);

/* ------------------------------------------------------------------------ */
/* Weighted softmax cross-entropy over node rows (csrc/node_loss.hip): the   */
/* loss of a full-graph node classifier. No reference counterpart: the       */
/* reference's examples call torch's F.cross_entropy / nll_loss             */
/* (examples/pytorch/gcn/gcn_spmv.py:113-118).                              */
/* ------------------------------------------------------------------------ */
/* Floats of the forward's workspace (per-workgroup partial sums). */
int dglhip_xent_workspace_floats(void);

/* *loss = sum_i w_i (logsumexp(z_i) - z_i[labels_i]) over num_rows rows of
 * num_classes (1..64) logits at row stride ld; weight NULL = all ones; rows
 * whose label is outside [0, num_classes) (ignore_index) add nothing. The sum
 * runs per lane, per workgroup in a fixed tree, then over the workgroups in
 * order: deterministic. loss and workspace are device pointers. */
int dglhip_xent_fwd_device(int64_t num_rows, int64_t num_classes, const float* logits,
                           int64_t ld, const int64_t* labels, const float* weight, float* loss,
                           float* workspace, void* stream);

/* dlogits_ij = g w_i (softmax(z_i)_j - [j == labels_i]) with g = *grad_loss
 * (a device scalar: no host round trip); ignored rows get zeros; dlogits at
 * row stride ldd. */
int dglhip_xent_bwd_device(int64_t num_rows, int64_t num_classes, const float* logits,
                           int64_t ld, const int64_t* labels, const float* weight,
                           const float* grad_loss, float* dlogits, int64_t ldd, void* stream);

/* Floats of the column-sum workspace of dglhip_xent_bwd_ex_device. */
int dglhip_xent_colsum_workspace_floats(int64_t num_classes);

/* dglhip_xent_bwd_device, plus two optional outputs taken from the gradient
 * rows as they are stored (no pass of their own):
 * - colsum[j] = sum_i dlogits_ij (the output layer's bias gradient): per wave
 *   in row order, per workgroup over its waves in order, then over the
 *   workgroups in 16 contiguous runs summed in order, the runs in order
 *   (deterministic). colsum NULL = no sums (workspace unused).
 * - dlogits_scaled[i, j] = dlogits_ij / divisor[i] (IEEE division) at row
 *   stride ld_scaled (a multiple of 4, >= num_classes, 16-byte aligned; pad
 *   columns zeroed): the mean aggregation's backward operand dC / deg in the
 *   padded rows its transposed g-SpMM gathers (dglhip_div_rows_device's
 *   output). dlogits_scaled NULL = none.
 * All pointers are device pointers. Replaces the separate column reduce of
 * the bias gradient (nn.Linear's autograd: torch's sum over dim 0) and the
 * mean backward's division pass. */
int dglhip_xent_bwd_ex_device(int64_t num_rows, int64_t num_classes, const float* logits,
                              int64_t ld, const int64_t* labels, const float* weight,
                              const float* grad_loss, float* dlogits, int64_t ldd, float* colsum,
                              float* workspace, const float* divisor, float* dlogits_scaled,
                              int64_t ld_scaled, void* stream);

/* Same contract on host memory (the CPU device of the engine; std::thread). */
int dglhip_gspmm_host(int msg_op, int reduce_op, int64_t num_rows,
                      int64_t feat_len, const int64_t* indptr,
                      const int32_t* indices, const int64_t* eid,
                      const float* ufeat, const float* efeat,
                      int64_t efeat_len, float* out, int64_t* arg_out,
                      int num_threads);

/* Knob: where the copy_u + sum kernel's row gathers (two floats per lane, a
 * wave per row) go through buffer descriptors built from the wave-uniform row
 * address (one 32-bit lane offset for every gather in flight instead of a
 * 64-bit address each) rather than global loads, as a bit mask: bit 0 the
 * one-launch rows and heavy-row chunk launches, bit 1 the source-blocked
 * schedule's item launches, the first block's included (the default, 2: 42
 * instead of 70 VGPRs there). Same values. */
int dglhip_set_gather_mode(int buffer_descriptors);

/* Resident waves of the headline g-SpMM kernel (F = 128 copy_u + sum) on
 * `device`: compute units x the kernel's occupancy per CU (blocks of 4 waves).
 * The heavy-row policy sizes its critical-path test and its chunk launches
 * from it (dgl.kernel._resident_waves). MI355X: 256 CUs x 28 = 7168. */
int dglhip_gspmm_resident_waves(int device, int64_t* waves);

/* ------------------------------------------------------------------------ */
/* g-SDDMM: per-edge products feeding the backward of u_mul_e and the GAT    */
/* edge attention (gat/train.py:74-96).                                      */
/*   DOT : out[eid[k], h] = sum_{d<D} lhs[r, hD+d] * rhs[indices[k], hD+d]   */
/*         (r = row of slot k, H = num_heads, D = feat_len / H)              */
/* eid may be NULL: out is then indexed by slot k (edge values laid out in   */
/* this CSR's slot order, as the g-SpMM reads them with a NULL eid).         */
/* ------------------------------------------------------------------------ */
#define DGLHIP_SDDMM_DOT 0
int dglhip_gsddmm_device(int op, int64_t num_rows, int64_t feat_len,
                         int64_t num_heads, const int64_t* indptr,
                         const int32_t* indices, const int64_t* eid,
                         const float* lhs, const float* rhs, float* out,
                         void* stream);
int dglhip_gsddmm_host(int op, int64_t num_rows, int64_t feat_len,
                       int64_t num_heads, const int64_t* indptr,
                       const int32_t* indices, const int64_t* eid,
                       const float* lhs, const float* rhs, float* out,
                       int num_threads);

/* GAT attention gradient (the backward of dglhip_gat_aggregate_device with
 * respect to the attention's pre-activation), in CSR slot order, one pass:
 *   t = DOT(dout[r, h], ft[indices[k], h])   (the g-SDDMM dot above, same bits)
 *   t = attn_drop ? (attn_drop[k, h] != 0 ? t * drop_scale : 0) : t
 *   t = dz ? t + dz[r, h] : t                (the normaliser's gradient)
 *   grad[k, h] = lo < a < hi ? (apply_exp ? (t * a) * s : t * s) : 0,
 *   a = attn[k, h], s = alpha where a <= 1 (exp) / a <= 0 (the logit <= 0, as
 *   torch's leaky_relu backward), else 1
 * attn, attn_drop, grad: [nnz, H] slot order; dout: [num_rows, F]; ft:
 * [num_src, F]; dz: [num_rows, H] or NULL; attn_drop NULL without dropout. */
int dglhip_gat_attention_grad_device(int64_t num_rows, int64_t feat_len, int64_t num_heads,
                                     const int64_t* indptr, const int32_t* indices,
                                     const float* dout, const float* ft, const float* attn,
                                     const float* attn_drop, const float* dz, float alpha,
                                     float clamp_lo, float clamp_hi, int apply_exp,
                                     float drop_scale, float* grad, void* stream);

/* Study knob: 1 = the sliced g-SDDMM dot runs at its alternative depth of
 * slots in flight (16 <-> 32, or 8 -> 16 for F >= 256), 0 = the default. */
int dglhip_set_sddmm_variant(int alternate);

/* GAT edge attention (gat/train.py:90-96), fused u_add_v SDDMM + activation:
 *   out[eid[k], h] = clamp(act(lhs[indices[k], h] + rhs[r, h]), lo, hi),
 *   act(x) = exp(leaky_relu(x, alpha)) if apply_exp else leaky_relu(x, alpha)
 * lhs: [num_src, H], rhs: [num_rows, H], out: [num_edges, H]; a NULL eid
 * indexes out by slot k (CSR slot order). */
int dglhip_gsddmm_attention_device(int64_t num_rows, int64_t num_heads,
                                   const int64_t* indptr, const int32_t* indices,
                                   const int64_t* eid, const float* lhs,
                                   const float* rhs, float alpha, float clamp_lo,
                                   float clamp_hi, int apply_exp, float* out,
                                   void* stream);
int dglhip_gsddmm_attention_host(int64_t num_rows, int64_t num_heads,
                                 const int64_t* indptr, const int32_t* indices,
                                 const int64_t* eid, const float* lhs, const float* rhs,
                                 float alpha, float clamp_lo, float clamp_hi,
                                 int apply_exp, float* out, int num_threads);

/* Fused GAT layer aggregation (gat/train.py:74-96: apply_edges(edge_attention),
 * attn_drop, update_all([src_mul_edge, copy_edge], [sum, sum])) in one pass,
 * one wave per destination row r, slots k of the row in CSR order, u = indices[k]:
 *   a[k, h]         = clamp(act(el[u, h] + er[r, h]), lo, hi)   (act as above)
 *   w[k, h]         = keep(s, k * H + h) ? a[k, h] / (1 - drop_p) : 0
 *                     (w = a when drop_p == 0), s = seed + *seed_offset
 *                     (seed_offset: a device int64, may be NULL: s = seed;
 *                     a counter on the device keeps HIP-graph replays drawing
 *                     fresh masks)
 *   out_ft[r, hD+d] = sum_k w[k, h] * ft[u, hD+d]   (fma chain in slot order)
 *   out_z[r, h]     = sum_k a[k, h]                 (add chain in slot order)
 * el, er: [num_src, H], [num_rows, H]; ft: [num_src, H*D] (num_src: the column
 * count, every index below it); out_ft: [num_rows,
 * H*D]; out_z: [num_rows, H]. attn_out / attn_drop_out ([nnz, H], CSR slot
 * order) may be NULL (nothing stored); with dropout both or neither. The
 * outputs equal dglhip_gsddmm_attention_device (slot order) followed by the
 * u_mul_e and copy_e sums bit for bit. keep(): dglhip_gat_dropout_mask_host.
 * row_order (int32[num_rows], may be NULL): launch schedule only. */
int dglhip_gat_aggregate_device(int64_t num_rows, int64_t num_src, int64_t num_heads,
                                int64_t head_dim, const int64_t* indptr, const int32_t* indices,
                                const int32_t* row_order, const float* el, const float* er,
                                const float* ft, float alpha, float clamp_lo, float clamp_hi,
                                int apply_exp, float drop_p, uint64_t seed,
                                const int64_t* seed_offset, float* out_ft, float* out_z,
                                float* attn_out, float* attn_drop_out, void* stream);

/* Sum over items: item i adds the messages of slots [item_ptr[i],
 * item_ptr[i+1]) of indices (and eid / efeat by slot) to output row
 * item_rows[i] — from zero, or with accumulate != 0 continuing the row's
 * chain from the value in out. Rows not listed are not touched. The
 * source-blocked schedule runs one call per source block, its items the rows
 * with slots in the block, longest first, their slots laid out in item order
 * (DESIGN.md §4.1): the three loads that start an item are independent and
 * the slot stream is sequential across items. ufeat rows at stride ufeat_ld
 * (0: feat_len). */
int dglhip_gspmm_items_device(int msg_op, int64_t num_items, int64_t feat_len,
                              const int32_t* item_rows, const int64_t* item_ptr, int accumulate,
                              const int32_t* indices, const int64_t* eid, const float* ufeat,
                              int64_t ufeat_ld, const float* efeat, int64_t efeat_len,
                              float* out, void* stream);

/* Narrow rows, two slots per gather (r06): the same items as
 * dglhip_gspmm_items_device (copy_u + sum, item i = row item_rows[i] over
 * slots [item_ptr[i], item_ptr[i + 1]), accumulate continuing the chains)
 * for source rows of 16..64 floats at an even stride ufeat_ld <= 64 (0 =
 * feat_len) over a table of num_src_rows rows under 2 GiB. The wave's halves
 * gather consecutive slots and the lower half adds them in slot order, so the
 * results equal dglhip_gspmm_items_device's bit for bit with half the gather
 * instructions. _ok: 1 when a shape qualifies (and the knob is on). */
int dglhip_gspmm_pair_items_ok(int msg_op, int64_t feat_len, int64_t ufeat_ld,
                               int64_t num_src_rows);
int dglhip_gspmm_pair_items_device(int64_t num_items, int64_t feat_len, int64_t ufeat_ld,
                                   int64_t num_src_rows, const int32_t* item_rows,
                                   const int64_t* item_ptr, int accumulate,
                                   const int32_t* indices, const float* ufeat, float* out,
                                   void* stream);
/* Study knob: the plan's blocked copy_u + sum takes the paired kernel where
 * it qualifies (1), or never (0, the default: measured slower, 4.15 vs 2.14
 * ms at F = 41 on the Reddit-shaped graph); env
 * DGLHIP_PAIR_SLOTS. */
int dglhip_set_pair_slots(int on);

/* Source-swept copy_u + sum (mean != 0: mean) of fp32 rows of feat_len = 64,
 * 128 or 256 floats over the CSR (indptr, indices), every row of out
 * written. Each wave keeps rows_per_wave rows' running sums in LDS for a
 * whole launch and walks their slots source block by source block (block b:
 * columns below col_lo + (b + 1) * block_cols; the last block takes the
 * rest), always in slot order — so the result is dglhip_gspmm_device's chain,
 * bit for bit, for any edge order; the blocks only set the L2 locality.
 * row_order (int32[num_rows], may be NULL): the degree-descending order rows
 * are dealt to waves from. rows_per_wave: 10 or 20 at 128 floats (0: 20),
 * 20 or 40 at 64, 5 or 10 at 256. DESIGN.md §4.1 "Source sweep". Replaces,
 * like dglhip_gspmm_device, the reference's F.spmm
 * (python/dgl/backend/pytorch/tensor.py:145-146). */
int dglhip_gspmm_sweep_device(int64_t num_rows, int64_t feat_len, const int64_t* indptr,
                              const int32_t* indices, const float* ufeat, float* out,
                              const int32_t* row_order, int64_t col_lo, int64_t block_cols,
                              int num_blocks, int mean, int rows_per_wave, void* stream);

/* The streamed form of the source sweep (a study, DESIGN.md §4.1 "Source
 * sweep"): the slots laid out per (launch, block, wave, row) in lay, wave w's
 * block-b run starting at seg_beg[w * num_blocks + b], counts[row *
 * num_blocks + b] slots of each of its rows back to back (the layout of
 * tools/r05/sweep_study.py stream_layout, exact for source-monotone rows);
 * waves_total a multiple of dglhip_gspmm_sweep_stream_geometry's waves per
 * launch. lag > 0: a soft barrier (a wave starts block b once every
 * workgroup that has begun has finished block b - lag, or after max_spin
 * polls) over
 * device-scope counters in arrive (arrive_len >= launches * (num_blocks * 8 +
 * 1) * 32 ints, zeroed by the call; concurrent calls need their own; a
 * workgroup not yet resident is not waited for); results never depend on it. mode 0 sum, 1 mean, 2 sum continuing each dealt row's chain
 * from its value in out (SUM_ACCUM); num_rows rows of row_order are dealt.
 * per_cu > 0 caps the workgroups per CU of a launch (room for kernels on
 * other streams, e.g. RCCL's); the layout's waves_total must be a multiple
 * of the geometry's waves per launch for the same rows_per_wave and per_cu. rows_per_wave 10 or 19;
 * feat_len 128. */
int dglhip_gspmm_sweep_stream_geometry(int rows_per_wave, int per_cu, int64_t* waves_per_launch);
/* The same for the kernel of a given mode (0 sum, 1 mean, 2 sum continuing
 * out) at the current dglhip_set_sweep_unroll: the geometry the launch of
 * dglhip_gspmm_sweep_stream_device with that mode checks its layout against
 * (the plain entry above is mode 0). */
int dglhip_gspmm_sweep_stream_geometry_mode(int rows_per_wave, int per_cu, int mode,
                                            int64_t* waves_per_launch);
int dglhip_gspmm_sweep_stream_device(int64_t num_rows, int64_t waves_total,
                                     const int32_t* row_order, const int32_t* counts,
                                     int num_blocks, const int64_t* seg_beg, const int32_t* lay,
                                     const int64_t* indptr, const float* ufeat, float* out,
                                     int mode, int rows_per_wave, int per_cu, int* arrive,
                                     int64_t arrive_len, int lag, int max_spin, void* stream);
/* Study knobs of the sweep kernels: workgroups per CU of a launch (0: the
 * occupancy limit) and row gathers in flight per wave (16 or 32). */
/* The plan's source-sweep schedule (DGLHIP_PLAN_PATH_SWEEP, DESIGN.md §4.1
 * "Source sweep"): taken for copy_u sum / mean of fp32 rows of 128 floats
 * over a source-monotone CSR whose referenced source table is table_min
 * bytes or more, in ceil(table / block_bytes) <= 256 blocks; lag and
 * max_spin are the soft barrier's (dglhip_gspmm_sweep_stream_device).
 * Accumulating runs (SUM_ACCUM: the pipelined multi-GPU segments) take it
 * from accum_table_min bytes with accum_min_slots slots per non-empty row,
 * at accum_per_cu workgroups per CU (0: the occupancy limit). Defaults: on
 * (DGLHIP_SWEEP=off: off), 256 MiB, 6 MiB, 4, 2000; 160 MiB, 64, 0
 * (DGLHIP_SWEEP_ACCUM_PER_CU). */
/* mean_add (DGLHIP_REDUCE_MEAN_ACCUM) on the source-blocked schedule: the
 * chains in workspace rows, sum / deg added to out at the end (the
 * one-launch store's bits); 1 on (the default), 0 the one-launch schedule
 * (env DGLHIP_BLOCKED_MEAN_ADD). Returns the previous setting. */
int dglhip_set_blocked_mean_add(int on);
int dglhip_set_sweep_schedule(int on, int64_t table_min, int64_t block_bytes, int lag,
                              int max_spin, int64_t accum_table_min, int64_t accum_min_slots,
                              int accum_per_cu);
int dglhip_get_sweep_schedule(int* on, int64_t* table_min, int64_t* block_bytes, int* lag,
                              int* max_spin, int64_t* accum_table_min,
                              int64_t* accum_min_slots, int* accum_per_cu);
/* The accumulating sweep's soft barrier (sweep_wait in csrc/sweep.hip) gives
 * up after max_spin polls; results never depend on it. This reads how many
 * waits ran out on the current device since the last reset (one count per
 * wave that stopped waiting), synchronously; reset != 0 zeroes it after the
 * read. New design: no reference counterpart. */
int dglhip_sweep_barrier_expiries(int reset, int64_t* out);
int dglhip_set_sweep_per_cu(int per_cu);
/* Rows per wave the plan lays the streamed sweep out for: 19 (running sums
 * in LDS), 35 or 51 (19 in LDS, 16 or 32 more in registers: a CU holds more
 * rows, so fewer launches re-sweep the source blocks; 51 is the default), 10.
 * Process-wide; env DGLHIP_SWEEP_ROWS. Same bits at every setting. */
int dglhip_set_sweep_rows(int rows_per_wave);
int dglhip_get_sweep_rows(int* rows_per_wave);
int dglhip_set_sweep_unroll(int unroll);

/* The max reducer of dglhip_gspmm_device over row ranges: row r's slots are
 * [row_beg[r], row_end[r]) of the CSR (argmax slot ids stay the CSR's: k,
 * mapped as dglhip_gspmm_device's), rows in row_order. With accumulate != 0
 * a row whose range starts past indptr[r] continues from out / arg_out (its
 * earlier slots' max) and a row with an empty range is left as it is; the
 * first range of a row starts it. Launches over the rows' source-block
 * sub-ranges in block order give the one-launch values and, ties included,
 * the one-launch argmax (strict > keeps the earliest slot). */
int dglhip_gspmm_max_ranges_device(int msg_op, int64_t num_rows, int64_t feat_len,
                                   const int64_t* indptr, const int64_t* row_beg,
                                   const int64_t* row_end, int accumulate,
                                   const int32_t* indices, const int64_t* eid,
                                   const float* ufeat, const float* efeat, int64_t efeat_len,
                                   float* out, int64_t* arg_out, const int32_t* row_order,
                                   void* stream);

/* dglhip_gsddmm_device over row ranges: row r's slots are
 * [row_beg[r], row_end[r]) (outputs still at eid[k], or slot k when eid is
 * NULL), rows launched in row_order (NULL: natural order). Every value is
 * independent of the others: launches over the rows' source-block
 * sub-ranges give the one-launch bits. */
int dglhip_gsddmm_ranges_device(int op, int64_t num_rows, int64_t feat_len, int64_t num_heads,
                                const int64_t* row_beg, const int64_t* row_end,
                                const int32_t* row_order, const int32_t* indices,
                                const int64_t* eid, const float* lhs, const float* rhs,
                                float* out, void* stream);

/* dglhip_gat_attention_grad_device over row ranges: row r's slots are
 * [row_beg[r], row_end[r]) (slot indices stay the CSR's), rows launched in
 * row_order (NULL: 0..num_rows-1; a degree-descending schedule starts the
 * longest rows first). Every slot's value is independent, so launches over
 * the source blocks' sub-ranges give the one-launch bits (the GAT backward
 * under the source-blocked schedule). */
int dglhip_gat_attention_grad_ranges_device(
    int64_t num_rows, int64_t feat_len, int64_t num_heads, const int64_t* row_beg,
    const int64_t* row_end, const int32_t* row_order, const int32_t* indices,
    const float* dout, const float* ft,
    const float* attn, const float* attn_drop, const float* dz, float alpha, float clamp_lo,
    float clamp_hi, int apply_exp, float drop_scale, float* grad, void* stream);

/* dglhip_gat_attention_grad_ranges_device that also adds, per row and head,
 * the values it stores (in slot order) to grad_rowsum[row, h] (float,
 * [num_rows, num_heads], zero-filled by the caller before the first range):
 * the attention logit's destination-side gradient (GAT's er), which the
 * reference's layer gets from a second pass, a copy_edge sum over the same
 * values (examples/pytorch/gat/train.py:74-96) — same chain, same bits. Needs
 * the sliced kernel: dglhip_gat_attention_grad_rowsum_ok(feat_len, num_heads)
 * and 16-B aligned dout / ft rows. */
int dglhip_gat_attention_grad_rowsum_ok(int64_t feat_len, int64_t num_heads);
int dglhip_gat_attention_grad_rowsum_ranges_device(
    int64_t num_rows, int64_t feat_len, int64_t num_heads, const int64_t* row_beg,
    const int64_t* row_end, const int32_t* row_order, const int32_t* indices,
    const float* dout, const float* ft, const float* attn, const float* attn_drop,
    const float* dz, float alpha, float clamp_lo, float clamp_hi, int apply_exp,
    float drop_scale, float* grad, float* grad_rowsum, void* stream);

/* The backward of dglhip_gat_aggregate_device in one pass over the
 * TRANSPOSED CSR (rows u = sources, columns v = destinations), 8 heads x 16
 * features (dglhip_gat_backward_t_ok). Per transposed slot (u -> v, forward
 * slot kf = fslot[slot]) it recomputes the forward's attention a and dropped
 * weight w from el[u], er[v] and the dropout hash of kf (seed as the forward's,
 * seed + *seed_offset), and
 *   d_ft[u] = sum w * dout[v]            (fma chain in the transpose's slot order)
 *   d_el[u] = sum g                      (add chain, same order)
 *   grad[kf, h] = g = epilogue of <dout[v, h], ft[u, h]> (the attention gradient
 *                 of dglhip_gat_attention_grad_device, same bits; d_er is then
 *                 the copy_e sum of grad over the forward CSR)
 * Items as dglhip_gspmm_items_device: item i is row item_row[i] (NULL: i) with
 * slots [item_beg[i], item_end[i]) of cols / fslot, or with by_row != 0 slots
 * [item_beg[row], item_end[row]); accumulate != 0 continues both chains from
 * d_ft / d_el (source blocks of the transpose in order). dz may be NULL;
 * grad may be NULL when d_er is not wanted (nothing stored). */
int dglhip_gat_backward_t_ok(int64_t num_heads, int64_t head_dim);
int dglhip_gat_backward_t_device(
    int64_t num_items, const int32_t* item_row, const int64_t* item_beg, const int64_t* item_end,
    int by_row, int accumulate, int64_t num_rows, int64_t num_src, int64_t num_heads,
    int64_t head_dim, const int32_t* cols, const int64_t* fslot, const float* ft, const float* el,
    const float* er, const float* dz, const float* dout, float alpha, float clamp_lo,
    float clamp_hi, int apply_exp, float drop_p, uint64_t seed, const int64_t* seed_offset,
    float* d_ft, float* d_el, float* grad, void* stream);

/* dglhip_gat_backward_t_device with er and dz as one [num_rows, 2H] table
 * erdz (row v: er[v, 0..H), then dz[v, 0..H)): a pair's two destination
 * operands in one 64-B run, one cache line per slot instead of two. The same
 * arithmetic and bits. */
int dglhip_gat_backward_t_packed_device(
    int64_t num_items, const int32_t* item_row, const int64_t* item_beg, const int64_t* item_end,
    int by_row, int accumulate, int64_t num_rows, int64_t num_src, int64_t num_heads,
    int64_t head_dim, const int32_t* cols, const int64_t* fslot, const float* ft, const float* el,
    const float* erdz, const float* dout, float alpha, float clamp_lo, float clamp_hi,
    int apply_exp, float drop_p, uint64_t seed, const int64_t* seed_offset, float* d_ft,
    float* d_el, float* grad, void* stream);

/* out[r, h] = sum over the slots k of row r of vals[k, h], 8 heads, as the
 * copy_e sum's chain ((0 + v0) + v1) + ... in slot order (the same bits as
 * dglhip_gspmm_device(COPY_E, SUM) with slot-ordered values), one wave per
 * row: the GAT backward's d_er. row_order may be NULL. */
int dglhip_rowsum_heads8_device(int64_t num_rows, const int64_t* indptr,
                                const int32_t* row_order, const float* vals, float* out,
                                void* stream);

/* dglhip_gat_attention_grad_rowsum_ranges_device with the dropout's keep
 * bits recomputed from the forward's hash (seed + *seed_offset, drop_p) instead
 * of read as attn_drop != 0: a kept pair whose attention is exactly 0 keeps
 * its gradient. grad_rowsum may be NULL. */
int dglhip_gat_attention_grad_keep_ranges_device(
    int64_t num_rows, int64_t feat_len, int64_t num_heads, const int64_t* row_beg,
    const int64_t* row_end, const int32_t* row_order, const int32_t* indices,
    const float* dout, const float* ft, const float* attn, const float* dz, float alpha,
    float clamp_lo, float clamp_hi, int apply_exp, float drop_p, uint64_t seed,
    const int64_t* seed_offset, float* grad, float* grad_rowsum, void* stream);

/* The attention gradient with the leaky_relu slope taken from the logit's
 * sign, x = el[u, h] + er[v, h] (the forward's sum): alpha where x <= 0, as
 * torch's leaky_relu backward. The entries above read it from the stored
 * attention (a <= 1 with exp), which differs only for 0 < x < 2^-24, where
 * exp(x) rounds to 1 (r04 ADVICE); the fused one-pass backward
 * (dglhip_gat_backward_t_device) has x and uses its sign too. Dropout: the hash
 * keep bits when drop_p > 0 (attn_drop must then be NULL), else attn_drop != 0
 * with drop_scale when attn_drop is given. grad_rowsum, dz may be NULL. */
int dglhip_gat_attention_grad_logits_ranges_device(
    int64_t num_rows, int64_t feat_len, int64_t num_heads, const int64_t* row_beg,
    const int64_t* row_end, const int32_t* row_order, const int32_t* indices,
    const float* dout, const float* ft, const float* attn, const float* attn_drop,
    const float* dz, const float* el, const float* er, float alpha, float clamp_lo,
    float clamp_hi, int apply_exp, float drop_scale, float drop_p, uint64_t seed,
    const int64_t* seed_offset, float* grad, float* grad_rowsum, void* stream);

/* GAT logits el[n, h] = sum_d ft[n, h, d] * attn_l[h, d] (and er with attn_r;
 * attn_r / er may both be NULL), ft [N, H, D], attn [H, D], el / er [N, H]:
 * the reference's bmm(head_ft, attn_l) (gat/train.py:66-67) in a fixed
 * association: at D = 16 the tree ((p0 + p1) + (p2 + p3)) + ((p4 + p5) +
 * (p6 + p7)) with p_l = fma(x[2l+1], a[2l+1], x[2l] * a[2l]), else one fma
 * chain over d. Host and device give the same bits. */
int dglhip_gat_logits_device(int64_t num_nodes, int64_t num_heads, int64_t head_dim,
                             const float* ft, const float* attn_l, const float* attn_r, float* el,
                             float* er, void* stream);
int dglhip_gat_logits_host(int64_t num_nodes, int64_t num_heads, int64_t head_dim,
                           const float* ft, const float* attn_l, const float* attn_r, float* el,
                           float* er, int num_threads);
/* dglhip_gat_aggregate_ranges_device with attn_l [H, D] given: with the
 * recompute switched on (dglhip_set_gat_logit_recompute(1); off by default,
 * slower on the Reddit-shaped layer: DESIGN.md §4.2.1) and where the 8-head x
 * 16 source-blocked kernel runs, each slot's el[u] is recomputed from the
 * gathered ft[u] row in dglhip_gat_logits_device's association instead of
 * gathered (4 lines per slot instead of 5). The caller guarantees el ==
 * dglhip_gat_logits(ft, attn_l) (the same bits then); otherwise the plain
 * entry. */
int dglhip_gat_aggregate_logits_ranges_device(
    int64_t num_rows, int64_t num_src, int64_t num_heads, int64_t head_dim,
    const int64_t* row_beg, const int64_t* row_end, int accumulate, const int32_t* indices,
    const int32_t* row_order, const float* el, const float* er, const float* ft,
    const float* attn_l, float alpha, float clamp_lo, float clamp_hi, int apply_exp,
    float drop_p, uint64_t seed, const int64_t* seed_offset, float* out_ft, float* out_z,
    float* attn_out, float* attn_drop_out, void* stream);
/* Study knob: 1 switches the recompute above on (default 0; same bits). */
/* Study knob: the 8 x 16 fused forward (row policy 2, logits gathered)
 * compiled for at least 5 or 6 waves per SIMD (0: as the compiler allocates). */
int dglhip_set_gat_fwd_waves(int waves);
int dglhip_set_gat_logit_recompute(int on);

/* dglhip_gat_aggregate_device over row ranges: row r's slots are
 * [row_beg[r], row_end[r]) of indices (slot indices, the dropout hash and the
 * attention positions stay the CSR's); with accumulate != 0 both chains
 * continue from out_ft / out_z and rows with an empty range are left as they
 * are. One launch per contiguous source block, in block order, over the
 * sub-ranges of rows whose sources never decrease in block along the row,
 * gives the one-launch bits (the source-blocked schedule).
 * dglhip_gat_aggregate_device is this with row_beg = indptr,
 * row_end = indptr + 1, accumulate = 0. */
int dglhip_gat_aggregate_ranges_device(
    int64_t num_rows, int64_t num_src, int64_t num_heads, int64_t head_dim,
    const int64_t* row_beg, const int64_t* row_end, int accumulate, const int32_t* indices,
    const int32_t* row_order, const float* el, const float* er, const float* ft, float alpha,
    float clamp_lo, float clamp_hi, int apply_exp, float drop_p, uint64_t seed,
    const int64_t* seed_offset, float* out_ft, float* out_z, float* attn_out,
    float* attn_drop_out, void* stream);

/* Study knob for dglhip_gat_aggregate_device: 0 (default) automatic; 1 = the
 * attention computed in every lane that consumes it; 2 = once per (slot,
 * head), shared through LDS (H in {1, 2, 4, 8, 16}). Same bits. */
int dglhip_set_gat_variant(int variant);

/* Study knob for dglhip_gat_backward_t_device: the attention gradient's store
 * (0 default, 1 non-temporal, 2 none — the gradient buffer is then left
 * unwritten, so d_er is not valid: timing only). */
int dglhip_set_gat_bwd_variant(int variant);

/* The attention-dropout mask of dglhip_gat_aggregate_device: keep[i] = 1 for
 * the kept (slot, head) pairs i = k * H + h, a stateless hash of (seed, i). */
int dglhip_gat_dropout_mask_host(int64_t num_slots, int64_t num_heads, float drop_p,
                                 uint64_t seed, uint8_t* keep);

/* ------------------------------------------------------------------------ */
/* Typed-edge block-diagonal g-SpMM (R-GCN block layer; replaces the        */
/* reference's edge UDF + builtin sum, examples/pytorch/rgcn/layers.py:      */
/* 121-132 and link_predict.py's RGCNBlockLayer): with Fi = nb*si,           */
/* Fo = nb*so,                                                               */
/*   out[r, b*so+j] = sum_{slot k of row r} norm[k] *                       */
/*                    sum_i ufeat[indices[k], b*si+i] * weight[rel[k],b,i,j] */
/* with rel / norm given per CSR slot (norm may be NULL = 1); weight is     */
/* float32[R, nb, si, so]. Rows are cut into chunks of DGLHIP_TYPED_CHUNK   */
/* slots: each chunk is one sequential fma chain in slot order, and a row   */
/* of several chunks is their partial sums added in chunk order. The host   */
/* entry points run the same chains (identical bits).                       */
/* ------------------------------------------------------------------------ */
#define DGLHIP_TYPED_CHUNK 64
/* Device form: the chunks as items. item_ptr[num_rows+1] = each row's first
 * item (a row of deg slots has max(1, ceil(deg / DGLHIP_TYPED_CHUNK))
 * items), item_row[num_items] = the row of each item (entries >= num_rows:
 * padding, skipped — an item list sized by its bound num_rows + nnz /
 * DGLHIP_TYPED_CHUNK needs no host sync), heavy_row[num_heavy] = the rows of
 * more than one item (NULL with num_heavy = num_rows: every row checked);
 * partial = num_items x Fo floats of workspace (only heavy rows' items are
 * written). */
int dglhip_typed_block_spmm_device(int64_t num_rows, int64_t num_items, int64_t num_blocks,
                                   int64_t in_block, int64_t out_block,
                                   const int64_t* indptr, const int64_t* item_ptr,
                                   const int32_t* item_row, int64_t num_heavy,
                                   const int32_t* heavy_row, const int32_t* indices,
                                   const int32_t* slot_rel, const float* slot_norm,
                                   const float* ufeat, const float* weight, float* out,
                                   float* partial, void* stream);
int dglhip_typed_block_spmm_host(int64_t num_rows, int64_t num_blocks,
                                 int64_t in_block, int64_t out_block,
                                 const int64_t* indptr, const int32_t* indices,
                                 const int32_t* slot_rel, const float* slot_norm,
                                 const float* ufeat, const float* weight, float* out,
                                 int num_threads);
/* Study knob: at most `slices` (1, 2, 4, 8) slices of 64 outputs per wave of
 * the typed-block g-SpMM (default 1: one wave per 64 outputs; 8: one wave per
 * item at R-GCN's 500 outputs, slower there). Same bits. */
int dglhip_set_typed_block_width(int slices);
/* Weight gradient: dweight[r,b,i,j] = sum over the edges k of relation r
 * (relation-major CSR rel_ptr[R+1] with per-edge rel_src / rel_dst /
 * rel_norm, norm may be NULL) of norm[k] * ufeat[src, b*si+i] *
 * dout[dst, b*so+j]; each relation's edge list chunked as the rows above
 * (items item_ptr / item_rel, heavy_rel, partial = num_items x nb*si*so
 * floats). */
int dglhip_typed_block_wgrad_device(int64_t num_rels, int64_t num_items, int64_t num_blocks,
                                    int64_t in_block, int64_t out_block,
                                    const int64_t* rel_ptr, const int64_t* item_ptr,
                                    const int32_t* item_rel, int64_t num_heavy,
                                    const int32_t* heavy_rel, const int32_t* rel_src,
                                    const int32_t* rel_dst, const float* rel_norm,
                                    const float* ufeat, const float* dout, float* dweight,
                                    float* partial, void* stream);
int dglhip_typed_block_wgrad_host(int64_t num_rels, int64_t num_blocks,
                                  int64_t in_block, int64_t out_block,
                                  const int64_t* rel_ptr, const int32_t* rel_src,
                                  const int32_t* rel_dst, const float* rel_norm,
                                  const float* ufeat, const float* dout, float* dweight,
                                  int num_threads);
/* The typed-block g-SpMM in two launches (r06), the same bits as
 * dglhip_typed_block_spmm_device:
 *   messages: msg[pos_slot[p] * Fo + b*so + j] = fma chain over i of
 *     ufeat[pos_row[p], b*si + i] * weight[r, b, i, j] (from 0), for every
 *     position p of the relation-major grouping (rel_ptr[R+1], chunked as
 *     items item_ptr / item_rel; pos_row = each position's operand row,
 *     pos_slot = the forward-CSR slot its message goes to; Fi, Fo <= 1024,
 *     in_block 1, 2, 4, 5, 8 or 16);
 *   sum: out[row] = fma(slot_norm[k], msg[slot_map[k]], acc) over the CSR
 *     row's slots k in order (slot_map NULL: the slot itself; slot_norm NULL:
 *     1), rows of several items combined as in the one-kernel form, times
 *     row_scale[row] when given (one rounding, as torch's `agg * norm`).
 * A message's operand row may be scaled too (row_scale of the message entry:
 * ufeat[row] * row_scale[row], the backward's dout * norm), and the weight
 * given as (R, nb, out_block, in_block) and read transposed
 * (weight_transposed = 1: the backward's blocks without a transposed copy). 
 * dglhip_typed_block_msg_ok: 1 when the message path is on (the default;
 * dglhip_set_typed_block_messages / env DGLHIP_TYPED_MESSAGES) and takes
 * these widths. The same switch moves dglhip_typed_block_wgrad_device to its
 * LDS-staged form (same bits). */
int dglhip_typed_block_msg_ok(int64_t num_blocks, int64_t in_block, int64_t out_block);
int dglhip_set_typed_block_messages(int on);
int dglhip_typed_block_msg_device(int64_t num_rels, int64_t num_items, int64_t num_blocks,
                                  int64_t in_block, int64_t out_block, const int64_t* rel_ptr,
                                  const int64_t* item_ptr, const int32_t* item_rel,
                                  const int32_t* pos_row, const int64_t* pos_slot,
                                  const float* ufeat, const float* row_scale,
                                  const float* weight, int weight_transposed, float* msg,
                                  void* stream);
int dglhip_typed_msg_sum_device(int64_t num_rows, int64_t num_items, int64_t feat_len,
                                const int64_t* indptr, const int64_t* item_ptr,
                                const int32_t* item_row, int64_t num_heavy,
                                const int32_t* heavy_row, const int64_t* slot_map,
                                const float* slot_norm, const float* msg,
                                const float* row_scale, float* out, float* partial,
                                void* stream);
/* The weight gradient with dout's rows scaled (dout[dst] * dout_scale[dst],
 * rounded as torch's product; NULL: unscaled, as
 * dglhip_typed_block_wgrad_device) on the message path's staged kernel. */
int dglhip_typed_block_wgrad_scaled_device(int64_t num_rels, int64_t num_items,
                                           int64_t num_blocks, int64_t in_block,
                                           int64_t out_block, const int64_t* rel_ptr,
                                           const int64_t* item_ptr, const int32_t* item_rel,
                                           int64_t num_heavy, const int32_t* heavy_rel,
                                           const int32_t* rel_src, const int32_t* rel_dst,
                                           const float* rel_norm, const float* ufeat,
                                           const float* dout, const float* dout_scale,
                                           float* dweight, float* partial, void* stream);

/* The typed-block entries' item list from a CSR-like ptr[num_rows+1]: item_ptr
 * [num_rows+1] (row r has max(1, ceil(deg / DGLHIP_TYPED_CHUNK)) items) and
 * item_row[bound] (each item's row; entries past the last item = num_rows),
 * bound >= the item count (num_rows + ceil(nnz / DGLHIP_TYPED_CHUNK) always
 * is). No host sync; workspace of dglhip_typed_items_workspace_bytes bytes. */
int64_t dglhip_typed_items_workspace_bytes(int64_t num_rows);
int dglhip_typed_items_device(int64_t num_rows, const int64_t* ptr, int64_t bound,
                              int64_t* item_ptr, int32_t* item_row, void* workspace,
                              int64_t workspace_bytes, void* stream);

/* Groupings of the typed-block and DistMult kernels, each one call (r06):
 *   positions: ptr[num_rows+1] and order[m] = the positions k of idx[m]
 *     grouped by idx[k], ascending k within a group (a stable sort; ids
 *     outside [0, num_rows) are clamped into it: check them first), and the
 *     item list over ptr as dglhip_typed_items_device makes it (bound >=
 *     num_rows + ceil(m / DGLHIP_TYPED_CHUNK));
 *   relations: the forward CSR's slots grouped by relation, etype[fwd_eid[s]]
 *     for slot s, ascending slot within a relation: ptr[num_rels+1], and per
 *     relation-major position the slot, its column (src) and its row (dst),
 *     with the item list over ptr (item_ptr / item_rel).
 * No host sync; workspace of the *_workspace_bytes size. */
int64_t dglhip_group_positions_workspace_bytes(int64_t num_rows, int64_t m);
int dglhip_group_positions_device(int64_t num_rows, int64_t m, const int64_t* idx,
                                  int64_t bound, int64_t* ptr, int32_t* order,
                                  int64_t* item_ptr, int32_t* item_row, void* workspace,
                                  int64_t workspace_bytes, void* stream);
int64_t dglhip_relation_groups_workspace_bytes(int64_t num_rels, int64_t nnz);
int dglhip_relation_groups_device(int64_t num_rels, int64_t fwd_rows, int64_t nnz,
                                  const int64_t* etype, const int64_t* fwd_indptr,
                                  const int32_t* fwd_indices, const int64_t* fwd_eid,
                                  int64_t bound, int64_t* ptr, int32_t* src, int64_t* slot,
                                  int32_t* dst, int64_t* item_ptr, int32_t* item_rel,
                                  void* workspace, int64_t workspace_bytes, void* stream);

/* DistMult decoder of R-GCN link prediction (the reference's calc_score,
 * examples/pytorch/rgcn/link_predict.py:50-55: s = h[subj] * w_rel[rel] *
 * h[obj], score = s.sum(1)), with no [num_samples, F] tensor in between.
 * score[i] = sum_f (h[subj[i], f] * w_rel[rel[i], f]) * h[obj[i], f]: 64 lane
 * chains over f = l, l + 64, ... then a xor butterfly (the host entry runs the
 * same association). Indices outside [0, num_nodes) / [0, num_rels) give NaN. */
int dglhip_distmult_score_device(int64_t num_samples, int64_t feat_len, int64_t num_nodes,
                                 int64_t num_rels, const int64_t* subj, const int64_t* rel,
                                 const int64_t* obj, const float* h, const float* w_rel,
                                 float* score, void* stream);
int dglhip_distmult_score_host(int64_t num_samples, int64_t feat_len, int64_t num_nodes,
                               int64_t num_rels, const int64_t* subj, const int64_t* rel,
                               const int64_t* obj, const float* h, const float* w_rel,
                               float* score, int num_threads);
/* Its gradients from dscore[num_samples], deterministic: out[row] = the chain
 * acc + term over the row's positions in ptr / order (a stable grouping of an
 * index array by row, cut into DGLHIP_TYPED_CHUNK-position items combined in
 * order, item_ptr / item_row as the typed-block entries; partial =
 * num_items x feat_len floats of workspace). Terms, as torch's autograd of
 * (h[subj] * w_rel[rel]) * h[obj]:
 *   task 0, rows = nodes, positions p in [0, 2 num_samples) over cat(subj, obj):
 *     p < n: (dscore[p] * h[obj[p]]) * w_rel[rel[p]];
 *     p >= n: dscore[i] * (h[subj[i]] * w_rel[rel[i]]), i = p - n;
 *   task 1, rows = relations, positions i over rel: (dscore[i] * h[obj[i]]) * h[subj[i]]. */
int dglhip_distmult_grad_device(int task, int64_t num_rows, int64_t num_items, int64_t feat_len,
                                int64_t num_samples, int64_t num_nodes, int64_t num_rels,
                                const int64_t* ptr, const int64_t* item_ptr,
                                const int32_t* item_row, const int32_t* order,
                                const int64_t* subj, const int64_t* rel, const int64_t* obj,
                                const float* dscore, const float* h, const float* w_rel,
                                float* out, float* partial, void* stream);
/* The R-GCN example's link-prediction loss fused (r06; the reference's
 * get_loss, examples/pytorch/rgcn/link_predict.py: BCE-with-logits of the
 * DistMult scores averaged over the samples, + reg * (mean(h^2) +
 * mean(w_rel^2))): loss[0] and score[num_samples] (the bits of
 * dglhip_distmult_score_device) in two launches, workspace of
 * dglhip_distmult_loss_workspace_floats floats. Its gradients: the entry
 * above with dscore = (sigmoid(score) - labels) * (g[0] / num_samples) formed
 * in the kernel, and 2 * reg * g[0] / (rows * feat_len) * h (task 0) or
 * * w_rel (task 1) added to every output row; g = the loss's upstream
 * gradient on the device (no host read). */
int64_t dglhip_distmult_loss_workspace_floats(int64_t num_samples, int64_t num_nodes,
                                              int64_t num_rels, int64_t feat_len);
int dglhip_distmult_loss_fwd_device(int64_t num_samples, int64_t feat_len, int64_t num_nodes,
                                    int64_t num_rels, const int64_t* subj, const int64_t* rel,
                                    const int64_t* obj, const float* h, const float* w_rel,
                                    const float* labels, float reg, float* score, float* loss,
                                    float* workspace, int64_t workspace_floats, void* stream);
int dglhip_distmult_loss_grad_device(int task, int64_t num_rows, int64_t num_items,
                                     int64_t feat_len, int64_t num_samples, int64_t num_nodes,
                                     int64_t num_rels, const int64_t* ptr, const int64_t* item_ptr,
                                     const int32_t* item_row, const int32_t* order,
                                     const int64_t* subj, const int64_t* rel, const int64_t* obj,
                                     const float* score, const float* labels, const float* g,
                                     float reg, const float* h, const float* w_rel, float* out,
                                     float* partial, void* stream);
int dglhip_distmult_grad_host(int task, int64_t num_rows, int64_t feat_len, int64_t num_samples,
                              int64_t num_nodes, int64_t num_rels, const int64_t* ptr,
                              const int32_t* order, const int64_t* subj, const int64_t* rel,
                              const int64_t* obj, const float* dscore, const float* h,
                              const float* w_rel, float* out, int num_threads);

/* ------------------------------------------------------------------------ */
/* Kernel timing (measurement support for bench.py): when enabled, every     */
/* g-SpMM launch is bracketed by a pair of hipEvents on its own stream.     */
/* ------------------------------------------------------------------------ */
int dglhip_timing_enable(int enable);
/* Tuning knob for copy_u + sum: force (vec floats/lane, lanes/row, gathers
 * per batch, software-pipelined batches) for subsequent launches; vec = 0
 * restores the automatic choice. Results are identical for every variant
 * (same per-element chain). */
int dglhip_set_spmm_variant(int vec, int group, int unroll, int pipelined);
/* Cache policy of copy_u + sum's source-row gathers and output stores (VEC 2 x
 * 64-lane shape; results are identical under every policy):
 *  -1 automatic (the default): non-temporal output stores when the output
 *     exceeds 512 MiB (twice the Infinity Cache), default policy otherwise;
 *   0 default policy; 1 all non-temporal; 2 "hot" rows (column id with bit 31
 *   set by the caller, on a CSR copy no other kernel reads) default and the
 *   rest non-temporal; 3 non-temporal output stores only. */
int dglhip_set_cache_policy(int policy);
/* Study knob: the cache policy of the running output rows that accumulating
 * copy_u + sum items (the source-blocked schedule's later launches) read and
 * rewrite (and the fused GAT layer's 8-head rows): 0 plain, 1 non-temporal
 * load and store, 2 non-temporal load + sc1 store (the default), 3 sc0 sc1
 * load + sc1 store, 4 plain load + sc1 store (2-4: the first launch's stores
 * with sc1 too). Item launches only, and only where no output cache policy
 * (dglhip_set_cache_policy, or the automatic non-temporal output past twice
 * the Infinity Cache) applies. Same values. */
int dglhip_set_row_policy(int policy);
/* Synchronises on the recorded events and returns the summed kernel time
 * (ms) and launch count since the last enable/reset. */
int dglhip_timing_read(double* total_ms, int64_t* launches);

/* ------------------------------------------------------------------------ */
/* PackedFunc registry (replaces the TVM-derived runtime's global registry, */
/* src/runtime/registry.cc:47,137 and c_runtime_api.cc:243-276, so that a    */
/* ctypes binding written for libdgl finds the engine's kernels by name).   */
/* ------------------------------------------------------------------------ */

/* Type codes (include/dgl/runtime/c_runtime_api.h:79-95, DLPack kDLInt=0,
 * kDLUInt=1, kDLFloat=2). */
#define DGLHIP_TC_INT 0
#define DGLHIP_TC_UINT 1
#define DGLHIP_TC_FLOAT 2
#define DGLHIP_TC_HANDLE 3
#define DGLHIP_TC_NULL 4
#define DGLHIP_TC_DGL_TYPE 5
#define DGLHIP_TC_DGL_CONTEXT 6
#define DGLHIP_TC_ARRAY_HANDLE 7
#define DGLHIP_TC_NODE_HANDLE 8
#define DGLHIP_TC_MODULE_HANDLE 9
#define DGLHIP_TC_FUNC_HANDLE 10
#define DGLHIP_TC_STR 11
#define DGLHIP_TC_BYTES 12
#define DGLHIP_TC_NDARRAY_CONTAINER 13

/* DLPack-compatible tensor (same layout as DLTensor with DLContext, which is
 * what include/dgl/runtime/ndarray.h:114 passes). device_type: 1 = CPU,
 * 10 = ROCm (kDLROCM, c_runtime_api.cc:36). */
typedef struct {
  void* data;
  int32_t device_type;
  int32_t device_id;
  int32_t ndim;
  uint8_t dtype_code;
  uint8_t dtype_bits;
  uint16_t dtype_lanes;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
} DGLHipTensor;

typedef union {
  int64_t v_int64;
  double v_float64;
  void* v_handle;
  const char* v_str;
} DGLHipValue;

/* DLManagedTensor (dlpack.h; the reference's include/dgl/runtime/ndarray.h
 * exchanges these with torch through DGLArrayFromDLPack / DGLArrayToDLPack). */
typedef struct DGLHipManagedTensor {
  DGLHipTensor dl_tensor;
  void* manager_ctx;
  void (*deleter)(struct DGLHipManagedTensor* self);
} DGLHipManagedTensor;

typedef void* DGLHipFunctionHandle;
typedef void* DGLHipModuleHandle;
typedef void* DGLHipStreamHandle;
/* A DGLArrayHandle points at a DGLHipTensor that is the first member of the
 * library's ref-counted array container. */
typedef DGLHipTensor* DGLHipArrayHandle;
typedef void* DGLHipRetValueHandle;
/* C callback types (c_runtime_api.h:300-314). */
typedef int (*DGLHipPackedCFunc)(DGLHipValue* args, int* type_codes, int num_args,
                                 DGLHipRetValueHandle ret, void* resource_handle);
typedef void (*DGLHipPackedCFuncFinalizer)(void* resource_handle);

/* Function registry and calls (c_runtime_api.h:233-375). */
int DGLFuncGetGlobal(const char* name, DGLHipFunctionHandle* out);
int DGLFuncListGlobalNames(int* out_size, const char*** out_array);
int DGLFuncCall(DGLHipFunctionHandle func, DGLHipValue* arg_values,
                int* type_codes, int num_args, DGLHipValue* ret_val,
                int* ret_type_code);
int DGLFuncFree(DGLHipFunctionHandle func);
int DGLFuncRegisterGlobal(const char* name, DGLHipFunctionHandle f, int override_);
int DGLFuncCreateFromCFunc(DGLHipPackedCFunc func, void* resource_handle,
                           DGLHipPackedCFuncFinalizer fin, DGLHipFunctionHandle* out);
int DGLCFuncSetReturn(DGLHipRetValueHandle ret, DGLHipValue* value, int* type_code,
                      int num_ret);
int DGLCbArgToReturn(DGLHipValue* value, int code);

/* NDArray (c_runtime_api.h:388-461). Host arrays are 64-B aligned host
 * memory; device_type 10 (ROCm) arrays are hipMalloc'ed on device_id. */
int DGLArrayAlloc(const int64_t* shape, int ndim, int dtype_code, int dtype_bits,
                  int dtype_lanes, int device_type, int device_id,
                  DGLHipArrayHandle* out);
int DGLArrayFree(DGLHipArrayHandle handle);
int DGLArrayCopyFromBytes(DGLHipArrayHandle handle, void* data, size_t nbytes);
int DGLArrayCopyToBytes(DGLHipArrayHandle handle, void* data, size_t nbytes);
int DGLArrayCopyFromTo(DGLHipArrayHandle from, DGLHipArrayHandle to,
                       DGLHipStreamHandle stream);
int DGLArrayFromDLPack(DGLHipManagedTensor* from, DGLHipArrayHandle* out);
int DGLArrayToDLPack(DGLHipArrayHandle from, DGLHipManagedTensor** out);
void DGLDLManagedTensorCallDeleter(DGLHipManagedTensor* dltensor);

/* Streams (c_runtime_api.h:471-520); HIP streams on ROCm, no-ops on CPU. */
int DGLStreamCreate(int device_type, int device_id, DGLHipStreamHandle* out);
int DGLStreamFree(int device_type, int device_id, DGLHipStreamHandle stream);
int DGLSetStream(int device_type, int device_id, DGLHipStreamHandle handle);
int DGLSynchronize(int device_type, int device_id, DGLHipStreamHandle stream);
int DGLStreamStreamSynchronize(int device_type, int device_id,
                               DGLHipStreamHandle src, DGLHipStreamHandle dst);

/* Modules / extension types (c_runtime_api.h:179-226). DGL never creates
 * runtime modules or extension types; kernels are built into this library.
 * These fail with a message (freeing NULL succeeds). */
int DGLModLoadFromFile(const char* file_name, const char* format,
                       DGLHipModuleHandle* out);
int DGLModImport(DGLHipModuleHandle mod, DGLHipModuleHandle dep);
int DGLModGetFunction(DGLHipModuleHandle mod, const char* func_name,
                      int query_imports, DGLHipFunctionHandle* out);
int DGLModFree(DGLHipModuleHandle mod);
int DGLExtTypeFree(void* handle, int type_code);

/* Registered names (argument lists are documented in csrc/registry.cc,
 * csrc/graph_index.cc and csrc/scheduler.cc):
 *   "dglhip._CAPI_GSpMM"        (msg, reduce, indptr, indices, eid, ufeat,
 *                                efeat|null, out, arg_out|null,
 *                                row_order|null, stream[, plan|null
 *                                [, edge_layout]]) — through the plan's
 *                                schedule (a plan made for the call when none
 *                                is given; edge_layout default BY_EID)
 *   "dglhip._CAPI_SpmmPlanCreate" (indptr, indices, num_cols, row_order|null,
 *                                stream) -> plan HANDLE
 *   "dglhip._CAPI_SpmmPlanFree"  (plan)
 *   "dglhip._CAPI_SpmmPlanSchedule" (plan, msg, reduce, feat_len, ufeat_ld,
 *                                num_src_rows, efeat_len, edge_layout,
 *                                stream) -> path * 2^32 + launches
 *   "dglhip._CAPI_SpmmPlanBlocked" (plan, row_bytes, block_bytes, blocks,
 *                                stream) -> NULL or an indexable function:
 *                                0 meta int64 [B, suffix, n_absent, L, then
 *                                per launch n_items, nnz, off, suffix],
 *                                1 indices, 2 pos, 3 absent, 4 + 2i rows of
 *                                launch i, 5 + 2i its ptr (global offsets)
 *   "dglhip._CAPI_SpmmPlanCuts"  (plan, row_bytes, block_bytes, blocks,
 *                                stream) -> NULL or int64 [n, rows] ranges
 *   "dglhip._CAPI_SpmmPlanSplit" (plan, threshold, skip_empty, chunk, stream)
 *                                -> indexable: 0 meta [n_light, n_heavy,
 *                                n_chunks], 1 light, 2 heavy, 3 chunk_ptr,
 *                                4 beg, 5 end
 *   "dglhip._CAPI_SpmmPlanTiers" (plan, skip_empty, threshold|0, stream) ->
 *                                indexable: 0 meta [n_long, n_tail, T, then
 *                                per tier maxd, n], 1 + 3t rows, 2 + 3t
 *                                slot_ptr, 3 + 3t slot_cols of tier t
 *   "dglhip._CAPI_GSDDMM"       (op, num_heads, indptr, indices, eid, lhs, rhs,
 *                                out, stream)
 *   "dglhip._CAPI_COOToCSR"     (num_rows, row, col, order, indptr, indices,
 *                                eid)
 *   "dglhip._CAPI_RowsByDegree" (indptr, row_order)
 *   "graph_index._CAPI_*"       the 45 graph-index functions of
 *                                src/graph/graph_apis.cc, same arguments and
 *                                returns (graphs as HANDLEs, id arrays as
 *                                int64 host NDArrays, edge/subgraph/adjacency
 *                                results as indexable FUNC_HANDLEs)
 *   "runtime.degree_bucketing._CAPI_*"  the 4 scheduler functions of
 *                                src/scheduler/scheduler_apis.cc:16-60
 * Tensors are DGLHipTensor* (type code 7 or 13); device is taken from the
 * tensor. A NULL stream argument means the stream set by DGLSetStream. */

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif  /* DGL_HIP_H_ */
