/*
 * TEST ORACLE — test infrastructure only, never part of the product path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / the timed CPU baseline.
 *
 * Plain-C restatement of the reference's hot-path arithmetic:
 *
 *   The reference (GaiYu0/dgl-1, DGL 0.1.3) computes update_all(copy_src,sum)
 *   as  torch.sparse.mm(A, H)  with A = torch.sparse_coo_tensor(idx, ones)
 *   built by python/dgl/graph_index.py:574-583 from the index of
 *   Graph::GetAdj (src/graph/graph.cc:509-524): idx = [dst_0..dst_{E-1};
 *   src_0..src_{E-1}] in edge-id order, values fp32 ones, UNCOALESCED
 *   (python/dgl/backend/pytorch/tensor.py:45-51, spmm at :145-146).
 *   src_mul_edge(+sum) rebuilds the same COO with the edge weights as values
 *   (python/dgl/runtime/ir/executor.py:535-566).
 *
 *   The arithmetic itself lives in the third-party dependency PyTorch
 *   (pinned here: torch 2.10.0, CPU kernel s_addmm_out_sparse_dense_worker in
 *   aten/src/ATen/native/sparse/SparseTensorMath.cpp — not vendored under
 *   /root/reference). Its published algorithm for an uncoalesced COO:
 *     r = 0;  for e in nnz order:  r[row_e,:] += val_e * H[col_e,:]   (axpy)
 *   Measured in this container (tests/golden/make_golden.py, fixtures under
 *   tests/golden/): the result equals, bit for bit, a per-element fused
 *   multiply-add chain in nnz order, r = fmaf(val_e, H, r) — duplicates are
 *   NOT merged. Its autograd (dH = A^T dC) is the same chain over the
 *   transposed COO, i.e. per source node in edge-id order.
 *
 *   max / mean have no SPMV in the reference: they run the degree-bucketing
 *   UDF path (python/dgl/runtime/degree_bucketing.py:13-190,
 *   function/reducer.py:52-97) = torch.max / torch.mean over each node's
 *   mailbox (messages in edge order); nodes without messages get the frame
 *   initializer (zeros).
 *
 * Pinned by: tests/golden/*.npz (torch.sparse.mm outputs on the reference's
 * COO), checked in tests/test_oracle.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* r = A @ H for an uncoalesced COO in nnz order (val == NULL -> ones). */
void oracle_spmm_coo(int64_t num_rows, int64_t F, int64_t nnz,
                     const int64_t* row, const int64_t* col, const float* val,
                     const float* H, float* out) {
  memset(out, 0, sizeof(float) * (size_t)(num_rows * F));
  for (int64_t e = 0; e < nnz; ++e) {
    const float w = val ? val[e] : 1.0f;
    float* o = out + row[e] * F;
    const float* h = H + col[e] * F;
    for (int64_t f = 0; f < F; ++f) o[f] = fmaf(w, h[f], o[f]);
  }
}

/* Stable grouping of COO entries by row (counting sort): the CSR whose row
 * slots keep nnz order. indptr[num_rows+1], indices[nnz] (col), pos[nnz]. */
void oracle_coo_to_csr(int64_t num_rows, int64_t nnz, const int64_t* row,
                       const int64_t* col, int64_t* indptr, int64_t* indices,
                       int64_t* pos) {
  int64_t* cursor = (int64_t*)calloc((size_t)num_rows + 1, sizeof(int64_t));
  memset(indptr, 0, sizeof(int64_t) * (size_t)(num_rows + 1));
  for (int64_t e = 0; e < nnz; ++e) indptr[row[e] + 1]++;
  for (int64_t r = 0; r < num_rows; ++r) indptr[r + 1] += indptr[r];
  for (int64_t r = 0; r < num_rows; ++r) cursor[r] = indptr[r];
  for (int64_t e = 0; e < nnz; ++e) {
    const int64_t p = cursor[row[e]]++;
    indices[p] = col[e];
    pos[p] = e;
  }
  free(cursor);
}

/* Same product from the grouped form, rows in parallel (OpenMP): identical
 * per-element operation order, so identical bits. This is also the timed
 * multi-core CPU baseline "(ii)" of BASELINE.md. val indexed by pos. */
void oracle_spmm_csr(int64_t num_rows, int64_t F, const int64_t* indptr,
                     const int64_t* indices, const int64_t* pos,
                     const float* val, const float* H, float* out,
                     int num_threads) {
#pragma omp parallel for schedule(dynamic, 64) num_threads(num_threads)
  for (int64_t r = 0; r < num_rows; ++r) {
    float* o = out + r * F;
    for (int64_t f = 0; f < F; ++f) o[f] = 0.0f;
    for (int64_t k = indptr[r]; k < indptr[r + 1]; ++k) {
      const float w = val ? val[pos[k]] : 1.0f;
      const float* h = H + indices[k] * F;
      for (int64_t f = 0; f < F; ++f) o[f] = fmaf(w, h[f], o[f]);
    }
  }
}

/* Degree-bucketing max over each row's mailbox of messages m[pos[k], :]
 * (torch.max over dim 1 is exact); empty rows = 0 (zero initializer). */
void oracle_max_mailbox(int64_t num_rows, int64_t F, const int64_t* indptr,
                        const int64_t* pos, const float* msg, float* out) {
  for (int64_t r = 0; r < num_rows; ++r) {
    float* o = out + r * F;
    if (indptr[r] == indptr[r + 1]) {
      for (int64_t f = 0; f < F; ++f) o[f] = 0.0f;
      continue;
    }
    for (int64_t f = 0; f < F; ++f) o[f] = msg[pos[indptr[r]] * F + f];
    for (int64_t k = indptr[r] + 1; k < indptr[r + 1]; ++k)
      for (int64_t f = 0; f < F; ++f) {
        const float x = msg[pos[k] * F + f];
        if (x > o[f]) o[f] = x;
      }
  }
}

/* Mean over each row's mailbox, accumulated in double (a reference value
 * for the tolerance check; torch.mean's own summation order is
 * implementation-defined). Empty rows = 0. */
void oracle_mean_mailbox(int64_t num_rows, int64_t F, const int64_t* indptr,
                         const int64_t* pos, const float* msg, float* out) {
  for (int64_t r = 0; r < num_rows; ++r) {
    const int64_t d = indptr[r + 1] - indptr[r];
    for (int64_t f = 0; f < F; ++f) {
      double s = 0.0;
      for (int64_t k = indptr[r]; k < indptr[r + 1]; ++k) s += msg[pos[k] * F + f];
      out[r * F + f] = d ? (float)(s / (double)d) : 0.0f;
    }
  }
}

/* Per-edge dot product <A[row_e], B[col_e]> in double (tolerance reference
 * for the u_mul_e weight gradient = sparse_mask(dC @ H^T)). */
void oracle_sddmm_dot(int64_t nnz, int64_t F, const int64_t* row,
                      const int64_t* col, const float* A, const float* B,
                      float* out) {
  for (int64_t e = 0; e < nnz; ++e) {
    double s = 0.0;
    for (int64_t f = 0; f < F; ++f) s += (double)A[row[e] * F + f] * B[col[e] * F + f];
    out[e] = (float)s;
  }
}
