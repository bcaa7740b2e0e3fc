/* Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5
 * "race / memory checking"): drives every host entry point of libdgl_hip
 * (the CSR builder, degree schedule, degree bucketing, g-SpMM for every
 * message / reducer, the ranges form, g-SDDMM, GAT attention, the typed-block
 * kernels and the registry's error path) together with the CPU oracle
 * (oracle/spmm_oracle.c, linked into this test binary), on random graphs and
 * the edge cases the reference's tests cover: empty graphs, rows without
 * in-edges, duplicate (multigraph) edges, F = 1, one huge row.
 *
 * Built and run by tests/test_sanitizers.py against the sanitized library
 * (make -C dgl-1_amd/csrc asan); any invalid access, leak in our code or UB
 * aborts with a report. Results are also checked: the library's host g-SpMM
 * equals the oracle bit for bit (same per-element chain). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dgl_hip.h"

void oracle_spmm_coo(int64_t num_rows, int64_t F, int64_t nnz, const int64_t* row,
                     const int64_t* col, const float* val, const float* H, float* out);
void oracle_max_mailbox(int64_t num_rows, int64_t F, const int64_t* indptr,
                        const int64_t* pos, const float* msg, float* out);
void oracle_coo_to_csr(int64_t num_rows, int64_t nnz, const int64_t* row,
                       const int64_t* col, int64_t* indptr, int64_t* indices, int64_t* pos);

static uint64_t g_state = 88172645463325252ull;
static uint64_t rnd(void) {
  g_state ^= g_state << 13;
  g_state ^= g_state >> 7;
  g_state ^= g_state << 17;
  return g_state;
}
static float frand(void) { return (float)((rnd() >> 40) * (1.0 / 16777216.0)) * 2.0f - 1.0f; }

#define CHECK(cond, ...)                                         \
  do {                                                           \
    if (!(cond)) {                                               \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);        \
      fprintf(stderr, __VA_ARGS__);                              \
      fprintf(stderr, "\n");                                     \
      exit(1);                                                   \
    }                                                            \
  } while (0)
#define OK(call) CHECK((call) == 0, "%s -> %s", #call, DGLGetLastError())

static void* xmalloc(size_t n) {
  void* p = malloc(n ? n : 1);
  CHECK(p != NULL, "out of memory");
  return p;
}

/* one graph: n rows/cols, nnz edges; `hub` sends a third of the edges to row 0 */
static void run_case(int64_t n, int64_t nnz, int64_t F, int hub, int nthreads) {
  int64_t* row = xmalloc(sizeof(int64_t) * nnz);
  int64_t* col = xmalloc(sizeof(int64_t) * nnz);
  for (int64_t e = 0; e < nnz; ++e) {
    row[e] = (hub && e % 3 == 0) ? 0 : (int64_t)(rnd() % (uint64_t)n);
    col[e] = (int64_t)(rnd() % (uint64_t)n);
    if (e % 7 == 0 && e > 0) { row[e] = row[e - 1]; col[e] = col[e - 1]; } /* duplicates */
  }
  float* H = xmalloc(sizeof(float) * n * F);
  float* W = xmalloc(sizeof(float) * (nnz ? nnz : 1));
  float* WF = xmalloc(sizeof(float) * (nnz ? nnz : 1) * F);
  for (int64_t i = 0; i < n * F; ++i) H[i] = frand();
  for (int64_t e = 0; e < nnz; ++e) W[e] = frand();
  for (int64_t i = 0; i < nnz * F; ++i) WF[i] = frand();

  int64_t* indptr = xmalloc(sizeof(int64_t) * (n + 1));
  int32_t* indices = xmalloc(sizeof(int32_t) * (nnz ? nnz : 1));
  int64_t* eid = xmalloc(sizeof(int64_t) * (nnz ? nnz : 1));
  OK(dglhip_coo_to_csr_host(n, n, nnz, row, col, DGLHIP_ORDER_EID, indptr, indices, eid));
  /* integer arrays equal the oracle's grouping */
  int64_t* oip = xmalloc(sizeof(int64_t) * (n + 1));
  int64_t* oix = xmalloc(sizeof(int64_t) * (nnz ? nnz : 1));
  int64_t* opos = xmalloc(sizeof(int64_t) * (nnz ? nnz : 1));
  oracle_coo_to_csr(n, nnz, row, col, oip, oix, opos);
  for (int64_t r = 0; r <= n; ++r) CHECK(indptr[r] == oip[r], "indptr[%lld]", (long long)r);
  for (int64_t k = 0; k < nnz; ++k)
    CHECK(indices[k] == oix[k] && eid[k] == opos[k], "slot %lld", (long long)k);
  int32_t* order = xmalloc(sizeof(int32_t) * (n ? n : 1));
  if (n) OK(dglhip_rows_by_degree_host(n, indptr, order));
  /* the (col, eid) order too */
  int64_t* ip2 = xmalloc(sizeof(int64_t) * (n + 1));
  int32_t* ix2 = xmalloc(sizeof(int32_t) * (nnz ? nnz : 1));
  int64_t* e2 = xmalloc(sizeof(int64_t) * (nnz ? nnz : 1));
  OK(dglhip_coo_to_csr_host(n, n, nnz, row, col, DGLHIP_ORDER_COL, ip2, ix2, e2));

  float* out = xmalloc(sizeof(float) * n * F);
  float* ref = xmalloc(sizeof(float) * n * F);
  int64_t* arg = xmalloc(sizeof(int64_t) * n * F);
  /* copy_u + sum and u_mul_e (scalar) + sum: bit-exact vs the oracle */
  OK(dglhip_gspmm_host(DGLHIP_MSG_COPY_U, DGLHIP_REDUCE_SUM, n, F, indptr, indices, eid, H,
                       NULL, 0, out, NULL, nthreads));
  oracle_spmm_coo(n, F, nnz, row, col, NULL, H, ref);
  CHECK(memcmp(out, ref, sizeof(float) * n * F) == 0, "copy_u sum differs");
  OK(dglhip_gspmm_host(DGLHIP_MSG_U_MUL_E, DGLHIP_REDUCE_SUM, n, F, indptr, indices, eid, H, W,
                       1, out, NULL, nthreads));
  oracle_spmm_coo(n, F, nnz, row, col, W, H, ref);
  CHECK(memcmp(out, ref, sizeof(float) * n * F) == 0, "u_mul_e sum differs");
  /* every other reducer / message / edge layout: run (sanitizers watch) */
  OK(dglhip_gspmm_host(DGLHIP_MSG_COPY_U, DGLHIP_REDUCE_MEAN, n, F, indptr, indices, eid, H,
                       NULL, 0, out, NULL, nthreads));
  OK(dglhip_gspmm_host(DGLHIP_MSG_COPY_U, DGLHIP_REDUCE_MAX, n, F, indptr, indices, eid, H,
                       NULL, 0, out, arg, nthreads));
  {
    /* max vs the oracle's mailbox max over the messages H[col] */
    float* msg = xmalloc(sizeof(float) * (nnz ? nnz : 1) * F);
    for (int64_t e = 0; e < nnz; ++e) memcpy(msg + e * F, H + col[e] * F, sizeof(float) * F);
    oracle_max_mailbox(n, F, oip, opos, msg, ref);
    CHECK(memcmp(out, ref, sizeof(float) * n * F) == 0, "copy_u max differs");
    free(msg);
  }
  OK(dglhip_gspmm_host(DGLHIP_MSG_U_MUL_E, DGLHIP_REDUCE_MAX, n, F, indptr, indices, eid, H,
                       WF, F, out, arg, nthreads));
  OK(dglhip_gspmm_host(DGLHIP_MSG_COPY_E, DGLHIP_REDUCE_SUM, n, F, indptr, indices, eid, NULL,
                       WF, F, out, NULL, nthreads));
  OK(dglhip_gspmm_host(DGLHIP_MSG_COPY_E, DGLHIP_REDUCE_SUM, n, F, indptr, indices, NULL, NULL,
                       WF, F, out, NULL, nthreads)); /* slot-ordered edge values */
  if (F % 2 == 0 && F >= 2) /* per-head weights: H = 2 heads */
    OK(dglhip_gspmm_host(DGLHIP_MSG_U_MUL_E, DGLHIP_REDUCE_SUM, n, F, indptr, indices, eid, H,
                         WF, 2, out, NULL, nthreads));
  memcpy(ref, out, sizeof(float) * n * F);
  OK(dglhip_gspmm_host(DGLHIP_MSG_COPY_U, DGLHIP_REDUCE_SUM_ACCUM, n, F, indptr, indices, eid,
                       H, NULL, 0, out, NULL, nthreads));
  /* ranges form: every row as one item, accumulate off */
  {
    int64_t* b = xmalloc(sizeof(int64_t) * (n ? n : 1));
    int64_t* t = xmalloc(sizeof(int64_t) * (n ? n : 1));
    for (int64_t r = 0; r < n; ++r) { b[r] = indptr[r]; t[r] = indptr[r + 1]; }
    OK(dglhip_gspmm_ranges_host(DGLHIP_MSG_COPY_U, n, F, b, t, 0, indices, eid, H, NULL, 0,
                                out, nthreads));
    oracle_spmm_coo(n, F, nnz, row, col, NULL, H, ref);
    CHECK(memcmp(out, ref, sizeof(float) * n * F) == 0, "ranges differ");
    free(b);
    free(t);
  }
  /* g-SDDMM dot (1 head and F heads) and GAT attention (eid and slot order) */
  float* dots = xmalloc(sizeof(float) * (nnz ? nnz : 1) * F);
  OK(dglhip_gsddmm_host(DGLHIP_SDDMM_DOT, n, F, 1, indptr, indices, eid, H, H, dots, nthreads));
  OK(dglhip_gsddmm_host(DGLHIP_SDDMM_DOT, n, F, F, indptr, indices, NULL, H, H, dots, nthreads));
  OK(dglhip_gsddmm_attention_host(n, F, indptr, indices, eid, H, H, 0.2f, -10.0f, 10.0f, 1,
                                  dots, nthreads));
  OK(dglhip_gsddmm_attention_host(n, F, indptr, indices, NULL, H, H, 0.2f, -INFINITY,
                                  INFINITY, 0, dots, nthreads));
  /* typed blocks: 3 relations, F = nb * 1 blocks of 1x1; relation and norm
     per slot; the relation-major grouping of the same edges for dW (rows past
     one chunk of DGLHIP_TYPED_CHUNK slots take the chunked chains) */
  {
    const int64_t R = 3, nb = F, si = 1, so = 1;
    int64_t* et = xmalloc(sizeof(int64_t) * (nnz ? nnz : 1));
    int32_t* srel = xmalloc(sizeof(int32_t) * (nnz ? nnz : 1));
    float* snrm = xmalloc(sizeof(float) * (nnz ? nnz : 1));
    float* w = xmalloc(sizeof(float) * R * nb * si * so);
    float* dw = xmalloc(sizeof(float) * R * nb * si * so);
    for (int64_t e = 0; e < nnz; ++e) et[e] = (int64_t)(rnd() % 3);
    for (int64_t k = 0; k < nnz; ++k) {
      srel[k] = (int32_t)et[eid[k]];
      snrm[k] = W[eid[k]];
    }
    for (int64_t i = 0; i < R * nb * si * so; ++i) w[i] = frand();
    OK(dglhip_typed_block_spmm_host(n, nb, si, so, indptr, indices, srel, snrm, H, w, out,
                                    nthreads));
    OK(dglhip_typed_block_spmm_host(n, nb, si, so, indptr, indices, srel, NULL, H, w, out,
                                    nthreads));
    int64_t* rp = xmalloc(sizeof(int64_t) * (R + 1));
    int32_t* rs = xmalloc(sizeof(int32_t) * (nnz ? nnz : 1));
    int64_t* re = xmalloc(sizeof(int64_t) * (nnz ? nnz : 1));
    int32_t* rd = xmalloc(sizeof(int32_t) * (nnz ? nnz : 1));
    float* rn = xmalloc(sizeof(float) * (nnz ? nnz : 1));
    OK(dglhip_coo_to_csr_host(R, n, nnz, et, col, DGLHIP_ORDER_EID, rp, rs, re));
    for (int64_t k = 0; k < nnz; ++k) {
      rd[k] = (int32_t)row[re[k]];
      rn[k] = W[re[k]];
    }
    OK(dglhip_typed_block_wgrad_host(R, nb, si, so, rp, rs, rd, rn, H, H, dw, nthreads));
    free(et); free(srel); free(snrm); free(w); free(dw); free(rp); free(rs); free(re);
    free(rd); free(rn);
  }
  /* degree bucketing of the messages by destination */
  {
    int64_t nbk = 0;
    int64_t* bdeg = xmalloc(sizeof(int64_t) * (n ? n : 1));
    int64_t* bptr = xmalloc(sizeof(int64_t) * (n + 1));
    int64_t* nodes = xmalloc(sizeof(int64_t) * (n ? n : 1));
    int64_t* mids = xmalloc(sizeof(int64_t) * (nnz ? nnz : 1));
    OK(dglhip_degree_bucketing_host(nnz, row, n, &nbk, bdeg, bptr, nodes, mids));
    int64_t total = 0;
    for (int64_t b = 0; b < nbk; ++b) total += bdeg[b] * (bptr[b + 1] - bptr[b]);
    CHECK(total == nnz, "bucketing lost messages");
    free(bdeg); free(bptr); free(nodes); free(mids);
  }
  free(row); free(col); free(H); free(W); free(WF); free(indptr); free(indices); free(eid);
  free(oip); free(oix); free(opos); free(order); free(ip2); free(ix2); free(e2);
  free(out); free(ref); free(arg); free(dots);
}

int main(void) {
  /* error convention: bad arguments fail with a message, nothing is touched */
  CHECK(dglhip_gspmm_host(9, 0, 1, 1, NULL, NULL, NULL, NULL, NULL, 0, NULL, NULL, 1) == -1,
        "unknown op accepted");
  CHECK(strlen(DGLGetLastError()) > 0, "no error message");
  {
    int64_t r[2] = {0, 5}, c[2] = {0, 0}, ip[3];
    int32_t ix[2];
    int64_t e[2];
    CHECK(dglhip_coo_to_csr_host(2, 2, 2, r, c, DGLHIP_ORDER_EID, ip, ix, e) == -1,
          "out-of-range row accepted");
  }
  run_case(0, 0, 4, 0, 2);        /* empty graph */
  run_case(5, 0, 3, 0, 2);        /* rows without in-edges */
  run_case(1, 40, 1, 0, 1);       /* one row, F = 1, duplicates */
  run_case(200, 3000, 7, 1, 4);   /* odd width, a hub row */
  run_case(1000, 20000, 16, 1, 8);
  run_case(300, 5000, 64, 0, 3);
  printf("sanitize_driver ok\n");
  return 0;
}
