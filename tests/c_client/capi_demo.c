/*
 * A plain-C caller of libdgl_hip.so, as a maintainer binding the reference's
 * C API from another language would write it: only
 * include/dgl_hip.h, plain pointers and the PackedFunc calling convention.
 *
 *  1. builds a multigraph in the native graph index through the registry
 *     (graph_index._CAPI_DGLGraphCreateMutable / AddVertices / AddEdges);
 *  2. reads its in-CSR back with graph_index._CAPI_DGLGraphGetAdj, an
 *     indexable packed function returning library-owned NDArrays;
 *  3. runs update_all(copy_src, sum) on host memory with dglhip_gspmm_host
 *     over a CSR from dglhip_coo_to_csr_host, and checks every element
 *     against a sequential loop in edge-id order (the reference's product);
 *  4. checks the error convention (-1 + DGLGetLastError) on a bad call.
 * Prints "capi_demo ok" and exits 0 on success. Host only: no GPU needed.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dgl_hip.h"

#define CHECK(x)                                                        \
  do {                                                                  \
    if ((x) != 0) {                                                     \
      fprintf(stderr, "%s:%d: %s failed: %s\n", __FILE__, __LINE__, #x, \
              DGLGetLastError());                                       \
      exit(1);                                                          \
    }                                                                   \
  } while (0)

static DGLHipFunctionHandle get(const char* name) {
  DGLHipFunctionHandle f = NULL;
  CHECK(DGLFuncGetGlobal(name, &f));
  if (!f) {
    fprintf(stderr, "missing %s\n", name);
    exit(1);
  }
  return f;
}

/* A 1-D int64 host array owned by the library. */
static DGLHipArrayHandle ids(const int64_t* v, int64_t n) {
  DGLHipArrayHandle a = NULL;
  CHECK(DGLArrayAlloc(&n, 1, 0, 64, 1, 1, 0, &a));
  CHECK(DGLArrayCopyFromBytes(a, (void*)v, (size_t)n * sizeof(int64_t)));
  return a;
}

int main(void) {
  enum { N = 6, E = 9, F = 4 };
  const int64_t src[E] = {0, 1, 2, 3, 4, 5, 0, 0, 5};
  const int64_t dst[E] = {1, 2, 3, 4, 5, 0, 1, 3, 1};

  /* 1. graph index through the registry */
  DGLHipValue args[3], ret;
  int codes[3], rcode;
  args[0].v_int64 = 1;  /* multigraph */
  codes[0] = DGLHIP_TC_INT;
  CHECK(DGLFuncCall(get("graph_index._CAPI_DGLGraphCreateMutable"), args, codes, 1, &ret,
                    &rcode));
  if (rcode != DGLHIP_TC_HANDLE) return 1;
  void* g = ret.v_handle;
  args[0].v_handle = g;
  codes[0] = DGLHIP_TC_HANDLE;
  args[1].v_int64 = N;
  codes[1] = DGLHIP_TC_INT;
  CHECK(DGLFuncCall(get("graph_index._CAPI_DGLGraphAddVertices"), args, codes, 2, &ret,
                    &rcode));
  DGLHipArrayHandle s = ids(src, E), d = ids(dst, E);
  args[1].v_handle = s;
  codes[1] = DGLHIP_TC_NDARRAY_CONTAINER;
  args[2].v_handle = d;
  codes[2] = DGLHIP_TC_NDARRAY_CONTAINER;
  CHECK(DGLFuncCall(get("graph_index._CAPI_DGLGraphAddEdges"), args, codes, 3, &ret, &rcode));
  CHECK(DGLFuncCall(get("graph_index._CAPI_DGLGraphNumEdges"), args, codes, 1, &ret, &rcode));
  if (rcode != DGLHIP_TC_INT || ret.v_int64 != E) return 2;

  /* 2. in-CSR back through GetAdj(transpose=False, "csr") */
  args[1].v_int64 = 0;
  codes[1] = DGLHIP_TC_INT;
  args[2].v_str = "csr";
  codes[2] = DGLHIP_TC_STR;
  CHECK(DGLFuncCall(get("graph_index._CAPI_DGLGraphGetAdj"), args, codes, 3, &ret, &rcode));
  if (rcode != DGLHIP_TC_FUNC_HANDLE) return 3;
  DGLHipFunctionHandle adj = ret.v_handle;
  int64_t gi_indptr[N + 1], gi_indices[E];
  for (int which = 0; which < 2; ++which) {
    DGLHipValue w;
    int wc = DGLHIP_TC_INT;
    w.v_int64 = which;
    CHECK(DGLFuncCall(adj, &w, &wc, 1, &ret, &rcode));
    if (rcode != DGLHIP_TC_NDARRAY_CONTAINER) return 4;
    DGLHipArrayHandle arr = (DGLHipArrayHandle)ret.v_handle;
    CHECK(DGLArrayCopyToBytes(arr, which == 0 ? (void*)gi_indptr : (void*)gi_indices,
                              (size_t)(which == 0 ? N + 1 : E) * sizeof(int64_t)));
    CHECK(DGLArrayFree(arr));
  }
  CHECK(DGLFuncFree(adj));

  /* 3. g-SpMM on host: the engine's CSR (int32 columns) and kernel */
  int64_t indptr[N + 1], eid[E];
  int32_t indices[E];
  CHECK(dglhip_coo_to_csr_host(N, N, E, dst, src, DGLHIP_ORDER_EID, indptr, indices, eid));
  for (int r = 0; r <= N; ++r)
    if (indptr[r] != gi_indptr[r]) return 5;
  for (int k = 0; k < E; ++k)
    if (indices[k] != gi_indices[k]) return 6;
  float h[N * F], out[N * F], ref[N * F];
  for (int i = 0; i < N * F; ++i) h[i] = (float)((i * 37) % 11) - 5.0f + 0.25f * (float)i;
  memset(ref, 0, sizeof(ref));
  for (int e = 0; e < E; ++e)
    for (int f = 0; f < F; ++f) ref[dst[e] * F + f] += h[src[e] * F + f];
  CHECK(dglhip_gspmm_host(DGLHIP_MSG_COPY_U, DGLHIP_REDUCE_SUM, N, F, indptr, indices, eid, h,
                          NULL, 0, out, NULL, 1));
  if (memcmp(out, ref, sizeof(ref)) != 0) return 7;

  /* 4. error convention */
  int64_t bad_dst[1] = {N};
  int64_t p2[N + 1], e2[1];
  int32_t i2[1];
  if (dglhip_coo_to_csr_host(N, N, 1, bad_dst, src, 0, p2, i2, e2) != -1) return 8;
  if (strlen(DGLGetLastError()) == 0) return 9;

  args[0].v_handle = g;
  codes[0] = DGLHIP_TC_HANDLE;
  CHECK(DGLFuncCall(get("graph_index._CAPI_DGLGraphFree"), args, codes, 1, &ret, &rcode));
  CHECK(DGLArrayFree(s));
  CHECK(DGLArrayFree(d));
  printf("capi_demo ok\n");
  return 0;
}
