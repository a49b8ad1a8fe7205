/*
 * capi_smoke.c -- a plain-C client of include/ppnp_amd.h (no Python, no torch).
 *
 * Builds the complete graph K5 plus an isolated node and a path P3 tail, runs
 * appnp_propagate, and checks the closed forms of SURVEY.md section 4:
 *   K_n (A+I = J):  Z_K = a H + (1-a) mean_rows(H)  for every K >= 1
 *   isolated node:  Z_K = H
 * plus error codes for invalid arguments.  Built by tests/test_native.py with gcc against the
 * HIP runtime headers; run on the GPU box.  Exit status 0 on success.
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "ppnp_amd.h"

#define CHECK_HIP(x)                                                              \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d HIP error %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 2;                                                                   \
    }                                                                             \
  } while (0)

#define CHECK_RC(x)                                                               \
  do {                                                                            \
    int rc_ = (x);                                                                \
    if (rc_ != APPNP_OK) {                                                        \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, appnp_strerror(rc_)); \
      return 3;                                                                   \
    }                                                                             \
  } while (0)

int main(void) {
  /* nodes 0..4: K5; node 5: isolated */
  enum { N = 6, F = 3, NNZ = 20 };
  int32_t indptr[N + 1];
  int32_t indices[NNZ];
  int p = 0;
  for (int i = 0; i < 5; ++i) {
    indptr[i] = p;
    for (int j = 0; j < 5; ++j)
      if (j != i) indices[p++] = j;
  }
  indptr[5] = p;
  indptr[6] = p;
  float H[N * F], Z[N * F];
  for (int i = 0; i < N * F; ++i) H[i] = (float)((i * 37) % 11) - 5.0f;

  if (appnp_abi_version() != PPNP_AMD_ABI_VERSION) return 4;
  appnp_graph* g = NULL;
  if (appnp_graph_create(NULL, NULL, NULL, N, NNZ, 0, NULL, &g) != APPNP_EINVAL) return 5;

  int32_t *d_ip, *d_ix;
  float *d_H, *d_Z;
  void* d_ws;
  CHECK_HIP(hipMalloc((void**)&d_ip, sizeof(indptr)));
  CHECK_HIP(hipMalloc((void**)&d_ix, sizeof(indices)));
  CHECK_HIP(hipMalloc((void**)&d_H, sizeof(H)));
  CHECK_HIP(hipMalloc((void**)&d_Z, sizeof(Z)));
  CHECK_HIP(hipMemcpy(d_ip, indptr, sizeof(indptr), hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_ix, indices, sizeof(indices), hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_H, H, sizeof(H), hipMemcpyHostToDevice));
  CHECK_RC(appnp_graph_create(d_ip, d_ix, NULL, N, NNZ, APPNP_NORM_SYM, NULL, &g));
  int64_t n, lo, hi, nnz_hat;
  int mode, sym;
  CHECK_RC(appnp_graph_info(g, &n, &lo, &hi, &nnz_hat, &mode, &sym));
  if (n != N || nnz_hat != NNZ + N || !sym) return 6;

  size_t ws_bytes = appnp_workspace_bytes(g, F, F, APPNP_F32);
  CHECK_HIP(hipMalloc(&d_ws, ws_bytes));
  const float alpha = 0.1f;
  for (int K = 1; K <= 10; K += 3) {
    CHECK_RC(appnp_propagate(g, d_H, F, d_Z, F, F, APPNP_F32, K, alpha, 0.0f, 0, d_ws, ws_bytes,
                             NULL));
    CHECK_HIP(hipDeviceSynchronize());
    CHECK_HIP(hipMemcpy(Z, d_Z, sizeof(Z), hipMemcpyDeviceToHost));
    for (int c = 0; c < F; ++c) {
      double mean = 0.0;
      for (int i = 0; i < 5; ++i) mean += H[i * F + c];
      mean /= 5.0;
      for (int i = 0; i < 5; ++i) {
        const double ref = alpha * H[i * F + c] + (1.0 - alpha) * mean;
        if (fabs(Z[i * F + c] - ref) > 1e-5) {
          fprintf(stderr, "K=%d node %d col %d: %f vs %f\n", K, i, c, Z[i * F + c], ref);
          return 7;
        }
      }
      if (fabs(Z[5 * F + c] - H[5 * F + c]) > 1e-6) return 8; /* isolated node */
    }
  }
  /* argument errors come back as codes */
  if (appnp_propagate(g, d_H, F, d_H, F, F, APPNP_F32, 3, alpha, 0.0f, 0, d_ws, ws_bytes, NULL) !=
      APPNP_EINVAL)
    return 9; /* aliasing H == Z */
  if (appnp_propagate(g, d_H, F, d_Z, F, F, APPNP_F32, 3, 1.5f, 0.0f, 0, d_ws, ws_bytes, NULL) !=
      APPNP_EINVAL)
    return 10; /* alpha out of range */
  if (appnp_propagate(g, d_H, F, d_Z, F, F, 7, 3, alpha, 0.0f, 0, d_ws, ws_bytes, NULL) !=
      APPNP_EINVAL)
    return 11; /* dtype */
  appnp_graph_destroy(g);
  hipFree(d_ip);
  hipFree(d_ix);
  hipFree(d_H);
  hipFree(d_Z);
  hipFree(d_ws);
  printf("capi_smoke ok\n");
  return 0;
}
