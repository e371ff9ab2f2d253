/* Plain-C client of the C ABI (include/wfpt_amd.h): what a non-Python host
 * (cgo, JNI, N-API, a C program) does. Built and run by tests/test_c_abi.py.
 * Prints: resident total, host-array total, sum of pdf_array log densities,
 * then the status codes of deliberately bad calls. */
#include <math.h>
#include <stdio.h>

#include "wfpt_amd.h"

#define N 1000

int main(void) {
  wfpt_ctx *ctx = NULL;
  if (wfpt_open(0, &ctx) != WFPT_OK) {
    fprintf(stderr, "wfpt_open: %s\n", wfpt_last_error());
    return 2;
  }
  static double rt[N], dens[N];
  for (int i = 0; i < N; ++i) rt[i] = ((i % 3) == 0 ? -1.0 : 1.0) * (0.35 + 0.002 * i);
  wfpt_ds *ds = NULL;
  if (wfpt_dataset_create(ctx, rt, N, NULL, 0, &ds) != WFPT_OK) {
    fprintf(stderr, "dataset: %s\n", wfpt_last_error());
    return 3;
  }
  const wfpt_params p = {.v = 0.5, .sv = 0.1, .a = 2.0, .z = 0.5, .sz = 0.1, .t = 0.3, .st = 0.1,
                         .p_outlier = 0.05};
  const wfpt_knobs k = {.err = 1e-4, .n_st = 2, .n_sz = 2, .use_adaptive = 1, .simps_err = 1e-3,
                        .w_outlier = 0.1};
  double lp_res = 0, lp_host = 0, lp_arr = 0;
  if (wfpt_wiener_like(ctx, ds, &p, &k, &lp_res) != WFPT_OK ||
      wfpt_wiener_like_host(ctx, rt, N, &p, &k, &lp_host) != WFPT_OK ||
      wfpt_pdf_array(ctx, rt, N, &p, &k, 1, dens) != WFPT_OK) {
    fprintf(stderr, "likelihood: %s\n", wfpt_last_error());
    return 4;
  }
  for (int i = 0; i < N; ++i) lp_arr += dens[i];
  printf("%.17g %.17g %.17g\n", lp_res, lp_host, lp_arr);
  /* error conventions: bad arguments are status codes, never numbers */
  double out = 0;
  const int rc_null = wfpt_wiener_like(ctx, NULL, &p, &k, &out);
  wfpt_params bad = p;
  bad.a = -1.0;
  static double cdf[N];
  const int rc_cdf = wfpt_dmat_cdf_array(ctx, rt, N, &bad, 0.1, cdf);
  wfpt_params po = p;
  po.p_outlier = 1.5;
  double lp_po = 0;
  const int rc_po = wfpt_wiener_like(ctx, ds, &po, &k, &lp_po);
  printf("%d %d %d %d\n", rc_null, rc_cdf, rc_po, isinf(lp_po) && lp_po < 0);
  wfpt_dataset_destroy(ds);
  wfpt_close(ctx);
  return 0;
}
