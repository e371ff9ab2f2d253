// wfpt_internal.h — launcher interface between the C ABI (wfpt_capi.cpp) and
// the kernels (wfpt_kernels.hip). Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/wfpt_amd.h"

namespace wfpt {
struct Params;
struct Knobs;

int stack_kind(const Knobs& K);
int64_t blocks_for(int64_t n);
// out_kind: 0 = block {sum, zeros}; 1 = per-trial density (logp => log); 2 = per-trial log p.
// Adaptive modes run a level-0 fast pass then a slow pass over the deferred
// trials: wl must hold blocks_for(n)*256 bytes and wl_n blocks_for(n) ints;
// OUT_SUM then leaves partials_for(n) block partials in out/zeros.
// fast_done (optional) is recorded right after the level-0 fast kernel.
void launch_trials(int out_kind, const double* x, int64_t n, const Params& P, const Knobs& K,
                   double* out, int* zeros, unsigned long long* evals, int* status, int logp,
                   unsigned char* wl, int* wl_n, hipStream_t s,
                   hipEvent_t fast_done = nullptr);
int64_t partials_for(int64_t n, const Params& P, const Knobs& K);
void final_partials(int64_t n, const Params& P, const Knobs& K, int64_t* off, int64_t* cnt);
void launch_slow_pass(const double* x, int64_t n, const Params& P, const Knobs& K, double* part,
                      int* zeros, int* status, unsigned char* wl, int* wl_n, hipStream_t s);
// Status bit the level-0 pass of a sum sets when it deferred trials (besides
// the error bits 1 = Simpson depth, 2 = evaluation budget).
constexpr int kStatusDeferred = 4;
// The level-0 pass alone (adaptive modes; false, nothing launched, otherwise):
// per-64-trial partials in part[0, ceil(n/64)) + worklists, and
// kStatusDeferred in *status if any trial still needs the slow pass.
bool launch_fast_pass(const double* x, int64_t n, const Params& P, const Knobs& K, double* part,
                      int* zeros, int* status, unsigned char* wl, int* wl_n, hipStream_t s,
                      hipEvent_t fast_done);
// res[0..2] (device) -> out[0..2] (mapped host), then out[3] = seq.
void launch_publish(const double* res, double* out, unsigned long long seq, hipStream_t s);
// out[0..2] = {sum, #zero trials, status flags & keep}, then out[3] = seq (as
// a 64-bit word) once they are visible; resets *status to 0.
void launch_finalize(const double* part, const int* zeros, int64_t nb, int* status, double* out,
                     unsigned long long seq, hipStream_t s, int keep = -1);
// mode: the integration family shared by every node (kDirect..kAdaptTZ: the
// two-pass fast path; d_idx / d_par hold up to n deferred trials, *n_defer
// must be 0 on the stream), or -1 (mixed / fixed
// Simpson: one generic per-trial kernel with a per-lane mode).
void launch_nodes(const double* x, const int32_t* node, int64_t n, const Params* P,
                  const Knobs& K, int mode, double* lp, int64_t* d_idx, Params* d_par,
                  int* n_defer, unsigned long long* evals, int* status, hipStream_t s);
// res (device, n_nodes) per-node sums; then out (mapped host): [0, n_nodes)
// the sums, [n_nodes] status flags, [n_nodes + 1] the 64-bit completion word.
void launch_segment_sum(const double* lp, const int64_t* off, int32_t n_nodes, double* res,
                        double* out, int* status, unsigned long long seq, hipStream_t s);
void launch_multi(const double* x, int64_t n, const double* const* arr, const double* scal,
                  const Knobs& K, double p_outlier, double* part, int* zeros, int* status,
                  hipStream_t s);
// cdfdif_kernels.hip: dmat_cdf_array over device x[n]; par = the wrapper's
// transformed (a, Ter, eta, z, sZ, st, nu) (cdfdif_wrapper.pyx:36-42).
// defer: n ints of workspace, n_defer: one device int.
void launch_dmat_cdf(const double* x, int64_t n, const double par[7], double p_outlier,
                     double w_outlier, double* out, int* defer, int* n_defer, hipStream_t s);
}  // namespace wfpt
