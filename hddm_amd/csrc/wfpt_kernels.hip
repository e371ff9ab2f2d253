// wfpt_kernels.hip — gfx950 kernels of the WFPT likelihood engine.
//
//   trial_kernel<MODE, STK, COUNT, OUT>   one trial per lane: full_pdf, the
//       outlier mixture (wfpt.pyx:69-70) and either the per-block
//       {sum log p, #zeros} (OUT_SUM, fused wave/LDS tree reduction) or the
//       per-trial density / log density (OUT_ARRAY, pdf_array), or per-trial
//       log p for the segmented per-node reduction (OUT_LOGP).
//   finalize_kernel       deterministic second pass over block partials.
//   segment_sum_kernel    per-node sums (one wave per node).
//   multi_kernel          per-trial parameters (wiener_like_multi).
// No float atomics on any likelihood value: every sum is a fixed-order tree.
#include "wfpt_device.hpp"
#include "wfpt_internal.h"

#pragma clang fp contract(off)

namespace wfpt {

constexpr int kBlock = 256;
// Threads per block of the level-0 fast kernel (barrier-free, one chunk of 64
// trials per wave): the block is only the hardware's dispatch unit.
#ifndef WFPT_FAST_BLOCK
#define WFPT_FAST_BLOCK 256
#endif
constexpr int kFastBlock = WFPT_FAST_BLOCK;
static inline int64_t fast_blocks(int64_t n) { return (n + kFastBlock - 1) / kFastBlock; }

// Minimum waves per SIMD requested for the level-0 fast kernels (0 = let the
// compiler choose): WFPT_FAST_WAVES for the 1-D / direct modes,
// WFPT_FAST_WAVES_TZ for the 2-D mode (5-wide z evaluation: 199 VGPRs, 2 waves
// spill-free; 3 waves spill 36). Chosen by tools/ab_variants.py on MI355X.
#ifndef WFPT_FAST_WAVES
#define WFPT_FAST_WAVES 3
#endif
#ifndef WFPT_FAST_WAVES_TZ
#define WFPT_FAST_WAVES_TZ 2
#endif
template <int MODE>
struct FastWaves {
  static constexpr int value = MODE == kAdaptTZ ? WFPT_FAST_WAVES_TZ : WFPT_FAST_WAVES;
};
// Minimum waves per SIMD of the general (recursive) kernels (slow pass, generic
// per-trial / per-node / per-trial-parameter kernels):
// left free their register use reaches 255 VGPRs + 2 AGPRs, one past the
// 2-wave budget (1 wave / SIMD); 2 keeps them at 256 with a little more scratch.
#ifndef WFPT_SLOW_WAVES
#define WFPT_SLOW_WAVES 2
#endif
// Blocks (one wave each) of the deferred-trial pass: one per SIMD slot it can
// occupy (256 CUs x 4 SIMDs x WFPT_SLOW_WAVES).
#ifndef WFPT_SLOW_GRID
#define WFPT_SLOW_GRID 2048
#endif

enum Out : int { OUT_SUM = 0, OUT_ARRAY = 1, OUT_LOGP = 2 };

__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ inline long long wave_sum_ll(long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block (256 lanes = 4 waves) reduction of (sum, zeros, evals); lane 0 returns.
template <bool COUNT>
__device__ inline void block_reduce(double& s, int& zeros, long long& ne) {
  __shared__ double ss[kBlock / 64];
  __shared__ int sz[kBlock / 64];
  __shared__ long long sn[kBlock / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  s = wave_sum(s);
  const unsigned long long zb = __ballot(zeros != 0);
  if (COUNT) ne = wave_sum_ll(ne);
  if (lane == 0) {
    ss[w] = s;
    sz[w] = __popcll(zb);
    if (COUNT) sn[w] = ne;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    s = ((ss[0] + ss[1]) + (ss[2] + ss[3]));
    zeros = sz[0] + sz[1] + sz[2] + sz[3];
    if (COUNT) ne = sn[0] + sn[1] + sn[2] + sn[3];
  }
}

struct TrialArgs {
  const double* x;
  int64_t n;
  Params P;
  Knobs K;
  double wp_outlier;      // w_outlier * p_outlier
  double* out;            // OUT_SUM: block sums; OUT_ARRAY/OUT_LOGP: per trial
  int* zeros;             // OUT_SUM: block zero counts
  unsigned long long* evals;
  int* status;            // set to 1 if a trial overflowed the Simpson stack
  int logp;               // OUT_ARRAY: return log density
};

template <int STK>
struct StackOf;
template <>
struct StackOf<0> {
  using type = RegStack<2>;
};
template <>
struct StackOf<1> {
  using type = RegStack<4>;
};
template <>
struct StackOf<2> {
  using type = MemStack<WFPT_MAX_DEPTH>;
};

template <int MODE, int STK, bool COUNT, int OUT>
__global__ __launch_bounds__(kBlock, WFPT_SLOW_WAVES) void trial_kernel(TrialArgs A) {
  using Stack = typename StackOf<STK>::type;
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  long long ne = 0;
  double lp = 0.0;
  int zero = 0, ovf = 0;
  if (i < A.n) {
    double p = full_pdf<MODE, Stack, COUNT>(A.x[i], A.P, A.K, ne, ovf);
    if (ovf) atomicOr(A.status, ovf);
    if (OUT == OUT_ARRAY) {
      p = p * (1 - A.P.p_outlier) + (A.K.w_outlier * A.P.p_outlier);  // wfpt.pyx:44
      A.out[i] = A.logp ? log(p) : p;
    } else {
      p = p * (1 - A.P.p_outlier) + A.wp_outlier;  // wfpt.pyx:70
      if (p == 0) zero = 1;
      else lp = log(p);
      if (OUT == OUT_LOGP) A.out[i] = zero ? -INFINITY : lp;
    }
  }
  if (OUT == OUT_SUM || COUNT) {
    block_reduce<COUNT>(lp, zero, ne);
    if (threadIdx.x == 0) {
      if (OUT == OUT_SUM) {
        A.out[blockIdx.x] = lp;
        A.zeros[blockIdx.x] = zero;
      }
      if (COUNT) atomicAdd(A.evals, (unsigned long long)ne);
    }
  }
}

// Level-0 fast pass (MODE in kDirect..kAdaptTZ). Trials whose root Simpson
// tests all pass are finished here; the others are compacted per WAVE into
// `wl` (lane ids, one byte each, 64 slots per wave) and counted in
// `wl_n[wave]` for slow_kernel. Barrier-free: every wave writes its own
// partial sum / zero count (A.out[wave], A.zeros[wave]) and worklist, so a
// wave that finishes early never waits for its block.
//
// fast_chunk: one 64-trial chunk of the level-0 pass for the calling wave: trial
// i = c*64 + lane with RT xi (ignored when i >= n). Writes the chunk's
// worklist, partial sum and zero count; returns the wave-reduced partial (lp,
// zs) and the deferred count.
template <int MODE, bool COUNT, int OUT>
__device__ __forceinline__ void fast_chunk(const TrialArgs& A, unsigned char* wl, int* wl_n,
                                           int64_t c, int lane, double xi, double& lp_out,
                                           int& zs_out, int& nslow_out) {
  const int64_t i = c * 64 + lane;
  const int64_t wave = c;
  long long ne = 0;
  double lp = 0.0;
  int zero = 0;
  bool slow = false;
  if (i < A.n) {
    int valid = 0;
    double p = fast_pdf<MODE>(xi, A.P, A.K, slow, valid);
    if (!slow) {
      if (COUNT && valid) ne = fast_evals(MODE);
      if (OUT == OUT_ARRAY) {
        p = p * (1 - A.P.p_outlier) + (A.K.w_outlier * A.P.p_outlier);  // wfpt.pyx:44
        A.out[i] = A.logp ? log(p) : p;
      } else {
        p = p * (1 - A.P.p_outlier) + A.wp_outlier;  // wfpt.pyx:70
        if (p == 0) zero = 1;
        else lp = log(p);
        if (OUT == OUT_LOGP) A.out[i] = zero ? -INFINITY : lp;
      }
    }
  }
  int nslow = 0;
  if (MODE != kDirect) {
    const unsigned long long b = __ballot(slow);
    if (slow) wl[wave * 64 + __popcll(b & ((1ull << lane) - 1ull))] = (unsigned char)lane;
    nslow = __popcll(b);
    if (lane == 0) wl_n[wave] = nslow;
    // tells the host this call deferred trials (the fast-only call sequence
    // of wfpt_capi.cpp relies on it)
    if (OUT == OUT_SUM && lane == 0 && nslow) atomicOr(A.status, kStatusDeferred);
  }
  int zs = 0;
  if (OUT == OUT_SUM || COUNT) {
    lp = wave_sum(lp);
    zs = __popcll(__ballot(zero != 0));
    if (COUNT) ne = wave_sum_ll(ne);
    if (lane == 0) {
      if (OUT == OUT_SUM) {
        A.out[wave] = lp;
        A.zeros[wave] = zs;
      }
      if (COUNT) atomicAdd(A.evals, (unsigned long long)ne);
    }
  }
  lp_out = lp;
  zs_out = zs;
  nslow_out = nslow;
}

template <int MODE, bool COUNT, int OUT>
__global__ __launch_bounds__(kFastBlock, FastWaves<MODE>::value > 0 ? FastWaves<MODE>::value : 1)
void fast_kernel(TrialArgs A, unsigned char* wl, int* wl_n) {
  // ascending |rt| in dispatch order: the costlier short-RT chunks start first
  // (dispatching largest |rt| first measured 3% slower)
  const int64_t i = (int64_t)blockIdx.x * kFastBlock + threadIdx.x;
  const int lane = threadIdx.x & 63;
  double lp;
  int zs, nslow;
  fast_chunk<MODE, COUNT, OUT>(A, wl, wl_n, i >> 6, lane, i < A.n ? A.x[i] : 0.0, lp, zs, nslow);
}

// General pass over the trials the fast pass deferred. The fast pass leaves
// one worklist and one partial per 64 trials (nl lists); this
// one-wave-per-block kernel runs on a bounded grid of kSlowGrid blocks — one
// wave per SIMD, which is all its register footprint (the general recursion,
// ~255 VGPRs) lets reside anyway — and block g walks lists g, g + G, ...,
// running the wl_n[b] deferred trials of list b on its first lanes (full
// adaptive quadrature, reference recursion order). An empty list costs one
// load, so a workload with (almost) nothing deferred pays one short
// launch. For OUT_SUM the block also folds the fast partials of its lists
// into its own (lane j takes list g + jG of each 64-list chunk) and writes
// A.out[nb + g] / A.zeros[nb + g]: finalize then sums G values. Fixed order
// for a given n.
constexpr int64_t kSlowGrid = WFPT_SLOW_GRID;

template <int MODE, int STK, bool COUNT, int OUT>
__global__ __launch_bounds__(64, WFPT_SLOW_WAVES) void slow_kernel(TrialArgs A, const unsigned char* wl,
                                                  const int* wl_n, int64_t nl, int64_t nb) {
  using Stack = typename StackOf<STK>::type;
  long long ne = 0;
  double lp = 0.0;
  long long zc = 0;
  int ovf = 0;
  const int lane = threadIdx.x;
  const int64_t G = gridDim.x;
  // chunks of 64 lists (g + j G, j = 0..63): one parallel load of their
  // counts and fast partials, then only the non-empty lists are walked
  for (int64_t b0 = blockIdx.x; b0 < nl; b0 += 64 * G) {
    const int64_t myb = b0 + lane * G;
    int mycnt = 0;
    if (myb < nl) {
      mycnt = wl_n[myb];
      if (OUT == OUT_SUM) {
        lp += A.out[myb];
        zc += A.zeros[myb];
      }
    }
    // one list at a time on its first lanes: the trials of a list are
    // neighbours in |rt| and refine alike (packing the 64 lists' trials into
    // full waves mixes distant |rt| and measured 3% slower on the stress set)
    unsigned long long work = __ballot(mycnt > 0);
    while (work) {
      const int j = __ffsll((long long)work) - 1;
      work &= work - 1;
      const int cnt = __shfl(mycnt, j, 64);
      const int64_t b = b0 + (int64_t)j * G;
      if (lane >= cnt) continue;
      const int64_t i = b * 64 + wl[b * 64 + lane];
      double p = full_pdf<MODE, Stack, COUNT>(A.x[i], A.P, A.K, ne, ovf);
      if (OUT == OUT_ARRAY) {
        p = p * (1 - A.P.p_outlier) + (A.K.w_outlier * A.P.p_outlier);
        A.out[i] = A.logp ? log(p) : p;
      } else {
        p = p * (1 - A.P.p_outlier) + A.wp_outlier;
        const bool z = p == 0;
        double l = 0.0;
        if (z) zc += 1;
        else l = log(p);
        lp += l;
        if (OUT == OUT_LOGP) A.out[i] = z ? -INFINITY : l;
      }
    }
  }
  if (ovf) atomicOr(A.status, ovf);
  if (OUT == OUT_SUM || COUNT) {
    lp = wave_sum(lp);
    zc = wave_sum_ll(zc);
    if (COUNT) ne = wave_sum_ll(ne);
    if (threadIdx.x == 0) {
      if (OUT == OUT_SUM) {
        A.out[nb + blockIdx.x] = lp;
        A.zeros[nb + blockIdx.x] = (int)zc;
      }
      if (COUNT) atomicAdd(A.evals, (unsigned long long)ne);
    }
  }
}

__host__ __device__ inline int64_t slow_grid(int64_t nl) { return nl < kSlowGrid ? nl : kSlowGrid; }

// out[0] = sum of partials, out[1] = number of zero trials, out[2] = the
// call's status flags (as doubles); the device status word is reset to 0 for
// the next call. `out` may be mapped pinned host memory: the 24-byte result
// then reaches the host with the kernel, without a copy. Fixed summation
// order for a given nb (4 independent accumulators per thread keep 4 loads
// in flight).
__global__ __launch_bounds__(1024) void finalize_kernel(const double* part, const int* zeros,
                                                        int64_t nb, int* status, double* out,
                                                        unsigned long long seq, int keep) {
  __shared__ double ss[16];
  __shared__ long long sz[16];
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  long long z = 0;
  int64_t b = threadIdx.x;
  for (; b + 3 * 1024 < nb; b += 4 * 1024) {
    s0 += part[b];
    s1 += part[b + 1024];
    s2 += part[b + 2048];
    s3 += part[b + 3072];
    z += (long long)zeros[b] + zeros[b + 1024] + zeros[b + 2048] + zeros[b + 3072];
  }
  for (; b < nb; b += 1024) {
    s0 += part[b];
    z += zeros[b];
  }
  double s = (s0 + s1) + (s2 + s3);
  s = wave_sum(s);
  z = wave_sum_ll(z);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    ss[w] = s;
    sz[w] = z;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    long long zz = 0;
    for (int k = 0; k < 16; ++k) {
      t += ss[k];
      zz += sz[k];
    }
    const int st = *status;
    *status = 0;
    out[0] = t;
    out[1] = (double)zz;
    out[2] = (double)(st & keep);
    __threadfence_system();
    // completion word, written after the results are visible: the host may
    // poll it instead of waiting on the stream
    reinterpret_cast<volatile unsigned long long*>(out)[3] = seq;
    __threadfence_system();
  }
}

// Copies a device result {sum, zeros, status} (after the RCCL all-reduce) to
// the mapped host slot, then writes the completion word (as finalize_kernel).
__global__ __launch_bounds__(64) void publish_kernel(const double* res, double* out,
                                                     unsigned long long seq) {
  if (threadIdx.x == 0) {
    out[0] = res[0];
    out[1] = res[1];
    out[2] = res[2];
    __threadfence_system();
    reinterpret_cast<volatile unsigned long long*>(out)[3] = seq;
    __threadfence_system();
  }
}

void launch_publish(const double* res, double* out, unsigned long long seq, hipStream_t s) {
  hipLaunchKernelGGL(publish_kernel, dim3(1), dim3(64), 0, s, res, out, seq);
}

// One wave per node: sums per-trial log p of [off[j], off[j+1]) in fixed order.
// res[j] = -inf if the node holds a zero-density trial (wfpt.pyx:71-72).
__global__ __launch_bounds__(256) void segment_sum_kernel(const double* lp, const int64_t* off,
                                                          int32_t n_nodes, double* res) {
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (j >= n_nodes) return;
  const int64_t lo = off[j], hi = off[j + 1];
  double s = 0.0;
  int zero = 0;
  for (int64_t i = lo + lane; i < hi; i += 64) {
    const double v = lp[i];
    if (v == -INFINITY) zero = 1;
    else s += v;
  }
  s = wave_sum(s);
  const bool anyz = __ballot(zero != 0) != 0ull;
  if (lane == 0) res[j] = anyz ? -INFINITY : s;
}

// One block: copies the per-node sums to the mapped host slot, then the
// call's status flags (out[n]) and, once all of it is visible, the 64-bit
// completion word (out[n + 1]); resets the device status word.
__global__ __launch_bounds__(256) void publish_nodes_kernel(const double* res, int32_t n,
                                                            int* status, double* out,
                                                            unsigned long long seq) {
  for (int j = threadIdx.x; j < n; j += 256) out[j] = res[j];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    out[n] = (double)atomicExch(status, 0);
    __threadfence_system();
    reinterpret_cast<volatile unsigned long long*>(out + n + 1)[0] = seq;
    __threadfence_system();
  }
}

// Per-node parameters (wfpt_wiener_like_nodes): trials of node j use P[j].
// The dataset is grouped by node, so a 256-trial block spans a short run of
// node ids; their parameter rows (P is the mapped pinned table the host
// filled for this call) are staged once per block in LDS and every trial
// reads its row there. Blocks spanning more than kStageRows ids (empty nodes
// between) read the table directly.
constexpr int kStageRows = 256;

template <int STK, bool COUNT>
__global__ __launch_bounds__(kBlock, WFPT_SLOW_WAVES) void node_kernel(const double* x, const int32_t* node,
                                                      int64_t n, const Params* P, Knobs K,
                                                      double* lp, unsigned long long* evals,
                                                      int* status) {
  using Stack = typename StackOf<STK>::type;
  __shared__ Params rows[kStageRows];
  const int64_t i0 = (int64_t)blockIdx.x * kBlock;
  const int64_t i = i0 + threadIdx.x;
  const int first = node[i0];
  const int last = node[(i0 + kBlock - 1 < n) ? i0 + kBlock - 1 : n - 1];
  const int span = last - first + 1;
  const bool staged = span <= kStageRows;
  if (staged) {
    const double* src = reinterpret_cast<const double*>(P + first);
    double* dst = reinterpret_cast<double*>(rows);
    for (int k = threadIdx.x; k < span * 8; k += kBlock) dst[k] = src[k];
  }
  __syncthreads();
  long long ne = 0;
  double out = 0.0;
  int zero = 0, ovf = 0;
  if (i < n) {
    const int nj = node[i];
    const Params Q = staged ? rows[nj - first] : P[nj];
    double p = full_pdf<kRuntime, Stack, COUNT>(x[i], Q, K, ne, ovf);
    if (ovf) atomicOr(status, ovf);
    const bool ok = (Q.p_outlier >= 0) & (Q.p_outlier <= 1);
    p = p * (1 - Q.p_outlier) + K.w_outlier * Q.p_outlier;
    if (!ok || p == 0) zero = 1;
    else out = log(p);
    lp[i] = zero ? -INFINITY : out;
  }
  if (COUNT) {
    double d = 0.0;
    block_reduce<COUNT>(d, zero, ne);
    if (threadIdx.x == 0) atomicAdd(evals, (unsigned long long)ne);
  }
}

// Two-pass per-node path (used when every node's parameters select the same
// integration family, the usual HDDM case: sv/sz/st are group-level):
// node_fast_kernel is fast_kernel with the node's parameter row (staged in
// LDS as in node_kernel) and per-trial log p out; a trial that needs
// refinement is appended — index and parameter row — to a dense deferred
// list (wave-aggregated atomic; the order does not matter, outputs are per
// trial), which node_slow_kernel runs 64 trials per wave.
__device__ inline double node_logp(double p, const Params& Q, const Knobs& K) {
  const bool ok = (Q.p_outlier >= 0) & (Q.p_outlier <= 1);  // wfpt.pyx:63-64 per node
  p = p * (1 - Q.p_outlier) + K.w_outlier * Q.p_outlier;
  return (!ok || p == 0) ? -INFINITY : log(p);
}

template <int MODE, bool COUNT>
__global__ __launch_bounds__(kBlock, FastWaves<MODE>::value > 0 ? FastWaves<MODE>::value : 1)
void node_fast_kernel(const double* x, const int32_t* node, int64_t n, const Params* P, Knobs K,
                      double* lp, int64_t* d_idx, Params* d_par, int* n_defer,
                      unsigned long long* evals) {
  __shared__ Params rows[kStageRows];
  const int64_t i0 = (int64_t)blockIdx.x * kBlock;
  const int64_t i = i0 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int first = node[i0];
  const int last = node[(i0 + kBlock - 1 < n) ? i0 + kBlock - 1 : n - 1];
  const int span = last - first + 1;
  const bool staged = span <= kStageRows;
  if (staged) {
    const double* src = reinterpret_cast<const double*>(P + first);
    double* dst = reinterpret_cast<double*>(rows);
    for (int k = threadIdx.x; k < span * 8; k += kBlock) dst[k] = src[k];
  }
  __syncthreads();
  long long ne = 0;
  bool slow = false;
  Params Q;
  if (i < n) {
    const int nj = node[i];
    Q = staged ? rows[nj - first] : P[nj];
    int valid = 0;
    const double p = fast_pdf<MODE>(x[i], Q, K, slow, valid);
    if (!slow) {
      if (COUNT && valid) ne = fast_evals(MODE);
      lp[i] = node_logp(p, Q, K);
    }
  }
  if (MODE != kDirect) {
    const unsigned long long b = __ballot(slow);
    if (b) {
      int base = 0;
      if (lane == 0) base = atomicAdd(n_defer, __popcll(b));
      base = __shfl(base, 0, 64);
      if (slow) {
        const int k = base + __popcll(b & ((1ull << lane) - 1ull));
        d_idx[k] = i;
        d_par[k] = Q;
      }
    }
  }
  if (COUNT) {
    ne = wave_sum_ll(ne);
    if (lane == 0) atomicAdd(evals, (unsigned long long)ne);
  }
}

template <int MODE, int STK, bool COUNT>
__global__ __launch_bounds__(64, WFPT_SLOW_WAVES) void node_slow_kernel(const double* x, Knobs K, double* lp,
                                                       const int64_t* d_idx, const Params* d_par,
                                                       const int* n_defer,
                                                       unsigned long long* evals, int* status) {
  using Stack = typename StackOf<STK>::type;
  const int nd = *n_defer;
  long long ne = 0;
  int ovf = 0;
  for (int64_t k = (int64_t)blockIdx.x * 64 + threadIdx.x; k < nd; k += (int64_t)gridDim.x * 64) {
    const int64_t i = d_idx[k];
    const Params Q = d_par[k];
    const double p = full_pdf<MODE, Stack, COUNT>(x[i], Q, K, ne, ovf);
    lp[i] = node_logp(p, Q, K);
  }
  if (ovf) atomicOr(status, ovf);
  if (COUNT) {
    ne = wave_sum_ll(ne);
    if (threadIdx.x == 0) atomicAdd(evals, (unsigned long long)ne);
  }
}

// wiener_like_multi (wfpt.pyx:244-274): per-trial parameters, ±999 = missing.
template <int STK>
__global__ __launch_bounds__(kBlock, WFPT_SLOW_WAVES) void multi_kernel(const double* x, int64_t n,
                                                       const double* const* arr,
                                                       const double* scal, Knobs K,
                                                       double p_outlier, double* out,
                                                       int* zeros, int* status) {
  using Stack = typename StackOf<STK>::type;
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double lp = 0.0;
  int zero = 0, ovf = 0;
  long long ne = 0;
  if (i < n) {
    double q[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) q[j] = arr[j] ? arr[j][i] : scal[j];
    Params Q;
    Q.v = q[0];
    Q.sv = q[1];
    Q.a = q[2];
    Q.z = q[3];
    Q.sz = q[4];
    Q.t = q[5];
    Q.st = q[6];
    Q.p_outlier = p_outlier;
    const double xi = x[i];
    double p;
    if (fabs(xi) != 999.) {
      p = full_pdf<kRuntime, Stack, false>(xi, Q, K, ne, ovf);
      if (ovf) atomicOr(status, ovf);
      p = p * (1 - p_outlier) + (K.w_outlier * p_outlier);
    } else if (xi == 999.) {
      p = prob_ub(Q.v, Q.a, Q.z);
    } else {
      p = 1 - prob_ub(Q.v, Q.a, Q.z);
    }
    // the reference has no early exit here: log(0) = -inf enters the sum
    lp = log(p);
  }
  block_reduce<false>(lp, zero, ne);
  if (threadIdx.x == 0) {
    out[blockIdx.x] = lp;
    zeros[blockIdx.x] = 0;
  }
}

// ---------------------------------------------------------------------------
// launchers

template <int MODE, int STK, bool COUNT, int OUT>
static void launch_generic(const TrialArgs& A, int64_t nb, hipStream_t s) {
  hipLaunchKernelGGL((trial_kernel<MODE, STK, COUNT, OUT>), dim3(nb), dim3(kBlock), 0, s, A);
}

// fast pass + (for adaptive modes) the slow pass on the deferred trials
template <int MODE, int STK, bool COUNT, int OUT>
static void launch_slow(const TrialArgs& A, int64_t nb, const unsigned char* wl, const int* wl_n,
                        hipStream_t s) {
  hipLaunchKernelGGL((slow_kernel<MODE, STK, COUNT, OUT>), dim3(slow_grid(nb)), dim3(64), 0, s, A,
                     wl, wl_n, nb, nb);
}

template <int MODE, bool COUNT, int OUT>
static void launch_two_pass(int stk, const TrialArgs& A, int64_t n, unsigned char* wl,
                            int* wl_n, hipStream_t s, hipEvent_t fast_done) {
  // both fast kernels leave one partial / worklist per 64 trials
  constexpr int TPB = 64;
  const int64_t nb = (n + TPB - 1) / TPB;
  hipLaunchKernelGGL((fast_kernel<MODE, COUNT, OUT>), dim3(fast_blocks(n)), dim3(kFastBlock), 0,
                     s, A, wl, wl_n);
  if (fast_done) (void)hipEventRecord(fast_done, s);
  if (MODE == kDirect) return;
  const int64_t g = slow_grid(nb);
  if (stk == 0)
    hipLaunchKernelGGL((slow_kernel<MODE, 0, COUNT, OUT>), dim3(g), dim3(TPB), 0, s, A, wl, wl_n,
                       nb, nb);
  else if (stk == 1)
    hipLaunchKernelGGL((slow_kernel<MODE, 1, COUNT, OUT>), dim3(g), dim3(TPB), 0, s, A, wl, wl_n,
                       nb, nb);
  else
    hipLaunchKernelGGL((slow_kernel<MODE, 2, COUNT, OUT>), dim3(g), dim3(TPB), 0, s, A, wl, wl_n,
                       nb, nb);
}

template <bool COUNT, int OUT>
static void launch_out(int mode, int stk, const TrialArgs& A, int64_t nb, unsigned char* wl,
                       int* wl_n, hipStream_t s, hipEvent_t ev) {
  switch (mode) {
    case kDirect: launch_two_pass<kDirect, COUNT, OUT>(stk, A, A.n, wl, wl_n, s, ev); break;
    case kAdaptT: launch_two_pass<kAdaptT, COUNT, OUT>(stk, A, A.n, wl, wl_n, s, ev); break;
    case kAdaptZ: launch_two_pass<kAdaptZ, COUNT, OUT>(stk, A, A.n, wl, wl_n, s, ev); break;
    case kAdaptTZ: launch_two_pass<kAdaptTZ, COUNT, OUT>(stk, A, A.n, wl, wl_n, s, ev); break;
    case kFixedT: launch_generic<kFixedT, 0, COUNT, OUT>(A, nb, s); break;
    case kFixedZ: launch_generic<kFixedZ, 0, COUNT, OUT>(A, nb, s); break;
    default: launch_generic<kFixedTZ, 0, COUNT, OUT>(A, nb, s); break;
  }
  if (ev && mode > kAdaptTZ) (void)hipEventRecord(ev, s);  // the single trial kernel
}

template <bool COUNT>
static void launch_count(int out_kind, int mode, int stk, const TrialArgs& A, int64_t nb,
                         unsigned char* wl, int* wl_n, hipStream_t s, hipEvent_t ev) {
  if (out_kind == OUT_SUM) launch_out<COUNT, OUT_SUM>(mode, stk, A, nb, wl, wl_n, s, ev);
  else if (out_kind == OUT_ARRAY) launch_out<COUNT, OUT_ARRAY>(mode, stk, A, nb, wl, wl_n, s, ev);
  else launch_out<COUNT, OUT_LOGP>(mode, stk, A, nb, wl, wl_n, s, ev);
}

// Where launch_trials(OUT_SUM) leaves the partials finalize must sum: the
// slow pass's G partials (which already fold the fast ones) for adaptive
// modes, else every fast / trial-kernel partial.
void final_partials(int64_t n, const Params& P, const Knobs& K, int64_t* off, int64_t* cnt) {
  const int mode = select_mode(P.sz, P.st, K.use_adaptive);
  const int64_t nw = (n + 63) / 64;
  if (mode == kAdaptT || mode == kAdaptZ || mode == kAdaptTZ) {
    *off = nw;
    *cnt = slow_grid(nw);
  } else {
    *off = 0;
    *cnt = (mode == kDirect) ? nw : blocks_for(n);
  }
}

// size of the partial buffers launch_trials(OUT_SUM) writes
int64_t partials_for(int64_t n, const Params& P, const Knobs& K) {
  const int mode = select_mode(P.sz, P.st, K.use_adaptive);
  const int64_t nw = (n + 63) / 64;  // fast (and slow) partials are per 64 trials
  if (mode == kAdaptT || mode == kAdaptZ || mode == kAdaptTZ) return nw + slow_grid(nw);
  if (mode == kDirect) return nw;
  return blocks_for(n);  // fixed Simpson: trial_kernel, one partial per 256-trial block
}

int stack_kind(const Knobs& K) {
  const int d = (K.n_st > K.n_sz) ? K.n_st : K.n_sz;
  return d <= 2 ? 0 : (d <= 4 ? 1 : 2);
}

int64_t blocks_for(int64_t n) { return (n + kBlock - 1) / kBlock; }

void launch_trials(int out_kind, const double* x, int64_t n, const Params& P, const Knobs& K,
                   double* out, int* zeros, unsigned long long* evals, int* status, int logp,
                   unsigned char* wl, int* wl_n, hipStream_t s, hipEvent_t fast_done) {
  TrialArgs A;
  A.x = x;
  A.n = n;
  A.P = P;
  A.K = K;
  A.wp_outlier = K.w_outlier * P.p_outlier;
  A.out = out;
  A.zeros = zeros;
  A.evals = evals;
  A.status = status;
  A.logp = logp;
  const int mode = select_mode(P.sz, P.st, K.use_adaptive);
  const int64_t nb = blocks_for(n);
  if (nb == 0) return;
  if (evals) launch_count<true>(out_kind, mode, stack_kind(K), A, nb, wl, wl_n, s, fast_done);
  else launch_count<false>(out_kind, mode, stack_kind(K), A, nb, wl, wl_n, s, fast_done);
}

static TrialArgs sum_args(const double* x, int64_t n, const Params& P, const Knobs& K,
                          double* part, int* zeros, int* status) {
  TrialArgs A;
  A.x = x;
  A.n = n;
  A.P = P;
  A.K = K;
  A.wp_outlier = K.w_outlier * P.p_outlier;
  A.out = part;
  A.zeros = zeros;
  A.evals = nullptr;
  A.status = status;
  A.logp = 0;
  return A;
}

bool launch_fast_pass(const double* x, int64_t n, const Params& P, const Knobs& K, double* part,
                      int* zeros, int* status, unsigned char* wl, int* wl_n, hipStream_t s,
                      hipEvent_t fast_done) {
  const int mode = select_mode(P.sz, P.st, K.use_adaptive);
  if (n <= 0 || mode < kAdaptT || mode > kAdaptTZ) return false;
  const TrialArgs A = sum_args(x, n, P, K, part, zeros, status);
  const dim3 g(fast_blocks(n)), b(kFastBlock);
  switch (mode) {
    case kAdaptT: hipLaunchKernelGGL((fast_kernel<kAdaptT, false, OUT_SUM>), g, b, 0, s, A, wl, wl_n); break;
    case kAdaptZ: hipLaunchKernelGGL((fast_kernel<kAdaptZ, false, OUT_SUM>), g, b, 0, s, A, wl, wl_n); break;
    default: hipLaunchKernelGGL((fast_kernel<kAdaptTZ, false, OUT_SUM>), g, b, 0, s, A, wl, wl_n); break;
  }
  if (fast_done) (void)hipEventRecord(fast_done, s);
  return true;
}

void launch_slow_pass(const double* x, int64_t n, const Params& P, const Knobs& K, double* part,
                      int* zeros, int* status, unsigned char* wl, int* wl_n, hipStream_t s) {
  const TrialArgs A = sum_args(x, n, P, K, part, zeros, status);
  const int64_t nb = (n + 63) / 64;
  const int mode = select_mode(P.sz, P.st, K.use_adaptive);
  const int stk = stack_kind(K);
#define SLOW(M_)                                                        \
  do {                                                                  \
    if (stk == 0) launch_slow<M_, 0, false, OUT_SUM>(A, nb, wl, wl_n, s); \
    else if (stk == 1) launch_slow<M_, 1, false, OUT_SUM>(A, nb, wl, wl_n, s); \
    else launch_slow<M_, 2, false, OUT_SUM>(A, nb, wl, wl_n, s);        \
  } while (0)
  switch (mode) {
    case kAdaptT: SLOW(kAdaptT); break;
    case kAdaptZ: SLOW(kAdaptZ); break;
    case kAdaptTZ: SLOW(kAdaptTZ); break;
    default: break;  // kDirect never defers
  }
#undef SLOW
}

void launch_finalize(const double* part, const int* zeros, int64_t nb, int* status, double* out,
                     unsigned long long seq, hipStream_t s, int keep) {
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(1024), 0, s, part, zeros, nb, status, out,
                     seq, keep);
}

template <int MODE, bool COUNT>
static void launch_nodes_two_pass(const double* x, const int32_t* node, int64_t n,
                                  const Params* P, const Knobs& K, double* lp, int64_t* d_idx,
                                  Params* d_par, int* n_defer, unsigned long long* evals,
                                  int* status, hipStream_t s) {
  hipLaunchKernelGGL((node_fast_kernel<MODE, COUNT>), dim3(blocks_for(n)), dim3(kBlock), 0, s, x,
                     node, n, P, K, lp, d_idx, d_par, n_defer, evals);
  if (MODE == kDirect) return;
  const int64_t nl = (n + 63) / 64;
  const int64_t g = nl < 2048 ? nl : 2048;
  const int stk = stack_kind(K);
  if (stk == 0)
    hipLaunchKernelGGL((node_slow_kernel<MODE, 0, COUNT>), dim3(g), dim3(64), 0, s, x, K, lp,
                       d_idx, d_par, n_defer, evals, status);
  else if (stk == 1)
    hipLaunchKernelGGL((node_slow_kernel<MODE, 1, COUNT>), dim3(g), dim3(64), 0, s, x, K, lp,
                       d_idx, d_par, n_defer, evals, status);
  else
    hipLaunchKernelGGL((node_slow_kernel<MODE, 2, COUNT>), dim3(g), dim3(64), 0, s, x, K, lp,
                       d_idx, d_par, n_defer, evals, status);
}

template <bool COUNT>
static void launch_nodes_mode(int mode, const double* x, const int32_t* node, int64_t n,
                              const Params* P, const Knobs& K, double* lp, int64_t* d_idx,
                              Params* d_par, int* n_defer, unsigned long long* evals,
                              int* status, hipStream_t s) {
#define TWO_PASS(M_) \
  launch_nodes_two_pass<M_, COUNT>(x, node, n, P, K, lp, d_idx, d_par, n_defer, evals, status, s)
  switch (mode) {
    case kDirect: TWO_PASS(kDirect); break;
    case kAdaptT: TWO_PASS(kAdaptT); break;
    case kAdaptZ: TWO_PASS(kAdaptZ); break;
    default: TWO_PASS(kAdaptTZ); break;
  }
#undef TWO_PASS
}

void launch_nodes(const double* x, const int32_t* node, int64_t n, const Params* P,
                  const Knobs& K, int mode, double* lp, int64_t* d_idx, Params* d_par,
                  int* n_defer, unsigned long long* evals, int* status, hipStream_t s) {
  const int64_t nb = blocks_for(n);
  if (nb == 0) return;
  if (mode >= kDirect && mode <= kAdaptTZ) {
    if (evals)
      launch_nodes_mode<true>(mode, x, node, n, P, K, lp, d_idx, d_par, n_defer, evals, status, s);
    else
      launch_nodes_mode<false>(mode, x, node, n, P, K, lp, d_idx, d_par, n_defer, evals, status,
                               s);
    return;
  }
  const int stk = stack_kind(K);
#define NODE_LAUNCH(S_, C_)                                                                  \
  hipLaunchKernelGGL((node_kernel<S_, C_>), dim3(nb), dim3(kBlock), 0, s, x, node, n, P, K, \
                     lp, evals, status)
  if (evals) {
    if (stk == 0) NODE_LAUNCH(0, true);
    else if (stk == 1) NODE_LAUNCH(1, true);
    else NODE_LAUNCH(2, true);
  } else {
    if (stk == 0) NODE_LAUNCH(0, false);
    else if (stk == 1) NODE_LAUNCH(1, false);
    else NODE_LAUNCH(2, false);
  }
#undef NODE_LAUNCH
}

void launch_segment_sum(const double* lp, const int64_t* off, int32_t n_nodes, double* res,
                        double* out, int* status, unsigned long long seq, hipStream_t s) {
  if (n_nodes <= 0) return;
  hipLaunchKernelGGL(segment_sum_kernel, dim3((n_nodes + 3) / 4), dim3(256), 0, s, lp, off,
                     n_nodes, res);
  hipLaunchKernelGGL(publish_nodes_kernel, dim3(1), dim3(256), 0, s, res, n_nodes, status, out,
                     seq);
}

void launch_multi(const double* x, int64_t n, const double* const* arr, const double* scal,
                  const Knobs& K, double p_outlier, double* part, int* zeros, int* status,
                  hipStream_t s) {
  const int64_t nb = blocks_for(n);
  if (nb == 0) return;
  const int stk = stack_kind(K);
  if (stk == 0)
    hipLaunchKernelGGL((multi_kernel<0>), dim3(nb), dim3(kBlock), 0, s, x, n, arr, scal, K,
                       p_outlier, part, zeros, status);
  else if (stk == 1)
    hipLaunchKernelGGL((multi_kernel<1>), dim3(nb), dim3(kBlock), 0, s, x, n, arr, scal, K,
                       p_outlier, part, zeros, status);
  else
    hipLaunchKernelGGL((multi_kernel<2>), dim3(nb), dim3(kBlock), 0, s, x, n, arr, scal, K,
                       p_outlier, part, zeros, status);
}

}  // namespace wfpt
