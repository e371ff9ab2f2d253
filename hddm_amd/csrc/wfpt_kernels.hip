// wfpt_kernels.hip — gfx950 kernels of the WFPT likelihood engine.
//
// Adaptive / direct integration families (the HDDM case), one call:
//   fast_kernel<MODE>     level-0 pass, one 64-trial chunk per wave: trials
//                         whose root Simpson tests pass finish here (mixture,
//                         log, per-chunk partial); the others are compacted per
//                         chunk into tree records (refinement) or exact records
//   gather_kernel         level-1 task list from the per-chunk counts
//   level_kernel<MODE,L>  tree level L breadth-first over all deferred trials:
//                         one task = one interval (2 new sample points + its
//                         stop test), refined intervals push their children
//   fold_kernel<MODE>     per chunk: the deferred trials' densities (tree
//                         re-walk, exact path, per-lane fallback), mixture and
//                         log, added to the chunk's partial in lane order
//   finalize_kernel       fixed-order sum of the chunk partials -> mapped slot
// The per-chunk partial of a chunk is the same value whether or not the call
// ran the deferred kernels (a chunk without deferred trials is never touched),
// so a likelihood is bitwise reproducible across call sequences. No float
// atomics on any likelihood value.
// Fixed Simpson (use_adaptive = 0): trial_kernel. Per-node and per-trial
// parameter variants: node_*_kernel, multi_kernel.
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
// WFPT_FAST_WAVES_TZ for the 2-D mode. Chosen by tools/ab_variants.py.
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
// Minimum waves per SIMD of the general (per-lane walk) kernels.
#ifndef WFPT_SLOW_WAVES
#define WFPT_SLOW_WAVES 2
#endif
// Blocks of the grid-stride deferred-trial kernels (level and fold).
#ifndef WFPT_LEVEL_GRID
#define WFPT_LEVEL_GRID 2048
#endif
#ifndef WFPT_FOLD_GRID
#define WFPT_FOLD_GRID 16384
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
__device__ inline unsigned long long lanemask_lt(int lane) { return (1ull << lane) - 1ull; }

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
  double* out;            // OUT_SUM: chunk / block partial sums; OUT_ARRAY/OUT_LOGP: per trial
  int* zeros;             // OUT_SUM: chunk / block zero counts
  unsigned long long* evals;
  int* status;            // error flags (kFlagDepth | kFlagBudget)
  int logp;               // OUT_ARRAY: return log density
};

// Trial output of a settled density p (wfpt.pyx:44 / :70).
template <int OUT>
__device__ inline void emit(const TrialArgs& A, int64_t i, double p, double& lp, int& zero) {
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

// ---------------------------------------------------------------------------
// Level-0 pass. One wave = one chunk of 64 consecutive trials c*64 + lane.
// Deferred trials of chunk c take slots c*64 + k (k = their rank among the
// chunk's tree trials, then among its exact trials), so the deferred state is
// slot-indexed without any atomic.
template <int MODE, bool COUNT, int OUT>
__global__ __launch_bounds__(kFastBlock, FastWaves<MODE>::value > 0 ? FastWaves<MODE>::value : 1)
void fast_kernel(TrialArgs A, Work W) {
  // ascending |rt| in dispatch order: the costlier short-RT chunks start first
  const int64_t i = (int64_t)blockIdx.x * kFastBlock + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int64_t c = i >> 6;
  double p = 0.0, f[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  long long ne = 0;
  int flags = 0, oc = kFinal;
  unsigned pend = 0u;
  if (i < A.n) oc = fast_level0<MODE>(A.x[i], A.P, A.K, p, f, ne, flags, pend);
  double lp = 0.0;
  int zero = 0;
  if (i < A.n && oc == kFinal) emit<OUT>(A, i, p, lp, zero);
  // tree records first, then exact records
  const unsigned long long bt = __ballot(oc == kTree), be = __ballot(oc == kExact);
  const int nt = __popcll(bt);
  if (oc != kFinal) {
    const int k = oc == kTree ? __popcll(bt & lanemask_lt(lane))
                              : nt + __popcll(be & lanemask_lt(lane));
    const int64_t slot = c * 64 + k;
    W.wl[slot] = (unsigned char)lane;
    W.rflag[slot] = oc == kExact ? (int)kFlagExact : 0;
    if (oc == kTree) {
      W.pend[slot] = pend;
#pragma unroll
      for (int j = 0; j < 5; ++j) W.F[(int64_t)(j * (kTreeW / 4)) * W.nslots + slot] = f[j];
    }
    if (COUNT) W.rcnt[slot] = oc == kTree ? (int)ne : 0;
  }
  if (lane == 0) W.wl_n[c] = nt | (__popcll(be) << 8);
  if (OUT == OUT_SUM) {
    lp = wave_sum(lp);
    const int zs = __popcll(__ballot(zero != 0));
    if (lane == 0) {
      A.out[c] = lp;
      A.zeros[c] = zs;
    }
  }
  if (COUNT) {
    const long long nf = wave_sum_ll(oc == kFinal ? ne : 0);
    if (lane == 0) atomicAdd(A.evals, (unsigned long long)nf);
  }
}

// Work lists of the tree records after the level-0 pass: a record whose root
// test asked for refinement gets both halves of its root interval in N_1; a
// record with z integrals awaiting refinement gets its root in RT_0. One
// block compacts 1024 slots (16 chunks; 4 consecutive slots per thread) in
// slot order with one atomic per list per block.
constexpr int kGatherSlots = 1024;
__global__ __launch_bounds__(256) void gather_kernel(int64_t nw, Work W) {
  __shared__ int sc[2][256];
  __shared__ int base[2];
  const int tid = threadIdx.x;
  const int64_t s0 = (int64_t)blockIdx.x * kGatherSlots + 4 * tid;
  int kind[4];  // 0: none, 1: N_1 (2 entries), 2: RT_0 (1 entry)
  int n1 = 0, n0 = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t slot = s0 + q;
    kind[q] = 0;
    const int64_t c = slot >> 6;
    if (c < nw && (slot & 63) < (W.wl_n[c] & 255)) {
      kind[q] = W.pend[slot] ? 2 : 1;
      if (kind[q] == 1) n1 += 2;
      else n0 += 1;
    }
  }
  sc[0][tid] = n1;
  sc[1][tid] = n0;
  __syncthreads();
  // block exclusive scans (Hillis-Steele in LDS)
  for (int o = 1; o < 256; o <<= 1) {
    const int a1 = tid >= o ? sc[0][tid - o] : 0, a0 = tid >= o ? sc[1][tid - o] : 0;
    __syncthreads();
    sc[0][tid] += a1;
    sc[1][tid] += a0;
    __syncthreads();
  }
  if (tid == 255) {
    base[0] = sc[0][255] ? atomicAdd(&W.ntask[1], sc[0][255]) : 0;
    base[1] = sc[1][255] ? atomicAdd(&W.ntask[kRepairCounter], sc[1][255]) : 0;
  }
  __syncthreads();
  int at1 = base[0] + sc[0][tid] - n1, at0 = base[1] + sc[1][tid] - n0;
  uint32_t* t1 = W.tasks + node_list(1, W.nslots);
  uint32_t* r0 = W.tasks + repair_list(0, W.nslots);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t e = (uint32_t)(s0 + q) << kBfDepth;
    if (kind[q] == 1) {
      t1[at1++] = e;
      t1[at1++] = e | 1u;
    } else if (kind[q] == 2) {
      r0[at0++] = e;
    }
  }
}

// Appends the wave's flagged entries to list `dst` (length counter *cnt), one
// atomic per wave; n_each entries per flagged lane: e, e + 1, ...
__device__ inline void wave_push(bool flag, uint32_t e, int n_each, uint32_t* dst, int* cnt) {
  const int lane = threadIdx.x & 63;
  const unsigned long long b = __ballot(flag);
  if (!b) return;
  int at = 0;
  if (lane == 0) at = atomicAdd(cnt, n_each * __popcll(b));
  at = __shfl(at, 0, 64);
  if (flag) {
    at += n_each * __popcll(b & lanemask_lt(lane));
    for (int k = 0; k < n_each; ++k) dst[at + k] = e + (uint32_t)k;
  }
}

// Tree levels, breadth-first over all tree records. Node (L, m) of a record
// is an interval of its adaptive tree (m's bits: left / right turns from the
// root); its geometry and S come from the reference's recursion over the
// stored values (tree_node).
//
// level_kernel<MODE, L> (L = 1..kBfDepth): one lane per interval of N_L.
// Evaluates f at the interval's d and e (the adaptiveSimpsonsAux
// evaluations, integrate.pxi:94-104 / 161-169) and stores them. If a z
// integral there needs refinement (kAdaptTZ) the interval goes to RT_L;
// otherwise its stop test runs here and a refinement pushes both halves to
// N_{L+1} (past kBfDepth: the record continues on the per-lane walk in
// fold_kernel). A near-tie or ambiguous decision marks the record exact; its
// other tasks then stop.
template <int MODE, int L>
__device__ inline void node_test(const TrialArgs& A, const Work& W, const TreeFn<MODE>& fn,
                                 const TreeNode& nd, int64_t slot, int m, int depth, int& fl,
                                 bool& push) {
  const int64_t ns = W.nslots;
  const double* F = W.F;
  auto FV = [&](int j) -> double { return F[(int64_t)j * ns + slot]; };
  const Simp s = simp5(nd.ub - nd.lb, FV(nd.pos), FV(nd.pos + nd.W / 4), FV(nd.pos + nd.W / 2),
                       FV(nd.pos + 3 * nd.W / 4), FV(nd.pos + nd.W));
  // the root's S comes from its own points, which a repair may just have
  // replaced; deeper intervals' S (the parent's Sleft / Sright) is final
  const bool refine = simpson_refine(L == 0 ? s.S : nd.S, s.S2, nd.err, depth - L, fl);
  if (!(fl & kFlagExact) && refine) {
    if (L < kBfDepth) push = true;
    else atomicOr(&W.rflag[slot], (int)kFlagFallback);
  }
}

template <int MODE, int L, bool COUNT>
__global__ __launch_bounds__(256) void level_kernel(TrialArgs A, Work W, int depth) {
  const int nt = W.ntask[L];
  const uint32_t* tl = W.tasks + node_list(L, W.nslots);
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t base = (int64_t)blockIdx.x * 256 + (threadIdx.x & ~63); base < nt; base += stride) {
    const int64_t t = base + lane;
    bool push = false, rep = false;
    uint32_t e = 0;
    if (t < nt) {
      e = tl[t];
      const int64_t slot = e >> kBfDepth;
      const int m = (int)(e & ((1u << kBfDepth) - 1u));
      if (!(W.rflag[slot] & (kFlagExact | kFlagFallback))) {
        const int64_t i = (slot >> 6) * 64 + W.wl[slot];
        TreeFn<MODE> fn;
        fn.setup(A.x[i], A.P, A.K);
        const int64_t ns = W.nslots;
        double* F = W.F;
        auto FV = [&](int j) -> double { return F[(int64_t)j * ns + slot]; };
        const TreeNode nd = tree_node(FV, fn.lb, fn.ub, A.K.simps_err, L, m);
        const double c = (nd.ub + nd.lb) / 2.;
        const double d = (nd.lb + c) / 2., ee = (c + nd.ub) / 2.;
        int fl = 0;
        long long ne = 0;
        unsigned pm = 0u;
        // the two new points from one evaluation site (one copy of the
        // 5-wide z root in the code: fewer live registers)
#pragma unroll 1
        for (int q = 1; q < 4; q += 2) {
          const double u = q == 1 ? d : ee;
          const int pos = nd.pos + q * (nd.W / 4);
          bool r = false;
          const double y = fn(u, A.P, A.K, fl, ne, r);
          if (fl & kFlagExact) break;
          F[(int64_t)pos * ns + slot] = y;
          if (r) pm |= 1u << pos;
        }
        if (!(fl & kFlagExact)) {
          if (pm) {
            atomicOr(&W.pend[slot], pm);
            rep = true;
          } else {
            node_test<MODE, L>(A, W, fn, nd, slot, m, depth, fl, push);
          }
        }
        if (fl & kFlagExact) atomicOr(&W.rflag[slot], (int)kFlagExact);
        if (COUNT) atomicAdd(&W.rcnt[slot], (int)ne);
      }
    }
    const int mb = (int)(e & ((1u << kBfDepth) - 1u));
    const uint32_t slot_e = e & ~((1u << kBfDepth) - 1u);
    if (L < kBfDepth)
      wave_push(push, slot_e | (uint32_t)(2 * mb), 2,
                W.tasks + node_list(L < kBfDepth ? L + 1 : 1, W.nslots), &W.ntask[L + 1]);
    wave_push(rep, e, 1, W.tasks + repair_list(L, W.nslots), &W.ntask[kRepairCounter + L]);
  }
}

// repair_kernel<MODE, L> (kAdaptTZ, L = 0..kBfDepth): one lane per interval
// of RT_L: the complete z integrals at its pending points (the root's five at
// L = 0, else d and e), then its stop test as in level_kernel. The lanes all
// run refinement walks, so none idles beside another lane's walk.
template <int MODE, int L, bool COUNT>
__global__ __launch_bounds__(256) void repair_kernel(TrialArgs A, Work W, int depth) {
  const int nt = W.ntask[kRepairCounter + L];
  const uint32_t* tl = W.tasks + repair_list(L, W.nslots);
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t base = (int64_t)blockIdx.x * 256 + (threadIdx.x & ~63); base < nt; base += stride) {
    const int64_t t = base + (threadIdx.x & 63);
    bool push = false;
    uint32_t e = 0;
    if (t < nt) {
      e = tl[t];
      const int64_t slot = e >> kBfDepth;
      const int m = (int)(e & ((1u << kBfDepth) - 1u));
      if (!(W.rflag[slot] & (kFlagExact | kFlagFallback))) {
        const int64_t i = (slot >> 6) * 64 + W.wl[slot];
        TreeFn<MODE> fn;
        fn.setup(A.x[i], A.P, A.K);
        const int64_t ns = W.nslots;
        double* F = W.F;
        auto FV = [&](int j) -> double { return F[(int64_t)j * ns + slot]; };
        const TreeNode nd = tree_node(FV, fn.lb, fn.ub, A.K.simps_err, L, m);
        const unsigned pm = W.pend[slot];
        const double c = (nd.ub + nd.lb) / 2.;
        const double d = (nd.lb + c) / 2., ee = (c + nd.ub) / 2.;
        int fl = 0;
        long long ne = 0;
#pragma unroll 1
        for (int q = (L == 0 ? 0 : 1); q < (L == 0 ? 5 : 4); q += (L == 0 ? 1 : 2)) {
          const int pos = nd.pos + q * (nd.W / 4);
          if (!((pm >> pos) & 1u) || (fl & kFlagExact)) continue;
          const double u = q == 0 ? nd.lb : q == 1 ? d : q == 2 ? c : q == 3 ? ee : nd.ub;
          ne -= 5;  // the full walk evaluates the root again
          F[(int64_t)pos * ns + slot] = fn.full(u, A.P, A.K, fl, ne);
        }
        if (fl & kFlagErrors) {
          atomicOr(&W.rflag[slot], (int)kFlagFallback);
          fl &= ~kFlagErrors;
        } else if (!(fl & kFlagExact)) {
          node_test<MODE, L>(A, W, fn, nd, slot, m, depth, fl, push);
        }
        if (fl & kFlagExact) atomicOr(&W.rflag[slot], (int)kFlagExact);
        if (COUNT) atomicAdd(&W.rcnt[slot], (int)ne);
      }
    }
    const int mb = (int)(e & ((1u << kBfDepth) - 1u));
    const uint32_t slot_e = e & ~((1u << kBfDepth) - 1u);
    if (L < kBfDepth)
      wave_push(push, slot_e | (uint32_t)(2 * mb), 2,
                W.tasks + node_list(L < kBfDepth ? L + 1 : 1, W.nslots), &W.ntask[L + 1]);
  }
}

// Settles every deferred trial and folds it into its chunk: block g walks
// chunks g, g + G, ... (64 chunk counts per parallel load); a chunk's deferred
// trials run on its first lanes: tree records re-walk their completed tree,
// exact records take the exact path, deeper trees the per-lane walk. OUT_SUM:
// chunk partial += wave sum of the deferred log densities (fixed lane order).
// Last kernel of the deferred sequence: resets the level counters.
template <int MODE, bool COUNT, int OUT>
__global__ __launch_bounds__(64, WFPT_SLOW_WAVES) void fold_kernel(TrialArgs A, Work W, int64_t nw,
                                                                 int depth) {
  const int lane = threadIdx.x;
  const int64_t G = gridDim.x;
  long long ne = 0;
  int errf = 0;
  for (int64_t b0 = blockIdx.x; b0 < nw; b0 += 64 * G) {
    const int64_t myc = b0 + lane * G;
    const int mycnt = myc < nw ? W.wl_n[myc] : 0;
    unsigned long long work = __ballot(mycnt != 0);
    while (work) {
      const int j = __ffsll((long long)work) - 1;
      work &= work - 1;
      const int wn = __shfl(mycnt, j, 64);
      const int ntot = (wn & 255) + (wn >> 8);
      const int64_t c = b0 + (int64_t)j * G;
      double lp = 0.0;
      int zero = 0;
      if (lane < ntot) {
        const int64_t slot = c * 64 + lane;
        const int64_t i = c * 64 + W.wl[slot];
        const double x = A.x[i];
        const int fl = W.rflag[slot];
        long long n1 = 0;
        double p;
        if (fl & kFlagExact) {
          p = exact_pdf(x, A.P, A.K, &n1, &errf);
        } else if (fl & kFlagFallback) {
          p = fallback_pdf<MODE>(x, A.P, A.K, &n1, &errf);
        } else {
          const Trial tr = trial_setup(x, A.P);
          double lb, ub;
          tree_root<MODE>(tr, A.P, lb, ub);
          const int64_t ns = W.nslots;
          const double* F = W.F;
          p = tree_value([&](int q) -> double { return F[(int64_t)q * ns + slot]; }, lb, ub,
                         A.K.simps_err, depth);
          if (COUNT) n1 = W.rcnt[slot];
          const bool structural = (MODE == kAdaptZ) ? tr.x - A.P.t <= 0 : tr.x - lb <= 0;
          p = settle(p, x, A.P, A.K, structural, n1, errf);
        }
        ne += n1;
        emit<OUT>(A, i, p, lp, zero);
      }
      if (OUT == OUT_SUM) {
        lp = wave_sum(lp);
        const int zs = __popcll(__ballot(zero != 0));
        if (lane == 0) {
          A.out[c] = A.out[c] + lp;
          A.zeros[c] = A.zeros[c] + zs;
        }
      }
    }
  }
  if (errf & kFlagErrors) atomicOr(A.status, errf & kFlagErrors);
  if (COUNT) {
    ne = wave_sum_ll(ne);
    if (lane == 0) atomicAdd(A.evals, (unsigned long long)ne);
  }
  if (blockIdx.x == 0 && lane < 16) W.ntask[lane] = 0;
}

// ---------------------------------------------------------------------------
// Fixed composite Simpson (use_adaptive = 0): one trial per lane, full_pdf +
// settle, per-block {sum, zeros} (OUT_SUM) or per-trial outputs.
template <int MODE, bool COUNT, int OUT>
__global__ __launch_bounds__(kBlock, WFPT_SLOW_WAVES) void trial_kernel(TrialArgs A) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  long long ne = 0;
  double lp = 0.0;
  int zero = 0, flags = 0;
  if (i < A.n) {
    const double x = A.x[i];
    double p = full_pdf<MODE, RegStack<2>>(x, A.P, A.K, ne, flags);
    p = settle(p, x, A.P, A.K, !trial_setup(x, A.P).valid, ne, flags);
    if (flags & kFlagErrors) atomicOr(A.status, flags & kFlagErrors);
    emit<OUT>(A, i, p, lp, zero);
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

// out[0] = sum of nb partials, out[1] = number of zero trials, out[2] = error
// flags encoded as counts that survive a sum over ranks (depth + 2^20 budget),
// out[3] = 1 if the level-0 pass deferred trials (wl_n non-null: any chunk
// count), then the 64-bit completion word out[4] once they are visible. `out`
// may be mapped pinned host memory. Resets the device status word. Fixed
// summation order for a given nb (4 accumulators per thread keep 4 loads in
// flight).
__global__ __launch_bounds__(1024) void finalize_kernel(const double* part, const int* zeros,
                                                        int64_t nb, const int* wl_n, int64_t nw,
                                                        int* status, double* out,
                                                        unsigned long long seq) {
  __shared__ double ss[16];
  __shared__ long long sz[16];
  __shared__ int sd[16];
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
  int def = 0;
  if (wl_n)
    for (int64_t c = threadIdx.x; c < nw; c += 1024) def |= wl_n[c];
  double s = (s0 + s1) + (s2 + s3);
  s = wave_sum(s);
  z = wave_sum_ll(z);
  const bool anyd = __ballot(def != 0) != 0ull;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    ss[w] = s;
    sz[w] = z;
    sd[w] = anyd;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    long long zz = 0;
    int dd = 0;
    for (int k = 0; k < 16; ++k) {
      t += ss[k];
      zz += sz[k];
      dd |= sd[k];
    }
    const int st = *status;
    *status = 0;
    out[0] = t;
    out[1] = (double)zz;
    out[2] = (double)(st & kFlagDepth) + ((st & kFlagBudget) ? kBudgetUnit : 0.0);
    out[3] = (double)dd;
    __threadfence_system();
    // completion word, written after the results are visible: the host may
    // poll it instead of waiting on the stream
    reinterpret_cast<volatile unsigned long long*>(out)[4] = seq;
    __threadfence_system();
  }
}

// Copies a device result {sum, zeros, errors} (after the RCCL all-reduce) to
// the mapped host slot, then writes the completion word.
__global__ __launch_bounds__(64) void publish_kernel(const double* res, double* out,
                                                     unsigned long long seq) {
  if (threadIdx.x == 0) {
    out[0] = res[0];
    out[1] = res[1];
    out[2] = res[2];
    out[3] = 0.0;
    __threadfence_system();
    reinterpret_cast<volatile unsigned long long*>(out)[4] = seq;
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
// call's encoded error flags (out[n]) and, once all of it is visible, the
// 64-bit completion word (out[n + 1]); resets the device status word.
__global__ __launch_bounds__(256) void publish_nodes_kernel(const double* res, int32_t n,
                                                            int* status, double* out,
                                                            unsigned long long seq) {
  for (int j = threadIdx.x; j < n; j += 256) out[j] = res[j];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const int st = atomicExch(status, 0);
    out[n] = (double)(st & kFlagDepth) + ((st & kFlagBudget) ? kBudgetUnit : 0.0);
    __threadfence_system();
    reinterpret_cast<volatile unsigned long long*>(out + n + 1)[0] = seq;
    __threadfence_system();
  }
}

// ---------------------------------------------------------------------------
// Per-node parameters (wfpt_wiener_like_nodes): trials of node j use P[j].
// The dataset is grouped by node, so a 256-trial block spans a short run of
// node ids; their parameter rows (P is the mapped pinned table the host
// filled for this call) are staged once per block in LDS and every trial
// reads its row there. Blocks spanning more than kStageRows ids (empty nodes
// between) read the table directly.
constexpr int kStageRows = 256;

template <int STK>
struct StackOf {
  using type = typename std::conditional<
      STK == 0, RegStack<2>,
      typename std::conditional<STK == 1, RegStack<4>, MemStack<WFPT_MAX_DEPTH>>::type>::type;
};

__device__ inline double node_logp(double p, const Params& Q, const Knobs& K) {
  const bool ok = (Q.p_outlier >= 0) & (Q.p_outlier <= 1);  // wfpt.pyx:63-64 per node
  p = p * (1 - Q.p_outlier) + K.w_outlier * Q.p_outlier;
  return (!ok || p == 0) ? -INFINITY : log(p);
}

template <int STK, bool COUNT>
__global__ __launch_bounds__(kBlock, WFPT_SLOW_WAVES) void node_kernel(
    const double* x, const int32_t* node, int64_t n, const Params* P, Knobs K, double* lp,
    unsigned long long* evals, int* status) {
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
  int zero = 0, flags = 0;
  if (i < n) {
    const int nj = node[i];
    const Params Q = staged ? rows[nj - first] : P[nj];
    double p = full_pdf<kRuntime, Stack>(x[i], Q, K, ne, flags);
    p = settle(p, x[i], Q, K, !trial_setup(x[i], Q).valid, ne, flags);
    if (flags & kFlagErrors) atomicOr(status, flags & kFlagErrors);
    lp[i] = node_logp(p, Q, K);
  }
  if (COUNT) {
    double d = 0.0;
    block_reduce<COUNT>(d, zero, ne);
    if (threadIdx.x == 0) atomicAdd(evals, (unsigned long long)ne);
  }
}

// Two-pass per-node path (used when every node's parameters select the same
// integration family, the usual HDDM case: sv/sz/st are group-level):
// node_fast_kernel is the level-0 pass with the node's parameter row (staged
// in LDS as in node_kernel) and per-trial log p out; a trial that needs
// refinement or the exact path is appended — index and parameter row — to a
// dense deferred list (wave-aggregated atomic; outputs are per trial, so the
// order does not matter), which node_slow_kernel runs 64 trials per wave.
template <int MODE, bool COUNT>
__global__ __launch_bounds__(kBlock, FastWaves<MODE>::value > 0 ? FastWaves<MODE>::value : 1)
void node_fast_kernel(const double* x, const int32_t* node, int64_t n, const Params* P, Knobs K,
                      double* lp, int64_t* d_idx, Params* d_par, int* n_defer,
                      unsigned long long* evals, int* status) {
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
  bool defer = false;
  Params Q;
  if (i < n) {
    const int nj = node[i];
    Q = staged ? rows[nj - first] : P[nj];
    double p, f[5];
    int flags = 0;
    unsigned pend;
    const int oc = fast_level0<MODE>(x[i], Q, K, p, f, ne, flags, pend);
    if (oc == kFinal) lp[i] = node_logp(p, Q, K);
    else defer = true;
  }
  const unsigned long long b = __ballot(defer);
  if (b) {
    int base = 0;
    if (lane == 0) base = atomicAdd(n_defer, __popcll(b));
    base = __shfl(base, 0, 64);
    if (defer) {
      const int k = base + __popcll(b & lanemask_lt(lane));
      d_idx[k] = i;
      d_par[k] = Q;
    }
  }
  if (COUNT) {
    ne = wave_sum_ll(defer ? 0 : ne);
    if (lane == 0) atomicAdd(evals, (unsigned long long)ne);
  }
}

template <int MODE, int STK, bool COUNT>
__global__ __launch_bounds__(64, WFPT_SLOW_WAVES) void node_slow_kernel(
    const double* x, Knobs K, double* lp, const int64_t* d_idx, const Params* d_par,
    const int* n_defer, unsigned long long* evals, int* status) {
  using Stack = typename StackOf<STK>::type;
  const int nd = *n_defer;
  long long ne = 0;
  int flags = 0;
  for (int64_t k = (int64_t)blockIdx.x * 64 + threadIdx.x; k < nd; k += (int64_t)gridDim.x * 64) {
    const int64_t i = d_idx[k];
    const Params Q = d_par[k];
    long long n1 = 0;
    int f1 = 0;
    double p = full_pdf<MODE, Stack>(x[i], Q, K, n1, f1);
    if (f1 & kFlagExact) p = __builtin_nan("");  // near-tie: settled exactly below
    flags |= f1 & kFlagErrors;
    p = settle(p, x[i], Q, K, false, n1, flags);
    ne += n1;
    lp[i] = node_logp(p, Q, K);
  }
  if (flags & kFlagErrors) atomicOr(status, flags & kFlagErrors);
  if (COUNT) {
    ne = wave_sum_ll(ne);
    if (threadIdx.x == 0) atomicAdd(evals, (unsigned long long)ne);
  }
}

// wiener_like_multi (wfpt.pyx:244-274): per-trial parameters, ±999 = missing.
template <int STK>
__global__ __launch_bounds__(kBlock, WFPT_SLOW_WAVES) void multi_kernel(
    const double* x, int64_t n, const double* const* arr, const double* scal, Knobs K,
    double p_outlier, double* out, int* zeros, int* status) {
  using Stack = typename StackOf<STK>::type;
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double lp = 0.0;
  int zero = 0, flags = 0;
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
      p = full_pdf<kRuntime, Stack>(xi, Q, K, ne, flags);
      p = settle(p, xi, Q, K, !trial_setup(xi, Q).valid, ne, flags);
      if (flags & kFlagErrors) atomicOr(status, flags & kFlagErrors);
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

int stack_kind(const Knobs& K) {
  const int d = (K.n_st > K.n_sz) ? K.n_st : K.n_sz;
  return d <= 2 ? 0 : (d <= 4 ? 1 : 2);
}

int64_t blocks_for(int64_t n) { return (n + kBlock - 1) / kBlock; }

static TrialArgs trial_args(const double* x, int64_t n, const Params& P, const Knobs& K,
                            double* out, int* zeros, unsigned long long* evals, int* status,
                            int logp) {
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
  return A;
}

template <int MODE, bool COUNT, int OUT>
static void run_fast(const TrialArgs& A, const Work& W, hipStream_t s, hipEvent_t fast_done) {
  hipLaunchKernelGGL((fast_kernel<MODE, COUNT, OUT>), dim3(fast_blocks(A.n)), dim3(kFastBlock), 0,
                     s, A, W);
  if (fast_done) (void)hipEventRecord(fast_done, s);
}

template <int MODE, bool COUNT, int OUT>
static void run_deferred(const TrialArgs& A, const Work& W, int depth, hipStream_t s) {
  const int64_t nw = (A.n + 63) / 64;
  if (MODE != kDirect && depth > 0) {
    hipLaunchKernelGGL(gather_kernel, dim3((nw * 64 + kGatherSlots - 1) / kGatherSlots), dim3(256),
                       0, s, nw, W);
    const int lv = depth < kBfDepth ? depth : kBfDepth;
    const int64_t gl = std::min<int64_t>(WFPT_LEVEL_GRID, (2 * nw * 64 + 255) / 256);
    const int64_t gr = std::min<int64_t>(WFPT_LEVEL_GRID, (nw * 64 + 255) / 256);
    constexpr bool TZ = MODE == kAdaptTZ;
    if (TZ)
      hipLaunchKernelGGL((repair_kernel<MODE, 0, COUNT>), dim3(gr), dim3(256), 0, s, A, W, depth);
    if (lv >= 1) {
      hipLaunchKernelGGL((level_kernel<MODE, 1, COUNT>), dim3(gl), dim3(256), 0, s, A, W, depth);
      if (TZ)
        hipLaunchKernelGGL((repair_kernel<MODE, 1, COUNT>), dim3(gr), dim3(256), 0, s, A, W,
                           depth);
    }
    if (lv >= 2) {
      constexpr int L2 = kBfDepth >= 2 ? 2 : 1;
      hipLaunchKernelGGL((level_kernel<MODE, L2, COUNT>), dim3(gl), dim3(256), 0, s, A, W, depth);
      if (TZ)
        hipLaunchKernelGGL((repair_kernel<MODE, L2, COUNT>), dim3(gr), dim3(256), 0, s, A, W,
                           depth);
    }
    if (lv >= 3) {
      constexpr int L3 = kBfDepth >= 3 ? 3 : 1;
      hipLaunchKernelGGL((level_kernel<MODE, L3, COUNT>), dim3(gl), dim3(256), 0, s, A, W, depth);
      if (TZ)
        hipLaunchKernelGGL((repair_kernel<MODE, L3, COUNT>), dim3(gr), dim3(256), 0, s, A, W,
                           depth);
    }
  }
  // one wave per chunk up to WFPT_FOLD_GRID waves (latency-bound loads of the
  // records' tree values: many waves in flight)
  const int64_t gf = std::min<int64_t>(WFPT_FOLD_GRID, nw);
  hipLaunchKernelGGL((fold_kernel<MODE, COUNT, OUT>), dim3(gf), dim3(64), 0, s, A, W, nw, depth);
}

template <bool COUNT, int OUT>
static void launch_mode(int mode, int part, const TrialArgs& A, const Work& W, int depth,
                        hipStream_t s, hipEvent_t fast_done) {
#define FAST_AND_DEFERRED(M_)                                               \
  do {                                                                      \
    if (part & kPassFast) run_fast<M_, COUNT, OUT>(A, W, s, fast_done);     \
    if (part & kPassDeferred) run_deferred<M_, COUNT, OUT>(A, W, depth, s); \
  } while (0)
  switch (mode) {
    case kDirect: FAST_AND_DEFERRED(kDirect); break;
    case kAdaptT: FAST_AND_DEFERRED(kAdaptT); break;
    case kAdaptZ: FAST_AND_DEFERRED(kAdaptZ); break;
    case kAdaptTZ: FAST_AND_DEFERRED(kAdaptTZ); break;
    case kFixedT:
      hipLaunchKernelGGL((trial_kernel<kFixedT, COUNT, OUT>), dim3(blocks_for(A.n)), dim3(kBlock),
                         0, s, A);
      break;
    case kFixedZ:
      hipLaunchKernelGGL((trial_kernel<kFixedZ, COUNT, OUT>), dim3(blocks_for(A.n)), dim3(kBlock),
                         0, s, A);
      break;
    default:
      hipLaunchKernelGGL((trial_kernel<kFixedTZ, COUNT, OUT>), dim3(blocks_for(A.n)),
                         dim3(kBlock), 0, s, A);
      break;
  }
#undef FAST_AND_DEFERRED
  if (fast_done && mode > kAdaptTZ) (void)hipEventRecord(fast_done, s);
}

static int tree_depth(const Params& P, const Knobs& K) {
  const int mode = select_mode(P.sz, P.st, K.use_adaptive);
  return mode == kAdaptZ ? K.n_sz : K.n_st;
}

bool has_deferred_pass(const Params& P, const Knobs& K) {
  return select_mode(P.sz, P.st, K.use_adaptive) <= kAdaptTZ;
}

int64_t partials_for(int64_t n, const Params& P, const Knobs& K) {
  return has_deferred_pass(P, K) ? (n + 63) / 64 : blocks_for(n);
}

void launch_trials(int out_kind, int part, const double* x, int64_t n, const Params& P,
                   const Knobs& K, double* out, int* zeros, unsigned long long* evals, int* status,
                   int logp, const Work& W, hipStream_t s, hipEvent_t fast_done) {
  if (n <= 0) return;
  const TrialArgs A = trial_args(x, n, P, K, out, zeros, evals, status, logp);
  const int mode = select_mode(P.sz, P.st, K.use_adaptive);
  const int depth = tree_depth(P, K);
  if (evals) {
    if (out_kind == OUT_SUM) launch_mode<true, OUT_SUM>(mode, part, A, W, depth, s, fast_done);
    else if (out_kind == OUT_ARRAY)
      launch_mode<true, OUT_ARRAY>(mode, part, A, W, depth, s, fast_done);
    else launch_mode<true, OUT_LOGP>(mode, part, A, W, depth, s, fast_done);
  } else {
    if (out_kind == OUT_SUM) launch_mode<false, OUT_SUM>(mode, part, A, W, depth, s, fast_done);
    else if (out_kind == OUT_ARRAY)
      launch_mode<false, OUT_ARRAY>(mode, part, A, W, depth, s, fast_done);
    else launch_mode<false, OUT_LOGP>(mode, part, A, W, depth, s, fast_done);
  }
}

void launch_finalize(const double* part, const int* zeros, int64_t nb, const int* wl_n, int64_t nw,
                     int* status, double* out, unsigned long long seq, hipStream_t s) {
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(1024), 0, s, part, zeros, nb, wl_n, nw, status,
                     out, seq);
}

template <int MODE, bool COUNT>
static void launch_nodes_two_pass(const double* x, const int32_t* node, int64_t n,
                                  const Params* P, const Knobs& K, double* lp, int64_t* d_idx,
                                  Params* d_par, int* n_defer, unsigned long long* evals,
                                  int* status, hipStream_t s) {
  hipLaunchKernelGGL((node_fast_kernel<MODE, COUNT>), dim3(blocks_for(n)), dim3(kBlock), 0, s, x,
                     node, n, P, K, lp, d_idx, d_par, n_defer, evals, status);
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
