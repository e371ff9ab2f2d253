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
// Blocks of the deferred-trial kernel (fold).
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
// Deferred trials. A trial the level-0 kernels cannot settle (kFlagExact: its
// value hinges on last-bit rounding; kFlagFallback: its tree is deeper than
// kTreeDepth) takes slot c * 64 + k of its chunk c (k = its rank among the
// chunk's deferred trials): no atomic, and fold_kernel finds a chunk's
// deferred trials on its first lanes.
__device__ inline void defer_slots(const Work& W, int64_t c, int lane, bool defer, int rflag) {
  const unsigned long long b = __ballot(defer);
  if (defer) {
    const int64_t slot = c * 64 + __popcll(b & lanemask_lt(lane));
    W.wl[slot] = (unsigned char)lane;
    W.rflag[slot] = rflag;
  }
  if (lane == 0) W.wl_n[c] = __popcll(b);
}

// Direct family (sz = st = 0): one pdf_sv per trial, one chunk of 64 trials
// per wave.
template <int MODE, bool COUNT, int OUT>
__global__ __launch_bounds__(kFastBlock, FastWaves<MODE>::value > 0 ? FastWaves<MODE>::value : 1)
void fast_kernel(TrialArgs A, Work W) {
  const int64_t i = (int64_t)blockIdx.x * kFastBlock + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int64_t c = i >> 6;
  double p = 0.0, f[5];
  long long ne = 0;
  int flags = 0, oc = kFinal;
  unsigned pend = 0u;
  if (i < A.n) oc = fast_level0<MODE>(A.x[i], A.P, A.K, p, f, ne, flags, pend);
  double lp = 0.0;
  int zero = 0;
  if (i < A.n && oc == kFinal) emit<OUT>(A, i, p, lp, zero);
  if (c * 64 >= A.n) return;  // a wave past the last chunk (wave-uniform)
  defer_slots(W, c, lane, oc != kFinal, kFlagExact);
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

// ---------------------------------------------------------------------------
// The engine of the adaptive families (kAdaptT, kAdaptZ, kAdaptTZ;
// integrate.pxi:72-206 driven by pdf.pxi:132-146). One wave owns a chunk of 64
// consecutive trials and completes their quadrature trees, up to kTreeDepth
// refinement levels per axis (HDDM's n_st = n_sz = 2), without leaving the
// wave:
//   * a task is one evaluation of a trial's integrand at one t node: a 5-wide
//     z grid (kAdaptZ, kAdaptTZ: tnode_pdf_sv_grid5) or one pdf_sv (kAdaptT).
//     Level 0 is each lane's own root interval (its 5 t nodes, or its root z
//     grid). The stop tests of level L (each lane its own tree, in the
//     reference's order and arithmetic) queue level L + 1's tasks in LDS;
//     rounds of 64 tasks spread them over the wave's lanes, so the cost of a
//     level is ceil(tasks / 64) rounds and a chunk with few refining trials
//     pays few rounds;
//   * kAdaptTZ: a t node whose z integral asks for refinement queues a z walk:
//     4 lanes evaluate its 4 z grids (the root again, L1, L2L, L2R: every z
//     node a depth-2 walk can reach, 16 walks per round), then one lane walks
//     the z tree over those 17 values (tree_value), in the reference's order;
//   * every evaluation goes through one code site (the loop of rounds), so the
//     series code is instantiated once.
// Data in LDS per wave: the trees' values F[point * 64 + owner lane], the z
// walks' values, the task queues, the owners' x and flags; per block: the z
// grids of both boundaries and the t tree's dyadic points.
// Trials whose value hinges on last-bit rounding (kFlagExact) or whose tree is
// deeper (kFlagFallback) become deferred slots for fold_kernel.
constexpr int kEngBlock = 256;
constexpr int kEngWaves = kEngBlock / 64;
constexpr int kZBatch = 16;                             // z walks per round
constexpr int kQCap = 2 * (1 << kTreeDepth) * 64;      // tasks of one level
constexpr int kFlagIdle = 16;                           // lane without a trial to integrate
constexpr int kFlagStop = kFlagExact | kFlagFallback | kFlagIdle;

struct EngWave {
  double F[kTreePoints * 64];       // tree values: point * 64 + owner
  double ZV[kZBatch * kTreePoints];  // the current round's z walks
  double X[64];                      // the owners' x
  ZGrid G[2][4];                     // [x > 0][GridSel]: z grids of each boundary's root z interval
  double tc[kTreePoints];            // the t tree's dyadic points
  double lbz[2], ubz[2], hz[2], iz[2];  // per boundary: z interval, width, 1 / width
  int fl[64];                        // the owners' flags
  int cnt[64];                       // the owners' pdf_sv evaluations (COUNT)
  uint16_t Q[kQCap];                 // tasks of the current level: owner | point << 6 | grid << 11
  uint16_t ZQ[kQCap];                // z walks of the current level: owner | point << 6
};

__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Appends `code` of every flagged lane to q[base...] in lane order; returns
// the new length (wave-uniform).
__device__ inline int wave_append(bool flag, int code, uint16_t* q, int base) {
  const int lane = threadIdx.x & 63;
  const unsigned long long b = __ballot(flag);
  if (flag) q[base + __popcll(b & lanemask_lt(lane))] = (uint16_t)code;
  return base + __popcll(b);
}

// Point of value y[j] of a grid (GridSel) and whether this grid supplies it.
__device__ inline int grid_point(int gs, int j) {
  const int k0 = gs == kGridRoot ? 0 : gs == kGridL1 ? 2 : gs == kGridL2L ? 1 : 7;
  return k0 + j * (gs <= kGridL1 ? 4 : 2);
}
__device__ inline bool grid_owns(int gs, int j) {
  return gs == kGridRoot ? true : gs == kGridL2R ? j > 0 : j < 4;
}

// WFPT_PHASE_TIMING (diagnostic builds): shader-clock time per engine phase,
// summed over waves into W.prof[11..15] in units of 1024 cycles (level 0,
// tables, z rounds, t rounds, tests + epilogue).
#ifdef WFPT_PHASE_TIMING
#define PHASE_MARK(k)                                    \
  do {                                                   \
    const long long now_ = __builtin_amdgcn_s_memtime(); \
    ph[k] += now_ - ph_t;                                \
    ph_t = now_;                                         \
  } while (0)
#else
#define PHASE_MARK(k) \
  do {                \
  } while (0)
#endif

template <int MODE, bool COUNT, int OUT>
__global__ __launch_bounds__(kEngBlock, 2) void engine_kernel(TrialArgs A, Work W) {
#ifdef WFPT_PHASE_TIMING
  long long ph[5] = {0, 0, 0, 0, 0};
  long long ph_t = __builtin_amdgcn_s_memtime();
#endif
  __shared__ EngWave wave_lds[kEngWaves];
  const int lane = threadIdx.x & 63;
  EngWave& wv = wave_lds[threadIdx.x >> 6];
  EngWave& sh = wv;  // per-wave tables: no block barrier anywhere
  const double v = A.P.v, sv = A.P.sv, a = A.P.a, z = A.P.z, t = A.P.t;
  const double err = A.K.err, se = A.K.simps_err;
  const int nsz = A.K.n_sz;
  const int depth = (MODE == kAdaptZ) ? A.K.n_sz : A.K.n_st;
  const int64_t i = (int64_t)blockIdx.x * kEngBlock + threadIdx.x;
  const int64_t c = i >> 6;
  // (little state lives across level 0: the trial's setup is redone after it)
  const double* xp = A.x + (i < A.n ? i : 0);
  // ---- level 0, each lane its own trial, in registers (fast_level0: the
  // root interval's 5 t nodes with shared series decisions and the q
  // recurrence, or the root z grid) ----
  double p = 0.0, f0[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  long long ne0 = 0;
  int fl0 = 0, oc = kFinal;
  unsigned pend0 = 0u;
  if (i < A.n) oc = fast_level0<MODE>(*xp, A.P, A.K, p, f0, ne0, fl0, pend0);
  PHASE_MARK(0);
  const double x0 = i < A.n ? *xp : 0.0;
  const Trial tr = trial_setup(x0, A.P);
  double lb, ub;
  tree_root<MODE>(tr, A.P, lb, ub);
  const double iw = (MODE == kAdaptZ) ? 0.0 : 1.0 / (ub - lb);
  wv.X[lane] = x0;
  wv.fl[lane] = oc == kTree ? 0 : (oc == kExact ? (int)kFlagExact : (int)kFlagIdle);
  if (COUNT) wv.cnt[lane] = (int)ne0;

  int L = 0, stage = 1, r = 0, nq = 0, nz = 0;
  unsigned act = 1u;  // own tree: the intervals of level L under test
  int pq1 = 0, pq2 = 0, prec = 0, pz0 = 0, pz1 = 0, pz2 = 0;  // COUNT: work tallies
  if (__ballot(oc == kTree)) {
    // the wave's tables (trial_setup's flip: x > 0 => v = -v, z = 1 - z):
    // lanes 0..7 one z grid each, lanes 8..24 one t point each
    if (MODE != kAdaptT && lane < 8) {
      const int flip = lane >> 2, sel = lane & 3;
      const double zf = flip ? 1. - z : z, vf = flip ? -v : v;
      const double zl = zf - A.P.sz / 2., zu = zf + A.P.sz / 2.;
      sh.G[flip][sel] = zgrid_of(zl, zu, sel, vf, sv, a);
      if (sel == 0) {
        sh.lbz[flip] = zl;
        sh.ubz[flip] = zu;
        sh.hz[flip] = zu - zl;
        sh.iz[flip] = 1.0 / (zu - zl);
      }
    }
    if (MODE != kAdaptZ && lane >= 8 && lane < 8 + kTreePoints)
      sh.tc[lane - 8] = dyadic_point(t - A.P.st / 2., t + A.P.st / 2., lane - 8);
    // the refining trials' root values (a pending z integral's value comes
    // from its z walk) and their pending z integrals (kAdaptTZ)
    if (oc == kTree) {
#pragma unroll
      for (int j = 0; j < 5; ++j) wv.F[j * (kTreeW / 4) * 64 + lane] = f0[j];
    }
    if (MODE == kAdaptTZ) {
#pragma unroll
      for (int j = 0; j < 5; ++j)
        nz = wave_append(oc == kTree && ((pend0 >> (j * (kTreeW / 4))) & 1u),
                         lane | ((j * (kTreeW / 4)) << 6), wv.ZQ, nz);
    }
    wave_sync();
    PHASE_MARK(1);
#pragma unroll 1
    for (;;) {
      if (stage == 0 && r * 64 >= nq) {
        stage = 1;
        r = 0;
      }
      if (stage == 1 && (MODE != kAdaptTZ || r * kZBatch >= nz)) stage = 2;
      if (stage == 2) {
        PHASE_MARK(2);  // (the t rounds are marked at their end)
        if (COUNT) {
          if (L == 0) pz0 = nz;
          else if (L == 1) pz1 = nz;
          else pz2 = nz;
        }
        // stop tests of level L, each lane its own tree (adaptiveSimpsonsAux,
        // integrate.pxi:105 / 170): refined intervals make their children
        // level L + 1's intervals
        unsigned nxt = 0u;
        if (!(wv.fl[lane] & kFlagStop)) {
          int f = 0;
          auto FV = [&](int k) -> double { return wv.F[k * 64 + lane]; };
          for (int m = 0; m < (1 << L); ++m) {
            if (!((act >> m) & 1u)) continue;
            const TreeNode nd = tree_node(FV, lb, ub, se, L, m);
            const Simp s = simp5(nd.ub - nd.lb, FV(nd.pos), FV(nd.pos + nd.W / 4),
                                 FV(nd.pos + nd.W / 2), FV(nd.pos + 3 * nd.W / 4),
                                 FV(nd.pos + nd.W));
            if (simpson_refine(nd.S, s.S2, nd.err, depth - L, f)) nxt |= 3u << (2 * m);
          }
          if (L == kTreeDepth && nxt) f |= kFlagFallback;  // deeper than the in-wave levels
          if (f) {
            wv.fl[lane] |= f;
            nxt = 0u;
          }
        }
        if (COUNT && L == 0) prec = __popcll(__ballot(nxt != 0u));
        if (L == kTreeDepth) break;
        act = nxt;
        // level L + 1's tasks, in lane order
        int n = 0;
        if (MODE == kAdaptZ) {
          for (int m = 0; m < (1 << L); ++m)
            n = wave_append((act >> (2 * m)) & 1u,
                            lane | ((L == 0 ? kGridL1 : kGridL2L + m) << 11), wv.Q, n);
        } else {
          const int wc = kTreeW >> (L + 1);  // width of a level-(L + 1) interval
          for (int k = 0; k < (2 << L); ++k)
            for (int q = 1; q < 4; q += 2)
              n = wave_append((act >> k) & 1u, lane | ((k * wc + q * (wc / 4)) << 6), wv.Q, n);
        }
        if (COUNT) {
          if (L == 0) pq1 = n;
          else pq2 = n;
        }
        nq = n;
        wave_sync();
        PHASE_MARK(4);
        if (nq == 0) break;
        ++L;
        stage = 0;
        r = 0;
        nz = 0;
        continue;
      }
      // ---- one round: at most one evaluation per lane ----
      int owner = lane, pos = 0, gs = kGridRoot;
      bool on;
      if (stage == 0) {
        const int e = r * 64 + lane;
        on = e < nq;
        if (on) {
          const int code = wv.Q[e];
          owner = code & 63;
          pos = (code >> 6) & 31;
          gs = code >> 11;
        }
      } else {
        const int e = r * kZBatch + (lane >> 2);
        on = e < nz;
        gs = lane & 3;
        if (on) {
          const int code = wv.ZQ[e];
          owner = code & 63;
          pos = (code >> 6) & 31;
        }
      }
      on = on && !(wv.fl[owner] & kFlagStop);
      double y[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
      int flip = 0;
      if (on) {
        const double xo = wv.X[owner];
        flip = xo > 0;
        const double vo = flip ? -v : v;
        const double xa = fabs(xo);
        const double xx = (MODE == kAdaptZ) ? xa - t : xa - sh.tc[pos];
        const TNode T = tnode_setup(xx, vo, sv, a, err);
        if (T.amb) atomicOr(&wv.fl[owner], (int)kFlagExact);
        if (MODE == kAdaptT) y[0] = tnode_pdf_sv(T, flip ? 1. - z : z, vo, sv, a);
        else tnode_pdf_sv_grid5(T, sh.G[flip][gs], vo, sv, a, y);
      }
      if (stage == 0) {
        bool pend = false;
        if (on) {
          if (MODE == kAdaptT) {
            wv.F[pos * 64 + owner] = y[0] * iw;
            if (COUNT) atomicAdd(&wv.cnt[owner], 1);
          } else if (MODE == kAdaptZ) {
            const double izf = sh.iz[flip];
#pragma unroll
            for (int j = 0; j < 5; ++j)
              if (grid_owns(gs, j)) wv.F[grid_point(gs, j) * 64 + owner] = y[j] * izf;
            if (COUNT) atomicAdd(&wv.cnt[owner], 4);
          } else {
            // kAdaptTZ: the z integral's prologue + root test (integrate.pxi:
            // 114-141); a refinement queues the z walk
            const double izf = sh.iz[flip];
            const Simp s = simp5(sh.hz[flip], y[0] * izf, y[1] * izf, y[2] * izf, y[3] * izf,
                                 y[4] * izf);
            int f = 0;
            pend = simpson_refine(s.S, s.S2, se, nsz, f);
            if (f) atomicOr(&wv.fl[owner], f);
            else if (!pend) wv.F[pos * 64 + owner] = (s.S2 + (s.S2 - s.S) / 15) * iw;
            if (COUNT) atomicAdd(&wv.cnt[owner], 5);
          }
        }
        if (MODE == kAdaptTZ) nz = wave_append(pend && on, owner | (pos << 6), wv.ZQ, nz);
      } else if (MODE == kAdaptTZ) {
        if (on) {
          const double izf = sh.iz[flip];
          double* zv = wv.ZV + (lane >> 2) * kTreePoints;
#pragma unroll
          for (int j = 0; j < 5; ++j)
            if (grid_owns(gs, j)) zv[grid_point(gs, j)] = y[j] * izf;
        }
        wave_sync();
        const int e = r * kZBatch + lane;
        if (lane < kZBatch && e < nz) {
          const int code = wv.ZQ[e];
          const int ow = code & 63, ps = (code >> 6) & 31;
          if (!(wv.fl[ow] & kFlagStop)) {
            const int fz = wv.X[ow] > 0;
            const double* zv = wv.ZV + lane * kTreePoints;
            int f = 0, nref = 0;
            const double zi = tree_value([&](int k) -> double { return zv[k]; }, sh.lbz[fz],
                                         sh.ubz[fz], se, nsz, f, nref);
            if (f) atomicOr(&wv.fl[ow], f);
            else wv.F[ps * 64 + ow] = zi * iw;
            if (COUNT) atomicAdd(&wv.cnt[ow], 4 * nref);
          }
        }
      }
      ++r;
      wave_sync();
      if (stage == 0) PHASE_MARK(3);
    }
    wave_sync();
  }
  // ---- the own trial: its density (level 0, or its tree's value: the
  // reference's recursion over the stored values), or a deferred slot ----
  bool defer = oc == kExact;
  int rf = kFlagExact;
  if (oc == kTree) {
    const int ff = wv.fl[lane];
    if (ff & (kFlagExact | kFlagFallback)) {
      defer = true;
      rf = (ff & kFlagExact) ? kFlagExact : kFlagFallback;
    } else {
      int f = 0, nref = 0;
      p = tree_value([&](int k) -> double { return wv.F[k * 64 + lane]; }, lb, ub, se, depth, f,
                     nref);
      // structural zero: no evaluation point with x - t_node > 0
      const bool structural = (MODE == kAdaptZ) ? tr.x - t <= 0 : tr.x - lb <= 0;
      defer = (f & (kFlagExact | kFlagFallback)) || !(p > kExactBelow || structural);
    }
  }
  double lp = 0.0;
  int zero = 0;
  if (i < A.n && !defer) emit<OUT>(A, i, p, lp, zero);  // invalid parameters: p = 0
  if (c * 64 >= A.n) return;  // a wave past the last chunk (wave-uniform)
  defer_slots(W, c, lane, defer, rf);
  if (OUT == OUT_SUM) {
    lp = wave_sum(lp);
    const int zs = __popcll(__ballot(zero != 0));
    if (lane == 0) {
      A.out[c] = lp;
      A.zeros[c] = zs;
    }
  }
#ifdef WFPT_PHASE_TIMING
  PHASE_MARK(4);
  if (lane == 0)
    for (int k = 0; k < 5; ++k) atomicAdd(&W.prof[11 + k], (int)(ph[k] >> 10));
#endif
  if (COUNT) {
    const long long nf = wave_sum_ll((i < A.n && !defer) ? (long long)wv.cnt[lane] : 0ll);
    if (lane == 0) {
      atomicAdd(A.evals, (unsigned long long)nf);
      // wfpt_profile_lists
      atomicAdd(&W.prof[1], pq1);
      atomicAdd(&W.prof[2], pq2);
      atomicAdd(&W.prof[4], prec);
      atomicAdd(&W.prof[7], pz0 + pz1 + pz2);
      atomicAdd(&W.prof[8], pz0);
      atomicAdd(&W.prof[9], pz1);
      atomicAdd(&W.prof[10], pz2);
    }
  }
}

// Settles every deferred trial and folds it into its chunk: block g walks
// chunks g, g + G, ... (64 chunk counts per parallel load); a chunk's deferred
// trials run on its first lanes (the exact path, or the per-lane walk for
// deeper trees). OUT_SUM: chunk partial += wave sum of the deferred log
// densities (fixed lane order).
template <int MODE, bool COUNT, int OUT>
__global__ __launch_bounds__(64, WFPT_SLOW_WAVES) void fold_kernel(TrialArgs A, Work W, int64_t nw) {
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
      const int ntot = __shfl(mycnt, j, 64);
      const int64_t c = b0 + (int64_t)j * G;
      double lp = 0.0;
      int zero = 0;
      if (lane < ntot) {
        const int64_t slot = c * 64 + lane;
        const int64_t i = c * 64 + W.wl[slot];
        const double x = A.x[i];
        const int fl = W.rflag[slot];
        long long n1 = 0;
        const double p = (fl & kFlagExact) ? exact_pdf(x, A.P, A.K, &n1, &errf)
                                           : fallback_pdf<MODE>(x, A.P, A.K, &n1, &errf);
        ne += n1;
        emit<OUT>(A, i, p, lp, zero);
        if (COUNT) atomicAdd(&W.prof[(fl & kFlagExact) ? 5 : 6], 1);
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
  if constexpr (MODE == kDirect)
    hipLaunchKernelGGL((fast_kernel<MODE, COUNT, OUT>), dim3(fast_blocks(A.n)), dim3(kFastBlock),
                       0, s, A, W);
  else
    hipLaunchKernelGGL((engine_kernel<MODE, COUNT, OUT>), dim3((A.n + kEngBlock - 1) / kEngBlock),
                       dim3(kEngBlock), 0, s, A, W);
  if (fast_done) (void)hipEventRecord(fast_done, s);
}

template <int MODE, bool COUNT, int OUT>
static void run_deferred(const TrialArgs& A, const Work& W, hipStream_t s) {
  // one wave per chunk up to WFPT_FOLD_GRID waves
  const int64_t nw = (A.n + 63) / 64;
  const int64_t gf = std::min<int64_t>(WFPT_FOLD_GRID, nw);
  hipLaunchKernelGGL((fold_kernel<MODE, COUNT, OUT>), dim3(gf), dim3(64), 0, s, A, W, nw);
}

template <bool COUNT, int OUT>
static void launch_mode(int mode, int part, const TrialArgs& A, const Work& W,
                        hipStream_t s, hipEvent_t fast_done) {
#define FAST_AND_DEFERRED(M_)                                               \
  do {                                                                      \
    if (part & kPassFast) run_fast<M_, COUNT, OUT>(A, W, s, fast_done);     \
    if (part & kPassDeferred) run_deferred<M_, COUNT, OUT>(A, W, s);        \
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
  if (evals) {
    if (out_kind == OUT_SUM) launch_mode<true, OUT_SUM>(mode, part, A, W, s, fast_done);
    else if (out_kind == OUT_ARRAY)
      launch_mode<true, OUT_ARRAY>(mode, part, A, W, s, fast_done);
    else launch_mode<true, OUT_LOGP>(mode, part, A, W, s, fast_done);
  } else {
    if (out_kind == OUT_SUM) launch_mode<false, OUT_SUM>(mode, part, A, W, s, fast_done);
    else if (out_kind == OUT_ARRAY)
      launch_mode<false, OUT_ARRAY>(mode, part, A, W, s, fast_done);
    else launch_mode<false, OUT_LOGP>(mode, part, A, W, s, fast_done);
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
