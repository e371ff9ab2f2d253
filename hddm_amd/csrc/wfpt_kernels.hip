// wfpt_kernels.hip — gfx950 kernels of the WFPT likelihood engine.
//
// Adaptive / direct integration families (the HDDM case), one resident call:
//   lean_kernel<MODE>     level 0 of every trial, one 64-trial chunk per wave,
//                         boundary-uniform root grids in scalar registers (4
//                         waves/SIMD): a chunk none of whose trials refines
//                         ends here (mixture, log, chunk partial); a chunk that
//                         refines is flagged for the engine's redo pass
//   engine_kernel<MODE>   level 0 + in-wave refinement rounds (z walks, t-node
//                         tasks, tree17) of a chunk per wave; heavy chunks
//                         recorded by the previous call run as 8 split units
//   small_kernel<MODE>    <= 256 trials (one HDDM node): level 0 and the
//                         finalize in one launch
//   fast_kernel<kDirect>  the simple DDM (one pdf_sv per trial)
//   fold_kernel<MODE>     one wave per chunk: its deferred trials (exact path,
//                         trees deeper than kTreeDepth) settled in lane
//                         order and added to the chunk's partial
//   finalize_kernel       fixed-order sum of the chunk partials -> mapped slot
// The per-chunk partial of a chunk is the same value whichever sequence ran
// it (lean, lean + redo, engine, split), so a likelihood is bitwise
// reproducible across call histories. No float atomics on any likelihood
// value. OUT_BOTH builds of the same kernels also write each trial's term
// (wfpt_wiener_like_trials: the per-trial check of the summing path).
// Fixed Simpson (use_adaptive = 0): trial_kernel. Per-node parameters
// (wfpt_wiener_like_nodes): node_fast_kernel (level 0, LDS-staged node rows)
// + node_chunk_kernel (the deferred trials one wave each when they are sparse
// in their chunks, else the listed chunks 64 trials per wave per node
// segment); generic node_kernel for mixed families. Per-trial parameters (wiener_like_multi): multi_fast_kernel +
// node_engine_kernel<..., MULTI> (one wave per deferred record), or the
// generic multi_kernel.
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
#define WFPT_FAST_WAVES_TZ 3
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

// OUT_BOTH (the per-trial check of the summing kernels, wfpt_wiener_like_trials):
// exactly OUT_SUM's chunk partials and zero words, plus each trial's log term
// (-inf for a zero density) in A.trial[i]: the same template with one more store.
enum Out : int { OUT_SUM = 0, OUT_ARRAY = 1, OUT_LOGP = 2, OUT_BOTH = 3 };
constexpr bool sum_out(int out) { return out == OUT_SUM || out == OUT_BOTH; }
// OUT_SUM per-chunk zero-count word: zero-density trials | kZeroDefer if the
// chunk's level-0 pass deferred trials (or left the chunk to the redo pass)
constexpr int kZeroDefer = 1 << 16;

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
  double* out;            // OUT_SUM/BOTH: chunk / block partial sums; OUT_ARRAY/OUT_LOGP: per trial
  int* zeros;             // OUT_SUM/BOTH: chunk / block zero counts
  double* trial;          // OUT_BOTH: per-trial log terms
  unsigned long long* evals;
  int* status;            // error flags (kFlagDepth | kFlagBudget)
  int logp;               // OUT_ARRAY: return log density
};

// Trial output of a settled density p (wfpt.pyx:44 / :70).
template <int OUT>
__device__ inline void emit(const TrialArgs& A, int64_t i, double p, double& lp, int& zero) {
  if (OUT == OUT_ARRAY) {
    p = p * (1 - A.P.p_outlier) + (A.K.w_outlier * A.P.p_outlier);  // wfpt.pyx:44
    A.out[i] = A.logp ? log_val(p) : p;
  } else {
    p = p * (1 - A.P.p_outlier) + A.wp_outlier;  // wfpt.pyx:70
    if (p == 0) zero = 1;
    else lp = log_val(p);
    if (OUT == OUT_LOGP) A.out[i] = zero ? -INFINITY : lp;
    if (OUT == OUT_BOTH) A.trial[i] = zero ? -INFINITY : lp;
  }
}

// ---------------------------------------------------------------------------
// Deferred trials. A trial the level-0 kernels cannot settle (kFlagExact: its
// value hinges on last-bit rounding; kFlagFallback: its tree is deeper than
// kTreeDepth) takes slot c * 64 + k of its chunk c (k = its rank among the
// chunk's deferred trials): no atomic, and fold_kernel finds a chunk's
// deferred trials on its first lanes.
// Returns whether the chunk deferred any trial (its zero-count word then
// carries kZeroDefer, which finalize reports).
__device__ inline bool defer_slots(const Work& W, int64_t c, int lane, bool defer, int rflag) {
  const unsigned long long b = __ballot(defer);
  const int64_t slot = c * 64 + __popcll(b & lanemask_lt(lane));
  if (defer) {
    W.wl[slot] = (unsigned char)lane;
    W.rflag[slot] = rflag;
  }
  if (lane == 0) W.wl_n[c] = __popcll(b);
  return b != 0ull;
}

// Direct family (sz = st = 0): one pdf_sv per trial, one chunk of 64 trials
// per wave.
template <int MODE, bool COUNT, int OUT>
__global__ __launch_bounds__(kFastBlock, FastWaves<MODE>::value > 0 ? FastWaves<MODE>::value : 1)
void fast_kernel(TrialArgs A, Work W) {
  exp_table_init();
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
  const bool anyd = defer_slots(W, c, lane, oc != kFinal, kFlagExact);
  if (sum_out(OUT)) {
    lp = wave_sum(lp);
    const int zs = __popcll(__ballot(zero != 0));
    if (lane == 0) {
      A.out[c] = lp;
      A.zeros[c] = zs | (anyd ? kZeroDefer : 0);
    }
  }
  if (COUNT) {
    const long long nf = wave_sum_ll(oc == kFinal ? ne : 0);
    if (lane == 0) atomicAdd(A.evals, (unsigned long long)nf);
  }
}

// The direct family's level-0 pass with the call's per-boundary constants
// (DirectArgs: v, w, sin / 2cos(pi w), (-v) a w, 1 / a^2 computed once on the
// host) instead of per-lane flips, sincospi and a division: the same outputs
// as fast_kernel<kDirect> bit for bit (direct_level0). As in the lean pass, a
// wave's trials are taken by boundary (datasets are ordered by boundary, then
// |rt|), so the constants are wave-uniform; only the wave at the boundary
// switch takes the second call site.
#ifndef WFPT_DIRECT_ARGS
#define WFPT_DIRECT_ARGS 1
#endif
template <bool COUNT, int OUT>
__global__ __launch_bounds__(kFastBlock, FastWaves<kDirect>::value > 0 ? FastWaves<kDirect>::value : 1)
void direct_kernel(TrialArgs A, Work W, DirectArgs D) {
  exp_table_init();
  const int64_t i = (int64_t)blockIdx.x * kFastBlock + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int64_t c = i >> 6;
  if (c * 64 >= A.n) return;  // a wave past the last chunk (wave-uniform)
  const bool own = i < A.n;
  const double x0 = own ? A.x[i] : 0.0;
  double p = 0.0;
  long long ne = 0;
  int flags = 0, oc = kFinal;
  const bool pos = x0 > 0;
  const unsigned long long bo = __ballot(own), bp = __ballot(own && pos);
  const int b = (bp == bo) ? 1 : 0;  // every trial upper: 1; otherwise lower first
  if (own && pos == (b != 0)) oc = direct_level0(x0, A.P, A.K, D, b, p, ne, flags);
  if (bp != 0ull && bp != bo) {  // mixed wave: its upper-boundary lanes
    if (own && pos) oc = direct_level0(x0, A.P, A.K, D, 1, p, ne, flags);
  }
  double lp = 0.0;
  int zero = 0;
  if (own && oc == kFinal) emit<OUT>(A, i, p, lp, zero);
  const bool anyd = defer_slots(W, c, lane, oc != kFinal, kFlagExact);
  if (sum_out(OUT)) {
    lp = wave_sum(lp);
    const int zs = __popcll(__ballot(zero != 0));
    if (lane == 0) {
      A.out[c] = lp;
      A.zeros[c] = zs | (anyd ? kZeroDefer : 0);
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
// refinement levels per axis (HDDM's n_st = n_sz = 2):
//   * level 0 runs in registers, each lane its own trial (fast_level0: its
//     root interval's 5 t nodes with shared series decisions and the q
//     recurrence, or its root z grid); a chunk none of whose trials refines
//     ends there;
//   * refinement runs in rounds (refine_rounds). A task is one evaluation of a
//     trial's integrand at one t node: a 5-wide z grid (kAdaptZ, kAdaptTZ:
//     tnode_pdf_sv_grid5) or one pdf_sv (kAdaptT). The stop tests of level L
//     (each lane its own tree: tree17, the reference's recursion in
//     straight-line form over the values in registers) queue level L + 1's
//     tasks in LDS, and each round gives every lane of the team one task;
//   * kAdaptTZ: a t node whose z integral asks for refinement queues a z walk:
//     4 lanes evaluate its 4 z grids (the root again, L1, L2L, L2R: every z
//     node a depth-2 walk can reach), then one lane runs tree17 over the z
//     tree's 17 values;
//   * every evaluation of the rounds goes through one code site.
// Heavy chunks: a chunk whose level 0 leaves more than kHeavyZ z walks (the
// shortest RTs, where every t node's z integral refines) would serialise
// tens of rounds in one wave and set the launch's length. On a resident
// dataset the engine records such chunks (Split, next_*); the following call
// runs each of them as kSplit units of kSplitTrials trials, one wave each,
// dispatched first: the unit's level 0 runs as tasks (l0_node, bit-identical
// to the per-lane loop) and its refinement spreads over the whole wave. The
// last unit of a chunk to finish folds the chunk's per-trial terms in the
// same order wave_sum uses, so a chunk's partial does not depend on whether
// it was split (likelihoods stay bitwise reproducible across call histories).
// Trials whose value hinges on last-bit rounding (kFlagExact) or whose tree is
// deeper (kFlagFallback) become deferred slots for fold_kernel.
#ifndef WFPT_ENG_BLOCK
#define WFPT_ENG_BLOCK 256
#endif
// waves per SIMD the engine kernel is built for (its LDS, 4 x 13.4 KB per
// block, allows 3; its registers fit 2 without spilling)
#ifndef WFPT_ENG_WAVES
#define WFPT_ENG_WAVES 2
#endif
#ifndef WFPT_HEAVY_Z
#define WFPT_HEAVY_Z 96
#endif
// WFPT_HEAVY_TOTAL=1: a chunk with more than kHeavyZ z walks over all its
// levels (not after level 0 alone) is heavy too: class 2, split while the
// dataset has few heavy chunks (Split::n2)
#ifndef WFPT_HEAVY_TOTAL
#define WFPT_HEAVY_TOTAL 1
#endif
constexpr int kEngBlock = WFPT_ENG_BLOCK;
constexpr int kEngWaves = kEngBlock / 64;
constexpr int kHeavyZ = WFPT_HEAVY_Z;
constexpr int kQCap = 2 * (1 << kTreeDepth) * 64;  // tasks (or z walks) of one level
constexpr int kFlagIdle = 16;                       // lane without a trial to integrate
constexpr int kFlagStop = kFlagExact | kFlagFallback | kFlagIdle;

// WFPT_ZWALK_LDS=1: a z walk's 17 values are staged in LDS (ZV) for the lane
// that runs its tree17; 0 (default): gathered by wave shuffles (no LDS, no
// barrier; 3-4% faster on the stress sets in the r04 interleaved A/B despite
// 28 B of engine scratch)
#ifndef WFPT_ZWALK_LDS
#define WFPT_ZWALK_LDS 0
#endif
// LDS of one chunk under refinement by a team of TW waves.
template <int TW>
struct ChunkLds {
  double F[kTreePoints * 64];              // tree values: point * 64 + owner lane
#if WFPT_ZWALK_LDS
  double ZV[16 * TW * kTreePoints];        // the current round's z walks
#endif
  double X[64];                            // the owners' x
  EngTables tab;                           // the call's tables
  int fl[64];                              // the owners' flags
  int cnt[64];                             // the owners' pdf_sv evaluations (COUNT)
  int qn[2];                               // lengths of Q and ZQ
  uint16_t Q[kQCap];                       // tasks of the level: owner | point << 6 | grid << 11
  uint16_t ZQ[kQCap];                      // z walks of the level: owner | point << 6
};

// WFPT_SYNC_FENCE: wave_sync is also a scheduling barrier (experiment)
#ifndef WFPT_SYNC_FENCE
#define WFPT_SYNC_FENCE 0
#endif
__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#if WFPT_SYNC_FENCE
  __builtin_amdgcn_sched_barrier(0);
#endif
}
template <int TW>
__device__ inline void team_sync() {
  if (TW == 1) wave_sync();
  else __syncthreads();
}

// Appends `code` of every flagged lane of this wave to q at the LDS length
// counter *n (one LDS atomic per wave). Read *n after the next team_sync.
__device__ inline void team_push(bool flag, int code, uint16_t* q, int* n) {
  const int lane = threadIdx.x & 63;
  const unsigned long long b = __ballot(flag);
  if (!b) return;
  int base = 0;
  if (lane == 0) base = atomicAdd(n, __popcll(b));
  base = __shfl(base, 0, 64);
  if (flag) q[base + __popcll(b & lanemask_lt(lane))] = (uint16_t)code;
}

// Point of value y[j] of a grid (GridSel) and whether this grid supplies it.
__device__ inline int grid_point(int gs, int j) {
  const int k0 = gs == kGridRoot ? 0 : gs == kGridL1 ? 2 : gs == kGridL2L ? 1 : 7;
  return k0 + j * (gs <= kGridL1 ? 4 : 2);
}
__device__ inline bool grid_owns(int gs, int j) {
  return gs == kGridRoot ? true : gs == kGridL2R ? j > 0 : j < 4;
}

template <int TW>
__device__ inline void load_tables(ChunkLds<TW>& cl, const EngTables& tab, int tid) {
  const double* src = reinterpret_cast<const double*>(&tab);
  double* dst = reinterpret_cast<double*>(&cl.tab);
  for (int k = tid; k < (int)(sizeof(EngTables) / sizeof(double)); k += 64 * TW) dst[k] = src[k];
}

// Own tree of owner lane `o` in registers.
template <int TW>
__device__ inline void load_tree(const ChunkLds<TW>& cl, int o, double (&f)[kTreePoints]) {
#pragma unroll
  for (int k = 0; k < kTreePoints; ++k) f[k] = cl.F[k * 64 + o];
}

// Work tallies of one chunk (COUNT builds; wfpt_profile_lists).
// Per-node path: deferred trials run as records (one wave per trial,
// node_engine_kernel) when they average at most kNodeRecPerChunk per listed
// chunk, else 64 trials per wave through their chunks (node_chunk_kernel),
// which re-runs every trial of a chunk. Both produce each trial's term with
// the same operations; the choice depends only on the call's inputs.
#ifndef WFPT_NODE_REC_PER_CHUNK
#define WFPT_NODE_REC_PER_CHUNK 8
#endif
constexpr int kNodeRecPerChunk = WFPT_NODE_REC_PER_CHUNK;
__device__ inline bool node_records_sparse(int n_records, int n_chunks) {
  return (long long)n_records <= (long long)kNodeRecPerChunk * n_chunks;
}

struct Tally {
  int t1 = 0, t2 = 0, rec = 0, z[3] = {0, 0, 0};
};

// WFPT_PHASE_TIMING (diagnostic builds): shader-clock time per engine phase,
// per wave in W.phase (level 0, tables, z rounds, t rounds, tests + epilogue;
// wfpt_profile_lists reports the sums in kilo-cycles, wfpt_debug_waves the
// per-wave records).
#ifdef WFPT_PHASE_TIMING
struct PhaseClock {
  long long ph[5] = {0, 0, 0, 0, 0};
  long long t = 0;
  int nz = 0, nt = 0;
  __device__ void start() { t = __builtin_amdgcn_s_memtime(); }
  __device__ void mark(int k) {
    const long long now = __builtin_amdgcn_s_memtime();
    ph[k] += now - t;
    t = now;
  }
};
#else
struct PhaseClock {
  int nz = 0, nt = 0;
  __device__ void start() {}
  __device__ void mark(int) {}
};
#endif

// Refinement rounds of one chunk by a team of TW waves (tid = 0..64 TW - 1;
// the chunk's owner lanes are tid < 64). Entry: stage 1 after level 0 with
// its values in F and its z walks queued (engine_kernel), or stage 0 with
// level 0's t nodes (root z grids) queued as tasks (split_unit: they take the
// level-0 hints, l0_hints, so their bits equal fast per-lane level 0's). All
// control is team-uniform.
template <int MODE, bool COUNT, int TW>
__device__ inline void refine_rounds(const TrialArgs& A, ChunkLds<TW>& cl, int tid, int stage,
                                     Tally& ty, PhaseClock& pc) {
  constexpr int NT = 64 * TW;
  const double v = A.P.v, sv = A.P.sv, a = A.P.a, z = A.P.z, t = A.P.t;
  const double err = A.K.err, se = A.K.simps_err;
  const int nsz = A.K.n_sz;
  const int depth = (MODE == kAdaptZ) ? A.K.n_sz : A.K.n_st;
  const double iwt = 1.0 / (cl.tab.tP[kTreeW] - cl.tab.tP[0]);
  const double ia2 = 1.0 / (a * a);  // as l0_hints: the same tt for the same t node
  int L = 0, r = 0;
#pragma unroll 1
  for (;;) {
    const int nq = cl.qn[0], nz = cl.qn[1];
    if (stage == 0 && r * NT >= nq) {
      stage = 1;
      r = 0;
    }
    if (stage == 1 && (MODE != kAdaptTZ || r * 16 * TW >= nz)) stage = 2;
    if (stage == 2) {
      pc.mark(2);
      // constant indices: a runtime index would put the tally in scratch
      if (L == 0) ty.z[0] = nz;
      else if (L == 1) ty.z[1] = nz;
      else if (L == 2) ty.z[2] = nz;
      // stop tests of level L, each owner lane its own tree
      unsigned need = 0u;
      if (tid < 64 && !(cl.fl[tid] & kFlagStop)) {
        double f[kTreePoints];
        load_tree(cl, tid, f);
        const double(&P)[kTreePoints] =
            (MODE == kAdaptZ) ? cl.tab.zP[cl.X[tid] > 0] : cl.tab.tP;
        int fl = 0, nref = 0;
        (void)tree17(f, P, se, depth, L, fl, need, nref);
        if (L == kTreeDepth && need) fl |= kFlagFallback;  // deeper than the in-wave levels
        if (fl & (kFlagExact | kFlagFallback)) {
          atomicOr(&cl.fl[tid], fl & (kFlagExact | kFlagFallback));
          need = 0u;
        }
      }
      if (COUNT && L == 0 && tid < 64) ty.rec = __popcll(__ballot(need != 0u));
      if (L == kTreeDepth) break;
      if (tid == 0) {
        cl.qn[0] = 0;
        cl.qn[1] = 0;
      }
      team_sync<TW>();
      // level L + 1's tasks: for each refining interval m of level L, the aux
      // nodes d, e of both its halves (kAdaptZ: one grid per interval)
      if (tid < 64) {
        if (MODE == kAdaptZ) {
          for (int m = 0; m < (1 << L); ++m)
            team_push((need >> m) & 1u, tid | ((L == 0 ? kGridL1 : kGridL2L + m) << 11), cl.Q,
                      &cl.qn[0]);
        } else {
          const int wm = kTreeW >> L;  // width of a level-L interval
          for (int m = 0; m < (1 << L); ++m)
            for (int q = 1; q < 8; q += 2)
              team_push((need >> m) & 1u, tid | ((m * wm + q * (wm / 8)) << 6), cl.Q, &cl.qn[0]);
        }
      }
      team_sync<TW>();
      pc.mark(4);
      if (COUNT) {
        if (L == 0) ty.t1 = cl.qn[0];
        else ty.t2 = cl.qn[0];
      }
      if (cl.qn[0] == 0) break;
      ++L;
      stage = 0;
      r = 0;
      continue;
    }
    // ---- one round: at most one evaluation per lane ----
    int owner = tid & 63, pos = 0, gs = kGridRoot, zslot = 0;
    bool on;
    if (stage == 0) {
      const int e = r * NT + tid;
      on = e < nq;
      if (on) {
        const int code = cl.Q[e];
        owner = code & 63;
        pos = (code >> 6) & 31;
        gs = code >> 11;
      }
    } else {
      zslot = tid >> 2;
      const int e = r * 16 * TW + zslot;
      on = e < nz;
      gs = tid & 3;
      if (on) {
        const int code = cl.ZQ[e];
        owner = code & 63;
        pos = (code >> 6) & 31;
      }
    }
    on = on && !(cl.fl[owner] & kFlagStop);
    double y[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    int flip = 0;
    bool ovf = false;  // a drift factor overflowed (tnode_pdf_sv_grid5)
    if (on) {
      const double xo = cl.X[owner];
      flip = xo > 0;
      const double vo = flip ? -v : v;
      const double xa = fabs(xo);
      const double xx = (MODE == kAdaptZ) ? xa - t : xa - cl.tab.tP[pos];
      // level-0 t nodes (split units): the per-lane loop's hints (l0_hints)
      double qh = -1.0;
      bool known = false;
      Decision kd{0, 0, 0};
      if (MODE != kAdaptZ && L == 0 && stage == 0) {
        const L0Hints H = l0_hints(xa, cl.tab.tP[0], cl.tab.tP[kTreeW], a, err);
        const int j = pos / (kTreeW / 4);
        qh = H.qh(j);
        known = j == 0 ? H.ok0 : (j == 4 ? H.ok4 : H.shared);
        kd = j == 4 ? H.D4 : H.D0;
      }
      const TNode T = tnode_setup_r(xx, vo, sv, a, ia2, err, qh, known, kd);
      if (T.amb) atomicOr(&cl.fl[owner], (int)kFlagExact);
      if (MODE == kAdaptT) y[0] = tnode_pdf_sv(T, flip ? 1. - z : z, vo, sv, a);
      else
        ovf = !tnode_pdf_sv_grid5(T, cl.tab.G[flip][gs], vo, sv, a, y);  // literal values
    }
    if (stage == 0) {
      bool pend = false;
      if (on) {
        if (MODE == kAdaptT) {
          cl.F[pos * 64 + owner] = y[0] * iwt;
          if (COUNT) atomicAdd(&cl.cnt[owner], 1);
        } else if (MODE == kAdaptZ) {
          const double izf = cl.tab.iz[flip];
#pragma unroll
          for (int j = 0; j < 5; ++j)
            if (grid_owns(gs, j)) cl.F[grid_point(gs, j) * 64 + owner] = y[j] * izf;
          if (COUNT) atomicAdd(&cl.cnt[owner], gs == kGridRoot ? 5 : 4);
        } else {
          // kAdaptTZ: the z integral's prologue + root test (integrate.pxi:
          // 114-141); a refinement queues the z walk
          // (inner_root's operations: the root grid's weights, simp_value)
          const double izf = cl.tab.iz[flip];
          const ZGrid& gr = cl.tab.G[flip][kGridRoot];
          const Simp s = simp5p(gr.h6, gr.h12, y[0] * izf, y[1] * izf, y[2] * izf, y[3] * izf,
                                y[4] * izf);
          int f = 0;
          // an overflowed root grid: the z walk (inner_root's rule)
          pend = simpson_refine(s.S, s.S2, se, nsz, f) || ovf;
          if (ovf) f = 0;
          if (f) atomicOr(&cl.fl[owner], f);
          else if (!pend) cl.F[pos * 64 + owner] = simp_value(s) * iwt;
          if (COUNT) atomicAdd(&cl.cnt[owner], 5);
        }
      }
      if (MODE == kAdaptTZ) {
        team_push(pend && on, owner | (pos << 6), cl.ZQ, &cl.qn[1]);
      }
      ++pc.nt;
    } else if (MODE == kAdaptTZ) {
      double zv[kTreePoints];
#if WFPT_ZWALK_LDS
      if (on) {
        const double izf = cl.tab.iz[flip];
        double* zw = cl.ZV + zslot * kTreePoints;
#pragma unroll
        for (int j = 0; j < 5; ++j)
          if (grid_owns(gs, j)) zw[grid_point(gs, j)] = y[j] * izf;
      }
      team_sync<TW>();
      if (tid < 16 * TW) {
#pragma unroll
        for (int k = 0; k < kTreePoints; ++k) zv[k] = cl.ZV[tid * kTreePoints + k];
      }
#else
      static_assert(TW == 1, "z walks gather their values by wave shuffles");
      // lane t < 16 runs walk t: its 17 values come from lanes 4t .. 4t + 3
      // (grid gs = source lane & 3; grid_point / grid_owns), by shuffles
      const double izf = on ? cl.tab.iz[flip] : 0.0;
      double yz[5];
#pragma unroll
      for (int j = 0; j < 5; ++j) yz[j] = y[j] * izf;
      const int b4 = (tid & 15) * 4;
#pragma unroll
      for (int j = 0; j < 5; ++j) zv[4 * j] = __shfl(yz[j], b4 + kGridRoot, 64);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        zv[2 + 4 * j] = __shfl(yz[j], b4 + kGridL1, 64);
        zv[1 + 2 * j] = __shfl(yz[j], b4 + kGridL2L, 64);
        zv[9 + 2 * j] = __shfl(yz[j + 1], b4 + kGridL2R, 64);
      }
#endif
      const int e = r * 16 * TW + tid;
      if (tid < 16 * TW && e < nz) {
        const int code = cl.ZQ[e];
        const int ow = code & 63, ps = (code >> 6) & 31;
        if (!(cl.fl[ow] & kFlagStop)) {
          int f = 0, nref = 0;
          unsigned need = 0u;
          const double zi = tree17(zv, cl.tab.zP[cl.X[ow] > 0], se, nsz, kTreeDepth, f, need, nref);
          if (need) f |= kFlagFallback;  // z tree deeper than the walk's levels
          if (f & (kFlagExact | kFlagFallback)) atomicOr(&cl.fl[ow], f & (kFlagExact | kFlagFallback));
          else cl.F[ps * 64 + ow] = zi * iwt;
          if (COUNT) atomicAdd(&cl.cnt[ow], 4 * nref);
        }
      }
      ++pc.nz;
    }
    ++r;
    team_sync<TW>();
    if (stage == 0) pc.mark(3);
  }
}

// Final density of owner lane o (a refined tree: tree17 over its stored
// values; the level tests already flagged ties and deeper trees).
template <int MODE, int TW>
__device__ inline void tree_density(const TrialArgs& A, const ChunkLds<TW>& cl, int o, double x,
                                    double& p, bool& defer, int& rf) {
  const int ff = cl.fl[o];
  if (ff & (kFlagExact | kFlagFallback)) {
    defer = true;
    rf = (ff & kFlagExact) ? kFlagExact : kFlagFallback;
    return;
  }
  double f[kTreePoints];
  load_tree(cl, o, f);
  const Trial tr = trial_setup(x, A.P);
  const double(&P)[kTreePoints] = (MODE == kAdaptZ) ? cl.tab.zP[x > 0] : cl.tab.tP;
  const int depth = (MODE == kAdaptZ) ? A.K.n_sz : A.K.n_st;
  int fl = 0, nref = 0;
  unsigned need = 0u;
  p = tree17(f, P, A.K.simps_err, depth, kTreeDepth, fl, need, nref);
  // structural zero: no evaluation point with x - t_node > 0
  const bool structural = (MODE == kAdaptZ) ? tr.x - A.P.t <= 0 : tr.x - P[0] <= 0;
  defer = (fl & kFlagExact) || need || !(p > kExactBelow || structural);
  if (defer && !(fl & kFlagExact) && !need && tiny_absorbed(p, A.P.p_outlier, A.K.w_outlier)) {
    defer = false;  // the mixture absorbs it (tiny_absorbed)
    p = 0.0;
  }
  rf = kFlagExact;
}

// Chunk outputs of the owner lanes (one wave): per-trial emit, deferred
// slots, the chunk partial and the evaluation count.
template <bool COUNT, int OUT>
__device__ inline void chunk_out(const TrialArgs& A, const Work& W, int64_t c, int lane, double p,
                                 bool defer, int rf, long long ne) {
  const int64_t i = c * 64 + lane;
  double lp = 0.0;
  int zero = 0;
  if (i < A.n && !defer) emit<OUT>(A, i, p, lp, zero);  // invalid parameters: p = 0
  const bool anyd = defer_slots(W, c, lane, defer, rf);
  if (sum_out(OUT)) {
    lp = wave_sum(lp);
    const int zs = __popcll(__ballot(zero != 0));
    if (lane == 0) {
      A.out[c] = lp;
      A.zeros[c] = zs | (anyd ? kZeroDefer : 0);
    }
  }
  if (COUNT) {
    const long long nf = wave_sum_ll((i < A.n && !defer) ? ne : 0ll);
    if (lane == 0) atomicAdd(A.evals, (unsigned long long)nf);
  }
}

__device__ inline void tally_out(const Work& W, const Tally& ty) {
  atomicAdd(&W.prof[1], ty.t1);
  atomicAdd(&W.prof[2], ty.t2);
  atomicAdd(&W.prof[4], ty.rec);
  atomicAdd(&W.prof[7], ty.z[0] + ty.z[1] + ty.z[2]);
  atomicAdd(&W.prof[8], ty.z[0]);
  atomicAdd(&W.prof[9], ty.z[1]);
  atomicAdd(&W.prof[10], ty.z[2]);
}

// Records chunk c for the next call's split (lane 0 of its last wave).
__device__ inline void record_heavy(const Split& S, int64_t c, int cls) {
  if (!S.next_pred) return;
  unsigned char flag = 0;
  if (cls) {
    const int half = S.cap / 2;
    const int slot = atomicAdd(S.next_n + (cls == 2 ? 2 : 0), 1);
    if (slot < half) {
      S.next_list[(cls == 2 ? half : 0) + slot] = (int)c;
      flag = (unsigned char)cls;
    }
  }
  S.next_pred[c] = flag;
}
// Heavy class of a chunk from its z walks after level 0 (z0) and over all
// levels (zt): 1, 2 (WFPT_HEAVY_TOTAL) or 0.
__device__ inline int heavy_class(int z0, int zt) {
  return z0 > kHeavyZ ? 1 : ((WFPT_HEAVY_TOTAL && zt > kHeavyZ) ? 2 : 0);
}

// Chunk outputs of a split unit's trials: per-trial outputs now, the chunk
// partial's terms to S.lp / S.meta; the chunk's last unit (agent-scope
// release / acquire hand-off) folds them in wave_sum's order and writes the
// chunk's deferred slots in lane order, exactly as an unsplit chunk's wave.
template <int MODE, bool COUNT, int OUT>
__device__ inline void split_out(const TrialArgs& A, const Work& W, const Split& S,
                                 const ChunkLds<1>& cl, int slot, int sub, int lane, double x0,
                                 int nz0, int nzt) {
  const int64_t c = S.list[slot < S.n ? slot : S.cap / 2 + (slot - S.n)];
  const int64_t i = c * 64 + sub * kSplitTrials + lane;
  const bool own = lane < kSplitTrials && i < A.n;
  double p = 0.0, lp = 0.0;
  bool defer = false;
  int rf = kFlagExact, zero = 0;
  if (own && !(cl.fl[lane] & kFlagIdle)) tree_density<MODE, 1>(A, cl, lane, x0, p, defer, rf);
  if (own && !defer) emit<OUT>(A, i, p, lp, zero);  // invalid parameters: p = 0
  if (lane < kSplitTrials) {
    const int k = slot * 64 + sub * kSplitTrials + lane;
    S.lp[k] = lp;
    S.meta[k] = zero | ((int)defer << 1) | (rf << 2);
  }
  if (COUNT) {
    const long long nf = wave_sum_ll((own && !defer) ? (long long)cl.cnt[lane] : 0ll);
    if (lane == 0) atomicAdd(A.evals, (unsigned long long)nf);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int prev = 0;
  if (lane == 0) {
    atomicAdd(&S.zn[slot], nz0 + (nzt << 16));
    prev = __hip_atomic_fetch_add(&S.done[slot], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  prev = __shfl(prev, 0, 64);
  if (prev != kSplit - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const double lpc = S.lp[slot * 64 + lane];
  const int m = S.meta[slot * 64 + lane];
  const bool anyd = defer_slots(W, c, lane, (m >> 1) & 1, m >> 2);
  if (sum_out(OUT)) {
    const double sum = wave_sum(lpc);
    const int zs = __popcll(__ballot((m & 1) != 0));
    if (lane == 0) {
      A.out[c] = sum;
      A.zeros[c] = zs | (anyd ? kZeroDefer : 0);
    }
  }
  if (lane == 0) {
    const int znc = __hip_atomic_load(&S.zn[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    record_heavy(S, c, heavy_class(znc & 0xffff, znc >> 16));
    S.done[slot] = 0;
    S.zn[slot] = 0;
  }
}

template <int MODE, bool COUNT, int OUT>
__global__ __launch_bounds__(kEngBlock, WFPT_ENG_WAVES) void engine_kernel(TrialArgs A, Work W, EngTables tab,
                                                              Split S) {
  exp_table_init();
  __shared__ ChunkLds<1> lds[kEngWaves];
  const int lane = threadIdx.x & 63;
  ChunkLds<1>& cl = lds[threadIdx.x >> 6];
  PhaseClock pc;
  pc.start();
#ifdef WFPT_PHASE_TIMING
  const long long rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  // work units: the split chunks' units first (dispatched first), then one
  // wave per chunk
  const int64_t u = (int64_t)blockIdx.x * kEngWaves + (threadIdx.x >> 6);
  const int ns = S.n + S.n2;  // split chunks: class 1's units, then class 2's
  const bool split = u < (int64_t)ns * kSplit;
  const int slot = split ? (int)(u / kSplit) : 0, sub = split ? (int)(u % kSplit) : 0;
  const int64_t c = split ? (int64_t)S.list[slot < S.n ? slot : S.cap / 2 + (slot - S.n)]
                          : u - (int64_t)ns * kSplit;
  // past the end / split in this call (class 2 only while n2 > 0)
  if (!split && (c * 64 >= A.n ||
                 (ns > 0 && (S.pred[c] == 1 || (S.pred[c] == 2 && S.n2 > 0)))))
    return;
  if (W.redo && !W.redo[c]) return;  // redo pass: only the chunks the lean pass flagged
  load_tables(cl, tab, lane);
  const int64_t i = split ? c * 64 + sub * kSplitTrials + lane : c * 64 + lane;
  const bool own = (split ? lane < kSplitTrials : true) && i < A.n;
  const double x0 = own ? A.x[i] : 0.0;
  wave_sync();
  double p = 0.0;
  long long ne0 = 0;
  int oc = kFinal, stage = 1;
  bool rounds;
  if (!split) {
    // ---- level 0, each lane its own trial, in registers ----
    double f0[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    unsigned pend0 = 0u;
    if (own) {
      const ZGrid G = cl.tab.G[x0 > 0][kGridRoot];
      oc = eng_level0<MODE>(x0, A.P, A.K, G, p, f0, ne0, pend0);
    }
    pc.mark(0);
    rounds = __ballot(oc == kTree) != 0ull;
    if (rounds) {
      cl.X[lane] = x0;
      cl.fl[lane] = oc == kTree ? 0 : (oc == kExact ? (int)kFlagExact : (int)kFlagIdle);
      if (COUNT) cl.cnt[lane] = (int)ne0;
      if (oc == kTree) {
#pragma unroll
        for (int j = 0; j < 5; ++j) cl.F[j * (kTreeW / 4) * 64 + lane] = f0[j];
      }
      if (lane == 0) {
        cl.qn[0] = 0;
        cl.qn[1] = 0;
      }
      wave_sync();
      // the pending z integrals of the refining trials (kAdaptTZ)
      if (MODE == kAdaptTZ) {
#pragma unroll
        for (int j = 0; j < 5; ++j)
          team_push(oc == kTree && ((pend0 >> (j * (kTreeW / 4))) & 1u),
                    lane | ((j * (kTreeW / 4)) << 6), cl.ZQ, &cl.qn[1]);
      }
    }
  } else {
    // ---- a split unit: its kSplitTrials trials' level 0 as tasks (t node j
    // of owner o, or owner o's root z grid) ----
    cl.X[lane] = x0;
    cl.fl[lane] = (own && trial_setup(x0, A.P).valid) ? 0 : kFlagIdle;
    if (COUNT) cl.cnt[lane] = 0;
    if (lane == 0) {
      cl.qn[0] = 0;
      cl.qn[1] = 0;
    }
    wave_sync();
    constexpr int n0 = (MODE == kAdaptZ) ? 1 : 5;
    const int o = lane % kSplitTrials, j = lane / kSplitTrials;
    team_push(j < n0 && !(cl.fl[o] & kFlagStop), o | ((j * (kTreeW / 4)) << 6), cl.Q, &cl.qn[0]);
    stage = 0;
    rounds = true;
  }
  Tally ty;
  int nz0 = 0, nzt = 0;
  if (rounds) {
    // chunks that refined in-wave (a split chunk once: its unit 0); finalize
    // reports the count, which picks the next call's level-0 pass
    if (lane == 0 && (!split || sub == 0)) atomicAdd(W.tree_any, 1);
    wave_sync();
    nz0 = cl.qn[1];
    pc.mark(1);
    refine_rounds<MODE, COUNT, 1>(A, cl, lane, stage, ty, pc);
    if (split) nz0 = ty.z[0];
    nzt = ty.z[0] + ty.z[1] + ty.z[2];  // the z walks of every level
  }
  if (split) {
    split_out<MODE, COUNT, OUT>(A, W, S, cl, slot, sub, lane, x0, nz0, nzt);
    if (COUNT && lane == 0) tally_out(W, ty);
#ifdef WFPT_PHASE_TIMING
    // split units in the upper half of the records (unit u at kPhaseWaves / 2 + u)
    if (lane == 0 && u < kPhaseWaves / 2) {
      unsigned long long* rec = W.phase + (kPhaseWaves / 2 + u) * 8;
      rec[0] = rt0;
      rec[1] = __builtin_amdgcn_s_memrealtime();
      for (int k = 0; k < 5; ++k) rec[2 + k] = pc.ph[k];
      rec[7] = (unsigned long long)pc.nz | ((unsigned long long)pc.nt << 32);
    }
#endif
    return;
  }
  if (lane == 0) {
    record_heavy(S, c, heavy_class(nz0, nzt));
    if (W.redo) W.redo[c] = 0;
  }
  bool defer = oc == kExact;
  int rf = kFlagExact;
  if (oc == kTree) tree_density<MODE, 1>(A, cl, lane, x0, p, defer, rf);
  chunk_out<COUNT, OUT>(A, W, c, lane, p, defer, rf, oc == kTree ? (long long)cl.cnt[lane] : ne0);
  pc.mark(4);
#ifdef WFPT_PHASE_TIMING
  if (lane == 0 && c < kPhaseWaves / 2) {
    unsigned long long* rec = W.phase + c * 8;
    rec[0] = rt0;
    rec[1] = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < 5; ++k) rec[2 + k] = pc.ph[k];
    rec[7] = (unsigned long long)pc.nz | ((unsigned long long)pc.nt << 32);
  }
#endif
  if (COUNT && lane == 0) tally_out(W, ty);
}

// The engine's level 0 alone (kPassLean), for resident datasets whose last
// call refined no chunk in-wave (the usual MCMC case at HDDM's knobs): no LDS,
// no refinement code, so the register allocation and occupancy are those of
// level 0 (FastWaves) instead of the engine's. Each lane runs eng_level0 on
// the table's root z grid, i.e. the same operations on the same inputs as the
// engine's level 0, and a chunk without refining trials leaves the bits the
// engine would (chunk_out). A chunk with a refining trial writes nothing but
// its redo flag and a nonzero deferred count; the engine's redo pass
// (kPassRedo) then processes it from scratch, as a full engine call would.
// Root z grid of boundary b (0: lower, 1: upper) with b wave-uniform: every
// field is a select between two kernel arguments on a uniform condition, so
// the grid stays in scalar registers.
// WFPT_ZGRID_REF: the grid is read through a reference into the kernel
// argument block (scalar loads at a uniform offset, on demand) instead of
// select-copied into registers.
#ifndef WFPT_ZGRID_REF
#define WFPT_ZGRID_REF 1
#endif
#if WFPT_ZGRID_REF
__device__ inline const ZGrid& zgrid_uniform(const RootGrids& R, int b) { return R.G[b]; }
#else
__device__ inline ZGrid zgrid_uniform(const RootGrids& R, int b) {
  const ZGrid& g0 = R.G[0];
  const ZGrid& g1 = R.G[1];
  ZGrid G;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    G.g[k] = b ? g1.g[k] : g0.g[k];
    G.A[k] = b ? g1.A[k] : g0.A[k];
  }
  G.h6 = b ? g1.h6 : g0.h6;
  G.h12 = b ? g1.h12 : g0.h12;
  G.s0 = b ? g1.s0 : g0.s0;
  G.c0 = b ? g1.c0 : g0.c0;
  G.s4 = b ? g1.s4 : g0.s4;
  G.c4 = b ? g1.c4 : g0.c4;
  G.sd = b ? g1.sd : g0.sd;
  G.cd = b ? g1.cd : g0.cd;
  return G;
}
#endif

// WFPT_SIN_TABLE=0: the lean pass evaluates the large-time sines per lane
// (the recurrence) instead of reading the call's table (same values).
#ifndef WFPT_SIN_TABLE
#define WFPT_SIN_TABLE 1
#endif

// Block size of the lean pass (WFPT_LEAN_BLOCK; its waves are independent:
// one chunk each, no block-level exchange). The launch bound's second
// argument is waves per SIMD (amdgpu_waves_per_eu), independent of the block
// size, so the register budget is the same for every block size.
#ifndef WFPT_LEAN_BLOCK
#define WFPT_LEAN_BLOCK 256
#endif
constexpr int kLeanBlock = WFPT_LEAN_BLOCK;
static_assert(kLeanBlock % 64 == 0 && kLeanBlock <= kFastBlock, "kLeanBlock");
template <int MODE, bool COUNT, int OUT>
__global__ __launch_bounds__(kLeanBlock, FastWaves<MODE>::value > 0 ? FastWaves<MODE>::value : 1)
void lean_kernel(TrialArgs A, Work W, RootGrids R) {
  exp_table_init();
#ifdef WFPT_PHASE_TIMING
  const long long rt0 = __builtin_amdgcn_s_memrealtime();
#endif
#if WFPT_LEAN_REVERSE
  // blocks dispatched last take the first chunks (timing experiment)
  const int64_t i = (int64_t)(gridDim.x - 1 - blockIdx.x) * kLeanBlock + threadIdx.x;
#else
  const int64_t i = (int64_t)blockIdx.x * kLeanBlock + threadIdx.x;
#endif
  const int lane = threadIdx.x & 63;
  const int64_t c = i >> 6;
  if (c * 64 >= A.n) return;  // a wave past the last chunk (wave-uniform)
  const bool own = i < A.n;
  const double x0 = own ? A.x[i] : 0.0;
  double p = 0.0, f0[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  long long ne0 = 0;
  unsigned pend0 = 0u;
  int oc = kFinal;
  // The wave's trials by boundary. Inside one boundary the root z grid and
  // the flipped v, z (pdf.pxi:116-118) are wave-uniform: they stay in scalar
  // registers (zgrid_uniform) instead of per-lane selects and copies.
  // Datasets are ordered by boundary, then |rt| (wfpt_dataset_create), so
  // only the wave at the boundary switch is mixed: its upper-boundary lanes
  // take the second call site.
  const bool pos = x0 > 0;
  const unsigned long long bo = __ballot(own), bp = __ballot(own && pos);
  const int b = (bp == bo) ? 1 : 0;  // every trial upper: 1; otherwise lower first
  if (own && pos == (b != 0))
    oc = eng_level0_t<MODE, false, WFPT_LEAN_UNROLL != 0>(trial_setup_b(x0, A.P, b != 0), A.P, A.K,
                                   zgrid_uniform(R, b), p, f0, ne0, pend0,
                                   WFPT_SIN_TABLE ? &R.S[b][0][0] : nullptr);
  if (bp != 0ull && bp != bo) {  // mixed wave: its upper-boundary lanes
    if (own && pos)
      oc = eng_level0_t<MODE, false, WFPT_LEAN_UNROLL != 0>(trial_setup_b(x0, A.P, true), A.P, A.K, R.G[1], p, f0,
                                     ne0, pend0, WFPT_SIN_TABLE ? &R.S[1][0][0] : nullptr);
  }
  if (__ballot(oc == kTree) != 0ull) {
    if (lane == 0) {
      W.redo[c] = 1;
      // finalize reports the call as deferred: the host runs the redo pass
      if (sum_out(OUT)) A.zeros[c] = kZeroDefer;
    }
    return;
  }
  chunk_out<COUNT, OUT>(A, W, c, lane, p, oc == kExact, kFlagExact, ne0);
#ifdef WFPT_PHASE_TIMING
  // per-wave start / end (the lean pass has no split units: every record)
  if (lane == 0 && c < kPhaseWaves) {
    unsigned long long* rec = W.phase + c * 8;
    rec[0] = rt0;
    rec[1] = __builtin_amdgcn_s_memrealtime();
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    rec[2] = hw;
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    rec[3] = xcc;
  }
#endif
}

// A node's trial term: mixture with the node's p_outlier, -inf for a zero
// density or a p_outlier outside [0, 1] (wfpt.pyx:63-72 per node).
__device__ inline double node_logp(double p, const Params& Q, const Knobs& K) {
  const bool ok = (Q.p_outlier >= 0) & (Q.p_outlier <= 1);  // wfpt.pyx:63-64 per node
  p = p * (1 - Q.p_outlier) + K.w_outlier * Q.p_outlier;
  return (!ok || p == 0) ? -INFINITY : log_val(p);
}

// The per-call tables (EngTables) of one trial's parameters, built by the lanes
// of a wave in parallel: lanes 0-7 the 8 z grids, then the dyadic points of the
// t tree and of both z trees, then 1 / (ub_z - lb_z). The same functions as
// the host's eng_tables.
__device__ inline void eng_tables_wave(const Params& P, EngTables& T, int lane) {
  constexpr int kP = kTreePoints;
  if (lane < 8) {
    const int flip = lane >> 2, sel = lane & 3;
    const double zf = flip ? 1. - P.z : P.z, vf = flip ? -P.v : P.v;
    T.G[flip][sel] = zgrid_of(zf - P.sz / 2., zf + P.sz / 2., sel, vf, P.sv, P.a);
  } else if (lane < 8 + kP) {
    T.tP[lane - 8] = dyadic_point(P.t - P.st / 2., P.t + P.st / 2., lane - 8);
  } else if (lane < 8 + 3 * kP) {
    const int idx = lane - 8 - kP, flip = idx / kP, k = idx % kP;
    const double zf = flip ? 1. - P.z : P.z;
    T.zP[flip][k] = dyadic_point(zf - P.sz / 2., zf + P.sz / 2., k);
  } else if (lane < 8 + 3 * kP + 2) {
    const int flip = lane - (8 + 3 * kP);
    const double zf = flip ? 1. - P.z : P.z;
    T.iz[flip] = 1.0 / ((zf + P.sz / 2.) - (zf - P.sz / 2.));
  }
  wave_sync();
}

// Deferred trials of the per-node and per-trial-parameter paths (records of
// index + parameter row; adaptive families). The per-lane recursion would
// leave one lane walking a trial's whole tree serially (~40 dependent
// evaluations at one-wave latency set the call's length); instead one wave
// takes one record and runs the engine's breadth-first rounds on the trial's
// own tables: its level-0 t nodes (or root z grid) as tasks, then refinement
// levels and z walks across the lanes, exactly as a split unit of the dataset
// engine. Trees deeper than kTreeDepth and rounding-critical values take the
// per-lane fallback / exact path on lane 0. MULTI: wiener_like_multi's term.
// One wave per record, wave ids w0, w0 + nwaves, ...: the record's tables in
// the wave's LDS, its level-0 t nodes as tasks, the refinement rounds, and on
// lane 0 its density (tree17, the exact path or the per-lane walk) and term.
// A record's index is virtual (t n_tab + i: trial i of parameter table t, the
// multi-table node call); its RT is x[i], its term lp[t n_tab + i].
__device__ inline int64_t tab_trial(int64_t v, int64_t n_tab) { return v < n_tab ? v : v % n_tab; }
// (the node path's rare list: see node_sum)
constexpr int kRareShift = 56;
constexpr int64_t kRareMask = (1LL << kRareShift) - 1;
constexpr int kRareExact = 1, kRareWalk = 2;
struct NodeRare {
  int64_t* v;
  int32_t* j;
  int* n;
};
__device__ inline void rare_push(const NodeRare& R, int64_t v, int32_t vj, int kind, double* lp) {
  const int k = atomicAdd(R.n, 1);
  R.v[k] = v | ((int64_t)kind << kRareShift);
  R.j[k] = vj;
  lp[v] = 0.0;  // a neutral addend until the summing kernel settles the trial
}

template <int MODE, bool COUNT, bool MULTI>
__device__ inline void node_records(ChunkLds<1>& cl, int lane, int w0, int nwaves,
                                    const double* x, const Knobs& K, double* lp,
                                    const int64_t* d_idx, const Params* d_par, int nd,
                                    unsigned long long* evals, int* status,
                                    int64_t n_tab = INT64_MAX, const NodeRare* R = nullptr,
                                    const int32_t* node = nullptr, int32_t n_nodes = 0) {
  long long ne = 0;
  int errf = 0;
  for (int k = w0; k < nd; k += nwaves) {
    const int64_t i = d_idx[k];
    const Params Q = d_par[k];
    TrialArgs A{};
    A.x = x;
    A.P = Q;
    A.K = K;
    A.wp_outlier = K.w_outlier * Q.p_outlier;
    const double x0 = x[tab_trial(i, n_tab)];
    eng_tables_wave(Q, cl.tab, lane);
    cl.X[lane] = lane == 0 ? x0 : 0.0;
    cl.fl[lane] = (lane == 0 && trial_setup(x0, Q).valid) ? 0 : (int)kFlagIdle;
    if (COUNT) cl.cnt[lane] = 0;
    if (lane == 0) {
      cl.qn[0] = 0;
      cl.qn[1] = 0;
    }
    wave_sync();
    constexpr int n0 = (MODE == kAdaptZ) ? 1 : 5;
    team_push(lane < n0 && !(cl.fl[0] & kFlagStop), (lane * (kTreeW / 4)) << 6, cl.Q, &cl.qn[0]);
    wave_sync();
    Tally ty;
    PhaseClock pc;
    refine_rounds<MODE, COUNT, 1>(A, cl, lane, 0, ty, pc);
    if (lane == 0) {
      double p = 0.0;
      bool defer = false;
      int rf = kFlagExact;
      long long n1 = 0;
      if (!(cl.fl[0] & kFlagIdle)) {
        tree_density<MODE, 1>(A, cl, 0, x0, p, defer, rf);
        if (COUNT) n1 = cl.cnt[0];
      }
      if constexpr (MULTI) {
        if (defer) {
          n1 = 0;
          p = (rf & kFlagExact) ? exact_pdf(x0, Q, K, &n1, &errf)
                                : fallback_pdf<MODE>(x0, Q, K, &n1, &errf);
        }
        ne += n1;
        lp[i] = log_val(p * (1 - Q.p_outlier) + (K.w_outlier * Q.p_outlier));
      } else {
        if (defer) {  // the node path's rare list (node_sum settles it)
          const int64_t t = i / n_tab;
          rare_push(*R, i, (int32_t)(t * n_nodes + node[i - t * n_tab]),
                    (rf & kFlagExact) ? kRareExact : kRareWalk, lp);
        } else {
          ne += n1;
          lp[i] = node_logp(p, Q, K);
        }
      }
    }
    wave_sync();  // the next record reuses this wave's LDS
  }
  if (errf & kFlagErrors) atomicOr(status, errf & kFlagErrors);
  if (COUNT) {
    ne = wave_sum_ll(ne);
    if (lane == 0) atomicAdd(evals, (unsigned long long)ne);
  }
}

template <int MODE, bool COUNT, bool MULTI>
__global__ __launch_bounds__(kEngBlock, 2) void node_engine_kernel(
    const double* x, Knobs K, double* lp, const int64_t* d_idx, const Params* d_par,
    const int* n_defer, unsigned long long* evals, int* status) {
  exp_table_init();
  __shared__ ChunkLds<1> lds[kEngWaves];
  const int lane = threadIdx.x & 63;
  node_records<MODE, COUNT, MULTI>(
      lds[threadIdx.x >> 6], lane,
      __builtin_amdgcn_readfirstlane((int)blockIdx.x * kEngWaves + (int)(threadIdx.x >> 6)),
      (int)gridDim.x * kEngWaves, x, K, lp, d_idx, d_par, *n_defer, evals, status);
}

// Folds every chunk's deferred trials into it, one wave per chunk: slot k of
// chunk c (its k-th deferred lane) on lane k, settled on the exact path
// (near-ties, ambiguous series decisions, subnormal densities) or the per-lane
// walk (trees deeper than kTreeDepth); the mixture and log (emit), and the
// wave sum added to the chunk's partial (a fixed order).
template <int MODE, bool COUNT, int OUT>
__global__ __launch_bounds__(256, WFPT_SLOW_WAVES) void fold_kernel(TrialArgs A, Work W, int64_t nw) {
  exp_table_init();
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  long long ne = 0;
  int errf = 0;
  for (int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); c < nw; c += nwaves) {
    const int ntot = W.wl_n[c];
    if (ntot == 0) continue;  // wave-uniform
    double lp = 0.0;
    int zero = 0;
    if (lane < ntot) {
      const int64_t slot = c * 64 + lane;
      const int64_t i = c * 64 + W.wl[slot];
      const int fl = W.rflag[slot];
      long long n1 = 0;
      const double p = (fl & kFlagExact) ? exact_pdf(A.x[i], A.P, A.K, &n1, &errf)
                                         : fallback_pdf<MODE>(A.x[i], A.P, A.K, &n1, &errf);
      ne += n1;
      if (COUNT) atomicAdd(&W.prof[(fl & kFlagExact) ? 5 : 6], 1);
      emit<OUT>(A, i, p, lp, zero);
    }
    if (sum_out(OUT)) {
      lp = wave_sum(lp);
      const int zs = __popcll(__ballot(zero != 0));
      if (lane == 0) {
        A.out[c] = A.out[c] + lp;
        A.zeros[c] = A.zeros[c] + zs;
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
  exp_table_init();
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
  if (sum_out(OUT) || COUNT) {
    block_reduce<COUNT>(lp, zero, ne);
    if (threadIdx.x == 0) {
      if (sum_out(OUT)) {
        A.out[blockIdx.x] = lp;
        A.zeros[blockIdx.x] = zero;
      }
      if (COUNT) atomicAdd(A.evals, (unsigned long long)ne);
    }
  }
}

// out[0] = sum of nb partials, out[1] = number of zero trials, out[2] = error
// flags encoded as counts that survive a sum over ranks (depth + 2^20 budget),
// out[3] = kResDeferred if some chunk's word carries kZeroDefer (defer_bits:
// per-chunk partials of the adaptive / direct families) | kResTree, then the
// 64-bit completion word out[4] once they are visible. `out` may be mapped
// pinned host memory. Resets the device status word. Fixed summation order
// for a given nb: thread k owns partials k + 1024 j, loaded kFinLoads at a
// time (all in flight together) and summed in j order; then a fixed tree.
// The completion word of a result slot in mapped host memory: a system-scope
// release store, after every result store the call's publication ordered
// before it; the host reads it with an acquire load (wait_word).
__device__ __forceinline__ void publish_word(unsigned long long* w, unsigned long long seq) {
  __hip_atomic_store(w, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The result slot of a call (finalize's last step, one thread): {sum, zero
// count, encoded errors, flags, -, heavy chunks, #tree} and then the
// completion word; resets the device status word.
__device__ inline void fin_write(double t, long long zz, int dd, int* status, double* out,
                                 unsigned long long seq, const int* split_rd, int* split_rs,
                                 int* tree_any, double* mirror) {
  const int st = *status;
  *status = 0;
  out[0] = t;
  out[1] = (double)zz;
  out[2] = (double)(st & kFlagDepth) + ((st & kFlagBudget) ? kBudgetUnit : 0.0);
  int res3 = dd ? kResDeferred : 0;
  double ntree = 0.0;
  if (tree_any) {
    if (*tree_any) res3 |= kResTree;
    ntree = (double)*tree_any;
    *tree_any = 0;
  }
  out[6] = ntree;
  out[3] = (double)res3;
  // heavy chunks recorded for the next call (Split)
  out[5] = split_rd ? (double)split_rd[0] : 0.0;  // class 1 (Split)
  out[7] = split_rd ? (double)split_rd[2] : 0.0;  // class 2
  if (split_rs) {
    split_rs[0] = 0;
    split_rs[2] = 0;
  }
  if (mirror) {  // device copy of the result (the RCCL exchange reads it)
    mirror[0] = out[0];
    mirror[1] = out[1];
    mirror[2] = out[2];
    mirror[3] = out[3];
    mirror[5] = out[5];
    mirror[6] = out[6];
    mirror[7] = out[7];
  }
  // completion word, a system-scope release store after the results (one
  // thread wrote them all): the host may poll it (acquire) instead of waiting
  // on the stream
  publish_word(reinterpret_cast<unsigned long long*>(out) + 4, seq);
}

// Large nb (C2's 10M trials: 156k partials): one block is bound by a single
// CU's load bandwidth (29 us), so gridDim.x = G > 1 blocks each reduce a
// contiguous range the same way into fin[g] (sum), fin[kFinMaxBlocks + g]
// (zero count), fin[2 kFinMaxBlocks + g] (defer bits), and the last block to
// finish (agent-scope ticket) adds the G block results in g order. Fixed
// order for a given (nb, G); G = 1 is the single-block order.
constexpr int kFinLoads = 16;
constexpr int kFinMaxBlocks = 64;
#ifndef WFPT_FIN_PER_BLOCK
#define WFPT_FIN_PER_BLOCK 8192
#endif
constexpr int64_t kFinPerBlock = WFPT_FIN_PER_BLOCK;  // partials per block when split
__global__ __launch_bounds__(1024) void finalize_kernel(const double* part, const int* zeros,
                                                        int64_t nb, int defer_bits,
                                                        int* status, double* out,
                                                        unsigned long long seq,
                                                        const int* split_rd, int* split_rs,
                                                        int* tree_any, double* mirror,
                                                        double* fin, int* ticket) {
  __shared__ double ss[16];
  __shared__ long long sz[16];
  __shared__ int sd[16];
  __shared__ int last;
  const int G = gridDim.x;
  int64_t lo = 0, hi = nb;
  if (G > 1) {
    const int64_t L = (nb + G - 1) / G;
    lo = (int64_t)blockIdx.x * L;
    hi = lo + L < nb ? lo + L : nb;
  }
  double s = 0.0;
  long long z = 0;
  int def = 0;
  for (int64_t b0 = lo + threadIdx.x; b0 < hi; b0 += kFinLoads * 1024) {
    double v[kFinLoads];
    int w[kFinLoads];
#pragma unroll
    for (int j = 0; j < kFinLoads; ++j) {
      const int64_t b = b0 + (int64_t)j * 1024;
      v[j] = b < hi ? part[b] : 0.0;
      w[j] = b < hi ? zeros[b] : 0;
    }
#pragma unroll
    for (int j = 0; j < kFinLoads; ++j) {
      s += v[j];
      z += w[j] & (kZeroDefer - 1);
      def |= w[j];
    }
  }
  def = defer_bits ? (def & kZeroDefer) : 0;
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
    if (G > 1) {
      fin[blockIdx.x] = t;
      fin[kFinMaxBlocks + blockIdx.x] = (double)zz;
      fin[2 * kFinMaxBlocks + blockIdx.x] = (double)dd;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      const int prev =
          __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = prev == G - 1;
    } else {
      last = 1;
    }
    if (G > 1 && last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      t = 0.0;
      zz = 0;
      dd = 0;
      for (int g = 0; g < G; ++g) {
        t += __hip_atomic_load(&fin[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        zz += (long long)__hip_atomic_load(&fin[kFinMaxBlocks + g], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
        dd |= (int)__hip_atomic_load(&fin[2 * kFinMaxBlocks + g], __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
      }
      *ticket = 0;  // ready for the next call (stream order)
    }
    if (!last) return;
    fin_write(t, zz, dd, status, out, seq, split_rd, split_rs, tree_any, mirror);
  }
}

// One-block calls (n <= kFastBlock trials: an HDDM node's 250, the drop-in's
// per-node call): the level-0 pass of the direct family (fast_kernel's
// operations) or of the adaptive families (lean_kernel's), then the finalize
// of the block's <= 4 chunk partials in the same launch, with finalize_kernel's
// exact operations on them (thread k holds partial k, one wave sum, then the
// 16 wave sums added in order, the 15 empty ones as +0.0), so the result and
// the completion word are bit for bit those of the two-launch sequence. The
// chunk partials and zero words are written as usual (a deferred pass after a
// misprediction reads them).
struct FinArgs {
  int* status;
  double* out;
  unsigned long long seq;
  int* tree_any;
  int defer_bits;
};

template <int MODE, int OUT>
__global__ __launch_bounds__(kFastBlock) void small_kernel(TrialArgs A, Work W, RootGrids R,
                                                           FinArgs F) {
  exp_table_init();
  __shared__ double fp[kFastBlock / 64];
  __shared__ int fz[kFastBlock / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t i = threadIdx.x, c = wv;
  const bool has = c * 64 < A.n;  // wave-uniform
  const bool own = i < A.n;
  double part = 0.0;
  int zw = 0;
  bool tree = false;  // lean: the chunk is left to the redo pass (no partial)
  if (has) {
    double p = 0.0, f0[5];
    long long ne0 = 0;
    unsigned pend0 = 0u;
    int oc = kFinal;
    if constexpr (MODE == kDirect) {
      int flags = 0;
      if (own) oc = fast_level0<MODE>(A.x[i], A.P, A.K, p, f0, ne0, flags, pend0);
      double lp = 0.0;
      int zero = 0;
      if (own && oc == kFinal) emit<OUT>(A, i, p, lp, zero);
      const bool anyd = defer_slots(W, c, lane, oc != kFinal, kFlagExact);
      part = wave_sum(lp);
      zw = __popcll(__ballot(zero != 0)) | (anyd ? kZeroDefer : 0);
    } else {
      const double x0 = own ? A.x[i] : 0.0;
      const bool pos = x0 > 0;
      const unsigned long long bo = __ballot(own), bp = __ballot(own && pos);
      const int b = (bp == bo) ? 1 : 0;
      if (own && pos == (b != 0))
        oc = eng_level0_t<MODE, false, WFPT_LEAN_UNROLL != 0>(
            trial_setup_b(x0, A.P, b != 0), A.P, A.K, zgrid_uniform(R, b), p, f0, ne0, pend0,
            WFPT_SIN_TABLE ? &R.S[b][0][0] : nullptr);
      if (bp != 0ull && bp != bo) {
        if (own && pos)
          oc = eng_level0_t<MODE, false, WFPT_LEAN_UNROLL != 0>(
              trial_setup_b(x0, A.P, true), A.P, A.K, R.G[1], p, f0, ne0, pend0,
              WFPT_SIN_TABLE ? &R.S[1][0][0] : nullptr);
      }
      if (__ballot(oc == kTree) != 0ull) {
        if (lane == 0) W.redo[c] = 1;  // the host runs the redo pass (lean_kernel)
        part = 0.0;                    // (discarded: the call is reported deferred)
        zw = kZeroDefer;
        tree = true;
      } else {
        double lp = 0.0;
        int zero = 0;
        const bool defer = oc == kExact;
        if (own && !defer) emit<OUT>(A, i, p, lp, zero);
        const bool anyd = defer_slots(W, c, lane, defer, kFlagExact);
        part = wave_sum(lp);
        zw = __popcll(__ballot(zero != 0)) | (anyd ? kZeroDefer : 0);
      }
    }
    if (lane == 0) {
      if (!tree) A.out[c] = part;
      A.zeros[c] = zw;
      fp[wv] = part;
      fz[wv] = zw;
    }
  }
  __syncthreads();
  if (wv != 0) return;
  const int nb = (int)((A.n + 63) / 64);
  double s = 0.0;
  long long z = 0;
  int def = 0;
  if (lane < nb) {
    s += fp[lane];
    z += fz[lane] & (kZeroDefer - 1);
    def |= fz[lane];
  }
  def = F.defer_bits ? (def & kZeroDefer) : 0;
  s = wave_sum(s);
  z = wave_sum_ll(z);
  const bool anyd = __ballot(def != 0) != 0ull;
  if (lane == 0) {
    double t = 0.0;
    long long zz = 0;
    int dd = 0;
    const double ss[2] = {s, 0.0};
    for (int k = 0; k < 16; ++k) {
      t += ss[k == 0 ? 0 : 1];
      zz += k == 0 ? z : 0ll;
      dd |= k == 0 ? (int)anyd : 0;
    }
    fin_write(t, zz, dd, F.status, F.out, F.seq, nullptr, nullptr, F.tree_any, nullptr);
  }
}

// One-block calls of the full DDM (kAdaptTZ: 25 pdf_sv evaluations per
// trial, the per-node drop-in call of HDDM with sv, sz, st) are one wave's
// latency in small_kernel: 64 trials per wave, each lane its trial's 5 t
// nodes in sequence. Here three lanes share a trial (768 threads: 3 waves per
// SIMD, so the generic t-node code fits its registers): lane s of trial k
// evaluates t nodes s and s + 3 (l0_node, the function the split units'
// level-0 tasks use, bit-identical to the per-lane loop) into LDS; then waves
// 0-3 take one trial per lane again (chunk c on wave c), run the root stop
// test and the value from the five values as eng_level0_t does, and continue
// exactly as small_kernel (chunk partials, zero words, deferred slots, the
// finalize), so every output is small_kernel's, bit for bit.
// WFPT_SMALL_SPLIT=0: small_kernel.
#ifndef WFPT_SMALL_SPLIT
#define WFPT_SMALL_SPLIT 1
#endif
#ifndef WFPT_SPLIT_LANES
#define WFPT_SPLIT_LANES 3
#endif
constexpr int kSplitLanes = WFPT_SPLIT_LANES;
constexpr int kSplitBlock = kSplitLanes * kFastBlock;

// eng_level0_t's tail (KEEP_F) for one trial, from its five t-node values.
template <int MODE>
__device__ inline int l0_finish(const Trial& tr, const Params& P, const Knobs& K, int flags,
                                unsigned pend, const double (&f)[5], double& p) {
  p = 0.0;
  if (!tr.valid) return kFinal;
  if (flags & kFlagExact) return kExact;
  if (pend) return kTree;
  double lb, ub;
  tree_root<MODE>(tr, P, lb, ub);
  const bool structural = tr.x - lb <= 0;
  const Simp s = simp5(ub - lb, f[0], f[1], f[2], f[3], f[4]);
  int fl = 0;
  const bool refine = simpson_refine(s.S, s.S2, K.simps_err, K.n_st, fl);
  if (fl & kFlagExact) return kExact;
  if (refine) return kTree;
  p = s.S2 + (s.S2 - s.S) / 15;
  if (p > kExactBelow || structural) return kFinal;
  if (!tiny_absorbed(p, P.p_outlier, K.w_outlier)) return kExact;
  p = 0.0;
  return kFinal;
}

template <int MODE, int OUT>
__global__ __launch_bounds__(kSplitBlock) void small_split_kernel(TrialArgs A, Work W,
                                                                 RootGrids R, FinArgs F) {
  exp_table_init();
  static_assert(MODE == kAdaptTZ, "t-node split of the full DDM");
  __shared__ double sf[5][kFastBlock];  // t-node values, node-major
  __shared__ int sfl[kSplitLanes][kFastBlock];
  __shared__ unsigned spd[kSplitLanes][kFastBlock];
  __shared__ double fp[kFastBlock / 64];
  __shared__ int fz[kFastBlock / 64];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int k = t / kSplitLanes, sub = t - k * kSplitLanes;  // this lane's trial and share
  const bool own = k < A.n;
  const double x0 = own ? A.x[k] : 0.0;
  const bool pos = x0 > 0;
  const unsigned long long bo = __ballot(own), bp = __ballot(own && pos);
  const int b = (bp == bo) ? 1 : 0;
  int flags = 0;
  unsigned pend = 0u;
  long long ne = 0;
  // pass 1: the lanes of boundary b (a single-boundary wave: all); pass 2: the
  // upper-boundary lanes of a mixed wave (wave-uniform grids, as small_kernel)
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    const bool mine = pass == 0 ? (own && pos == (b != 0)) : (bp != 0ull && bp != bo && own && pos);
    if (!mine) continue;
    const int bb = pass == 0 ? b : 1;
    const Trial tr = trial_setup_b(x0, A.P, bb != 0);
    if (!tr.valid) continue;
    double lb, ub;
    tree_root<MODE>(tr, A.P, lb, ub);
    const L0Hints H = l0_hints(tr.x, lb, ub, A.P.a, A.K.err);
#pragma unroll 1
    for (int j = sub; j < 5; j += kSplitLanes) {
      bool pj = false;
      sf[j][k] = l0_node<MODE>(tr, A.P, A.K, lb, ub, H, j, zgrid_uniform(R, bb), flags, pj, ne,
                               WFPT_SIN_TABLE ? &R.S[bb][0][0] : nullptr);
      if (pj) pend |= 1u << (j * (kTreeW / 4));
    }
  }
  if (own) {
    sfl[sub][k] = flags;
    spd[sub][k] = pend;
  }
  __syncthreads();
  // one trial per lane again: chunk c on wave c (small_kernel's operations)
  if (wv < kFastBlock / 64) {
    const int i = t, c = wv;
    if (c * 64 < A.n) {  // wave-uniform
      const bool own1 = i < A.n;
      int oc = kFinal;
      double p = 0.0;
      if (own1) {
        const double xi = A.x[i];
        int fl = 0;
        unsigned pd = 0u;
#pragma unroll
        for (int q = 0; q < kSplitLanes; ++q) {
          fl |= sfl[q][i];
          pd |= spd[q][i];
        }
        const double f[5] = {sf[0][i], sf[1][i], sf[2][i], sf[3][i], sf[4][i]};
        oc = l0_finish<MODE>(trial_setup_b(xi, A.P, xi > 0), A.P, A.K, fl, pd, f, p);
      }
      double part = 0.0;
      int zw = 0;
      bool tree = false;
      if (__ballot(oc == kTree) != 0ull) {
        if (lane == 0) W.redo[c] = 1;  // the host runs the redo pass (lean_kernel)
        zw = kZeroDefer;
        tree = true;
      } else {
        double lp = 0.0;
        int zero = 0;
        const bool defer = oc == kExact;
        if (own1 && !defer) emit<OUT>(A, i, p, lp, zero);
        const bool anyd = defer_slots(W, c, lane, defer, kFlagExact);
        part = wave_sum(lp);
        zw = __popcll(__ballot(zero != 0)) | (anyd ? kZeroDefer : 0);
      }
      if (lane == 0) {
        if (!tree) A.out[c] = part;
        A.zeros[c] = zw;
        fp[wv] = part;
        fz[wv] = zw;
      }
    }
  }
  __syncthreads();
  if (wv != 0) return;
  const int nb = (int)((A.n + 63) / 64);
  double s = 0.0;
  long long z = 0;
  int def = 0;
  if (lane < nb) {
    s += fp[lane];
    z += fz[lane] & (kZeroDefer - 1);
    def |= fz[lane];
  }
  def = F.defer_bits ? (def & kZeroDefer) : 0;
  s = wave_sum(s);
  z = wave_sum_ll(z);
  const bool anyd = __ballot(def != 0) != 0ull;
  if (lane == 0) {
    double tt = 0.0;
    long long zz = 0;
    int dd = 0;
    const double ss[2] = {s, 0.0};
    for (int q = 0; q < 16; ++q) {
      tt += ss[q == 0 ? 0 : 1];
      zz += q == 0 ? z : 0ll;
      dd |= q == 0 ? (int)anyd : 0;
    }
    fin_write(tt, zz, dd, F.status, F.out, F.seq, nullptr, nullptr, F.tree_any, nullptr);
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
    out[3] = res[3];
    out[5] = res[5];
    out[6] = res[6];
    publish_word(reinterpret_cast<unsigned long long*>(out) + 4, seq);
  }
}

void launch_publish(const double* res, double* out, unsigned long long seq, hipStream_t s) {
  hipLaunchKernelGGL(publish_kernel, dim3(1), dim3(64), 0, s, res, out, seq);
}

__global__ __launch_bounds__(64) void poison_kernel(double* res) {
  if (threadIdx.x < 8) res[threadIdx.x] = threadIdx.x == 2 ? kPeerFailUnit : 0.0;
}

void launch_poison(double* res, hipStream_t s) {
  hipLaunchKernelGGL(poison_kernel, dim3(1), dim3(64), 0, s, res);
}

// The node path's rare trials -- the exact path (near-ties, ambiguous series
// decisions, densities below kExactBelow) and trees deeper than kTreeDepth --
// are not settled by the level-0 / record / chunk kernels: they append the
// trial to a list and leave lp[v] = +0.0, and the summing kernel settles each
// node's rare trials (exact_pdf / fallback_pdf, one lane each) before it
// publishes the node. Their code (wfpt_exact.hpp's double-double libm, the
// per-lane walk's memory stack) is thus out of the hot kernels' registers and
// scratch: node_fast_kernel<kDirect> 168 -> ~54 VGPRs (3 -> 8 waves/SIMD),
// node_chunk_kernel without its 7.5 KB/lane of scratch.
// Entry k: v[k] = virtual trial index (t n + i) | kind << kRareShift, j[k] =
// its virtual node (t m + node[i]); *n the count (0 at rest: the summing
// kernel's last block resets it).

// Node vj's sum, one wave (vj = t m + jr: the trials [t n + off[jr],
// t n + off[jr + 1]) of lp): each lane adds its strided terms in order, then
// a wave_sum; -inf if any term is -inf (wfpt.pyx:71-72 per node). The rare
// trials' terms are in lp by then (node_rare_kernel).
__device__ inline double node_sum(const double* lp, const int64_t* off, int32_t vj, int32_t m,
                                  int64_t n, int lane) {
  const int tab = vj / m, jr = vj - tab * m;
  const int64_t lo = tab * n + off[jr], hi = tab * n + off[jr + 1];
  double s = 0.0;
  int zero = 0;
  // four strided terms per lane loaded together, then added in order (one
  // memory latency per 256 trials instead of per 64)
  for (int64_t i0 = lo + lane; i0 < hi; i0 += 256) {
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = i0 + 64 * u < hi ? lp[i0 + 64 * u] : 0.0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (v[u] == -INFINITY) zero = 1;
      else s += v[u];
    }
  }
  s = wave_sum(s);
  return __ballot(zero != 0) != 0ull ? -INFINITY : s;
}

// node_sum of NB nodes of one wave at once (vj[b], on[b]): the same per-node
// operations -- each lane's strided terms in the same order, the same 0.0
// additions past a segment's end inside an active batch, one wave_sum per
// node -- with every node's loads issued before any node's additions, so the
// wave waits one memory latency per batch instead of one per node.
template <int NB>
__device__ inline void node_sums(const double* lp, const int64_t* off, const int32_t (&vj)[NB],
                                 const bool (&on)[NB], int32_t m, int64_t n, int lane,
                                 double (&out)[NB]) {
  int64_t lo[NB], hi[NB];
  double s[NB];
  int zero[NB];
  int64_t len = 0;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int tab = on[b] ? vj[b] / m : 0, jr = on[b] ? vj[b] - tab * m : 0;
    lo[b] = on[b] ? tab * n + off[jr] : 0;
    hi[b] = on[b] ? tab * n + off[jr + 1] : 0;
    len = hi[b] - lo[b] > len ? hi[b] - lo[b] : len;
    s[b] = 0.0;
    zero[b] = 0;
  }
  for (int64_t q = lane; q < len; q += 256) {
    double v[NB][4];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = lo[b] + q + 64 * u;
        v[b][u] = i < hi[b] ? lp[i] : 0.0;
      }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (lo[b] + q < hi[b]) {  // node_sum's iteration i0 = lo + q is active
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (v[b][u] == -INFINITY) zero[b] = 1;
          else s[b] += v[b][u];
        }
      }
    }
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const double t = wave_sum(s[b]);
    out[b] = __ballot(zero[b] != 0) != 0ull ? -INFINITY : t;
  }
}

// The rare trials of a node call (rare_push), one lane each: the exact path
// or the per-lane walk of the trial's family, its node term into lp. Launched
// only when the publication found the list non-empty (the host re-publishes;
// a call with no rare trial -- nearly all of them -- never runs this code, and
// its kernels carry neither its registers nor its scratch). n_tab: trials per
// table, m: nodes per table (table t's node j at t m + j).
__global__ __launch_bounds__(64, WFPT_SLOW_WAVES) void node_rare_kernel(NodeRare R, double* lp, const double* x,
                                                          const Params* P, int32_t m,
                                                          int64_t n_tab, Knobs K, int mode,
                                                          int* status, unsigned long long* evals) {
  const int nr = *R.n;
  int errf = 0;
  long long ne = 0;
  for (int k = blockIdx.x * 64 + threadIdx.x; k < nr; k += gridDim.x * 64) {
    const int64_t r = R.v[k];
    const int64_t v = r & kRareMask;
    const int kind = (int)(r >> kRareShift);
    const int32_t vj = R.j[k];
    const int64_t i = v - (int64_t)(vj / m) * n_tab;
    const Params Q = P[vj];
    long long n1 = 0;
    double p;
    if (kind == kRareExact) p = exact_pdf(x[i], Q, K, &n1, &errf);
    else if (mode == kAdaptT) p = fallback_pdf<kAdaptT>(x[i], Q, K, &n1, &errf);
    else if (mode == kAdaptZ) p = fallback_pdf<kAdaptZ>(x[i], Q, K, &n1, &errf);
    else p = fallback_pdf<kAdaptTZ>(x[i], Q, K, &n1, &errf);
    ne += n1;
    lp[v] = node_logp(p, Q, K);
  }
  if (errf & kFlagErrors) atomicOr(status, errf & kFlagErrors);
  if (evals && ne) atomicAdd(evals, (unsigned long long)ne);
}

// One wave per node (grid-stride): the per-node sums into res (the node
// all-reduce's vector and wfpt_wiener_like_nodes_local).
__global__ __launch_bounds__(256) void segment_sum_kernel(const double* lp, const int64_t* off,
                                                          int32_t n_nodes, double* res) {
  const int lane = threadIdx.x & 63;
  for (int j = blockIdx.x * 4 + (threadIdx.x >> 6); j < n_nodes; j += gridDim.x * 4) {
    const double s = node_sum(lp, off, j, n_nodes, 0, lane);
    if (lane == 0) res[j] = s;
  }
}

// segment_sum_kernel's per-node sums and publish_nodes_kernel's publication in
// one launch. The ordering is the memory model's, not the hardware's (LLVM
// AMDGPUUsage memory model for GFX942/GFX950, the HSA / OpenCL 2.0 scoped
// model: happens-before is the transitive closure of program order and scoped
// synchronizes-with edges, each edge between threads inside its scope):
//   1. lane 0 of node j's wave stores res[j] (device memory; an agent-scope
//      atomic store, performed at agent scope before the wave goes on);
//   2. __syncthreads (workgroup-scope release + acquire): every store of the
//      block happens-before thread 0's next operation;
//   3. thread 0: acq_rel fetch_add on the agent-scope ticket. The ticket's
//      RMWs form one release sequence, so the block that draws G - 1
//      synchronizes-with every earlier block's release;
//   4. __syncthreads: the last block's threads happen-after all G releases,
//      read res[] and store it to the mapped slot;
//   5. __syncthreads, then thread 0 stores the completion word with a
//      system-scope release; the host polls it with an acquire load
//      (wfpt_capi.cpp: wait_word), so every sum is visible when it reads.
// r05 let each wave store its sum straight into the mapped slot, ordered
// before the completion word by nothing: one GPU-suite run read a node sum
// of the previous call (profiles/r06/stale_diag/ shows the test catching that
// order deterministically in the WFPT_PUB_DIAG build). The last block also
// resets the call's counters (the node path's n_defer words and the ticket:
// 0 at rest, stream order).
//
// WFPT_PUB_DIAG=1 (diagnostic builds only, never the shipped library): every
// block but the last takes its ticket *first* and writes its nodes' sums into
// the mapped slot ~70 us later, i.e. the completion word deterministically
// overtakes the sums -- the failure the regression test must be able to see.
#ifndef WFPT_PUB_DIAG
#define WFPT_PUB_DIAG 0
#endif
#ifndef WFPT_PUB_BLOCKS
#define WFPT_PUB_BLOCKS 128
#endif
constexpr int32_t kPubBlocks = WFPT_PUB_BLOCKS;
// nodes a publishing wave sums at once (node_sums; 1: one node at a time)
#ifndef WFPT_PUB_NODES
#define WFPT_PUB_NODES 4
#endif
constexpr int kPubNodes = WFPT_PUB_NODES;
// Multi-table calls: n_nodes = T m virtual nodes, node j of table t at
// t m + j, summing trials [t n + off[j], t n + off[j + 1]) of lp.
// check_rare: a call whose level-0 / record / chunk kernels left rare trials
// (*n_rare > 0) is not summed: the last block writes kRarePending in the
// error slot and the completion word, the host runs node_rare_kernel and
// launches this kernel again with check_rare = 0.
constexpr double kRarePending = -1.0;  // (error counts are >= 0)
__global__ __launch_bounds__(256) void segment_publish_kernel(const double* lp, const int64_t* off,
                                                              int32_t n_nodes, int* status,
                                                              double* res, double* out,
                                                              unsigned long long seq, int* ticket,
                                                              int* counters, int32_t m_tab,
                                                              int64_t n_tab, int check_rare) {
  __shared__ int last;
  const int lane = threadIdx.x & 63;
  const int nwv = (int)gridDim.x * 4;  // waves; wave w sums nodes w, w + nwv, ...
  const int j0 = blockIdx.x * 4 + (threadIdx.x >> 6);
  // (written by the call's earlier kernels: stream order)
  const bool pending = check_rare && counters[1] > 0;
  double sum = 0.0;  // (the diagnostic build's: one node per wave)
#if WFPT_PUB_DIAG
  for (int j = pending ? n_nodes : j0; j < n_nodes; j += nwv)
    sum = node_sum(lp, off, j, m_tab, n_tab, lane);
#else
  // wave w sums nodes w, w + nwv, ..., kPubNodes of them at a time
  for (int j = pending ? n_nodes : j0; j < n_nodes; j += kPubNodes * nwv) {
    int32_t vj[kPubNodes];
    bool on[kPubNodes];
    double sums[kPubNodes];
#pragma unroll
    for (int b = 0; b < kPubNodes; ++b) {
      vj[b] = j + b * nwv;
      on[b] = vj[b] < n_nodes;
    }
    node_sums<kPubNodes>(lp, off, vj, on, m_tab, n_tab, lane, sums);
    if (lane == 0) {  // (1)
#pragma unroll
      for (int b = 0; b < kPubNodes; ++b)
        if (on[b]) __hip_atomic_store(&res[vj[b]], sums[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
#endif
  // the storing wave waits for its agent-scope stores (and status atomics) to
  // be performed: LLVM's workgroup barrier does not wait for other waves'
  // vector memory operations (non-tgsplit gfx950 emits only lgkmcnt(0) before
  // s_barrier), and thread 0's release below waits only for its own wave's
  if (!WFPT_PUB_DIAG) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // (2)
  if (threadIdx.x == 0)  // (3)
    last = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
           (int)gridDim.x - 1;
  __syncthreads();  // (4)
  if (pending) {  // the host settles the rare trials and publishes again
    if (!last) return;
    if (threadIdx.x == 0) {
      *ticket = 0;
      out[n_nodes] = kRarePending;
    }
    __syncthreads();
    if (threadIdx.x == 0)
      publish_word(reinterpret_cast<unsigned long long*>(out + n_nodes + 1), seq);
    return;
  }
#if WFPT_PUB_DIAG
  if (!last) {
    for (int r = 0; r < 20; ++r) __builtin_amdgcn_s_sleep(127);
    if (j0 < n_nodes && lane == 0) out[j0] = sum;  // after the word: stale reads follow
    return;
  }
  if (j0 < n_nodes && lane == 0) out[j0] = sum;
#else
  if (!last) return;
  // plain loads: every block's stores happen-before them (the acquire above
  // invalidates this XCD's caches at agent scope); sixteen in flight per
  // thread, then the stores (the compiler does not move a load of res above a
  // store to out: they may alias)
  for (int k0 = threadIdx.x; k0 < n_nodes; k0 += 16 * 256) {
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = k0 + 256 * u < n_nodes ? res[k0 + 256 * u] : 0.0;
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (k0 + 256 * u < n_nodes) out[k0 + 256 * u] = v[u];
  }
#endif
  if (threadIdx.x == 0) {
    *ticket = 0;
    counters[0] = 0;
    counters[1] = 0;  // the rare list's count
    counters[2] = 0;
    const int st = atomicExch(status, 0);
    out[n_nodes] = (double)(st & kFlagDepth) + ((st & kFlagBudget) ? kBudgetUnit : 0.0);
  }
  __syncthreads();  // (5)
  if (threadIdx.x == 0)
    publish_word(reinterpret_cast<unsigned long long*>(out + n_nodes + 1), seq);
}

// Node all-reduce (wfpt_wiener_like_nodes_allreduce): the encoded error
// count of this rank's node pass appended to its per-node sums (res[n]),
// status reset; or a failed rank's poisoned vector {0 ..., kPeerFailUnit}.
__global__ __launch_bounds__(64) void node_status_kernel(double* res, int32_t n, int* status,
                                                         int poison, int* counters) {
  if (threadIdx.x == 0) {
    counters[0] = 0;  // the node path's n_defer words: 0 at rest
    counters[1] = 0;
    counters[2] = 0;
    const int st = atomicExch(status, 0);
    res[n] = poison ? kPeerFailUnit
                    : (double)(st & kFlagDepth) + ((st & kFlagBudget) ? kBudgetUnit : 0.0);
  }
}
__global__ __launch_bounds__(256) void node_poison_kernel(double* res, int32_t n) {
  for (int j = blockIdx.x * 256 + threadIdx.x; j < n; j += gridDim.x * 256) res[j] = 0.0;
}
// The all-reduced vector (n sums + the error count) to mapped memory, then
// the completion word out[n + 1].
__global__ __launch_bounds__(256) void publish_vec_kernel(const double* res, int32_t n,
                                                          double* out, unsigned long long seq) {
  for (int j = threadIdx.x; j <= n; j += 256) out[j] = res[j];
  __syncthreads();  // every thread's stores happen-before thread 0's release
  if (threadIdx.x == 0) publish_word(reinterpret_cast<unsigned long long*>(out + n + 1), seq);
}

// ---------------------------------------------------------------------------
// Per-node parameters (wfpt_wiener_like_nodes): trials of node j use P[j].
// The dataset is grouped by node, so a 256-trial block spans a short run of
// node ids; their parameter rows (P is the mapped pinned table the host
// filled for this call) are staged once per block in LDS and every trial
// reads its row there. Blocks spanning more than kStageRows ids (empty nodes
// between) read the table directly.
constexpr int kStageRows = 256;
// node_fast_kernel: root grids staged per block for up to this many nodes
// (WFPT_NODE_L0T; a block of 256 stored trials spans 2 HDDM nodes of 250)
#ifndef WFPT_NODE_L0T
#define WFPT_NODE_L0T 0
#endif
constexpr int kNodeGridRows = 4;

template <int STK>
struct StackOf {
  using type = typename std::conditional<
      STK == 0, RegStack<2>,
      typename std::conditional<STK == 1, RegStack<4>, MemStack<WFPT_MAX_DEPTH>>::type>::type;
};


template <int STK, bool COUNT>
__global__ __launch_bounds__(kBlock, WFPT_SLOW_WAVES) void node_kernel(
    const double* x, const int32_t* node, int64_t n, const Params* P, Knobs K, double* lp,
    unsigned long long* evals, int* status) {
  exp_table_init();
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
// in LDS as in node_kernel) and per-trial log p out. Adaptive families: a wave
// (64 consecutive stored trials: a chunk) with a trial that needs refinement
// or the exact path appends its chunk id to a dense list (one atomic per
// wave), which node_chunk_kernel completes 64 trials per wave. Direct family:
// the rare exact-path trials are appended as (index, parameter row) records
// for node_slow_kernel.
// node_fast_kernel's level 0 without f[] (WFPT_NODE_KEEP_F=0; the deferred
// chunks' level 0 is redone by node_chunk_kernel)
#ifndef WFPT_NODE_KEEP_F
#define WFPT_NODE_KEEP_F 1
#endif
template <int MODE, bool COUNT>
__global__ __launch_bounds__(kBlock, FastWaves<MODE>::value > 0 ? FastWaves<MODE>::value : 1)
void node_fast_kernel(const double* x, const int32_t* node, int64_t n, const Params* P, Knobs K,
                      double* lp, int64_t* d_idx, Params* d_par, int* n_defer, int* clist,
                      int* n_chunks, unsigned long long* evals, int* status, int* prof,
                      int32_t n_nodes, int64_t nw_tab, NodeRare R) {
#ifdef WFPT_NODE_DEBUG_FAST
  const long long dbg_t0 = __builtin_amdgcn_s_memrealtime();
#endif
  exp_table_init();
  // parameter table blockIdx.y (multi-table calls: T tables x the same
  // trials): its rows, its terms lp[t n + i], its records' virtual indices
  // t n + i and its chunks' ids t nw_tab + c
  const int64_t tab = blockIdx.y;
  double* const lp0 = lp;
  P += tab * n_nodes;
  lp += tab * n;
  const int64_t vbase = tab * n, cbase = tab * nw_tab;
  __shared__ Params rows[kStageRows];
  __shared__ RootGrids grids[kNodeGridRows];
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
  // the full DDM with few nodes per block: each staged node's root z grids and
  // sine tables once per block (root_grids: the engine's zgrid_of operations),
  // and the lean pass's level 0 over them (eng_level0_t, the same bits as the
  // engine's level 0) instead of a grid set up per lane
  const bool gridded = WFPT_NODE_L0T && MODE == kAdaptTZ && staged && span <= kNodeGridRows;
  if (gridded) {
    if ((int)threadIdx.x < span) root_grids(rows[threadIdx.x], grids[threadIdx.x]);
    __syncthreads();
  }
  long long ne = 0;
  bool defer = false;
  Params Q;
  int nj = 0;
  if (i < n) {
    nj = node[i];
    Q = staged ? rows[nj - first] : P[nj];
    double p, f[5];
    int flags = 0;
    unsigned pend;
    int oc;
    if (gridded) {
      const double xi = x[i];
      const bool flip = xi > 0;
      const RootGrids& R = grids[nj - first];
      oc = eng_level0_t<MODE, false, true>(trial_setup_b(xi, Q, flip), Q, K, R.G[flip], p, f, ne,
                                           pend, WFPT_SIN_TABLE ? &R.S[flip][0][0] : nullptr);
    } else {
      oc = fast_level0<MODE, WFPT_NODE_KEEP_F != 0>(x[i], Q, K, p, f, ne, flags, pend);
    }
    if (oc == kFinal) lp[i] = node_logp(p, Q, K);
    else defer = true;
  }
  const unsigned long long b = __ballot(defer);
  if (b) {
    if (MODE == kDirect) {
      // the rare exact-path trials (near-ties, densities below kExactBelow:
      // fast_level0's kExact) go to the rare list; the summing kernel settles
      // them with exact_pdf -- what full_pdf + settle gives such a trial
      if (defer) {
        rare_push(R, vbase + i, (int32_t)(tab * n_nodes + nj), kRareExact, lp0);
        if (COUNT) ne = 0;  // (the summing kernel counts the exact path's evaluations)
      }
    } else {
      // the chunk for node_chunk_kernel and the trials as records for
      // node_engine_kernel (fast-pass records counted in n_chunks[2])
      int base = 0;
      if (lane == 0) {
        clist[atomicAdd(n_chunks, 1)] = (int)(cbase + (i >> 6));
        base = atomicAdd(n_chunks + 2, __popcll(b));
      }
      base = __shfl(base, 0, 64);
      if (defer) {
        const int k = base + __popcll(b & lanemask_lt(lane));
        d_idx[k] = vbase + i;
        d_par[k] = Q;
      }
    }
  }
#ifdef WFPT_NODE_DEBUG_FAST
  // diagnostic builds: lane 0's term of every wave is replaced by
  // -(1e6 + the wave's elapsed 100 MHz ticks) (tools/node_fast_debug.py)
  if (lane == 0 && i < n)
    lp[i] = -(1e6 + (double)(__builtin_amdgcn_s_memrealtime() - dbg_t0));
#endif
  if (COUNT) {
    ne = wave_sum_ll((defer && MODE != kDirect) ? 0 : ne);
    if (lane == 0) {
      atomicAdd(evals, (unsigned long long)ne);
      if (b && MODE != kDirect) atomicAdd(&prof[3], __popcll(b));
    }
  }
}

// Split per-node level 0 (the adaptive t families: kAdaptT, kAdaptTZ -- the
// full DDM of config 4). A batched node call of ~100k trials is ~1.5k waves:
// fewer than the chip's SIMDs, so node_fast_kernel's one-lane-per-trial level
// 0 lasts one wave's latency (25 dependent evaluations per lane). Here block c
// takes chunk c (64 stored trials) with kNodeSplit = 5 waves: wave j evaluates
// t node j of all 64 trials (l0_node: the function of the per-lane loop and of
// the split units, bit-identical to it; j is wave-uniform), on the trial's
// node row (the mapped table) and its root z grid (zgrid_setup per lane, as
// fast_level0). Then wave 0 takes one trial per lane again: the root
// stop test and value from the five node values (l0_finish, as
// small_split_kernel), the term, and -- exactly as node_fast_kernel -- a chunk
// with a trial that refines or needs the exact path is listed for
// node_chunk_kernel with its deferred trials as records.
constexpr int kNodeSplit = 5;
template <int MODE>
__global__ __launch_bounds__(kNodeSplit * 64) void node_split_kernel(
    const double* x, const int32_t* node, int64_t n, const Params* P, Knobs K, double* lp,
    int64_t* d_idx, Params* d_par, int* clist, int* n_chunks) {
  exp_table_init();
  static_assert(MODE == kAdaptT || MODE == kAdaptTZ, "t-node split");
  __shared__ double sf[kNodeSplit][64];
  __shared__ int sfl[kNodeSplit][64];
  __shared__ int spd[kNodeSplit][64];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t c = blockIdx.x;
  const int64_t i = c * 64 + lane;
  const bool own = i < n;
  const double x0 = own ? x[i] : 0.0;
  const int nj = own ? node[i] : 0;
  const Params Q = P[nj];  // the mapped table the host filled for this call
  const Trial tr = trial_setup(x0, Q);
  double y = 0.0;
  int flags = 0;
  bool pj = false;
  if (own && tr.valid) {
    double lb, ub;
    tree_root<MODE>(tr, Q, lb, ub);
    const L0Hints H = l0_hints(tr.x, lb, ub, Q.a, K.err);
    long long ne = 0;
    // the trial's root z grid per lane, as fast_level0 builds it (the
    // large-time sines by the per-lane recurrence: no table loads in the
    // series loop)
    ZGrid G{};
    if (MODE == kAdaptTZ) G = zgrid_setup(tr.z - tr.sz / 2., tr.z + tr.sz / 2., tr.v, Q.sv, Q.a);
    y = l0_node<MODE>(tr, Q, K, lb, ub, H, wv, G, flags, pj, ne, nullptr);
  }
  sf[wv][lane] = y;
  sfl[wv][lane] = flags;
  spd[wv][lane] = pj ? 1 : 0;
  __syncthreads();
  if (wv != 0) return;
  int fl = 0;
  unsigned pd = 0u;
#pragma unroll
  for (int q = 0; q < kNodeSplit; ++q) {
    fl |= sfl[q][lane];
    if (spd[q][lane]) pd |= 1u << (q * (kTreeW / 4));
  }
  const double f[5] = {sf[0][lane], sf[1][lane], sf[2][lane], sf[3][lane], sf[4][lane]};
  double p = 0.0;
  int oc = kFinal;
  if (own) oc = l0_finish<MODE>(tr, Q, K, fl, pd, f, p);
  const bool defer = own && oc != kFinal;
  if (own && !defer) lp[i] = node_logp(p, Q, K);
  const unsigned long long b = __ballot(defer);
  if (b) {  // node_fast_kernel's listing: the chunk, and its deferred trials as records
    int base = 0;
    if (lane == 0) {
      clist[atomicAdd(n_chunks, 1)] = (int)c;
      base = atomicAdd(n_chunks + 2, __popcll(b));
    }
    base = __shfl(base, 0, 64);
    if (defer) {
      const int k = base + __popcll(b & lanemask_lt(lane));
      d_idx[k] = i;
      d_par[k] = Q;
    }
  }
}

// Speculative record (non-counting node calls of the adaptive t families,
// with the call's node tables): a deferred trial of a sparse call is one
// wave's work, and the breadth-first rounds (node_records) walk its tree
// level by level -- six or more dependent rounds of one grid evaluation each.
// Here the wave evaluates EVERY value the reference's recursion can reach at
// n_st = n_sz = kTreeDepth in two rounds: the 17 dyadic t points x the 4 z
// grids (kAdaptTZ; kAdaptT: the 17 t points), plus the level-0 t points' root
// grids once more with the level-0 hints, exactly as the engine evaluates
// them (its stage-0 tasks of level 0 take l0_hints, its z walks do not).
// Then 17 lanes settle each t point's value as the engine's task completion
// does (the root test, simp_value, or the z walk's tree17 over its 17
// values), and lane 0 runs tree17 over the t points. Only the points that
// recursion reads (tree17's `used`) contribute their flags (ambiguous
// decisions, ties, deeper trees), so the trial's density and its deferral
// are the engine's; the extra values are never read. LDS: buf (>= 314
// doubles: the walk values and the hinted root grids), tv (17 t values),
// pf (>= 39 ints of point flags); lp[i] gets the node term.
constexpr int kOvfBit = 1 << 8;  // a grid's drift factor overflowed (literal values)
// The record's tables (eng_tables_wave's values) built by a team of NW waves:
// with NW = 4 each wave computes one group (the 8 z grids, the t points, the
// z points, the interval reciprocals), so the divergent groups run side by
// side instead of one after another.
template <int NW>
__device__ inline void eng_tables_team(const Params& P, EngTables& T, int wave, int lane) {
  if (NW == 1) {
    eng_tables_wave(P, T, lane);
    return;
  }
  constexpr int kP = kTreePoints;
  if (wave == 0) {
    if (lane < 8) {
      const int flip = lane >> 2, sel = lane & 3;
      const double zf = flip ? 1. - P.z : P.z, vf = flip ? -P.v : P.v;
      T.G[flip][sel] = zgrid_of(zf - P.sz / 2., zf + P.sz / 2., sel, vf, P.sv, P.a);
    }
  } else if (wave == 1) {
    if (lane < kP) T.tP[lane] = dyadic_point(P.t - P.st / 2., P.t + P.st / 2., lane);
  } else if (wave == 2) {
    if (lane < 2 * kP) {
      const int flip = lane / kP, k = lane % kP;
      const double zf = flip ? 1. - P.z : P.z;
      T.zP[flip][k] = dyadic_point(zf - P.sz / 2., zf + P.sz / 2., k);
    }
  } else if (lane < 2) {
    const int flip = lane;
    const double zf = flip ? 1. - P.z : P.z;
    T.iz[flip] = 1.0 / ((zf + P.sz / 2.) - (zf - P.sz / 2.));
  }
}
// WFPT_REC_FENCE: a scheduling barrier between the record's phases. Without
// them the compiler's schedule over the record's divergent phases makes the
// call's records 1.5x slower (node_chunk_kernel 24.0 -> 15.6 us at config 4's
// generating parameters, same code otherwise).
#ifndef WFPT_REC_FENCES
#define WFPT_REC_FENCES 1
#endif
#if WFPT_REC_FENCES
#define WFPT_REC_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define WFPT_REC_FENCE() ((void)0)
#endif
template <int NW>
__device__ inline void record_sync() {
  if (NW == 1) wave_sync();
  else __syncthreads();
}
// NW waves per record (NW = 1: the wave alone; NW = kEngWaves: the block,
// every wave calling with the same record, wave = its index): the NE
// evaluations are dealt to the waves in contiguous runs of t points, so each
// wave's lanes take similar x - t (similar code paths: a round costs the
// union of its lanes' paths), and the waves evaluate side by side. The
// values, and so every output bit, are the same for any NW.
template <int MODE, int NW>
__device__ inline void node_record_spec(double* buf, double* tv, int* pf, EngTables& T, int wave,
                                        int lane, const double* x, const Knobs& K, double* lp,
                                        int64_t i, const Params& Q, const NodeRare& R,
                                        double* lp_base, int64_t v, int32_t vj,
                                        long long dbg_entry = 0) {
  constexpr int NP = kTreePoints;
  constexpr int NG = MODE == kAdaptTZ ? 4 : 1;  // grids per t point
  constexpr int NE = NP * NG + (MODE == kAdaptTZ ? 5 : 0);
  constexpr int kPer = (NE + NW - 1) / NW;  // evaluations per wave (NW > 1: one trip)
  static_assert(NW == 1 || kPer <= 64, "record team");
  double* zv = buf;             // [NP][NP] the unhinted grids' values (the z walks)
  double* hv = buf + NP * NP;   // [5][5] the hinted root grids of the level-0 t points
  int* fu = pf;                 // [NP] unhinted root grid: kFlagExact (ambiguous) | kOvfBit
  int* fh = pf + NP;            // [5] hinted root grid: the same
  int* fp = pf + NP + 5;        // [NP] the t point's settled flags
  const double x0 = x[i];
  const Trial tr = trial_setup(x0, Q);
  if (!tr.valid) {  // (never deferred: p = 0 settles at level 0)
    if (wave == 0 && lane == 0) lp[i] = node_logp(0.0, Q, K);
    return;
  }
#ifdef WFPT_NODE_DEBUG
  const long long dbg0 = __builtin_amdgcn_s_memrealtime();
#endif
  WFPT_REC_FENCE();
  eng_tables_team<NW>(Q, T, wave, lane);  // the record's tables in LDS
  record_sync<NW>();
#ifdef WFPT_NODE_DEBUG
  const long long dbg1 = __builtin_amdgcn_s_memrealtime();
#endif
  WFPT_REC_FENCE();
  const int flip = x0 > 0 ? 1 : 0;
  const double a = Q.a, sv = Q.sv;
  const double iwt = 1.0 / (T.tP[kTreeW] - T.tP[0]);
  const double ia2 = 1.0 / (a * a);  // as l0_hints / refine_rounds
  const L0Hints H = l0_hints(tr.x, T.tP[0], T.tP[kTreeW], a, K.err);
  const double izf = T.iz[flip];
  const int e_lo = NW == 1 ? 0 : wave * kPer;
  const int e_hi = NW == 1 ? NE : ((wave + 1) * kPer < NE ? (wave + 1) * kPer : NE);
  for (int e0 = e_lo; e0 < e_hi; e0 += 64) {
    const int e = e0 + lane;
    if (e >= e_hi) continue;
    int k, gs, jh = -1;
    if (e < NP * NG) {
      k = e / NG;
      gs = e - k * NG;
      if (MODE == kAdaptT && (k & 3) == 0) jh = k >> 2;  // kAdaptT level 0: hinted
    } else {
      jh = e - NP * NG;
      k = jh * (kTreeW / 4);
      gs = kGridRoot;
    }
    double qh = -1.0;
    bool known = false;
    Decision kd{0, 0, 0};
    if (jh >= 0) {
      qh = H.qh(jh);
      known = jh == 0 ? H.ok0 : (jh == 4 ? H.ok4 : H.shared);
      kd = jh == 4 ? H.D4 : H.D0;
    }
    const TNode N = tnode_setup_r(tr.x - T.tP[k], tr.v, sv, a, ia2, K.err, qh, known, kd);
    const int amb = N.amb ? (int)kFlagExact : 0;
    if (MODE == kAdaptT) {
      tv[k] = tnode_pdf_sv(N, tr.z, tr.v, sv, a) * iwt;
      fp[k] = amb;
    } else {
      double y[5];
      const bool ok = tnode_pdf_sv_grid5(N, T.G[flip][gs], tr.v, sv, a, y);  // literal values
      if (jh < 0) {
#pragma unroll
        for (int j = 0; j < 5; ++j)
          if (grid_owns(gs, j)) zv[k * NP + grid_point(gs, j)] = y[j] * izf;
        if (gs == kGridRoot) fu[k] = amb | (ok ? 0 : kOvfBit);
      } else {
#pragma unroll
        for (int j = 0; j < 5; ++j) hv[jh * 5 + j] = y[j] * izf;
        fh[jh] = amb | (ok ? 0 : kOvfBit);
      }
    }
  }
  record_sync<NW>();
#ifdef WFPT_NODE_DEBUG
  const long long dbg2 = __builtin_amdgcn_s_memrealtime();
#endif
  WFPT_REC_FENCE();
  if (MODE == kAdaptTZ && wave == 0 && lane < NP) {
    // t point k's task completion (refine_rounds stage 0): the root test on
    // its root grid (hinted at level 0), then -- if it refines or the grid
    // overflowed -- the z walk over the unhinted grids
    const int k = lane;
    const bool l0 = (k & 3) == 0;
    const double* r = l0 ? hv + (k >> 2) * 5 : nullptr;
    const double r0 = l0 ? r[0] : zv[k * NP], r1 = l0 ? r[1] : zv[k * NP + 4],
                 r2 = l0 ? r[2] : zv[k * NP + 8], r3 = l0 ? r[3] : zv[k * NP + 12],
                 r4 = l0 ? r[4] : zv[k * NP + 16];
    const int rf = l0 ? fh[k >> 2] : fu[k];
    const ZGrid& gr = T.G[flip][kGridRoot];
    const Simp sm = simp5p(gr.h6, gr.h12, r0, r1, r2, r3, r4);
    int f = 0;
    const bool ovf = (rf & kOvfBit) != 0;
    const bool pend = simpson_refine(sm.S, sm.S2, K.simps_err, K.n_sz, f) || ovf;
    if (ovf) f = 0;
    int flags = (rf & kFlagExact) | f;
    double val;
    if (!pend) {
      val = simp_value(sm) * iwt;
    } else {
      flags |= fu[k] & kFlagExact;  // the walk's own (unhinted) t node
      const double(&zk)[kTreePoints] =
          *reinterpret_cast<const double(*)[kTreePoints]>(zv + k * NP);
      int f2 = 0, nref = 0;
      unsigned need = 0u;
      const double zi = tree17(zk, T.zP[flip], K.simps_err, K.n_sz, kTreeDepth, f2, need, nref);
      if (need) f2 |= kFlagFallback;  // z tree deeper than the walk's levels
      flags |= f2 & (kFlagExact | kFlagFallback);
      val = zi * iwt;
    }
    tv[k] = val;
    fp[k] = flags;
  }
  if (wave == 0) wave_sync();
#ifdef WFPT_NODE_DEBUG
  const long long dbg3 = __builtin_amdgcn_s_memrealtime();
#endif
  WFPT_REC_FENCE();
  if (wave == 0 && lane == 0) {
    const double(&tk)[kTreePoints] = *reinterpret_cast<const double(*)[kTreePoints]>(tv);
    unsigned need = 0u, used = 0u;
    int fl = 0, nref = 0;
    double p = tree17(tk, T.tP, K.simps_err, K.n_st, kTreeDepth, fl, need, nref, &used);
#pragma unroll 1
    for (int k = 0; k < NP; ++k)
      if ((used >> k) & 1u) fl |= fp[k];
    if (need) fl |= kFlagFallback;  // t tree deeper than kTreeDepth
    fl &= kFlagExact | kFlagFallback;
    // tree_density's settlement
    const bool structural = tr.x - T.tP[0] <= 0;
    bool defer = fl != 0 || !(p > kExactBelow || structural);
    if (defer && fl == 0 && tiny_absorbed(p, Q.p_outlier, K.w_outlier)) {
      defer = false;
      p = 0.0;
    }
    // the rare list (node_sum settles it): the exact path, or the per-lane
    // walk for a tree deeper than kTreeDepth
    if (defer)
      rare_push(R, v, vj, (fl & kFlagExact) || fl == 0 ? kRareExact : kRareWalk, lp_base);
    else
      lp[i] = node_logp(p, Q, K);
#if defined(WFPT_NODE_DEBUG) && !defined(WFPT_NODE_DEBUG_NOOUT)
    // diagnostic builds: the record's phase times (100 MHz ticks: tables,
    // evaluations, z settlement, t tree + settlement) in place of its term
    const long long dbg4 = __builtin_amdgcn_s_memrealtime();
    lp[i] = -((double)(dbg1 - dbg0) * 1e12 + (double)(dbg2 - dbg1) * 1e8 +
              (double)(dbg3 - dbg2) * 1e4 + (double)(dbg4 - dbg3));
#ifdef WFPT_NODE_DEBUG_ENTRY
    // the kernel's entry -> record start and the record's total instead
    lp[i] = -((double)(dbg0 - dbg_entry) * 1e8 + (double)(dbg4 - dbg0));
#endif
#endif
  }
  record_sync<NW>();  // the next record reuses the LDS
}

// The node path's completion of the chunks node_fast_kernel listed: one wave
// per chunk, as the dataset engine (engine_kernel) runs a chunk, per node
// segment of the chunk (nodes are contiguous and |rt|-ordered: a chunk holds
// one node, or the end of one and the start of the next). Per segment: the
// node's parameter row (wave-uniform), its tables built by the lanes in
// parallel into the wave's LDS (eng_tables_wave), level 0 per lane on the
// segment's trials, the in-wave refinement rounds over all of them together,
// then each trial's density (tree17 over its values; the exact path or the
// per-lane walk for the rare trials the rounds hand on) and its term. Every
// trial of a listed chunk is rewritten (the same level-0 operations as the
// fast pass), so a chunk's terms do not depend on which lanes deferred.
// A call where most trials refine (an MCMC proposal far in the tails) runs
// 64 trials per wave this way; when the deferred trials are sparse in their
// chunks (node_records_sparse: the usual MCMC call) the same launch runs the
// fast pass's records one wave each instead (node_records), which skips the
// level 0 of the chunks' settled trials. Trials the rounds hand on (the exact
// path, trees deeper than kTreeDepth) are settled on their own lane (rare).
// WFPT_NODE_REC_TEAM: a speculative record is one block's work (its waves
// evaluate side by side), else one wave's.
#ifndef WFPT_NODE_REC_TEAM
#define WFPT_NODE_REC_TEAM 1
#endif
// Team records (one block each, ~12 us) while the call's records fit in one
// round of resident blocks (2 per CU: the kernel's 68 KB of LDS); beyond, one
// wave per record (~21 us, but 4x as many side by side): multi-table calls of
// several chains defer thousands of trials
#ifndef WFPT_REC_TEAM_MAX
#define WFPT_REC_TEAM_MAX 512
#endif
// waves per SIMD the node chunk engine is compiled for (register budget)
#ifndef WFPT_NODE_CHUNK_WAVES
#define WFPT_NODE_CHUNK_WAVES 2
#endif
template <int MODE, bool COUNT>
__global__ __launch_bounds__(kEngBlock, WFPT_NODE_CHUNK_WAVES) void node_chunk_kernel(
    const double* x, const int32_t* node, int64_t n, const Params* P, Knobs K, double* lp,
    const int* clist, const int* n_chunks, const int64_t* r_idx, const Params* r_par,
    unsigned long long* evals, int* status, int* prof, int spec, int32_t n_nodes,
    int64_t nw_tab, NodeRare R) {
#ifdef WFPT_NODE_DEBUG
  const long long dbg_entry = __builtin_amdgcn_s_memrealtime();
#else
  const long long dbg_entry = 0;
#endif
  exp_table_init();
  __shared__ ChunkLds<1> lds[kEngWaves];
  const int lane = threadIdx.x & 63;
  ChunkLds<1>& cl = lds[threadIdx.x >> 6];
  const int nc = n_chunks[0], nrec = n_chunks[2];
  const int nwaves = (int)gridDim.x * kEngWaves;
  const int w0 =
      __builtin_amdgcn_readfirstlane((int)blockIdx.x * kEngWaves + (int)(threadIdx.x >> 6));
  if (node_records_sparse(nrec, nc)) {  // a few deferred trials: one wave each
    if constexpr (!COUNT && (MODE == kAdaptT || MODE == kAdaptTZ)) {
      if (spec) {  // every tree point in two rounds (node_record_spec)
        if (WFPT_NODE_REC_TEAM && nrec <= WFPT_REC_TEAM_MAX) {
          // one block per record, its waves side by side (wave 0's LDS)
          ChunkLds<1>& c0 = lds[0];
          const int wv = threadIdx.x >> 6;
          for (int k = (int)blockIdx.x; k < nrec; k += (int)gridDim.x) {
            const int64_t v = r_idx[k];  // virtual: table t's trial i at t n + i
            const int64_t t = v / n, ix = v - t * n;
            node_record_spec<MODE, kEngWaves>(c0.F, c0.X, c0.fl, c0.tab, wv, lane, x + ix, K,
                                              lp + v, 0, r_par[k], R, lp, v,
                                              (int32_t)(t * n_nodes + node[ix]), dbg_entry);
          }
        } else {
          for (int k = w0; k < nrec; k += nwaves) {
            const int64_t v = r_idx[k];
            const int64_t t = v / n, ix = v - t * n;
            node_record_spec<MODE, 1>(cl.F, cl.X, cl.fl, cl.tab, 0, lane, x + ix, K, lp + v, 0,
                                      r_par[k], R, lp, v, (int32_t)(t * n_nodes + node[ix]),
                                      dbg_entry);  // F: 1088 doubles, fl: 64 ints
          }
        }
        return;
      }
    }
    node_records<MODE, COUNT, false>(cl, lane, w0, nwaves, x, K, lp, r_idx, r_par, nrec, evals,
                                     status, n, &R, node, n_nodes);
    return;
  }
  long long ne = 0;
  int nseg = 0, nex = 0, nwk = 0;
  Tally ty;
  for (int k = w0; k < nc; k += nwaves) {
    const int64_t vc = clist[k];  // virtual: table t's chunk c at t nw_tab + c
    const int64_t tab = vc / nw_tab;
    const int64_t c = vc - tab * nw_tab;
    const Params* Pt = P + tab * n_nodes;
    double* lpt = lp + tab * n;
    const int64_t i = c * 64 + lane;
    const bool own = i < n;
    const double x0 = own ? x[i] : 0.0;
    const int nj = own ? node[i] : -1;
    bool todo = own;
    for (unsigned long long left = __ballot(todo); left; left = __ballot(todo)) {
      // the next node segment: the node of the first lane still to do
      const int jn = __shfl(nj, __ffsll((long long)left) - 1, 64);
      const bool mine = todo && nj == jn;
      todo = todo && !mine;
      ++nseg;
      const Params Q = Pt[__builtin_amdgcn_readfirstlane(jn)];
      TrialArgs A{};
      A.x = x;
      A.n = n;
      A.P = Q;
      A.K = K;
      A.wp_outlier = K.w_outlier * Q.p_outlier;
      eng_tables_wave(Q, cl.tab, lane);
      double p = 0.0, f0[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
      long long ne0 = 0;
      unsigned pend0 = 0u;
      int oc = kFinal;
      if (mine) oc = eng_level0<MODE>(x0, Q, K, cl.tab.G[x0 > 0][kGridRoot], p, f0, ne0, pend0);
      if (__ballot(mine && oc == kTree) != 0ull) {
        cl.X[lane] = x0;
        cl.fl[lane] = (mine && oc == kTree) ? 0 : (mine && oc == kExact ? (int)kFlagExact
                                                                         : (int)kFlagIdle);
        if (COUNT) cl.cnt[lane] = (int)ne0;
        if (mine && oc == kTree) {
#pragma unroll
          for (int j = 0; j < 5; ++j) cl.F[j * (kTreeW / 4) * 64 + lane] = f0[j];
        }
        if (lane == 0) {
          cl.qn[0] = 0;
          cl.qn[1] = 0;
        }
        wave_sync();
        if (MODE == kAdaptTZ) {
#pragma unroll
          for (int j = 0; j < 5; ++j)
            team_push(mine && oc == kTree && ((pend0 >> (j * (kTreeW / 4))) & 1u),
                      lane | ((j * (kTreeW / 4)) << 6), cl.ZQ, &cl.qn[1]);
        }
        wave_sync();
        PhaseClock pc;
        Tally t1;
        refine_rounds<MODE, COUNT, 1>(A, cl, lane, 1, t1, pc);
        if (COUNT) {
          ty.t1 += t1.t1;
          ty.t2 += t1.t2;
          ty.rec += t1.rec;
          for (int q = 0; q < 3; ++q) ty.z[q] += t1.z[q];
        }
      }
      bool defer = mine && oc == kExact;
      int rf = kFlagExact;
      long long n1 = ne0;
      if (mine && oc == kTree) {
        tree_density<MODE, 1>(A, cl, lane, x0, p, defer, rf);
        if (COUNT) n1 = cl.cnt[lane];
      }
      if (defer) {  // rare: the exact path or the per-lane walk, by node_sum
        rare_push(R, tab * n + i, (int32_t)(tab * n_nodes + jn),
                  (rf & kFlagExact) ? kRareExact : kRareWalk, lp);
        n1 = 0;
        if (COUNT) ++((rf & kFlagExact) ? nex : nwk);
      }
      if (mine && !defer) {
        if (oc != kFinal) ne += n1;  // node_fast_kernel counted the trials it settled
        lpt[i] = node_logp(p, Q, K);
      }
      wave_sync();  // the next segment rebuilds this wave's LDS
    }
  }
  if (COUNT) {
    ne = wave_sum_ll(ne);
    nex = (int)wave_sum_ll(nex);
    nwk = (int)wave_sum_ll(nwk);
    if (lane == 0) {
      atomicAdd(evals, (unsigned long long)ne);
      atomicAdd(&prof[0], nseg);
      atomicAdd(&prof[5], nex);
      atomicAdd(&prof[6], nwk);
      atomicAdd(&prof[1], ty.t1);
      atomicAdd(&prof[2], ty.t2);
      atomicAdd(&prof[4], ty.rec);
      atomicAdd(&prof[7], ty.z[0] + ty.z[1] + ty.z[2]);
      atomicAdd(&prof[8], ty.z[0]);
      atomicAdd(&prof[9], ty.z[1]);
      atomicAdd(&prof[10], ty.z[2]);
    }
  }
}

// MULTI: wiener_like_multi's trial term (wfpt.pyx:266-272: the mixture with
// the call's p_outlier and a plain log, no range check) instead of a node's.
template <int MODE, int STK, bool COUNT, bool MULTI = false>
__global__ __launch_bounds__(64, WFPT_SLOW_WAVES) void node_slow_kernel(
    const double* x, Knobs K, double* lp, const int64_t* d_idx, const Params* d_par,
    const int* n_defer, unsigned long long* evals, int* status) {
  exp_table_init();
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
    lp[i] = MULTI ? log_val(p * (1 - Q.p_outlier) + (K.w_outlier * Q.p_outlier)) : node_logp(p, Q, K);
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
    double p_outlier, double* out, int* zeros, int* status, double* lpo) {
  exp_table_init();
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
    lp = log_val(p);
    if (lpo) lpo[i] = lp;
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

// wiener_like_multi's level-0 pass when the integration family is uniform
// (sz and st are scalars, adaptive): one trial per lane with its own
// parameters (per-trial arrays, or the scalars), the same fast_level0 as the
// per-node path; trials whose root test refines (or hinge on rounding) go to
// node_slow_kernel<..., MULTI> as (index, parameter row) records. |x| = 999
// trials are scored by prob_ub (wfpt.pyx:267-271). lp[i] = the trial's term.
template <int MODE, bool COUNT>
__global__ __launch_bounds__(kBlock, FastWaves<MODE>::value > 0 ? FastWaves<MODE>::value : 1)
void multi_fast_kernel(const double* x, int64_t n, const double* const* arr, const double* scal,
                       Knobs K, double p_outlier, double* lp, int64_t* d_idx, Params* d_par,
                       int* n_defer, unsigned long long* evals) {
  exp_table_init();
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int lane = threadIdx.x & 63;
  long long ne = 0;
  bool defer = false;
  Params Q;
  if (i < n) {
    double q[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) q[j] = arr[j] ? arr[j][i] : scal[j];
    Q.v = q[0];
    Q.sv = q[1];
    Q.a = q[2];
    Q.z = q[3];
    Q.sz = q[4];
    Q.t = q[5];
    Q.st = q[6];
    Q.p_outlier = p_outlier;
    const double xi = x[i];
    if (fabs(xi) != 999.) {
      double p, f[5];
      int flags = 0;
      unsigned pend;
      const int oc = fast_level0<MODE>(xi, Q, K, p, f, ne, flags, pend);
      if (oc == kFinal) lp[i] = log_val(p * (1 - p_outlier) + (K.w_outlier * p_outlier));
      else defer = true;
    } else {
      const double pu = prob_ub(Q.v, Q.a, Q.z);
      lp[i] = log_val(xi == 999. ? pu : 1 - pu);
    }
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

// Fixed-order per-block sums of per-trial terms (finalize adds the blocks).
__global__ __launch_bounds__(kBlock) void lp_sum_kernel(const double* lp, int64_t n, double* part,
                                                        int* zeros) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double s = i < n ? lp[i] : 0.0;
  int zero = 0;
  long long ne = 0;
  block_reduce<false>(s, zero, ne);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = s;
    zeros[blockIdx.x] = 0;
  }
}

static TrialArgs trial_args(const double* x, int64_t n, const Params& P, const Knobs& K,
                            double* out, int* zeros, unsigned long long* evals, int* status,
                            int logp, double* trial = nullptr) {
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
  A.trial = trial;
  return A;
}

template <int MODE, bool COUNT, int OUT>
static void run_fast(const TrialArgs& A, const Work& W, const EngTables& T, const Split& S,
                     bool lean, hipStream_t s, hipEvent_t fast_done) {
  if constexpr (MODE == kDirect) {
    if (WFPT_DIRECT_ARGS) {
      DirectArgs D;
      direct_args(A.P, D);
      hipLaunchKernelGGL((direct_kernel<COUNT, OUT>), dim3(fast_blocks(A.n)), dim3(kFastBlock), 0,
                         s, A, W, D);
    } else {
      hipLaunchKernelGGL((fast_kernel<MODE, COUNT, OUT>), dim3(fast_blocks(A.n)),
                         dim3(kFastBlock), 0, s, A, W);
    }
  } else if (lean) {
    RootGrids R;
    root_grids(A.P, R);
    hipLaunchKernelGGL((lean_kernel<MODE, COUNT, OUT>), dim3((A.n + kLeanBlock - 1) / kLeanBlock),
                       dim3(kLeanBlock), 0, s, A, W, R);
  } else {
    const int64_t units = (int64_t)(S.n + S.n2) * kSplit + (A.n + 63) / 64;
    hipLaunchKernelGGL((engine_kernel<MODE, COUNT, OUT>),
                       dim3((units + kEngWaves - 1) / kEngWaves), dim3(kEngBlock), 0, s, A, W, T,
                       S);
  }
  if (fast_done) (void)hipEventRecord(fast_done, s);
}

template <int MODE, bool COUNT, int OUT>
static void run_deferred(const TrialArgs& A, const Work& W, const EngTables& T, bool redo,
                         hipStream_t s) {
  const int64_t nw = (A.n + 63) / 64;
  if constexpr (MODE != kDirect) {
    if (redo)  // the engine over the chunks the lean pass flagged (one wave each)
      hipLaunchKernelGGL((engine_kernel<MODE, COUNT, OUT>), dim3((nw + kEngWaves - 1) / kEngWaves),
                         dim3(kEngBlock), 0, s, A, W, T, Split{});
  }
  // the fold: one wave per chunk, up to WFPT_FOLD_GRID blocks of 4
  const int64_t gf = std::min<int64_t>(WFPT_FOLD_GRID, (nw + 3) / 4);
  hipLaunchKernelGGL((fold_kernel<MODE, COUNT, OUT>), dim3(gf), dim3(256), 0, s, A, W, nw);
}

template <bool COUNT, int OUT>
static void launch_mode(int mode, int part, const TrialArgs& A, const Work& W, const Split& S,
                        hipStream_t s, hipEvent_t fast_done) {
  // the engine's tables (the lean pass alone needs only its root grids)
  EngTables T;
  const bool engine = ((part & kPassFast) && !(part & kPassLean)) || (part & kPassRedo);
  if (mode >= kAdaptT && mode <= kAdaptTZ && engine) eng_tables(A.P, T);
  // W.redo is live only in the lean and redo passes (a full engine
  // launch processes every chunk); the host never combines kPassRedo with a
  // full engine level-0 pass
  Work F = W;
  F.redo = (part & (kPassLean | kPassRedo)) ? W.redo : nullptr;
#define FAST_AND_DEFERRED(M_)                                                       \
  do {                                                                              \
    if (part & kPassFast)                                                           \
      run_fast<M_, COUNT, OUT>(A, F, T, S, (part & kPassLean) != 0, s, fast_done);        \
    if (part & kPassDeferred)                                                       \
      run_deferred<M_, COUNT, OUT>(A, F, T, (part & kPassRedo) != 0, s);            \
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
                   int logp, const Work& W, hipStream_t s, hipEvent_t fast_done,
                   const Split* split, double* trial) {
  if (n <= 0) return;
  Split S{};
  if (split) S = *split;
  const TrialArgs A = trial_args(x, n, P, K, out, zeros, evals, status, logp, trial);
  const int mode = select_mode(P.sz, P.st, K.use_adaptive);
  if (out_kind == OUT_BOTH) {  // the per-trial check (no evaluation counting)
    launch_mode<false, OUT_BOTH>(mode, part, A, W, S, s, fast_done);
    return;
  }
  if (evals) {
    if (out_kind == OUT_SUM) launch_mode<true, OUT_SUM>(mode, part, A, W, S, s, fast_done);
    else if (out_kind == OUT_ARRAY)
      launch_mode<true, OUT_ARRAY>(mode, part, A, W, S, s, fast_done);
    else launch_mode<true, OUT_LOGP>(mode, part, A, W, S, s, fast_done);
  } else {
    if (out_kind == OUT_SUM) launch_mode<false, OUT_SUM>(mode, part, A, W, S, s, fast_done);
    else if (out_kind == OUT_ARRAY)
      launch_mode<false, OUT_ARRAY>(mode, part, A, W, S, s, fast_done);
    else launch_mode<false, OUT_LOGP>(mode, part, A, W, S, s, fast_done);
  }
}

int launch_small(const double* x, int64_t n, const Params& P, const Knobs& K, double* part,
                 int* zeros, int* status, const Work& W, double* out, unsigned long long seq,
                 int* tree_any, hipStream_t s, double* trial) {
  if (n <= 0 || n > kFastBlock) return kSmallNone;
  const int mode = select_mode(P.sz, P.st, K.use_adaptive);
  if (mode > kAdaptTZ) return kSmallNone;
  const TrialArgs A = trial_args(x, n, P, K, part, zeros, nullptr, status, 0, trial);
  Work F = W;
  F.redo = mode == kDirect ? nullptr : W.redo;
  RootGrids R{};
  if (mode != kDirect) root_grids(P, R);
  const FinArgs Fa{status, out, seq, tree_any, 1};
#define SMALL_MODES(O_)                                                                      \
  switch (mode) {                                                                            \
    case kDirect:                                                                            \
      hipLaunchKernelGGL((small_kernel<kDirect, O_>), dim3(1), dim3(kFastBlock), 0, s, A, F, R, \
                         Fa);                                                                \
      break;                                                                                 \
    case kAdaptT:                                                                            \
      hipLaunchKernelGGL((small_kernel<kAdaptT, O_>), dim3(1), dim3(kFastBlock), 0, s, A, F, R, \
                         Fa);                                                                \
      break;                                                                                 \
    case kAdaptZ:                                                                            \
      hipLaunchKernelGGL((small_kernel<kAdaptZ, O_>), dim3(1), dim3(kFastBlock), 0, s, A, F, R, \
                         Fa);                                                                \
      break;                                                                                 \
    default:                                                                                 \
      if (WFPT_SMALL_SPLIT)                                                                  \
        hipLaunchKernelGGL((small_split_kernel<kAdaptTZ, O_>), dim3(1), dim3(kSplitBlock), 0, s, \
                           A, F, R, Fa);                                                     \
      else                                                                                   \
        hipLaunchKernelGGL((small_kernel<kAdaptTZ, O_>), dim3(1), dim3(kFastBlock), 0, s, A, F, \
                           R, Fa);                                                           \
      break;                                                                                 \
  }
  if (trial) {
    SMALL_MODES(OUT_BOTH)
  } else {
    SMALL_MODES(OUT_SUM)
  }
#undef SMALL_MODES
  return (mode == kAdaptTZ && WFPT_SMALL_SPLIT) ? kSmallSplit : kSmallOne;
}

void launch_finalize(const double* part, const int* zeros, int64_t nb, int defer_bits,
                     int* status, double* out, unsigned long long seq, hipStream_t s,
                     const int* split_rd, int* split_rs, int* tree_any, double* mirror,
                     double* fin, int* ticket) {
  int64_t g = 1;
  if (fin && ticket && nb > 2 * kFinPerBlock)
    g = std::min<int64_t>(kFinMaxBlocks, (nb + kFinPerBlock - 1) / kFinPerBlock);
  hipLaunchKernelGGL(finalize_kernel, dim3((unsigned)g), dim3(1024), 0, s, part, zeros, nb,
                     defer_bits, status, out, seq, split_rd, split_rs, tree_any, mirror, fin,
                     ticket);
}

template <int MODE, bool COUNT>
static void launch_nodes_two_pass(const double* x, const int32_t* node, int64_t n,
                                  const Params* P, const Knobs& K, double* lp, int64_t* d_idx,
                                  Params* d_par, int* n_defer, int* clist,
                                  unsigned long long* evals, int* status, int* prof,
                                  hipStream_t s, const NodeTables* nt) {
  bool split = false, spec = false;
  const int T = nt ? std::max(nt->n_tables, 1) : 1;
  const int32_t m = nt ? nt->n_nodes : 0;
  const int64_t nw = (n + 63) / 64;
  if constexpr ((MODE == kAdaptT || MODE == kAdaptTZ) && !COUNT) {
    spec = nt && nt->spec;
    if (nt && nt->split && nt->n_nodes > 0 && T == 1) {
      // the call's node tables, then the t-node split level 0; the chunk
      // engine / records below read the device copy of the rows
      hipLaunchKernelGGL((node_split_kernel<MODE>), dim3((n + 63) / 64), dim3(kNodeSplit * 64), 0,
                         s, x, node, n, P, K, lp, d_idx, d_par, clist, n_defer);
      split = true;
    }
  }
  const NodeRare R{nt ? nt->rare_v : nullptr, nt ? nt->rare_j : nullptr, n_defer + 1};
  if (!split)
    hipLaunchKernelGGL((node_fast_kernel<MODE, COUNT>), dim3(blocks_for(n), T), dim3(kBlock), 0, s,
                       x, node, n, P, K, lp, d_idx, d_par, n_defer, clist, n_defer, evals, status,
                       prof, m, nw, R);
  if constexpr (MODE != kDirect) {
    // adaptive families, one launch: the fast pass's records one wave each
    // when they are sparse in their chunks, else one wave per listed chunk
    // (node_chunk_kernel reads the counts and picks)
    const int64_t nb = std::min<int64_t>((T * nw + kEngWaves - 1) / kEngWaves, 2048);
    hipLaunchKernelGGL((node_chunk_kernel<MODE, COUNT>), dim3(nb), dim3(kEngBlock), 0, s, x, node,
                       n, P, K, lp, clist, n_defer, d_idx, d_par, evals, status, prof,
                       spec ? 1 : 0, m, nw, R);
  }
  // direct family: node_fast_kernel settles its exact-path trials itself
}

template <bool COUNT>
static void launch_nodes_mode(int mode, const double* x, const int32_t* node, int64_t n,
                              const Params* P, const Knobs& K, double* lp, int64_t* d_idx,
                              Params* d_par, int* n_defer, int* clist,
                              unsigned long long* evals, int* status, int* prof, hipStream_t s,
                              const NodeTables* nt) {
#define TWO_PASS(M_)                                                                           \
  launch_nodes_two_pass<M_, COUNT>(x, node, n, P, K, lp, d_idx, d_par, n_defer, clist, evals,  \
                                   status, prof, s, nt)
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
                  int* n_defer, int* clist, unsigned long long* evals, int* status, int* prof,
                  hipStream_t s, const NodeTables* nt) {
  const int64_t nb = blocks_for(n);
  if (nb == 0) return;
  if (mode >= kDirect && mode <= kAdaptTZ) {
    if (evals)
      launch_nodes_mode<true>(mode, x, node, n, P, K, lp, d_idx, d_par, n_defer, clist, evals,
                              status, prof, s, nt);
    else
      launch_nodes_mode<false>(mode, x, node, n, P, K, lp, d_idx, d_par, n_defer, clist, evals,
                               status, prof, s, nt);
    return;
  }
  const int stk = stack_kind(K);
  // mixed families: the generic per-trial kernel once per parameter table
  const int T = nt ? std::max(nt->n_tables, 1) : 1;
  for (int t = 0; t < T; ++t) {
    const Params* Pt = P + (int64_t)t * (nt ? nt->n_nodes : 0);
    double* lpt = lp + (int64_t)t * n;
#define NODE_LAUNCH(S_, C_)                                                                     \
  hipLaunchKernelGGL((node_kernel<S_, C_>), dim3(nb), dim3(kBlock), 0, s, x, node, n, Pt, K, \
                     lpt, evals, status)
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
}

void launch_segment_res(double* lp, const int64_t* off, int32_t n_nodes, double* res,
                        int* status, bool poison, hipStream_t s, int* counters,
                        const NodeSum* ns) {
  if (poison) {
    hipLaunchKernelGGL(node_poison_kernel, dim3(std::max<int32_t>((n_nodes + 255) / 256, 1)),
                       dim3(256), 0, s, res, n_nodes);
  } else if (n_nodes > 0) {
    // the all-reduce / local paths have no host round trip before their sums:
    // the rare kernel always runs first (it exits at once on an empty list)
    launch_node_rare(lp, *ns, counters, n_nodes, 0, s);
    hipLaunchKernelGGL(segment_sum_kernel,
                       dim3(std::min<int32_t>((n_nodes + 3) / 4, kPubBlocks)), dim3(256), 0, s,
                       lp, off, n_nodes, res);
  }
  hipLaunchKernelGGL(node_status_kernel, dim3(1), dim3(64), 0, s, res, n_nodes, status,
                     poison ? 1 : 0, counters);
}

void launch_publish_vec(const double* res, int32_t n, double* out, unsigned long long seq,
                        hipStream_t s) {
  hipLaunchKernelGGL(publish_vec_kernel, dim3(1), dim3(256), 0, s, res, n, out, seq);
}

void launch_node_rare(double* lp, const NodeSum& ns, int* counters, int32_t m, int64_t n,
                      hipStream_t s) {
  const NodeRare R{ns.rare_v, ns.rare_j, counters + 1};
  hipLaunchKernelGGL(node_rare_kernel, dim3(64), dim3(64), 0, s, R, lp, ns.x, ns.P, m, n, *ns.K,
                     ns.mode, ns.status, ns.evals);
}

void launch_segment_sum(const double* lp, const int64_t* off, int32_t n_nodes, double* res,
                        double* out, int* status, unsigned long long seq, hipStream_t s,
                        int* ticket, int* counters, int32_t n_tables, int64_t n,
                        int check_rare) {
  if (n_nodes <= 0) return;
  const int32_t nv = n_nodes * std::max(n_tables, 1);  // virtual nodes t m + j
  // one node per wave up to kPubBlocks blocks, then several per wave: the
  // blocks' ticket releases serialise on one word (the diagnostic build keeps
  // one node per wave)
  const int32_t nb = WFPT_PUB_DIAG ? (nv + 3) / 4 : std::min<int32_t>((nv + 3) / 4, kPubBlocks);
  hipLaunchKernelGGL(segment_publish_kernel, dim3(nb), dim3(256), 0, s, lp, off, nv, status, res,
                     out, seq, ticket, counters, n_nodes, n, check_rare);
}

template <int MODE, bool COUNT>
static void launch_multi_two_pass(const double* x, int64_t n, const double* const* arr,
                                  const double* scal, const Knobs& K, double p_outlier, double* lp,
                                  int64_t* d_idx, Params* d_par, int* n_defer,
                                  unsigned long long* evals, int* status, hipStream_t s) {
  hipLaunchKernelGGL((multi_fast_kernel<MODE, COUNT>), dim3(blocks_for(n)), dim3(kBlock), 0, s, x,
                     n, arr, scal, K, p_outlier, lp, d_idx, d_par, n_defer, evals);
  if constexpr (MODE != kDirect) {
    // adaptive families: one wave per deferred record (node_engine_kernel)
    const int64_t nb = std::min<int64_t>(std::max<int64_t>((n + kEngBlock - 1) / kEngBlock, 1), 256);
    hipLaunchKernelGGL((node_engine_kernel<MODE, COUNT, true>), dim3(nb), dim3(kEngBlock), 0, s, x,
                       K, lp, d_idx, d_par, n_defer, evals, status);
  } else {
    // direct family: only exact-path records, one lane each
    const int64_t nl = (n + 63) / 64;
    const int64_t g = nl < 64 ? nl : 64;  // rare exact-path records; kilobytes of scratch per lane
    hipLaunchKernelGGL((node_slow_kernel<MODE, 0, COUNT, true>), dim3(g), dim3(64), 0, s, x, K, lp,
                       d_idx, d_par, n_defer, evals, status);
  }
}

void launch_multi_fast(int mode, const double* x, int64_t n, const double* const* arr,
                       const double* scal, const Knobs& K, double p_outlier, double* lp,
                       int64_t* d_idx, Params* d_par, int* n_defer, double* part, int* zeros,
                       unsigned long long* evals, int* status, hipStream_t s) {
#define MULTI_TWO_PASS(M_, C_)                                                                  \
  launch_multi_two_pass<M_, C_>(x, n, arr, scal, K, p_outlier, lp, d_idx, d_par, n_defer, evals, \
                                status, s)
#define MULTI_MODES(C_)                            \
  switch (mode) {                                  \
    case kDirect: MULTI_TWO_PASS(kDirect, C_); break; \
    case kAdaptT: MULTI_TWO_PASS(kAdaptT, C_); break; \
    case kAdaptZ: MULTI_TWO_PASS(kAdaptZ, C_); break; \
    default: MULTI_TWO_PASS(kAdaptTZ, C_); break;     \
  }
  if (evals) {
    MULTI_MODES(true)
  } else {
    MULTI_MODES(false)
  }
#undef MULTI_MODES
#undef MULTI_TWO_PASS
  hipLaunchKernelGGL(lp_sum_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, s, lp, n, part, zeros);
}

void launch_multi(const double* x, int64_t n, const double* const* arr, const double* scal,
                  const Knobs& K, double p_outlier, double* part, int* zeros, int* status,
                  hipStream_t s, double* lp) {
  const int64_t nb = blocks_for(n);
  if (nb == 0) return;
  const int stk = stack_kind(K);
  if (stk == 0)
    hipLaunchKernelGGL((multi_kernel<0>), dim3(nb), dim3(kBlock), 0, s, x, n, arr, scal, K,
                       p_outlier, part, zeros, status, lp);
  else if (stk == 1)
    hipLaunchKernelGGL((multi_kernel<1>), dim3(nb), dim3(kBlock), 0, s, x, n, arr, scal, K,
                       p_outlier, part, zeros, status, lp);
  else
    hipLaunchKernelGGL((multi_kernel<2>), dim3(nb), dim3(kBlock), 0, s, x, n, arr, scal, K,
                       p_outlier, part, zeros, status, lp);
}

}  // namespace wfpt
