// wfpt_internal.h — launcher interface between the C ABI (wfpt_capi.cpp) and
// the kernels (wfpt_kernels.hip). Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "../../include/wfpt_amd.h"

namespace wfpt {
struct Params;
struct Knobs;

// Deferred-trial state of one call, slot-indexed (slot = chunk * 64 + rank
// of the trial among its chunk's deferred trials; nslots = chunks * 64). The
// deferred trials are the rare ones the level-0 engine hands on: the exact
// path (near-ties, ambiguous series decisions, subnormal densities) and trees
// deeper than its in-wave levels.
struct Work {
  unsigned char* wl;  // [nslots] lane of the trial in slot
  int* wl_n;          // [chunks] deferred trials of the chunk
  int* rflag;         // [nslots] kFlagExact | kFlagFallback of the trial in slot
  int* prof;          // [16] refinement work counters (evaluation counting only)
  unsigned long long* phase;  // [8 * kPhaseWaves] per-wave engine timing (WFPT_PHASE_TIMING)
  // Lean level-0 pass (kPassLean) and the engine's redo pass (kPassRedo): 1 =
  // the chunk needs in-wave refinement, which the lean pass leaves to the
  // engine (0 at rest: the redo pass clears what it handles). Null in a
  // launch that is not the redo pass.
  unsigned char* redo;        // [chunks]
  int* tree_any;              // device word: some chunk of the call refined (0 at rest)
  int64_t nslots;
};

constexpr int kPhaseWaves = 16384;

// Heavy chunks of a resident dataset (wfpt_kernels.hip: engine_kernel). The
// engine records the chunks whose level 0 leaves more than kHeavyZ z walks
// (next_*); the following call splits those chunks into kSplit units of
// kSplitTrials trials, one wave each. All pointers null / n = 0: no split, no
// record (host arrays, non-engine families).
#ifndef WFPT_SPLIT
#define WFPT_SPLIT 8  // units per heavy chunk (kSplitTrials trials each)
#endif
constexpr int kSplit = WFPT_SPLIT, kSplitTrials = 64 / kSplit;
// Two classes (WFPT_HEAVY_TOTAL): 1 = more than kHeavyZ z walks after level
// 0 (always split), 2 = more than kHeavyZ over all levels only (split while
// the dataset has few heavy chunks: the host sets n2 = 0 otherwise). The
// lists hold class 1 in [0, cap / 2) and class 2 in [cap / 2, cap).
struct Split {
  int n;                       // class-1 chunks split in this call (their units come first)
  int n2;                      // class-2 chunks split in this call (units after class 1's)
  int cap;                     // capacity of the chunk lists and per-chunk state
  const int* list;             // [cap] their chunk ids (class 1 from 0, class 2 from cap / 2)
  const unsigned char* pred;   // [chunks] 1 / 2 = recorded heavy of that class last call
  unsigned char* next_pred;    // [chunks] this call's record for the next call
  int* next_list;              // [cap]
  int* next_n;                 // device counters [0] class 1, [2] class 2 (0 at the call's start)
  double* lp;                  // [cap * 64] per-trial log terms of split chunks
  int* meta;                   // [cap * 64] zero | defer << 1 | rflag << 2
  int* done;                   // [cap] units finished (0 at rest)
  int* zn;                     // [cap] z walks summed over units: level 0 | all levels << 16
};

// Error flags encoded as counts in one double that survives an RCCL sum:
// (#ranks with a depth error) + kBudgetUnit * (#ranks with a budget error)
// + kPeerFailUnit * (#ranks whose local pass failed before the exchange: a
// failing rank still enters the collective with this poisoned count, so no
// peer waits on it forever). All sums stay exact integers in a double.
constexpr double kBudgetUnit = 1048576.0;
constexpr double kPeerFailUnit = 1099511627776.0;  // 2^40

int stack_kind(const Knobs& K);
int64_t blocks_for(int64_t n);
// true: adaptive / direct family (level-0 pass + deferred pass); false: fixed
// Simpson (one trial kernel).
bool has_deferred_pass(const Params& P, const Knobs& K);
// partials a sum leaves in out/zeros: one per 64-trial chunk (adaptive /
// direct) or per 256-trial block (fixed Simpson)
int64_t partials_for(int64_t n, const Params& P, const Knobs& K);

// out_kind: 0 = partial {sum, zeros}; 1 = per-trial density (logp => log);
// 2 = per-trial log p; 3 = 0's partials + each trial's log term in trial[n]
// (the per-trial check of the summing kernels). part: kPassFast (level-0 pass, or the whole fixed
// Simpson kernel) | kPassDeferred (the deferred trials + fold). Adaptive
// families only: kPassLean makes the level-0 pass the lean kernel (level 0
// without the in-wave refinement; a chunk that refines is flagged in W.redo
// and counted as deferred), and kPassRedo runs the engine over the flagged
// chunks (before the fold). fast_done (optional) is recorded right after the
// level-0 / trial kernel.
constexpr int kPassFast = 1, kPassDeferred = 2, kPassAll = 3, kPassLean = 4, kPassRedo = 8;
void launch_trials(int out_kind, int part, const double* x, int64_t n, const Params& P,
                   const Knobs& K, double* out, int* zeros, unsigned long long* evals, int* status,
                   int logp, const Work& W, hipStream_t s, hipEvent_t fast_done = nullptr,
                   const Split* split = nullptr, double* trial = nullptr);
// out[0..3] = {sum of nb partials, #zero trials, encoded error flags,
// kResDeferred (defer_bits: some chunk's zero word carries kZeroDefer) |
// kResTree (*tree_any; then *tree_any = 0)}, out[6] = *tree_any (chunks that
// refined in-wave), out[5] = *split_rd (the heavy chunks the call
// recorded, or 0; then *split_rs = 0), then out[4] = seq (a 64-bit word) once
// they are visible; resets *status to 0. mirror (optional, device memory):
// out[0..3] and out[5] written there too.
constexpr int kResDeferred = 1, kResTree = 2;
void launch_finalize(const double* part, const int* zeros, int64_t nb, int defer_bits,
                     int* status, double* out, unsigned long long seq, hipStream_t s,
                     const int* split_rd = nullptr, int* split_rs = nullptr,
                     int* tree_any = nullptr, double* mirror = nullptr,
                     double* fin = nullptr, int* ticket = nullptr);
// One-block call (n <= 256, direct or adaptive family, level-0 pass + the
// finalize in one launch: the same result bits and completion word as
// launch_trials(kPassFast [| kPassLean]) + launch_finalize). kSmallNone: not
// eligible, nothing launched; kSmallOne: small_kernel; kSmallSplit: the full
// DDM's small_split_kernel (three lanes per trial). trial (nullable): out_kind
// 3's per-trial terms.
constexpr int kSmallNone = 0, kSmallOne = 1, kSmallSplit = 2;
int launch_small(const double* x, int64_t n, const Params& P, const Knobs& K, double* part,
                 int* zeros, int* status, const Work& W, double* out, unsigned long long seq,
                 int* tree_any, hipStream_t s, double* trial = nullptr);
// fin (device, 3 * 64 doubles) + ticket (device int, 0 at rest): scratch of the
// multi-block finalize for large nb (nullptr: one block)
// res[0..3], res[5] (device) -> out[0..3], out[5] (mapped host), then
// out[4] = seq.
void launch_publish(const double* res, double* out, unsigned long long seq, hipStream_t s);
// res[0..2] = wfpt_result_poison's triple {0, 0, kPeerFailUnit}, res[3..7] = 0
// (one thread, stream order: the all-reduce of a rank whose local pass failed)
void launch_poison(double* res, hipStream_t s);
// mode: the integration family shared by every node (kDirect..kAdaptTZ: the
// two-pass fast path; n_defer[0..2] must be 0 on the stream: the direct
// family's deferred (index, row) records in d_idx / d_par (up to n) counted in
// n_defer[0]; the adaptive families' listed chunks in clist (up to
// (n + 63) / 64) counted in n_defer[0] and the fast pass's deferred trials as
// (index, row) records in d_idx / d_par counted in n_defer[2]; n_defer[1] is
// unused), or -1 (mixed /
// fixed Simpson: one generic per-trial kernel with a per-lane mode). prof
// (COUNT builds, evals != null): the node tallies of wfpt_profile_lists.
// nt (optional): the call's node tables (device); with them the adaptive t
// families (kAdaptT, kAdaptTZ) of a non-counting call run node_grid_kernel +
// node_split_kernel (five lanes per trial) instead of node_fast_kernel.
// split: the adaptive t families take node_split_kernel; spec: the sparse
// deferred trials take node_record_spec (non-counting calls)
// n_tables: T parameter tables (P holds T x n_nodes rows, table t's node j at
// t n_nodes + j) over the same trials in one launch; table t's terms land in
// lp[t n, (t + 1) n), its deferred records carry virtual indices t n + i and
// its listed chunks t ceil(n / 64) + c (d_idx / d_par up to T n records, clist
// up to T ceil(n / 64) chunks).
// rare_v / rare_j (T n entries each): the node path's rare trials (exact
// path, trees deeper than kTreeDepth), counted in n_defer[1] and settled by
// the summing kernel (launch_segment_sum / launch_segment_res, NodeSum).
struct NodeTables {
  int32_t n_nodes;
  bool split, spec;
  int32_t n_tables = 1;
  int64_t* rare_v = nullptr;
  int32_t* rare_j = nullptr;
};
// What the summing kernels need to settle the rare trials before they sum:
// the dataset, the call's (T x n_nodes) parameter table, the knobs and the
// family (mode: the two-pass family; -1 / generic calls push none), evals
// (nullable) for the exact path's evaluation counts.
struct NodeSum {
  const double* x;
  const int32_t* node;
  const Params* P;
  const Knobs* K;
  int mode;
  int64_t* rare_v;
  int32_t* rare_j;
  unsigned long long* evals;
  int* status;
};
// The rare trials of the call (counters[1] of them): each one's node term into
// lp (exact path / per-lane walk). m: nodes per table, n: trials per table.
void launch_node_rare(double* lp, const NodeSum& ns, int* counters, int32_t m, int64_t n,
                      hipStream_t s);
void launch_nodes(const double* x, const int32_t* node, int64_t n, const Params* P,
                  const Knobs& K, int mode, double* lp, int64_t* d_idx, Params* d_par,
                  int* n_defer, int* clist, unsigned long long* evals, int* status, int* prof,
                  hipStream_t s, const NodeTables* nt = nullptr);
// res (device, n_nodes) per-node sums; then out (mapped host): [0, n_nodes)
// the sums, [n_nodes] encoded error flags, [n_nodes + 1] the completion word.
// Node all-reduce: res[0, n_nodes) per-node sums (or zeros when poison),
// res[n_nodes] the encoded error count (kPeerFailUnit when poison; the device
// status word is reset); then, after the exchange, res -> out[0, n_nodes] and
// the completion word out[n_nodes + 1].
// counters: the node path's n_defer words, reset to 0 (0 at rest)
void launch_segment_res(double* lp, const int64_t* off, int32_t n_nodes, double* res,
                        int* status, bool poison, hipStream_t s, int* counters,
                        const NodeSum* ns);
void launch_publish_vec(const double* res, int32_t n, double* out, unsigned long long seq,
                        hipStream_t s);
// One launch (segment_publish_kernel): the per-node sums into res, then the
// last block (ticket, 0 at rest) publishes them to out with the error word
// and the completion word and resets counters[0..2] (0 at rest).
// n_tables > 1: the T n_nodes sums of a multi-table call (table t's node j at
// t n_nodes + j, its trials at t n + off[j] of lp; n = trials per table).
// check_rare: a call with rare trials (counters[1] > 0) is not summed: out[T
// n_nodes] = kRarePending (-1) and the completion word; the host then runs
// launch_node_rare and this launch again with check_rare = 0.
constexpr double kRarePendingHost = -1.0;
void launch_segment_sum(const double* lp, const int64_t* off, int32_t n_nodes, double* res,
                        double* out, int* status, unsigned long long seq, hipStream_t s,
                        int* ticket, int* counters, int32_t n_tables, int64_t n,
                        int check_rare);
// wiener_like_multi with a uniform adaptive / direct family (mode): level-0
// pass + deferred trials (d_idx / d_par hold up to n records, *n_defer must
// be 0 on the stream) into lp[n], then per-block sums into part / zeros
// (blocks_for(n) of them) for launch_finalize.
void launch_multi_fast(int mode, const double* x, int64_t n, const double* const* arr,
                       const double* scal, const Knobs& K, double p_outlier, double* lp,
                       int64_t* d_idx, Params* d_par, int* n_defer, double* part, int* zeros,
                       unsigned long long* evals, int* status, hipStream_t s);
// lp (nullable): each trial's term too
void launch_multi(const double* x, int64_t n, const double* const* arr, const double* scal,
                  const Knobs& K, double p_outlier, double* part, int* zeros, int* status,
                  hipStream_t s, double* lp = nullptr);
// cdfdif_kernels.hip: dmat_cdf_array over device x[n]; par = the wrapper's
// transformed (a, Ter, eta, z, sZ, st, nu) (cdfdif_wrapper.pyx:36-42).
// defer: n ints of workspace, n_defer: one device int.
constexpr int kCdfTableDoubles = 1344 + 512 * 48;  // per-call tables of launch_dmat_cdf
void launch_dmat_cdf(const double* x, int64_t n, const double par[7], double p_outlier,
                     double w_outlier, double* out, double* tab, int* defer, int* n_defer,
                     hipStream_t s);
}  // namespace wfpt
