// wfpt_capi.cpp — C ABI of the MI355X WFPT engine (include/wfpt_amd.h).
//
// Host runtime: one context per GPU (HIP stream, grow-only device workspaces,
// pinned result slot, optional RCCL communicator), resident datasets, and the
// call sequences  fast pass -> slow pass -> finalize  per likelihood. The last
// kernel writes {sum, #zeros, status} straight into mapped pinned host memory
// (no copy, no memset, no stream sync).
// Calls into one context are serialised by its mutex; the ctypes binding
// releases the GIL around every call.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/wfpt_amd.h"
#include "wfpt_device.hpp"
#include "wfpt_internal.h"

static thread_local std::string g_last_error;
extern "C" int wfpt_decode_result(const double r[3], double* out);

static int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
// the last-error slot for wfpt_rendezvous.cpp
int wfpt_rdv_fail(int code, const std::string& msg) { return fail(code, msg); }

// roctx range around each C-ABI entry point (rocprofv3 --marker-trace shows
// the host side of a call next to its kernels); WFPT_ROCTX=0 turns them off.
static bool roctx_on() {
  static const bool on = [] {
    const char* e = std::getenv("WFPT_ROCTX");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  return on;
}
namespace {
struct RoctxRange {
  bool on;
  explicit RoctxRange(const char* name) : on(roctx_on()) {
    if (on) roctxRangePushA(name);
  }
  ~RoctxRange() {
    if (on) roctxRangePop();
  }
};
}  // namespace
#define WFPT_RANGE(name) RoctxRange wfpt_range_(name)

#define HIP_TRY(expr)                                                                 \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess)                                                             \
      return fail(WFPT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define NCCL_TRY(expr)                                                                 \
  do {                                                                                 \
    ncclResult_t r_ = (expr);                                                          \
    if (r_ != ncclSuccess)                                                             \
      return fail(WFPT_ERR_COMM, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
  } while (0)

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;
  hipError_t reserve(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n, 256);
    hipError_t e = hipMalloc((void**)&p, want * sizeof(T));
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Pinned host memory mapped into the device address space (fine-grained,
// coherent): the host writes per-call inputs / reads results there directly.
template <class T>
struct MappedBuf {
  T* h = nullptr;  // host pointer
  T* d = nullptr;  // device alias
  size_t cap = 0;
  hipError_t reserve(size_t n) {
    if (n <= cap) return hipSuccess;
    release();
    const size_t want = std::max<size_t>(n, 64);
    hipError_t e = hipHostMalloc((void**)&h, want * sizeof(T),
                                 hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&d, h, 0);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (h) (void)hipHostFree(h);
    h = nullptr;
    d = nullptr;
    cap = 0;
  }
};

struct wfpt_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  DevBuf<double> x;       // uploads of host arrays
  DevBuf<double> part;    // block partial sums
  DevBuf<int> zero;       // block zero counts
  DevBuf<double> res;     // per-node results
  double* ar = nullptr;   // device: this rank's {sum, zeros, errors, ...} of an all-reduce
                          // call (8 doubles, allocated at open: a failed workspace reserve
                          // cannot keep a rank out of the exchange)
  DevBuf<double> lp;      // per-trial outputs
  DevBuf<double> marr;    // wiener_like_multi parameter arrays
  DevBuf<double*> mptr;
  DevBuf<double> mscal;
  // deferred-trial state of adaptive calls (wfpt_internal.h: Work), sized for
  // the largest call so far: slot-indexed, nslots = 64 * chunks
  DevBuf<unsigned char> wl;  // lane of the deferred trial in each slot
  DevBuf<int> wl_n;          // per chunk: deferred trials
  DevBuf<int> rflag;         // per slot: kFlagExact | kFlagFallback
  DevBuf<unsigned char> redo;  // per chunk: the lean pass left it to the engine (0 at rest)
  int* tree_any = nullptr;   // device: some chunk refined in-wave (finalize reports + clears)
  double* fin = nullptr;     // device: multi-block finalize scratch (3 x 64 doubles)
  int* fin_ticket = nullptr; // device: its last-block ticket (0 at rest)
  int* prof = nullptr;       // device: 16 refinement work counters (PROF_EVALS)
  unsigned long long* phase = nullptr;  // device: engine phase cycles (diagnostic builds)
  DevBuf<int> defer;         // dmat_cdf_array: deferred trial indices + count
  DevBuf<double> cdf_tab;    // dmat_cdf_array: the call's parameter-only tables
  DevBuf<int64_t> nd_idx;    // wiener_like_nodes: deferred trial indices
  DevBuf<int64_t> rare_v;    // wiener_like_nodes: the rare trials (wfpt_kernels.hip: NodeRare)
  DevBuf<int32_t> rare_j;
  DevBuf<wfpt::Params> nd_par;  // ... and their parameter rows
  DevBuf<int> nd_chunks;     // wiener_like_nodes: chunks the level-0 pass left to the chunk engine
  int* ncnt = nullptr;       // device [4]: the node path's listed chunks / records counters and
                             // [3] the publish ticket (0 at rest: the call's last kernel resets
                             // them; a failed call restores them)
  int* n_defer = nullptr;    // device [4]: the per-node path's listed chunks, chunk-path records,
                             // fast-pass records (0 at rest)
  unsigned long long* evals = nullptr;
  int* status = nullptr;      // device: Simpson-stack overflow flag
  int* host_status = nullptr; // pinned mirror
  double* mres = nullptr;      // mapped pinned {sum, zeros, errors, deferred, word, heavy, #tree}
  double* mres_dev = nullptr;  // its device alias
  unsigned long long seq = 0;  // completion word finalize writes to mres[4]
  MappedBuf<wfpt::Params> mnodep;  // per-node parameter table of wiener_like_nodes
  DevBuf<wfpt::Params> dnodep;     // its device copy (node_table_dev: WFPT_NODE_TABLE_DEV=1)
  // WFPT_HOST_TIMING=1: host time of the multi-table node calls by phase
  // (table rows, launches, wait, copy-out; ns summed), printed at wfpt_close
  bool host_timing = false;
  std::chrono::steady_clock::time_point ht_mark;
  double ht[5] = {0, 0, 0, 0, 0};
  int64_t ht_calls = 0;
  bool node_table_dev = false;
  MappedBuf<double> mnode;         // per-node sums + status + completion word
  bool spin = true;            // poll mres[3] instead of hipStreamSynchronize
  bool nodes_generic = false;  // WFPT_NODES=generic: per-trial generic node kernel only
  // WFPT_NODE_SPLIT=1: the per-node level 0 of the adaptive t families split
  // over five lanes per trial (node_split_kernel; measured slower on config 4:
  // the per-lane grid and hints are redone by every lane); WFPT_NODE_SPEC=0:
  // sparse deferred trials through the breadth-first rounds instead of
  // node_record_spec
  bool node_split = false;
  bool node_spec = true;
  bool fast_only = true;       // WFPT_FAST_ONLY=0: resident calls always enqueue the slow pass
  bool lean = true;            // WFPT_LEAN=0: resident calls never use the lean level-0 pass
  bool small = true;           // WFPT_SMALL=0: one-block calls keep the separate finalize
  // WFPT_LEAN_TREE: the largest fraction of refining chunks (last call) for
  // which the lean pass + engine redo of those chunks beats the engine over
  // every chunk
  double lean_tree_max = 0.0;
  bool profile = false;      // HIP events around the main kernel
  bool count = false;        // pdf_sv evaluation counting
  double k_ms = 0.0;
  int64_t launches = 0;
  int64_t n_evals = 0;
  // per-trial check (wfpt_wiener_like_trials): device buffer of the call's
  // per-trial log terms (the summing kernels' OUT_BOTH build), else null
  double* trial = nullptr;
  int path = 0;  // WFPT_PATH_* bits of the kernels the last likelihood call launched
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  // the context's live datasets: wfpt_close releases their device memory and
  // detaches them (a dataset destroyed after its context only frees itself)
  std::vector<wfpt_ds*> dsets;
};

constexpr int64_t kSplitCap = 16384;  // heavy chunks a dataset records per call (both classes)
// class-2 heavy chunks (Split::n2) are split while the dataset's heavy chunks
// are at most 1 / kHeavyFewDiv of its chunks: then they are the launch's
// tail; when many chunks are heavy, splitting them only adds waves
constexpr int64_t kHeavyFewDiv = 16;

struct wfpt_ds {
  wfpt_ctx* ctx = nullptr;
  int64_t n = 0;
  double* x = nullptr;
  int32_t* node = nullptr;
  int64_t* off = nullptr;
  int32_t n_nodes = 0;
  // the last call on this dataset deferred no trial: the next one runs the
  // level-0 pass + finalize only (run_sum_fast), no slow pass
  mutable bool no_defer = false;
  // the last call on this dataset refined no chunk in-wave: the next one's
  // level-0 pass is the lean kernel (kPassLean)
  mutable bool no_tree = false;
  // fraction of chunks that refined in-wave in the last call: up to
  // lean_tree_max the lean pass still runs, the engine redoing those chunks
  mutable double tree_frac = 1.0;
  bool input_order = false;  // WFPT_DS_INPUT_ORDER: trials kept in the caller's order
  // heavy-chunk record (wfpt_internal.h: Split), double-buffered by call
  // parity: the engine writes [1 - parity] while it reads [parity]
  int64_t nw = 0;
  int split_cap = 0;
  unsigned char* hpred[2] = {nullptr, nullptr};
  int* hlist[2] = {nullptr, nullptr};
  int* hcount = nullptr;  // [4]: class 1 by parity, then class 2 by parity
  double* hlp = nullptr;
  int* hmeta = nullptr;
  int* hdone = nullptr;
  int* hzn = nullptr;
  mutable int nsplit = 0;  // class-1 chunks the next call splits
  mutable int nsplit2 = 0; // class-2 chunks the next call splits
  mutable int parity = 0;
  // device: the caller's index of each stored trial (per-trial outputs of the
  // diagnostic calls are returned in the caller's order; kept in HBM, not in
  // host memory: 8 B per trial); null = identity (WFPT_DS_INPUT_ORDER)
  int64_t* perm = nullptr;
  bool identity = true;  // stored order == the caller's order (perm never allocated)
};

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    (void)hipGetDevice(&prev);
    if (prev != dev) (void)hipSetDevice(dev);
    // a stale error of an earlier, already reported runtime call must not be
    // read as this call's launch failure (hipGetLastError after launches)
    (void)hipGetLastError();
  }
  ~DeviceGuard() {
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
  }
};

void ds_free_device(wfpt_ds* d);  // defined with wfpt_dataset_destroy

wfpt::Params to_params(const wfpt_params* p) {
  wfpt::Params q;
  q.v = p->v;
  q.sv = p->sv;
  q.a = p->a;
  q.z = p->z;
  q.sz = p->sz;
  q.t = p->t;
  q.st = p->st;
  q.p_outlier = p->p_outlier;
  return q;
}

wfpt::Knobs to_knobs(const wfpt_knobs* k) {
  wfpt::Knobs q;
  q.err = k->err;
  q.n_st = k->n_st;
  q.n_sz = k->n_sz;
  q.use_adaptive = k->use_adaptive != 0;  // `bint` in the reference signatures
  q.simps_err = k->simps_err;
  q.w_outlier = k->w_outlier;
  return q;
}

bool p_outlier_in_range(double p) { return (p >= 0) & (p <= 1); }  // wfpt.pyx:50-51


// Paths without finalize_kernel (pdf_array, nodes): clear the overflow flag
// before the launch, copy it back (and clear it again) before the stream sync.
int begin_status(wfpt_ctx* c) {
  HIP_TRY(hipMemsetAsync(c->status, 0, sizeof(int), c->stream));
  return WFPT_OK;
}
int fetch_status(wfpt_ctx* c) {
  HIP_TRY(hipMemcpyAsync(c->host_status, c->status, sizeof(int), hipMemcpyDeviceToHost,
                         c->stream));
  HIP_TRY(hipMemsetAsync(c->status, 0, sizeof(int), c->stream));  // 0 at rest
  return WFPT_OK;
}
int check_status_value(double enc);
// the raw device flag word (kFlagDepth | kFlagBudget) in the encoded form
double encode_status(int st) {
  return (double)(st & wfpt::kFlagDepth) + ((st & wfpt::kFlagBudget) ? wfpt::kBudgetUnit : 0.0);
}
int check_status(wfpt_ctx* c) { return check_status_value(encode_status(*c->host_status)); }

// Deferred-trial state for adaptive calls over up to n trials (grow-only).
int reserve_work(wfpt_ctx* c, int64_t n, wfpt::Work* W) {
  const int64_t nw = std::max<int64_t>((n + 63) / 64, 1);
  const int64_t ns = nw * 64;
  HIP_TRY(c->wl.reserve(ns));
  HIP_TRY(c->wl_n.reserve(nw));
  HIP_TRY(c->rflag.reserve(ns));
  if (c->redo.cap < (size_t)nw) {
    HIP_TRY(c->redo.reserve(nw));
    HIP_TRY(hipMemsetAsync(c->redo.p, 0, c->redo.cap, c->stream));
  }
  W->redo = c->redo.p;
  W->tree_any = c->tree_any;
  W->wl = c->wl.p;
  W->wl_n = c->wl_n.p;
  W->rflag = c->rflag.p;
  W->prof = c->prof;
  W->phase = c->phase;
  W->nslots = ns;
  return WFPT_OK;
}

// Status words are 0 at rest: finalize_kernel resets the device flag after
// reporting it, and the other paths clear it before their launch. enc:
// #depth errors + kBudgetUnit * #budget errors (summed over ranks).
int check_status_value(double enc) {
  if (enc == 0) return WFPT_OK;
  const double peers = std::floor(enc / wfpt::kPeerFailUnit);
  enc -= peers * wfpt::kPeerFailUnit;
  const double budget = std::floor(enc / wfpt::kBudgetUnit);
  const double depth = enc - budget * wfpt::kBudgetUnit;
  std::string msg;
  if (peers > 0)
    msg = std::to_string((long long)peers) +
          " rank(s) failed before the likelihood exchange (their own call returned the error)";
  if (depth > 0) {
    if (!msg.empty()) msg += "; ";
    msg += "adaptive Simpson refinement deeper than WFPT_MAX_DEPTH=" +
           std::to_string(WFPT_MAX_DEPTH) + " levels (lower n_st/n_sz or raise simps_err)";
  }
  if (budget > 0) {
    if (!msg.empty()) msg += "; ";
    msg += "a trial exceeded WFPT_EVAL_BUDGET pdf_sv evaluations (raise simps_err)";
  }
  return fail((depth > 0 || budget > 0) ? WFPT_ERR_UNSUPPORTED : WFPT_ERR_COMM, msg);
}

// The dataset's heavy-chunk state for one engine call (null: no split, no
// record).
wfpt::Split split_of(const wfpt_ds* d) {
  wfpt::Split S{};
  if (!d || !d->hcount) return S;
  const int cur = d->parity, nx = 1 - cur;
  S.n = d->nsplit;
  S.n2 = d->nsplit2;
  S.cap = d->split_cap;
  S.list = d->hlist[cur];
  S.pred = d->hpred[cur];
  S.next_pred = d->hpred[nx];
  S.next_list = d->hlist[nx];
  S.next_n = d->hcount + nx;
  S.lp = d->hlp;
  S.meta = d->hmeta;
  S.done = d->hdone;
  S.zn = d->hzn;
  return S;
}

// After a call's result r is in host memory: the next call splits the heavy
// chunks this one recorded (engine calls), or none.
void split_advance(const wfpt_ds* d, bool engine, const double* r) {
  if (!d) return;
  if (!engine || !d->hcount) {
    d->nsplit = 0;
    d->nsplit2 = 0;
    return;
  }
  const int half = d->split_cap / 2;
  d->nsplit = (int)std::min<double>(r[5], (double)half);
  const int n2 = (int)std::min<double>(r[7], (double)half);
  d->nsplit2 = (int64_t)(d->nsplit + n2) * kHeavyFewDiv <= d->nw ? n2 : 0;
  d->parity = 1 - d->parity;
}

bool engine_family(const wfpt::Params& P, const wfpt::Knobs& K) {
  const int m = wfpt::select_mode(P.sz, P.st, K.use_adaptive);
  return m >= wfpt::kAdaptT && m <= wfpt::kAdaptTZ;
}

// Likelihood sum over device x[n]: adaptive / direct families run the level-0
// pass and (part & kPassDeferred) the deferred-trial pass, fixed Simpson one
// trial kernel; then finalize writes {sum, zeros, errors, deferred} + the
// completion word to `out` (mapped host memory or device).
int run_sum(wfpt_ctx* c, const double* dx, int64_t n, const wfpt::Params& P,
            const wfpt::Knobs& K, double* out, int part = wfpt::kPassAll,
            const wfpt_ds* d = nullptr, double* mirror = nullptr) {
  const int64_t nb = wfpt::partials_for(n, P, K);
  HIP_TRY(c->part.reserve(std::max<int64_t>(nb, 1)));
  HIP_TRY(c->zero.reserve(std::max<int64_t>(nb, 1)));
  wfpt::Work W;
  if (int rc = reserve_work(c, n, &W)) return rc;
  const bool adaptive = wfpt::has_deferred_pass(P, K);
  if (part & wfpt::kPassFast) c->path = 0;  // a call sequence starts
  if (c->count && (part & wfpt::kPassFast))
    HIP_TRY(hipMemsetAsync(c->evals, 0, sizeof(unsigned long long), c->stream));
  // profiling: ev0..ev1 bracket the level-0 fast kernel (the dominant kernel,
  // the one rocprofv3 reports as fast_kernel<...>)
  const bool prof = c->profile && (part & wfpt::kPassFast);
  if (prof) HIP_TRY(hipEventRecord(c->ev0, c->stream));
  // heavy-chunk splitting belongs to full engine calls (not the lean / redo
  // passes)
  const bool eng = d && d->hcount && engine_family(P, K) &&
                   !(part & (wfpt::kPassLean | wfpt::kPassRedo));
  // one block of trials, level-0 pass only (direct family, or the lean pass):
  // level 0 and finalize in one launch (WFPT_SMALL=0: two launches)
  const bool level0_only = adaptive && (engine_family(P, K)
                                            ? part == (wfpt::kPassFast | wfpt::kPassLean)
                                            : part == wfpt::kPassFast);
  const bool direct = adaptive && !engine_family(P, K);
  if (c->small && level0_only && !prof && !c->count && !mirror) {
    const int sk = wfpt::launch_small(dx, n, P, K, c->part.p, c->zero.p, c->status, W, out,
                                      c->seq + 1, c->tree_any, c->stream, c->trial);
    if (sk != wfpt::kSmallNone) {
      ++c->seq;
      HIP_TRY(hipGetLastError());
      c->path |= WFPT_PATH_SMALL | (direct ? WFPT_PATH_DIRECT : WFPT_PATH_LEAN) |
                 (sk == wfpt::kSmallSplit ? WFPT_PATH_SMALL_SPLIT : 0);
      return WFPT_OK;
    }
  }
  const wfpt::Split S = eng ? split_of(d) : wfpt::Split{};
  wfpt::launch_trials(c->trial ? 3 : 0, adaptive ? part : wfpt::kPassAll, dx, n, P, K, c->part.p,
                      c->zero.p, c->count ? c->evals : nullptr, c->status, 0, W, c->stream,
                      prof ? c->ev1 : nullptr, &S, c->trial);
  if (!adaptive) {
    c->path |= WFPT_PATH_FIXED;
  } else {
    if (part & wfpt::kPassFast)
      c->path |= direct ? WFPT_PATH_DIRECT
                        : (part & wfpt::kPassLean)
                              ? WFPT_PATH_LEAN
                              : (WFPT_PATH_ENGINE | (S.n + S.n2 > 0 ? WFPT_PATH_SPLIT : 0));
    if (!direct && (part & wfpt::kPassRedo)) c->path |= WFPT_PATH_REDO;
    if (part & wfpt::kPassDeferred) c->path |= WFPT_PATH_FOLD;
  }
  HIP_TRY(hipGetLastError());
  wfpt::launch_finalize(c->part.p, c->zero.p, nb, adaptive ? 1 : 0,
                        c->status, out, ++c->seq, c->stream, eng ? S.next_n : nullptr,
                        eng ? d->hcount + d->parity : nullptr, c->tree_any, mirror, c->fin,
                        c->fin_ticket);
  HIP_TRY(hipGetLastError());
  return WFPT_OK;
}

int finish_profile(wfpt_ctx* c) {
  if (c->profile) {
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    c->k_ms += ms;
    c->launches += 1;
  }
  if (c->count) {
    unsigned long long ev = 0;
    HIP_TRY(hipMemcpy(&ev, c->evals, sizeof(ev), hipMemcpyDeviceToHost));
    c->n_evals += (int64_t)ev;
  }
  return WFPT_OK;
}

// Waits for the completion word `word` (mapped host memory) to reach c->seq:
// the last kernel of a call writes it after its results (a stream sync's
// wake-up costs several microseconds per call). Every 4096 polls the stream is
// asked whether it failed; after 5 s, or if the stream is idle without the
// word, it falls back to a stream sync so a device error is reported, never a
// stale number.
int wait_word(wfpt_ctx* c, const void* word) {
  if (c->spin) {
    // the word is the device's system-scope release store (fin_write,
    // segment_publish_kernel, publish_*): read it with acquire semantics, so
    // every result store the device ordered before it is visible below
    const unsigned long long* w = reinterpret_cast<const unsigned long long*>(word);
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 1;; ++it) {
      if (__atomic_load_n(w, __ATOMIC_ACQUIRE) == c->seq) {
        if (c->profile) HIP_TRY(hipEventSynchronize(c->ev1));
        return WFPT_OK;
      }
      if ((it & 4095u) == 0) {
        const hipError_t q = hipStreamQuery(c->stream);
        if (q != hipSuccess && q != hipErrorNotReady)
          return fail(WFPT_ERR_HIP, std::string("likelihood kernels: ") + hipGetErrorString(q));
        if (q == hipSuccess && __atomic_load_n(w, __ATOMIC_ACQUIRE) != c->seq)
          break;  // idle: let the stream sync decide
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) break;
      }
    }
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (*reinterpret_cast<const volatile unsigned long long*>(word) != c->seq)
    return fail(WFPT_ERR_HIP, "the call's completion word was not written");
  return WFPT_OK;
}

int wait_result(wfpt_ctx* c, const double* r) {
  if (r == c->mres) return wait_word(c, r + 4);
  HIP_TRY(hipStreamSynchronize(c->stream));
  return WFPT_OK;
}

// Decodes {sum, zeros, errors, deferred} from host memory `r` of a finished
// call; *deferred (if given) = the level-0 pass deferred trials.
bool res_deferred(const double* r) { return ((int)r[3] & wfpt::kResDeferred) != 0; }
bool res_tree(const double* r) { return ((int)r[3] & wfpt::kResTree) != 0; }
int decode_sum(wfpt_ctx* c, const double* r, double* out, bool* deferred = nullptr) {
  if (deferred) *deferred = res_deferred(r);
  if (int rc = wfpt_decode_result(r, out)) return rc;
  return finish_profile(c);
}

// Waits for the call and decodes its result.
int read_sum(wfpt_ctx* c, const double* r, double* out, bool* deferred = nullptr) {
  if (int rc = wait_result(c, r)) return rc;
  return decode_sum(c, r, out, deferred);
}

// The dataset's in-wave refinement record from a finished call's result.
void note_tree(const wfpt_ds* d, const double* r) {
  d->no_tree = !res_tree(r);
  d->tree_frac = d->nw > 0 ? r[6] / (double)d->nw : 0.0;
}
// The lean level-0 pass is predicted to pay: nothing refined last time, or
// few enough chunks that their engine redo beats an engine pass over all.
bool lean_predicted(const wfpt_ctx* c, const wfpt_ds* d) {
  return c->lean && (d->no_tree || d->tree_frac <= c->lean_tree_max);
}

// Waits for a resident call, updates the dataset's predictions from its
// result and decodes it.
int finish_sum(wfpt_ctx* c, const wfpt_ds* d, const wfpt::Params& P, const wfpt::Knobs& K,
               double* out, bool lean) {
  if (int rc = wait_result(c, c->mres)) return rc;
  const bool eng = engine_family(P, K);
  split_advance(d, eng && !lean, c->mres);
  bool deferred = true;
  const int rc = decode_sum(c, c->mres, out, &deferred);
  if (rc == WFPT_OK) {
    d->no_defer = c->fast_only && !deferred;
    if (eng) note_tree(d, c->mres);
  }
  return rc;
}

// Resident-data sums with a predicted call sequence (from the dataset's last
// call), each giving the full sequence's result bit for bit:
//   * no deferred trial predicted: level-0 pass + finalize only (no fold
//     launch). If the pass did defer this time (finalize reports it), the
//     deferred pass and a second finalize run over the intact chunk partials;
//     only that call pays a host round trip.
//   * no in-wave refinement predicted (engine families): the level-0 pass is
//     the lean kernel; chunks that do refine are flagged and the engine's redo
//     pass processes them before the fold (as part of the deferred pass).
// Returns -1 when neither prediction applies (nothing launched).
int run_sum_fast(wfpt_ctx* c, const wfpt_ds* d, const wfpt::Params& P, const wfpt::Knobs& K,
                 double* out) {
  const int64_t n = d->n;
  if (c->count || n <= 0 || !wfpt::has_deferred_pass(P, K)) return -1;
  const bool eng = engine_family(P, K);
  const bool lean = eng && lean_predicted(c, d);
  const bool fast = c->fast_only && d->no_defer;
  if (!lean && !fast) return -1;
  const int lp = lean ? wfpt::kPassLean : 0;
  if (!fast) {  // deferred trials expected: the whole sequence at once
    if (int rc = run_sum(c, d->x, n, P, K, c->mres_dev, wfpt::kPassAll | lp | wfpt::kPassRedo, d))
      return rc;
  } else {
    if (int rc = run_sum(c, d->x, n, P, K, c->mres_dev, wfpt::kPassFast | lp, d)) return rc;
    if (int rc = wait_result(c, c->mres)) return rc;
    if (res_deferred(c->mres)) {
      if (int rc = check_status_value(c->mres[2])) return rc;
      if (int rc = run_sum(c, d->x, n, P, K, c->mres_dev,
                           wfpt::kPassDeferred | (lean ? wfpt::kPassRedo : 0), d))
        return rc;
    }
  }
  return finish_sum(c, d, P, K, out, lean);
}

// |a| < |b| with NaN RTs last: a strict weak order for any input (the
// dataset sorts must not hit std::stable_sort's undefined behaviour)
// Stored order of a dataset: |rt| ascending with NaN RTs last (a strict weak
// order for any input), as an unsigned key: |rt|'s bits (monotone for
// non-negative doubles), every NaN one key above +inf. `upper_last` adds the boundary bit
// (x > 0 sorts after x <= 0). Keys are equal exactly when neither comparator
// orders the pair, so a stable sort by key is the stable comparator sort.
uint64_t order_key(double r, bool upper_last) {
  uint64_t b;
  std::memcpy(&b, &r, sizeof(b));
  b &= 0x7fffffffffffffffull;
  if (std::isnan(r)) b = 0x7ff8000000000000ull;
  return (upper_last && r > 0) ? (b | 0x8000000000000000ull) : b;
}

// Stable sort of idx by key[idx] (ties keep idx order): LSD radix, 16-bit
// digits, for large datasets (C5's 100M trials: seconds instead of a minute
// of comparator sorting); the comparator sort below 64k trials.
void stable_order(std::vector<int64_t>& idx, const double* rt, bool upper_last) {
  const size_t n = idx.size();
  if (n < (1u << 16)) {
    std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) {
      return order_key(rt[a], upper_last) < order_key(rt[b], upper_last);
    });
    return;
  }
  std::vector<uint64_t> k(n), k2(n);
  std::vector<int64_t> i2(n);
  for (size_t j = 0; j < n; ++j) k[j] = order_key(rt[idx[j]], upper_last);
  std::vector<size_t> cnt(1u << 16);
  for (int sh = 0; sh < 64; sh += 16) {
    std::fill(cnt.begin(), cnt.end(), 0);
    for (size_t j = 0; j < n; ++j) cnt[(k[j] >> sh) & 0xffffu]++;
    if (cnt[(k[0] >> sh) & 0xffffu] == n) continue;  // one digit value: nothing moves
    size_t acc = 0;
    for (auto& c : cnt) {
      const size_t t = c;
      c = acc;
      acc += t;
    }
    for (size_t j = 0; j < n; ++j) {
      const size_t p = cnt[(k[j] >> sh) & 0xffffu]++;
      k2[p] = k[j];
      i2[p] = idx[j];
    }
    k.swap(k2);
    idx.swap(i2);
  }
}

// Per-trial values of a dataset's stored order (device) -> the caller's order
// (host) through the dataset's stored permutation (diagnostic calls only).
int trials_to_caller(const wfpt_ds* d, const double* dev, double* out) {
  if (d->n <= 0) return WFPT_OK;
  std::vector<double> h(d->n);
  HIP_TRY(hipMemcpy(h.data(), dev, d->n * sizeof(double), hipMemcpyDeviceToHost));
  if (!d->perm) {
    std::memcpy(out, h.data(), d->n * sizeof(double));
    return WFPT_OK;
  }
  std::vector<int64_t> perm(d->n);
  HIP_TRY(hipMemcpy(perm.data(), d->perm, d->n * sizeof(int64_t), hipMemcpyDeviceToHost));
  for (int64_t i = 0; i < d->n; ++i) out[perm[i]] = h[i];
  return WFPT_OK;
}

int upload(wfpt_ctx* c, const double* x, int64_t n) {
  HIP_TRY(c->x.reserve(std::max<int64_t>(n, 1)));
  if (n > 0)
    HIP_TRY(hipMemcpyAsync(c->x.p, x, n * sizeof(double), hipMemcpyHostToDevice, c->stream));
  return WFPT_OK;
}

}  // namespace

extern "C" {

const char* wfpt_last_error(void) { return g_last_error.c_str(); }

int wfpt_result_poison(double r[3]) {
  if (!r) return fail(WFPT_ERR_ARG, "null pointer");
  r[0] = 0.0;
  r[1] = 0.0;
  r[2] = wfpt::kPeerFailUnit;
  return WFPT_OK;
}

int wfpt_decode_result(const double r[3], double* out) {
  if (!r || !out) return fail(WFPT_ERR_ARG, "null pointer");
  if (int rc = check_status_value(r[2])) return rc;
  *out = (r[1] > 0) ? -INFINITY : r[0];  // any zero-density trial: -inf (wfpt.pyx:71-72)
  return WFPT_OK;
}

int wfpt_device_count(int* n) {
  if (!n) return fail(WFPT_ERR_ARG, "null pointer");
  HIP_TRY(hipGetDeviceCount(n));
  return WFPT_OK;
}

int wfpt_open(int device, wfpt_ctx** out) {
  if (!out) return fail(WFPT_ERR_ARG, "null pointer");
  int nd = 0;
  HIP_TRY(hipGetDeviceCount(&nd));
  if (device < 0 || device >= nd)
    return fail(WFPT_ERR_ARG, "device " + std::to_string(device) + " not present (" +
                                  std::to_string(nd) + " visible)");
  DeviceGuard g(device);
  HIP_TRY(hipSetDevice(device));
  auto* c = new wfpt_ctx();
  c->device = device;
  if (const char* sm = std::getenv("WFPT_SYNC")) c->spin = std::strcmp(sm, "stream") != 0;
  if (const char* nm = std::getenv("WFPT_NODES")) c->nodes_generic = std::strcmp(nm, "generic") == 0;
  if (const char* ns = std::getenv("WFPT_NODE_SPLIT")) c->node_split = std::strcmp(ns, "0") != 0;
  if (const char* nq = std::getenv("WFPT_NODE_SPEC")) c->node_spec = std::strcmp(nq, "0") != 0;
  if (const char* ht = std::getenv("WFPT_HOST_TIMING")) c->host_timing = std::strcmp(ht, "0") != 0;
  if (const char* nt = std::getenv("WFPT_NODE_TABLE_DEV"))
    c->node_table_dev = std::strcmp(nt, "0") != 0;
  if (const char* fm = std::getenv("WFPT_FAST_ONLY")) c->fast_only = std::strcmp(fm, "0") != 0;
  if (const char* lm = std::getenv("WFPT_LEAN")) c->lean = std::strcmp(lm, "0") != 0;
  if (const char* sm = std::getenv("WFPT_SMALL")) c->small = std::strcmp(sm, "0") != 0;
  if (const char* lt = std::getenv("WFPT_LEAN_TREE")) c->lean_tree_max = std::atof(lt);
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreate(&c->ev0);
  if (e == hipSuccess) e = hipEventCreate(&c->ev1);
  if (e == hipSuccess) e = hipMalloc((void**)&c->evals, sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMalloc((void**)&c->status, sizeof(int));
  if (e == hipSuccess) e = hipHostMalloc((void**)&c->host_status, sizeof(int), hipHostMallocDefault);
  if (e == hipSuccess) e = hipMemset(c->status, 0, sizeof(int));
  if (e == hipSuccess)
    e = hipHostMalloc((void**)&c->mres, 8 * sizeof(double),
                      hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&c->mres_dev, c->mres, 0);
  if (e == hipSuccess) e = hipMalloc((void**)&c->n_defer, 4 * sizeof(int));
  if (e == hipSuccess) e = hipMemset(c->n_defer, 0, 4 * sizeof(int));
  if (e == hipSuccess) e = hipMalloc((void**)&c->ncnt, 4 * sizeof(int));
  if (e == hipSuccess) e = hipMemset(c->ncnt, 0, 4 * sizeof(int));
  if (e == hipSuccess) e = hipMalloc((void**)&c->tree_any, sizeof(int));
  if (e == hipSuccess) e = hipMemset(c->tree_any, 0, sizeof(int));
  if (e == hipSuccess) e = hipMalloc((void**)&c->fin, 3 * 64 * sizeof(double));
  if (e == hipSuccess) e = hipMalloc((void**)&c->ar, 8 * sizeof(double));
  if (e == hipSuccess) e = hipMemset(c->ar, 0, 8 * sizeof(double));
  if (e == hipSuccess) e = hipMalloc((void**)&c->fin_ticket, sizeof(int));
  if (e == hipSuccess) e = hipMemset(c->fin_ticket, 0, sizeof(int));
  if (e == hipSuccess) e = hipMalloc((void**)&c->prof, 16 * sizeof(int));
  if (e == hipSuccess) e = hipMemset(c->prof, 0, 16 * sizeof(int));
  if (e == hipSuccess)
    e = hipMalloc((void**)&c->phase, 8 * wfpt::kPhaseWaves * sizeof(unsigned long long));
  if (e == hipSuccess)
    e = hipMemset(c->phase, 0, 8 * wfpt::kPhaseWaves * sizeof(unsigned long long));
  if (e == hipSuccess) std::memset(c->mres, 0, 8 * sizeof(double));
  if (e != hipSuccess) {
    wfpt_close(c);
    return fail(WFPT_ERR_HIP, std::string("wfpt_open: ") + hipGetErrorString(e));
  }
  *out = c;
  return WFPT_OK;
}

void wfpt_close(wfpt_ctx* c) {
  if (!c) return;
  if (c->host_timing && c->ht_calls > 0)
    std::fprintf(stderr,
                 "wfpt host timing over %lld multi-table node calls (us per call): rows %.1f, "
                 "launches %.1f, wait %.1f, copy-out %.1f, total %.1f\n",
                 (long long)c->ht_calls, c->ht[0] / c->ht_calls / 1e3, c->ht[1] / c->ht_calls / 1e3,
                 c->ht[2] / c->ht_calls / 1e3, c->ht[3] / c->ht_calls / 1e3,
                 c->ht[4] / c->ht_calls / 1e3);
  DeviceGuard g(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (wfpt_ds* d : c->dsets) {  // detached: destroying one later frees only its host part
    ds_free_device(d);
    d->ctx = nullptr;
  }
  c->dsets.clear();
  if (c->comm) (void)ncclCommDestroy(c->comm);
  c->x.release();
  c->part.release();
  c->zero.release();
  c->res.release();
  c->lp.release();
  c->marr.release();
  c->mptr.release();
  c->mscal.release();
  c->wl.release();
  c->wl_n.release();
  c->rflag.release();
  if (c->prof) (void)hipFree(c->prof);
  if (c->phase) (void)hipFree(c->phase);
  c->defer.release();
  c->cdf_tab.release();
  c->nd_idx.release();
  c->dnodep.release();
  c->rare_v.release();
  c->rare_j.release();
  c->nd_par.release();
  c->nd_chunks.release();
  if (c->n_defer) (void)hipFree(c->n_defer);
  if (c->ncnt) (void)hipFree(c->ncnt);

  if (c->tree_any) (void)hipFree(c->tree_any);
  if (c->fin) (void)hipFree(c->fin);
  if (c->fin_ticket) (void)hipFree(c->fin_ticket);
  if (c->ar) (void)hipFree(c->ar);
  c->redo.release();
  if (c->evals) (void)hipFree(c->evals);
  if (c->status) (void)hipFree(c->status);
  if (c->host_status) (void)hipHostFree(c->host_status);
  if (c->mres) (void)hipHostFree(c->mres);
  c->mnodep.release();
  c->mnode.release();

  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

void wfpt_shard_range(int64_t n, int nranks, int rank, int64_t* lo, int64_t* hi) {
  if (nranks < 1) nranks = 1;
  const int64_t base = n / nranks, rem = n % nranks;
  const int64_t l = rank * base + std::min<int64_t>(rank, rem);
  *lo = l;
  *hi = l + base + (rank < rem ? 1 : 0);
}

int wfpt_dataset_create(wfpt_ctx* c, const double* rt, int64_t n, const int32_t* node_id,
                        int32_t n_nodes, wfpt_ds** out) {
  return wfpt_dataset_create_ex(c, rt, n, node_id, n_nodes, 0, out);
}

int wfpt_dataset_create_ex(wfpt_ctx* c, const double* rt, int64_t n, const int32_t* node_id,
                           int32_t n_nodes, int flags, wfpt_ds** out) {
  if (!c || !out || (n > 0 && !rt) || n < 0) return fail(WFPT_ERR_ARG, "bad dataset arguments");
  if (flags & ~WFPT_DS_INPUT_ORDER) return fail(WFPT_ERR_ARG, "unknown dataset flags");
  if (node_id && n_nodes <= 0) return fail(WFPT_ERR_ARG, "node ids need n_nodes > 0");
  WFPT_RANGE("wfpt_dataset_create_ex");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  // host-side layout: group by node, order by |rt| inside a node so that each
  // wavefront sees one series branch / similar quadrature depth.
  const bool keep_order = (flags & WFPT_DS_INPUT_ORDER) ||
                          (std::getenv("WFPT_DATASET_ORDER") &&
                           std::strcmp(std::getenv("WFPT_DATASET_ORDER"), "input") == 0);
  std::vector<int64_t> idx(n);
  for (int64_t i = 0; i < n; ++i) idx[i] = i;
  std::vector<int64_t> off;
  if (node_id) {
    for (int64_t i = 0; i < n; ++i)
      if (node_id[i] < 0 || node_id[i] >= n_nodes)
        return fail(WFPT_ERR_ARG, "node id out of range at trial " + std::to_string(i));
    std::vector<int64_t> cnt(n_nodes + 1, 0);
    for (int64_t i = 0; i < n; ++i) cnt[node_id[i] + 1]++;
    for (int32_t j = 0; j < n_nodes; ++j) cnt[j + 1] += cnt[j];
    off = cnt;
    // |rt| order first (stable), then a stable counting placement by node:
    // grouped by node, |rt|-ordered inside a node, ties in input order
    std::vector<int64_t> ord(n);
    for (int64_t i = 0; i < n; ++i) ord[i] = i;
    if (!keep_order) stable_order(ord, rt, false);
    std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1);
    for (int64_t q : ord) idx[pos[node_id[q]]++] = q;
  } else if (!keep_order) {
    // boundary first (x > 0 is the upper boundary, pdf.pxi:116), then |rt|:
    // the lean pass keeps a wave's root z grid in scalar registers when the
    // wave holds one boundary (wfpt_kernels.hip: lean_kernel)
    // (NaN RTs last in their group: a strict weak order for any input)
    stable_order(idx, rt, true);
  }
  std::vector<double> hx(n);
  std::vector<int32_t> hn(node_id ? n : 0);
  for (int64_t i = 0; i < n; ++i) {
    hx[i] = rt[idx[i]];
    if (node_id) hn[i] = node_id[idx[i]];
  }
  auto* d = new wfpt_ds();
  d->ctx = c;
  d->n = n;
  d->input_order = (flags & WFPT_DS_INPUT_ORDER) != 0;
  d->n_nodes = node_id ? n_nodes : 0;
  hipError_t e = hipMalloc((void**)&d->x, std::max<int64_t>(n, 1) * sizeof(double));
  if (e == hipSuccess && n > 0)
    e = hipMemcpy(d->x, hx.data(), n * sizeof(double), hipMemcpyHostToDevice);
  d->identity = !((!keep_order || node_id) && n > 0);
  if (e == hipSuccess && !d->identity) {
    e = hipMalloc((void**)&d->perm, n * sizeof(int64_t));
    if (e == hipSuccess) e = hipMemcpy(d->perm, idx.data(), n * sizeof(int64_t), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess && node_id) {
    e = hipMalloc((void**)&d->node, std::max<int64_t>(n, 1) * sizeof(int32_t));
    if (e == hipSuccess && n > 0)
      e = hipMemcpy(d->node, hn.data(), n * sizeof(int32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc((void**)&d->off, (n_nodes + 1) * sizeof(int64_t));
    if (e == hipSuccess)
      e = hipMemcpy(d->off, off.data(), (n_nodes + 1) * sizeof(int64_t), hipMemcpyHostToDevice);
  }
  // heavy-chunk record (Split): lists sized for up to kSplitCap chunks
  d->nw = (n + 63) / 64;
  d->split_cap = (int)std::min<int64_t>(std::max<int64_t>(d->nw, 1), kSplitCap);
  const int64_t nwb = std::max<int64_t>(d->nw, 1);
  for (int k = 0; k < 2 && e == hipSuccess; ++k) {
    e = hipMalloc((void**)&d->hpred[k], nwb);
    if (e == hipSuccess) e = hipMemset(d->hpred[k], 0, nwb);
    if (e == hipSuccess) e = hipMalloc((void**)&d->hlist[k], d->split_cap * sizeof(int));
  }
  if (e == hipSuccess) e = hipMalloc((void**)&d->hcount, 4 * sizeof(int));
  if (e == hipSuccess) e = hipMemset(d->hcount, 0, 4 * sizeof(int));
  if (e == hipSuccess) e = hipMalloc((void**)&d->hlp, (size_t)d->split_cap * 64 * sizeof(double));
  if (e == hipSuccess) e = hipMalloc((void**)&d->hmeta, (size_t)d->split_cap * 64 * sizeof(int));
  if (e == hipSuccess) e = hipMalloc((void**)&d->hdone, d->split_cap * sizeof(int));
  if (e == hipSuccess) e = hipMemset(d->hdone, 0, d->split_cap * sizeof(int));
  if (e == hipSuccess) e = hipMalloc((void**)&d->hzn, d->split_cap * sizeof(int));
  if (e == hipSuccess) e = hipMemset(d->hzn, 0, d->split_cap * sizeof(int));
  if (e != hipSuccess) {
    ds_free_device(d);
    delete d;
    return fail(WFPT_ERR_HIP, std::string("wfpt_dataset_create: ") + hipGetErrorString(e));
  }
  c->dsets.push_back(d);
  *out = d;
  return WFPT_OK;
}

namespace {
void ds_free_device(wfpt_ds* d) {
  if (d->x) (void)hipFree(d->x);
  if (d->node) (void)hipFree(d->node);
  if (d->off) (void)hipFree(d->off);
  if (d->perm) (void)hipFree(d->perm);
  d->perm = nullptr;
  for (int k = 0; k < 2; ++k) {
    if (d->hpred[k]) (void)hipFree(d->hpred[k]);
    if (d->hlist[k]) (void)hipFree(d->hlist[k]);
  }
  if (d->hcount) (void)hipFree(d->hcount);
  if (d->hlp) (void)hipFree(d->hlp);
  if (d->hmeta) (void)hipFree(d->hmeta);
  if (d->hdone) (void)hipFree(d->hdone);
  if (d->hzn) (void)hipFree(d->hzn);
  d->x = nullptr;
  d->node = nullptr;
  d->off = nullptr;
  d->hpred[0] = d->hpred[1] = nullptr;
  d->hlist[0] = d->hlist[1] = nullptr;
  d->hcount = nullptr;
  d->hlp = nullptr;
  d->hmeta = nullptr;
  d->hdone = nullptr;
  d->hzn = nullptr;
}
}  // namespace

void wfpt_dataset_destroy(wfpt_ds* d) {
  if (!d) return;
  if (wfpt_ctx* c = d->ctx) {
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    (void)hipStreamSynchronize(c->stream);
    c->dsets.erase(std::remove(c->dsets.begin(), c->dsets.end(), d), c->dsets.end());
    ds_free_device(d);
  }
  delete d;
}

int64_t wfpt_dataset_size(const wfpt_ds* d) { return d ? d->n : -1; }

int wfpt_wiener_like(wfpt_ctx* c, const wfpt_ds* d, const wfpt_params* p, const wfpt_knobs* k,
                     double* out) {
  if (!c || !d || !p || !k || !out) return fail(WFPT_ERR_ARG, "null pointer");
  if (d->ctx != c) return fail(WFPT_ERR_ARG, "dataset belongs to another context");
  const wfpt::Params P = to_params(p);
  const wfpt::Knobs K = to_knobs(k);
  if (!p_outlier_in_range(P.p_outlier)) {  // wfpt.pyx:63-64
    *out = -INFINITY;
    return WFPT_OK;
  }
  WFPT_RANGE("wfpt_wiener_like");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  const int rc = run_sum_fast(c, d, P, K, out);
  if (rc >= 0) return rc;
  if (int rc2 = run_sum(c, d->x, d->n, P, K, c->mres_dev, wfpt::kPassAll, d)) return rc2;
  return finish_sum(c, d, P, K, out, false);
}

int wfpt_wiener_like_trials(wfpt_ctx* c, const wfpt_ds* d, const wfpt_params* p,
                            const wfpt_knobs* k, double* out, double* out_trial) {
  if (!c || !d || !p || !k || !out || (!out_trial && d && d->n > 0))
    return fail(WFPT_ERR_ARG, "null pointer");
  if (d->ctx != c) return fail(WFPT_ERR_ARG, "dataset belongs to another context");
  const wfpt::Params P = to_params(p);
  const wfpt::Knobs K = to_knobs(k);
  if (!p_outlier_in_range(P.p_outlier)) {  // wfpt.pyx:63-64: no trial is scored
    *out = -INFINITY;
    for (int64_t i = 0; i < d->n; ++i) out_trial[i] = -INFINITY;
    return WFPT_OK;
  }
  WFPT_RANGE("wfpt_wiener_like_trials");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  HIP_TRY(c->lp.reserve(std::max<int64_t>(d->n, 1)));
  c->trial = c->lp.p;
  int rc = run_sum_fast(c, d, P, K, out);
  if (rc < 0) {
    rc = run_sum(c, d->x, d->n, P, K, c->mres_dev, wfpt::kPassAll, d);
    if (rc == WFPT_OK) rc = finish_sum(c, d, P, K, out, false);
  }
  c->trial = nullptr;
  if (rc != WFPT_OK) return rc;
  return trials_to_caller(d, c->lp.p, out_trial);
}

int wfpt_dataset_order(const wfpt_ds* d, int64_t* perm) {
  if (!d || (!perm && d->n > 0)) return fail(WFPT_ERR_ARG, "null pointer");
  if (d->identity) {  // identity order (input-order or empty dataset): host only
    for (int64_t i = 0; i < d->n; ++i) perm[i] = i;
    return WFPT_OK;
  }
  if (!d->ctx || !d->perm) return fail(WFPT_ERR_ARG, "the dataset's context was closed");
  wfpt_ctx* c = d->ctx;
  std::lock_guard<std::mutex> lk(c->mu);  // serialised with calls on the context
  DeviceGuard g(c->device);
  HIP_TRY(hipMemcpyAsync(perm, d->perm, d->n * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return WFPT_OK;
}

int wfpt_debug_partials(wfpt_ctx* c, double* part, int32_t* zero, int64_t n) {
  if (!c || n < 0 || (n > 0 && (!part || !zero))) return fail(WFPT_ERR_ARG, "bad arguments");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  if ((size_t)n > c->part.cap || (size_t)n > c->zero.cap)
    return fail(WFPT_ERR_ARG, "more partials requested than the last calls wrote");
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (n > 0) {
    HIP_TRY(hipMemcpy(part, c->part.p, n * sizeof(double), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(zero, c->zero.p, n * sizeof(int32_t), hipMemcpyDeviceToHost));
  }
  return WFPT_OK;
}

int wfpt_last_path(wfpt_ctx* c, int* path) {
  if (!c || !path) return fail(WFPT_ERR_ARG, "null pointer");
  std::lock_guard<std::mutex> lk(c->mu);
  *path = c->path;
  return WFPT_OK;
}

int wfpt_wiener_like_host(wfpt_ctx* c, const double* x, int64_t n, const wfpt_params* p,
                          const wfpt_knobs* k, double* out) {
  if (!c || (!x && n > 0) || !p || !k || !out || n < 0) return fail(WFPT_ERR_ARG, "bad arguments");
  const wfpt::Params P = to_params(p);
  const wfpt::Knobs K = to_knobs(k);
  if (!p_outlier_in_range(P.p_outlier)) {
    *out = -INFINITY;
    return WFPT_OK;
  }
  WFPT_RANGE("wfpt_wiener_like_host");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  if (int rc = upload(c, x, n)) return rc;
  if (int rc = run_sum(c, c->x.p, n, P, K, c->mres_dev)) return rc;
  return read_sum(c, c->mres, out);
}

int wfpt_pdf_array(wfpt_ctx* c, const double* x, int64_t n, const wfpt_params* p,
                   const wfpt_knobs* k, int logp, double* out) {
  if (!c || (!x && n > 0) || !p || !k || (!out && n > 0) || n < 0)
    return fail(WFPT_ERR_ARG, "bad arguments");
  const wfpt::Params P = to_params(p);
  const wfpt::Knobs K = to_knobs(k);
  if (n == 0) return WFPT_OK;
  WFPT_RANGE("wfpt_pdf_array");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  if (int rc = upload(c, x, n)) return rc;
  HIP_TRY(c->lp.reserve(n));
  if (int rc = begin_status(c)) return rc;
  wfpt::Work W;
  if (int rc = reserve_work(c, n, &W)) return rc;
  wfpt::launch_trials(1, wfpt::kPassAll, c->x.p, n, P, K, c->lp.p, nullptr, nullptr, c->status,
                      logp == 1, W, c->stream);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out, c->lp.p, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  if (int rc = fetch_status(c)) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  return check_status(c);
}

int wfpt_full_pdf(wfpt_ctx* c, double x, const wfpt_params* p, const wfpt_knobs* k,
                  double* out) {
  if (!p || !k) return fail(WFPT_ERR_ARG, "null pointer");
  wfpt_params q = *p;
  q.p_outlier = 0.0;
  wfpt_knobs kk = *k;
  kk.w_outlier = 0.0;
  return wfpt_pdf_array(c, &x, 1, &q, &kk, 0, out);
}

int wfpt_wiener_like_nodes(wfpt_ctx* c, const wfpt_ds* d, const wfpt_params* per_node,
                           const wfpt_knobs* k, double* out) {
  return wfpt_wiener_like_nodes_ex(c, d, per_node, k, out, nullptr);
}

}  // extern "C"

namespace {
// The per-node pass of a node dataset (everything before the per-node sums):
// the parameter table into mapped pinned memory (node_fast_kernel stages the
// rows each block needs in LDS: no H2D copy per call), the family every node
// selects, and the level-0 / chunk-engine / record kernels writing each
// trial's term to c->lp.
int nodes_launch(wfpt_ctx* c, const wfpt_ds* d, const wfpt_params* per_node,
                 const wfpt::Knobs& K, wfpt::NodeSum* ns, int32_t n_tables = 1) {
  const int32_t m = d->n_nodes;
  const int64_t T = std::max<int32_t>(n_tables, 1);
  const int64_t rows = T * m;  // table t's node j at t m + j
  HIP_TRY(c->mnodep.reserve(std::max<int64_t>(rows, 1)));
  int mode = -2;  // the integration family every node of every table selects, or -1 if mixed
  for (int64_t j = 0; j < rows; ++j) {
    c->mnodep.h[j] = to_params(&per_node[j]);
    const int mj = wfpt::select_mode(per_node[j].sz, per_node[j].st, K.use_adaptive);
    mode = (mode == -2 || mode == mj) ? mj : -1;
  }
  if (c->host_timing) c->ht_mark = std::chrono::steady_clock::now();
  if (mode > wfpt::kAdaptTZ) mode = -1;  // fixed Simpson: generic kernel
  if (c->nodes_generic) mode = -1;
  HIP_TRY(c->res.reserve((size_t)rows + 1));
  if (mode >= 0) {  // deferred records / listed chunks of the per-node fast path
    HIP_TRY(c->nd_idx.reserve(std::max<int64_t>(T * d->n, 1)));
    HIP_TRY(c->nd_par.reserve(std::max<int64_t>(T * d->n, 1)));
    HIP_TRY(c->nd_chunks.reserve(std::max<int64_t>(T * ((d->n + 63) / 64), 1)));
    HIP_TRY(c->rare_v.reserve(std::max<int64_t>(T * d->n, 1)));
    HIP_TRY(c->rare_j.reserve(std::max<int64_t>(T * d->n, 1)));
  }
  // the split level 0 (adaptive t families, non-counting one-table calls):
  // the call's node rows + root z grids in device memory
  const bool split = (mode == wfpt::kAdaptT || mode == wfpt::kAdaptTZ) && !c->count &&
                     c->node_split && T == 1;
  wfpt::NodeTables nt{m, split, !c->count && c->node_spec};
  nt.n_tables = (int32_t)T;
  nt.rare_v = c->rare_v.p;
  nt.rare_j = c->rare_j.p;
  *ns = wfpt::NodeSum{d->x, d->node, c->mnodep.d, &K, mode, c->rare_v.p, c->rare_j.p,
                      c->count ? c->evals : nullptr, c->status};
  c->path = split ? WFPT_PATH_NODE_SPLIT : 0;
  HIP_TRY(c->mnode.reserve((size_t)rows + 2));
  HIP_TRY(c->lp.reserve(std::max<int64_t>(T * d->n, 1)));
  if (c->count) HIP_TRY(hipMemsetAsync(c->evals, 0, sizeof(unsigned long long), c->stream));
  const wfpt::Params* table = c->mnodep.d;
  if (c->node_table_dev && rows > 0) {  // one H2D copy instead of per-block mapped reads
    HIP_TRY(c->dnodep.reserve(rows));
    HIP_TRY(hipMemcpyAsync(c->dnodep.p, c->mnodep.h, rows * sizeof(wfpt::Params),
                           hipMemcpyHostToDevice, c->stream));
    table = c->dnodep.p;
    ns->P = table;
  }
  if (c->profile) HIP_TRY(hipEventRecord(c->ev0, c->stream));
  wfpt::launch_nodes(d->x, d->node, d->n, table, K, mode, c->lp.p, c->nd_idx.p,
                     c->nd_par.p, c->ncnt, c->nd_chunks.p, c->count ? c->evals : nullptr,
                     c->status, c->prof, c->stream, &nt);
  HIP_TRY(hipGetLastError());
  if (c->profile) HIP_TRY(hipEventRecord(c->ev1, c->stream));
  return WFPT_OK;
}

// A node call that failed after its kernels were enqueued: the node counters
// (0 at rest, reset by the call's last kernel) may be left set; restore them.
int nodes_recover(wfpt_ctx* c, int rc) {
  (void)hipStreamSynchronize(c->stream);
  (void)hipMemset(c->ncnt, 0, 4 * sizeof(int));
  return rc;
}

// The per-node sums of the call's n_tables x n_nodes virtual nodes into the
// mapped slot (segment_publish_kernel). A call whose kernels left rare trials
// (the exact path, trees deeper than kTreeDepth: nearly never) is reported
// pending by that launch; its rare trials are then settled (node_rare_kernel)
// and the sums published again: one more host round trip, that call only.
int nodes_publish(wfpt_ctx* c, const wfpt_ds* d, const wfpt::NodeSum& ns, int32_t n_tables) {
  const int32_t m = d->n_nodes;
  const int32_t rows = n_tables * m;
  for (int pass = 0; pass < 2; ++pass) {
    ++c->seq;
    wfpt::launch_segment_sum(c->lp.p, d->off, m, c->res.p, c->mnode.d, c->status, c->seq,
                             c->stream, c->ncnt + 3, c->ncnt, n_tables, d->n, pass == 0);
    if (hipGetLastError() != hipSuccess)
      return nodes_recover(c, fail(WFPT_ERR_HIP, "segment_publish_kernel launch failed"));
    if (int rc = wait_word(c, c->mnode.h + rows + 1)) return nodes_recover(c, rc);
    if (c->mnode.h[rows] != wfpt::kRarePendingHost) break;
    c->path |= WFPT_PATH_NODE_RARE;
    wfpt::launch_node_rare(c->lp.p, ns, c->ncnt, m, d->n, c->stream);
    if (hipGetLastError() != hipSuccess)
      return nodes_recover(c, fail(WFPT_ERR_HIP, "node_rare_kernel launch failed"));
  }
  return check_status_value(c->mnode.h[rows]);
}

int nodes_check(wfpt_ctx* c, const wfpt_ds* d, const wfpt_params* per_node, const wfpt_knobs* k,
                const void* out) {
  if (!c || !d || !per_node || !k || !out) return fail(WFPT_ERR_ARG, "null pointer");
  if (d->ctx != c) return fail(WFPT_ERR_ARG, "dataset belongs to another context");
  if (!d->node) return fail(WFPT_ERR_ARG, "dataset was created without node ids");
  return WFPT_OK;
}
}  // namespace

extern "C" {

int wfpt_wiener_like_nodes_ex(wfpt_ctx* c, const wfpt_ds* d, const wfpt_params* per_node,
                              const wfpt_knobs* k, double* out, double* out_trial) {
  if (int rc = nodes_check(c, d, per_node, k, out)) return rc;
  const wfpt::Knobs K = to_knobs(k);
  WFPT_RANGE("wfpt_wiener_like_nodes");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  const int32_t m = d->n_nodes;
  wfpt::NodeSum ns{};
  if (int rc = nodes_launch(c, d, per_node, K, &ns)) return nodes_recover(c, rc);
  if (m > 0) {
    // per-node sums, status and the completion word land in mapped memory
    // (one launch; its last block resets the node counters)
    if (int rc = nodes_publish(c, d, ns, 1)) return rc;
  } else {
    HIP_TRY(hipStreamSynchronize(c->stream));
  }
  if (int rc = finish_profile(c)) return rc;
  std::memcpy(out, c->mnode.h, m * sizeof(double));
  // each trial's term (node_logp: the node's mixture, log, -inf for a zero
  // density or p_outlier outside [0, 1]) in the caller's trial order
  if (out_trial) return trials_to_caller(d, c->lp.p, out_trial);
  return WFPT_OK;
}

int wfpt_wiener_like_nodes_multi_ex(wfpt_ctx* c, const wfpt_ds* d, const wfpt_params* tables,
                                    int32_t n_tables, const wfpt_knobs* k, double* out,
                                    double* out_trial) {
  if (int rc = nodes_check(c, d, tables, k, out)) return rc;
  if (n_tables < 1) return fail(WFPT_ERR_ARG, "n_tables < 1");
  const int32_t m = d->n_nodes;
  if ((int64_t)n_tables * m > (int64_t)INT32_MAX / 2)
    return fail(WFPT_ERR_ARG, "n_tables x n_nodes too large");
  const wfpt::Knobs K = to_knobs(k);
  WFPT_RANGE("wfpt_wiener_like_nodes_multi");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  const int32_t rows = n_tables * m;
  using clk = std::chrono::steady_clock;
  const auto h0 = clk::now();
  wfpt::NodeSum ns{};
  if (int rc = nodes_launch(c, d, tables, K, &ns, n_tables)) return nodes_recover(c, rc);
  const auto h1 = clk::now();
  if (rows > 0) {
    if (int rc = nodes_publish(c, d, ns, n_tables)) return rc;
  } else {
    if (hipStreamSynchronize(c->stream) != hipSuccess)
      return nodes_recover(c, fail(WFPT_ERR_HIP, "node pass failed on the device"));
    (void)hipMemset(c->ncnt, 0, 4 * sizeof(int));
  }
  if (int rc = finish_profile(c)) return rc;
  const auto h2 = clk::now();
  std::memcpy(out, c->mnode.h, (size_t)rows * sizeof(double));
  if (c->host_timing) {
    const auto h3 = clk::now();
    auto ns_ = [](clk::duration d_) {
      return (double)std::chrono::duration_cast<std::chrono::nanoseconds>(d_).count();
    };
    c->ht[0] += ns_(c->ht_mark - h0);
    c->ht[1] += ns_(h1 - c->ht_mark);
    c->ht[2] += ns_(h2 - h1);
    c->ht[3] += ns_(h3 - h2);
    c->ht[4] += ns_(h3 - h0);
    ++c->ht_calls;
  }
  if (out_trial)
    for (int32_t t = 0; t < n_tables; ++t)
      if (int rc = trials_to_caller(d, c->lp.p + (int64_t)t * d->n, out_trial + (int64_t)t * d->n))
        return rc;
  return WFPT_OK;
}

int wfpt_wiener_like_nodes_multi(wfpt_ctx* c, const wfpt_ds* d, const wfpt_params* tables,
                                 int32_t n_tables, const wfpt_knobs* k, double* out) {
  return wfpt_wiener_like_nodes_multi_ex(c, d, tables, n_tables, k, out, nullptr);
}

int wfpt_wiener_like_nodes_local(wfpt_ctx* c, const wfpt_ds* d, const wfpt_params* per_node,
                                 const wfpt_knobs* k, double* out) {
  if (int rc = nodes_check(c, d, per_node, k, out)) return rc;
  const wfpt::Knobs K = to_knobs(k);
  WFPT_RANGE("wfpt_wiener_like_nodes_local");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  const int32_t m = d->n_nodes;
  wfpt::NodeSum ns{};
  if (int rc = nodes_launch(c, d, per_node, K, &ns)) return nodes_recover(c, rc);
  // every exit after nodes_launch restores the node counters (0 at rest)
  wfpt::launch_segment_res(c->lp.p, d->off, m, c->res.p, c->status, false, c->stream, c->ncnt,
                           &ns);
  if (hipGetLastError() != hipSuccess)
    return nodes_recover(c, fail(WFPT_ERR_HIP, "segment_res launch failed"));
  if (hipMemcpyAsync(out, c->res.p, ((size_t)m + 1) * sizeof(double), hipMemcpyDeviceToHost,
                     c->stream) != hipSuccess)
    return nodes_recover(c, fail(WFPT_ERR_HIP, "node vector copy failed"));
  if (hipStreamSynchronize(c->stream) != hipSuccess)
    return nodes_recover(c, fail(WFPT_ERR_HIP, "node pass failed on the device"));
  return finish_profile(c);
}

int wfpt_wiener_like_nodes_allreduce(wfpt_ctx* c, const wfpt_ds* d, const wfpt_params* per_node,
                                     int32_t n_nodes, const wfpt_knobs* k, double* out) {
  if (!c) return fail(WFPT_ERR_ARG, "null context");
  if (!c->comm) return fail(WFPT_ERR_ARG, "wfpt_comm_init was not called");
  // the exchange's count comes from the argument every rank passes, never
  // from this rank's dataset: a rank with a bad dataset still all-reduces
  // the same n_nodes + 1 doubles as its peers
  if (n_nodes < 0) return fail(WFPT_ERR_ARG, "n_nodes < 0 (no exchange entered)");
  WFPT_RANGE("wfpt_wiener_like_nodes_allreduce");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  // every exit once the communicator exists goes through the exchange: a
  // rank whose pass fails enters it with a poisoned vector
  int lrc = nodes_check(c, d, per_node, k, out);
  const int32_t m = n_nodes;
  if (lrc == WFPT_OK && d->n_nodes != n_nodes)
    lrc = fail(WFPT_ERR_ARG, "dataset has " + std::to_string(d->n_nodes) +
                                 " nodes, the call passes n_nodes = " + std::to_string(n_nodes));
  const wfpt::Knobs K = k ? to_knobs(k) : wfpt::Knobs{};  // (null k: nodes_check failed)
  wfpt::NodeSum ns{};
  if (lrc == WFPT_OK) lrc = nodes_launch(c, d, per_node, K, &ns);
  // fault injection for the failure path's tests (WFPT_FAULT=nodes_allreduce_local:
  // this rank's per-node pass reports a failure after it was enqueued)
  if (lrc == WFPT_OK) {
    const char* fi = std::getenv("WFPT_FAULT");
    if (fi && std::strcmp(fi, "nodes_allreduce_local") == 0)
      lrc = fail(WFPT_ERR_HIP, "injected local failure (WFPT_FAULT=nodes_allreduce_local)");
  }
  std::string lmsg = lrc != WFPT_OK ? g_last_error : std::string();
  if (c->res.cap < (size_t)m + 1) {  // the node vector of an early failure
    if (c->res.reserve((size_t)m + 1) != hipSuccess) {
      (void)ncclCommAbort(c->comm);
      c->comm = nullptr;
      return fail(WFPT_ERR_HIP, "node all-reduce: no device buffer for the exchange "
                                "(RCCL communicator aborted)");
    }
  }
  wfpt::launch_segment_res(lrc == WFPT_OK ? c->lp.p : nullptr, lrc == WFPT_OK ? d->off : nullptr,
                           m, c->res.p, c->status, lrc != WFPT_OK, c->stream, c->ncnt, &ns);
  if (hipGetLastError() != hipSuccess) {
    (void)ncclCommAbort(c->comm);
    c->comm = nullptr;
    return nodes_recover(c, fail(lrc != WFPT_OK ? lrc : WFPT_ERR_HIP,
                                 lmsg + " (device stream unusable: RCCL communicator aborted)"));
  }
  // per-node sums (and the error count) of every rank summed: a node's
  // -inf on any rank reaches every rank (wfpt.pyx:71-72 per node)
  const ncclResult_t nr = ncclAllReduce(c->res.p, c->res.p, (size_t)m + 1, ncclDouble, ncclSum,
                                        c->comm, c->stream);
  if (lrc != WFPT_OK) return nodes_recover(c, fail(lrc, lmsg));
  if (nr != ncclSuccess)
    return nodes_recover(c, fail(WFPT_ERR_COMM, std::string("ncclAllReduce: ") +
                                                    ncclGetErrorString(nr)));
  wfpt::launch_publish_vec(c->res.p, m, c->mnode.d, ++c->seq, c->stream);
  if (hipGetLastError() != hipSuccess)
    return nodes_recover(c, fail(WFPT_ERR_HIP, "publish_vec_kernel launch failed"));
  if (int rc = wait_word(c, c->mnode.h + m + 1)) return nodes_recover(c, rc);
  if (int rc = check_status_value(c->mnode.h[m])) return rc;
  if (int rc = finish_profile(c)) return rc;
  std::memcpy(out, c->mnode.h, m * sizeof(double));
  return WFPT_OK;
}

}  // extern "C"

namespace {
// wiener_like_multi over device x[n]: the per-trial parameter arrays go up for
// this call; a uniform adaptive / direct family (sz and st scalar) takes the
// level-0 pass + deferred records (launch_multi_fast), anything else the
// generic per-trial kernel.
int run_multi(wfpt_ctx* c, const double* dx, int64_t n, const double* const arrays[7],
              const double scalars[7], const wfpt::Knobs& K, double p_outlier, double* out,
              double* out_trial) {
  int na = 0;
  for (int j = 0; j < 7; ++j) na += arrays[j] != nullptr;
  HIP_TRY(c->marr.reserve(std::max<int64_t>((int64_t)na * n, 1)));
  HIP_TRY(c->mptr.reserve(7));
  HIP_TRY(c->mscal.reserve(7));
  double* hptr[7];
  int slot = 0;
  for (int j = 0; j < 7; ++j) {
    if (arrays[j]) {
      hptr[j] = c->marr.p + (int64_t)slot * n;
      if (n > 0)
        HIP_TRY(hipMemcpyAsync(hptr[j], arrays[j], n * sizeof(double), hipMemcpyHostToDevice,
                               c->stream));
      ++slot;
    } else {
      hptr[j] = nullptr;
    }
  }
  HIP_TRY(hipMemcpyAsync(c->mptr.p, hptr, sizeof(hptr), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->mscal.p, scalars, 7 * sizeof(double), hipMemcpyHostToDevice,
                         c->stream));
  const int64_t nb = wfpt::blocks_for(n);
  HIP_TRY(c->part.reserve(std::max<int64_t>(nb, 1)));
  HIP_TRY(c->zero.reserve(std::max<int64_t>(nb, 1)));
  const int mode = (arrays[4] || arrays[6]) ? -1 : wfpt::select_mode(scalars[4], scalars[6],
                                                                     K.use_adaptive);
  if (c->count) HIP_TRY(hipMemsetAsync(c->evals, 0, sizeof(unsigned long long), c->stream));
  if (c->profile) HIP_TRY(hipEventRecord(c->ev0, c->stream));
  if (mode >= 0 && mode <= wfpt::kAdaptTZ && n > 0) {
    HIP_TRY(c->lp.reserve(n));
    HIP_TRY(c->nd_idx.reserve(n));
    HIP_TRY(c->nd_par.reserve(n));
    HIP_TRY(hipMemsetAsync(c->n_defer, 0, sizeof(int), c->stream));
    wfpt::launch_multi_fast(mode, dx, n, c->mptr.p, c->mscal.p, K, p_outlier, c->lp.p,
                            c->nd_idx.p, c->nd_par.p, c->n_defer, c->part.p, c->zero.p,
                            c->count ? c->evals : nullptr, c->status, c->stream);
  } else {
    if (out_trial && n > 0) HIP_TRY(c->lp.reserve(n));
    wfpt::launch_multi(dx, n, c->mptr.p, c->mscal.p, K, p_outlier, c->part.p, c->zero.p,
                       c->status, c->stream, (out_trial && n > 0) ? c->lp.p : nullptr);
  }
  HIP_TRY(hipGetLastError());
  if (c->profile) HIP_TRY(hipEventRecord(c->ev1, c->stream));
  wfpt::launch_finalize(c->part.p, c->zero.p, nb, 0, c->status, c->mres_dev, ++c->seq,
                        c->stream, nullptr, nullptr, nullptr, nullptr, c->fin, c->fin_ticket);
  HIP_TRY(hipGetLastError());
  if (int rc = wait_result(c, c->mres)) return rc;
  if (int rc = check_status_value(c->mres[2])) return rc;
  if (int rc = finish_profile(c)) return rc;
  *out = c->mres[0];
  // each trial's term log(p (1 - p_outlier) + w_outlier p_outlier), or the
  // log prob_ub of a missing response (wfpt.pyx:261-272), in trial order
  if (out_trial && n > 0)
    HIP_TRY(hipMemcpy(out_trial, c->lp.p, n * sizeof(double), hipMemcpyDeviceToHost));
  return WFPT_OK;
}
}  // namespace

extern "C" {

int wfpt_wiener_like_multi(wfpt_ctx* c, const double* x, int64_t n,
                           const double* const arrays[7], const double scalars[7],
                           const wfpt_knobs* k, double p_outlier, double* out) {
  return wfpt_wiener_like_multi_ex(c, x, n, arrays, scalars, k, p_outlier, out, nullptr);
}

int wfpt_wiener_like_multi_ex(wfpt_ctx* c, const double* x, int64_t n,
                              const double* const arrays[7], const double scalars[7],
                              const wfpt_knobs* k, double p_outlier, double* out,
                              double* out_trial) {
  if (!c || (!x && n > 0) || !arrays || !scalars || !k || !out || n < 0)
    return fail(WFPT_ERR_ARG, "bad arguments");
  const wfpt::Knobs K = to_knobs(k);
  WFPT_RANGE("wfpt_wiener_like_multi");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  if (int rc = upload(c, x, n)) return rc;
  return run_multi(c, c->x.p, n, arrays, scalars, K, p_outlier, out, out_trial);
}

int wfpt_wiener_like_multi_resident(wfpt_ctx* c, const wfpt_ds* d, const double* const arrays[7],
                                    const double scalars[7], const wfpt_knobs* k,
                                    double p_outlier, double* out) {
  return wfpt_wiener_like_multi_resident_ex(c, d, arrays, scalars, k, p_outlier, out, nullptr);
}

int wfpt_wiener_like_multi_resident_ex(wfpt_ctx* c, const wfpt_ds* d,
                                       const double* const arrays[7], const double scalars[7],
                                       const wfpt_knobs* k, double p_outlier, double* out,
                                       double* out_trial) {
  if (!c || !d || !arrays || !scalars || !k || !out) return fail(WFPT_ERR_ARG, "null pointer");
  if (d->ctx != c) return fail(WFPT_ERR_ARG, "dataset belongs to another context");
  if (!d->input_order || d->node)
    return fail(WFPT_ERR_ARG,
                "wiener_like_multi on a dataset needs one created with WFPT_DS_INPUT_ORDER "
                "and no node ids (per-trial arrays follow the caller's trial order)");
  const wfpt::Knobs K = to_knobs(k);
  WFPT_RANGE("wfpt_wiener_like_multi_resident");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  return run_multi(c, d->x, d->n, arrays, scalars, K, p_outlier, out, out_trial);
}

int wfpt_dmat_cdf_array(wfpt_ctx* c, const double* x, int64_t n, const wfpt_params* p,
                        double w_outlier, double* out) {
  if (!c || (!x && n > 0) || !p || (!out && n > 0) || n < 0)
    return fail(WFPT_ERR_ARG, "bad arguments");
  const double v = p->v, sv = p->sv, a = p->a, z = p->z, sz = p->sz, t = p->t, st = p->st;
  const double po = p->p_outlier;
  // cdfdif_wrapper.pyx:23-25
  if ((sv < 0) || (a <= 0) || (z < 0) || (z > 1) || (sz < 0) || (sz > 1) || (z + sz / 2. > 1) ||
      (z - sz / 2. < 0) || (t - st / 2. < 0) || (t < 0) || (st < 0) || !p_outlier_in_range(po))
    return fail(WFPT_ERR_ARG, "at least one of the parameters is out of the support");
  if (n == 0) return WFPT_OK;
  if (n >= (int64_t)1 << 31) return fail(WFPT_ERR_ARG, "dmat_cdf_array: n must be < 2^31");
  // cdfdif_wrapper.pyx:35-42 (the model's units: a and z scaled by 1/10, s = 0.1)
  const double epsi = 1e-10;
  const double par[7] = {a / 10., t, sv / 10. + epsi, z * (a / 10.), sz * (a / 10.) + epsi,
                         st + epsi, v / 10.};
  WFPT_RANGE("wfpt_dmat_cdf_array");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  if (int rc = upload(c, x, n)) return rc;
  HIP_TRY(c->lp.reserve(n));
  if (c->profile) HIP_TRY(hipEventRecord(c->ev0, c->stream));
  HIP_TRY(c->defer.reserve(n + 1));
  HIP_TRY(c->cdf_tab.reserve(wfpt::kCdfTableDoubles));
  HIP_TRY(hipMemsetAsync(c->defer.p + n, 0, sizeof(int), c->stream));
  wfpt::launch_dmat_cdf(c->x.p, n, par, po, w_outlier, c->lp.p, c->cdf_tab.p, c->defer.p,
                        c->defer.p + n, c->stream);
  HIP_TRY(hipGetLastError());
  if (c->profile) HIP_TRY(hipEventRecord(c->ev1, c->stream));
  HIP_TRY(hipMemcpyAsync(out, c->lp.p, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (c->profile) {
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    c->k_ms += ms;
    c->launches += 1;
  }
  return WFPT_OK;
}

int wfpt_comm_unique_id(unsigned char id[128]) {
  if (!id) return fail(WFPT_ERR_ARG, "null pointer");
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId u;
  NCCL_TRY(ncclGetUniqueId(&u));
  std::memcpy(id, &u, 128);
  return WFPT_OK;
}

int wfpt_comm_init(wfpt_ctx* c, int nranks, int rank, const unsigned char id[128]) {
  if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(WFPT_ERR_ARG, "bad communicator arguments");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  HIP_TRY(hipSetDevice(c->device));
  ncclUniqueId u;
  std::memcpy(&u, id, 128);
  if (c->comm) {
    (void)ncclCommDestroy(c->comm);
    c->comm = nullptr;
  }
  NCCL_TRY(ncclCommInitRank(&c->comm, nranks, u, rank));
  c->nranks = nranks;
  c->rank = rank;
  return WFPT_OK;
}

int wfpt_comm_init_tcp(wfpt_ctx* c, int nranks, int rank, const char* host, int port,
                       int timeout_ms) {
  if (!c || !host || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(WFPT_ERR_ARG, "bad communicator arguments");
  WFPT_RANGE("wfpt_comm_init_tcp");
  unsigned char id[128];
  std::memset(id, 0, sizeof(id));
  if (rank == 0)
    if (int rc = wfpt_comm_unique_id(id)) return rc;
  if (int rc = wfpt_comm_exchange_id(nranks, rank, host, port, timeout_ms, id)) return rc;
  return wfpt_comm_init(c, nranks, rank, id);
}

int wfpt_comm_init_all(wfpt_ctx* const* ctxs, int n) {
  if (!ctxs || n < 1) return fail(WFPT_ERR_ARG, "bad communicator arguments");
  std::vector<int> devs(n);
  for (int i = 0; i < n; ++i) {
    if (!ctxs[i]) return fail(WFPT_ERR_ARG, "null context");
    devs[i] = ctxs[i]->device;
    for (int j = 0; j < i; ++j)
      if (ctxs[j] == ctxs[i] || devs[j] == devs[i])
        return fail(WFPT_ERR_ARG, "wfpt_comm_init_all: one context per distinct device");
  }
  WFPT_RANGE("wfpt_comm_init_all");
  std::vector<ncclComm_t> comms(n, nullptr);
  for (int i = 0; i < n; ++i) {
    std::lock_guard<std::mutex> lk(ctxs[i]->mu);
    if (ctxs[i]->comm) {
      DeviceGuard g(ctxs[i]->device);
      (void)ncclCommDestroy(ctxs[i]->comm);
      ctxs[i]->comm = nullptr;
    }
  }
  NCCL_TRY(ncclCommInitAll(comms.data(), n, devs.data()));
  for (int i = 0; i < n; ++i) {
    std::lock_guard<std::mutex> lk(ctxs[i]->mu);
    ctxs[i]->comm = comms[i];
    ctxs[i]->nranks = n;
    ctxs[i]->rank = i;
  }
  return WFPT_OK;
}

}  // extern "C"

namespace {
// One rank's local part of an all-reduce likelihood, in two steps so that a
// single process can overlap its devices (wfpt_wiener_like_allreduce_group):
// ar_launch enqueues the level-0 pass (+ the deferred pass unless the lean
// prediction applies) whose finalize leaves {sum, #zeros, errors} in the
// context's dedicated device triple c->ar; ar_settle waits for a lean call's
// level-0 result and, on a misprediction, enqueues the redo + fold passes and
// a second finalize over the intact chunk partials (an unconditional redo
// launch would dispatch one wave per chunk: ~48k blocks at 12.5M trials).
// After ar_settle, c->ar holds the rank's triple in stream order.
struct ArState {
  bool eng = false, lean = false, launched = false;
};
int ar_launch(wfpt_ctx* c, const wfpt_ds* d, const wfpt::Params& P, const wfpt::Knobs& K,
              ArState* st) {
  st->eng = engine_family(P, K);
  st->lean = st->eng && lean_predicted(c, d) && !c->count;
  st->launched = true;
  if (st->lean)
    return run_sum(c, d->x, d->n, P, K, c->mres_dev, wfpt::kPassFast | wfpt::kPassLean, d, c->ar);
  return run_sum(c, d->x, d->n, P, K, c->ar, wfpt::kPassAll, d);
}
int ar_settle(wfpt_ctx* c, const wfpt_ds* d, const wfpt::Params& P, const wfpt::Knobs& K,
              const ArState& st) {
  if (!st.lean) return WFPT_OK;
  if (int rc = wait_result(c, c->mres)) return rc;
  if (res_deferred(c->mres))
    return run_sum(c, d->x, d->n, P, K, c->mres_dev, wfpt::kPassDeferred | wfpt::kPassRedo, d,
                   c->ar);
  return WFPT_OK;
}
// After the exchange: the summed triple to the mapped slot with a fresh
// completion word (the local finalize used the previous one), then decode.
int ar_finish(wfpt_ctx* c, const wfpt_ds* d, const ArState& st, double* out) {
  wfpt::launch_publish(c->ar, c->mres_dev, ++c->seq, c->stream);
  HIP_TRY(hipGetLastError());
  if (int rc = wait_result(c, c->mres)) return rc;
  split_advance(d, st.eng && !st.lean, c->mres);
  const int rc = decode_sum(c, c->mres, out);
  if (rc == WFPT_OK && st.eng) note_tree(d, c->mres);
  return rc;
}
// A call that failed after its passes may have been enqueued: the dataset's
// heavy-chunk record (written by an engine pass into the next parity's list)
// and its predictions are reset, so the next call starts from a consistent
// state (no split, the full call sequence).
void ar_reset(wfpt_ctx* c, const wfpt_ds* d) {
  if (!d) return;
  (void)hipStreamSynchronize(c->stream);
  d->nsplit = 0;
  d->nsplit2 = 0;
  d->no_defer = false;
  d->no_tree = false;
  d->tree_frac = 1.0;
  if (d->hcount) (void)hipMemset(d->hcount, 0, 4 * sizeof(int));
}
}  // namespace

extern "C" {

int wfpt_wiener_like_allreduce(wfpt_ctx* c, const wfpt_ds* d, const wfpt_params* p,
                               const wfpt_knobs* k, double* out) {
  if (!c) return fail(WFPT_ERR_ARG, "null context");
  // no communicator: no collective exists that a peer could be waiting in
  if (!c->comm) return fail(WFPT_ERR_ARG, "wfpt_comm_init was not called");
  // every exit below, once the communicator exists, goes through the exchange
  if (p && !p_outlier_in_range(p->p_outlier) && d && k && out &&
      d->ctx == c) {
    *out = -INFINITY;  // the same parameters on every rank: no exchange needed
    return WFPT_OK;
  }
  WFPT_RANGE("wfpt_wiener_like_allreduce");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  ArState st;
  int lrc = WFPT_OK;
  if (!d || !p || !k || !out) lrc = fail(WFPT_ERR_ARG, "null pointer");
  else if (d->ctx != c) lrc = fail(WFPT_ERR_ARG, "dataset belongs to another context");
  if (lrc == WFPT_OK) {
    const wfpt::Params P = to_params(p);
    const wfpt::Knobs K = to_knobs(k);
    lrc = ar_launch(c, d, P, K, &st);
    if (lrc == WFPT_OK) lrc = ar_settle(c, d, P, K, st);
  }
  // fault injection for the failure path's tests (WFPT_FAULT=allreduce_local:
  // this rank's local pass reports a failure after it ran)
  if (lrc == WFPT_OK) {
    const char* fi = std::getenv("WFPT_FAULT");
    if (fi && std::strcmp(fi, "allreduce_local") == 0)
      lrc = fail(WFPT_ERR_HIP, "injected local failure (WFPT_FAULT=allreduce_local)");
  }
  std::string lmsg;
  if (lrc != WFPT_OK) {
    // A rank that failed locally still enters the collective, with a
    // poisoned triple (kPeerFailUnit) written by a one-thread kernel into its
    // preallocated device triple (nothing on the host stack is read after
    // this call returns), so no peer waits on it forever; every peer then
    // decodes "a rank failed" and this rank returns its own error. Only a
    // broken stream (a sticky device fault) cannot enqueue the exchange: the
    // communicator is then aborted.
    lmsg = g_last_error;
    wfpt::launch_poison(c->ar, c->stream);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      (void)ncclCommAbort(c->comm);
      c->comm = nullptr;
      if (st.launched) ar_reset(c, d);
      return fail(lrc, lmsg + " (device stream unusable: RCCL communicator aborted; "
                              "re-create it with wfpt_comm_init)");
    }
  }
  // {sum, zeros, encoded errors} of every rank summed: any zero trial or
  // failure anywhere reaches every rank (wfpt_internal.h: the error counts
  // stay apart under the sum)
  const ncclResult_t nr = ncclAllReduce(c->ar, c->ar, 3, ncclDouble, ncclSum, c->comm, c->stream);
  if (lrc != WFPT_OK) {
    (void)hipStreamSynchronize(c->stream);
    if (st.launched) ar_reset(c, d);
    return fail(lrc, lmsg);
  }
  if (nr != ncclSuccess) {
    if (st.launched) ar_reset(c, d);
    return fail(WFPT_ERR_COMM, std::string("ncclAllReduce: ") + ncclGetErrorString(nr));
  }
  return ar_finish(c, d, st, out);
}

int wfpt_wiener_like_local(wfpt_ctx* c, const wfpt_ds* d, const wfpt_params* p,
                           const wfpt_knobs* k, double triple[3]) {
  if (!c || !d || !p || !k || !triple) return fail(WFPT_ERR_ARG, "null pointer");
  if (d->ctx != c) return fail(WFPT_ERR_ARG, "dataset belongs to another context");
  const wfpt::Params P = to_params(p);
  const wfpt::Knobs K = to_knobs(k);
  if (!p_outlier_in_range(P.p_outlier)) {  // -inf on every rank: one zero trial
    triple[0] = 0.0;
    triple[1] = 1.0;
    triple[2] = 0.0;
    return WFPT_OK;
  }
  WFPT_RANGE("wfpt_wiener_like_local");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  ArState st;
  int rc = ar_launch(c, d, P, K, &st);
  if (rc == WFPT_OK) rc = ar_settle(c, d, P, K, st);
  if (rc != WFPT_OK) {
    ar_reset(c, d);
    return rc;
  }
  double h[8];
  HIP_TRY(hipMemcpyAsync(h, c->ar, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  split_advance(d, st.eng && !st.lean, h);
  if (st.eng) note_tree(d, h);
  d->no_defer = false;
  (void)finish_profile(c);
  triple[0] = h[0];
  triple[1] = h[1];
  triple[2] = h[2];
  return WFPT_OK;
}

int wfpt_wiener_like_allreduce_group(wfpt_ctx* const* ctxs, const wfpt_ds* const* dss, int n,
                                     const wfpt_params* p, const wfpt_knobs* k, double* out) {
  if (!ctxs || !dss || n < 1 || !p || !k || !out) return fail(WFPT_ERR_ARG, "null pointer");
  for (int i = 0; i < n; ++i) {
    if (!ctxs[i] || !dss[i]) return fail(WFPT_ERR_ARG, "null context or dataset");
    if (dss[i]->ctx != ctxs[i]) return fail(WFPT_ERR_ARG, "dataset belongs to another context");
    if (!ctxs[i]->comm || ctxs[i]->nranks != n || ctxs[i]->rank != i)
      return fail(WFPT_ERR_ARG, "contexts need wfpt_comm_init_all over the same list");
  }
  const wfpt::Params P = to_params(p);
  const wfpt::Knobs K = to_knobs(k);
  if (!p_outlier_in_range(P.p_outlier)) {
    *out = -INFINITY;
    return WFPT_OK;
  }
  WFPT_RANGE("wfpt_wiener_like_allreduce_group");
  std::vector<std::unique_lock<std::mutex>> locks;
  for (int i = 0; i < n; ++i) locks.emplace_back(ctxs[i]->mu);
  int prev = 0;
  (void)hipGetDevice(&prev);
  std::vector<ArState> st(n);
  // every device's local pass in flight before any wait; a failure on any
  // device ends the call before the collective (no device has entered it)
  int rc = WFPT_OK;
  for (int i = 0; i < n && rc == WFPT_OK; ++i) {
    (void)hipSetDevice(ctxs[i]->device);
    rc = ar_launch(ctxs[i], dss[i], P, K, &st[i]);
  }
  for (int i = 0; i < n && rc == WFPT_OK; ++i) {
    (void)hipSetDevice(ctxs[i]->device);
    rc = ar_settle(ctxs[i], dss[i], P, K, st[i]);
  }
  if (rc == WFPT_OK) {
    ncclResult_t r = ncclGroupStart();
    for (int i = 0; i < n && r == ncclSuccess; ++i)
      r = ncclAllReduce(ctxs[i]->ar, ctxs[i]->ar, 3, ncclDouble, ncclSum, ctxs[i]->comm,
                        ctxs[i]->stream);
    const ncclResult_t r2 = ncclGroupEnd();
    if (r == ncclSuccess) r = r2;
    if (r != ncclSuccess)
      rc = fail(WFPT_ERR_COMM, std::string("ncclAllReduce (group): ") + ncclGetErrorString(r));
  }
  double v = 0.0;
  for (int i = 0; i < n && rc == WFPT_OK; ++i) {
    (void)hipSetDevice(ctxs[i]->device);
    double vi = 0.0;
    rc = ar_finish(ctxs[i], dss[i], st[i], &vi);
    if (i == 0) v = vi;
  }
  if (rc != WFPT_OK) {
    // as the single-context path: a device whose passes were enqueued may
    // hold a half-written heavy-chunk record; every such dataset restarts
    // from the full call sequence
    const std::string msg = g_last_error;
    for (int i = 0; i < n; ++i) {
      if (!st[i].launched) continue;
      (void)hipSetDevice(ctxs[i]->device);
      ar_reset(ctxs[i], dss[i]);
    }
    g_last_error = msg;
  }
  (void)hipSetDevice(prev);
  if (rc == WFPT_OK) *out = v;
  return rc;
}

int wfpt_profile_enable(wfpt_ctx* c, int flags) {
  if (!c) return fail(WFPT_ERR_ARG, "null pointer");
  std::lock_guard<std::mutex> lk(c->mu);
  c->profile = (flags & WFPT_PROF_EVENTS) != 0;
  c->count = (flags & WFPT_PROF_EVALS) != 0;
  return WFPT_OK;
}

int wfpt_profile_read(wfpt_ctx* c, double* kernel_ms, int64_t* launches, int64_t* n_evals,
                      int reset) {
  if (!c) return fail(WFPT_ERR_ARG, "null pointer");
  std::lock_guard<std::mutex> lk(c->mu);
  if (kernel_ms) *kernel_ms = c->k_ms;
  if (launches) *launches = c->launches;
  if (n_evals) *n_evals = c->n_evals;
  if (reset) {
    c->k_ms = 0.0;
    c->launches = 0;
    c->n_evals = 0;
  }
  return WFPT_OK;
}

int wfpt_profile_lists(wfpt_ctx* c, int64_t counts[16], int reset) {
  if (!c || !counts) return fail(WFPT_ERR_ARG, "null pointer");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  int h[16];
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipMemcpy(h, c->prof, sizeof(h), hipMemcpyDeviceToHost));
  for (int k = 0; k < 16; ++k) counts[k] = h[k];
  std::vector<unsigned long long> ph(8 * wfpt::kPhaseWaves);
  HIP_TRY(hipMemcpy(ph.data(), c->phase, ph.size() * sizeof(ph[0]), hipMemcpyDeviceToHost));
  for (int k = 0; k < 5; ++k) {
    unsigned long long t = 0;
    for (int w = 0; w < wfpt::kPhaseWaves; ++w) t += ph[w * 8 + 2 + k];
    counts[11 + k] = (int64_t)(t / 1000);
  }
  if (reset) {
    HIP_TRY(hipMemset(c->prof, 0, sizeof(h)));
    HIP_TRY(hipMemset(c->phase, 0, ph.size() * sizeof(ph[0])));
  }
  return WFPT_OK;
}

int wfpt_debug_waves(wfpt_ctx* c, uint64_t* out, int64_t max_records) {
  if (!c || !out) return fail(WFPT_ERR_ARG, "null pointer");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  HIP_TRY(hipStreamSynchronize(c->stream));
  const int64_t n = std::min<int64_t>(max_records, wfpt::kPhaseWaves);
  HIP_TRY(hipMemcpy(out, c->phase, n * 8 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return WFPT_OK;
}

int wfpt_synchronize(wfpt_ctx* c) {
  if (!c) return fail(WFPT_ERR_ARG, "null pointer");
  DeviceGuard g(c->device);
  HIP_TRY(hipStreamSynchronize(c->stream));
  return WFPT_OK;
}

}  // extern "C"
