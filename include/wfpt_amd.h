/*
 * wfpt_amd — MI355X (gfx950) Wiener first-passage-time likelihood engine.
 *
 * C ABI that replaces the reference's `wfpt` Cython extension module on its
 * hot path. Plain pointers and sizes only; device memory, streams and RCCL
 * communicators live behind opaque handles. Every entry point returns a
 * status (WFPT_OK == 0); a non-zero status is a device / argument error and is
 * never folded into a numeric result. Numeric failure keeps the reference's
 * conventions exactly: -inf for an impossible likelihood, 0 for an invalid
 * parameter set per trial, NaN where the reference yields NaN (a == 0).
 *
 * Reference interfaces replaced (file:line under the reference tree):
 *   wfpt_wiener_like*      <- wfpt.wiener_like         src/wfpt.pyx:54-76
 *   wfpt_pdf_array         <- wfpt.pdf_array           src/wfpt.pyx:32-48
 *   wfpt_full_pdf          <- wfpt.full_pdf (cpdef)    src/pdf.pxi:104-146
 *   wfpt_wiener_like_nodes <- one wfpt_like per PyMC node, batched
 *   wfpt_wiener_like_nodes_multi <- the same for several parameter tables (chains)
 *                             hddm/likelihoods.py:52-73 via base.py:754-757
 *   wfpt_wiener_like_multi <- wfpt.wiener_like_multi   src/wfpt.pyx:244-274
 *   wfpt_dmat_cdf_array    <- cdfdif_wrapper.dmat_cdf_array
 *                             src/cdfdif_wrapper.pyx:16-53, src/cdfdif.c:59-221
 * The Python binding that keeps the reference signatures is
 * hddm_amd/wfpt.py (ctypes); INTEGRATION.md shows the drop-in.
 */
#ifndef WFPT_AMD_H
#define WFPT_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WFPT_OK 0
#define WFPT_ERR_HIP 1         /* HIP runtime / kernel failure */
#define WFPT_ERR_ARG 2         /* bad argument (null pointer, size, depth) */
#define WFPT_ERR_COMM 3        /* RCCL failure */
#define WFPT_ERR_UNSUPPORTED 4 /* e.g. n_st/n_sz beyond WFPT_MAX_DEPTH */

/* Maximum adaptive-Simpson recursion depth (n_st, n_sz) supported on device.
 * The reference recurses without bound; 2^24 leaves per trial is far past any
 * practical use (HDDM passes 2, wiener_like's default is 10). */
#define WFPT_MAX_DEPTH 24
/* Per-trial cap on pdf_sv evaluations (2^24). The heaviest call in the
 * reference's own tests needs 1.2e5 (wiener_like defaults n=10,
 * simps_err=1e-8). Exceeding either limit fails the call with
 * WFPT_ERR_UNSUPPORTED; no value is returned. */
#define WFPT_EVAL_BUDGET (1ll << 24)

typedef struct wfpt_ctx wfpt_ctx;
typedef struct wfpt_ds wfpt_ds;

/* DDM parameters of one likelihood call (src/wfpt.pyx:54: v sv a z sz t st
 * p_outlier). */
typedef struct wfpt_params {
    double v, sv, a, z, sz, t, st, p_outlier;
} wfpt_params;

/* Numerical knobs (src/wfpt.pyx:55-56). All explicit: the reference's own
 * defaults differ between wiener_like and pdf_array. */
typedef struct wfpt_knobs {
    double err;           /* series truncation error (pdf.pxi:36-47) */
    int32_t n_st;         /* max recursion depth over st */
    int32_t n_sz;         /* max recursion depth over sz */
    int32_t use_adaptive; /* 0 => fixed Simpson with n_st/n_sz panels */
    double simps_err;     /* adaptive Simpson tolerance */
    double w_outlier;     /* outlier density */
} wfpt_knobs;

/* ---- context ---------------------------------------------------------- */
int wfpt_device_count(int *n);
int wfpt_open(int device, wfpt_ctx **out);
void wfpt_close(wfpt_ctx *ctx);
/* message of the last failing call on this thread ("" if none) */
const char *wfpt_last_error(void);

/* ---- resident datasets ------------------------------------------------- */
/* Uploads rt[n] (signed RTs, sign = boundary, hddm/utils.py:15-37) once.
 * node_id (nullable) assigns each trial to one of n_nodes likelihood nodes
 * (hierarchical models); trials are regrouped by node and, inside a node,
 * ordered by |rt| so one wavefront sees one series branch.
 * The caller's arrays are not retained. */
int wfpt_dataset_create(wfpt_ctx *ctx, const double *rt, int64_t n, const int32_t *node_id,
                        int32_t n_nodes, wfpt_ds **out);
/* As wfpt_dataset_create; flags: WFPT_DS_INPUT_ORDER keeps the trials in the
 * caller's order (no |rt| ordering), as wfpt_wiener_like_multi_resident's
 * per-trial parameter arrays require. */
#define WFPT_DS_INPUT_ORDER 1
int wfpt_dataset_create_ex(wfpt_ctx *ctx, const double *rt, int64_t n, const int32_t *node_id,
                           int32_t n_nodes, int flags, wfpt_ds **out);
void wfpt_dataset_destroy(wfpt_ds *ds);
int64_t wfpt_dataset_size(const wfpt_ds *ds);
/* The i-th rank's contiguous shard [lo, hi) of n trials (multi-GPU). */
void wfpt_shard_range(int64_t n, int nranks, int rank, int64_t *lo, int64_t *hi);

/* ---- likelihoods -------------------------------------------------------- */
/* Sum of log mixture densities over a resident dataset (wfpt.pyx:54-76). */
int wfpt_wiener_like(wfpt_ctx *ctx, const wfpt_ds *ds, const wfpt_params *p,
                     const wfpt_knobs *k, double *out_logp);
/* wfpt_wiener_like with each trial's addend of the sum too (the
 * `log(p * (1 - p_outlier) + wp_outlier)` terms of wfpt.pyx:66-74; -inf for a
 * zero mixture density) in out_trial[n], in the caller's trial order. It takes
 * the same predicted call sequence (lean level-0 pass, one-launch small path,
 * engine, redo, fold) as wfpt_wiener_like would, with the same kernels built
 * with one extra store per trial, and leaves the same chunk partials: the
 * per-trial check of the summing path (tests), not a hot-path call. */
int wfpt_wiener_like_trials(wfpt_ctx *ctx, const wfpt_ds *ds, const wfpt_params *p,
                            const wfpt_knobs *k, double *out_logp, double *out_trial);
/* perm[i] = the caller's index of the dataset's stored trial i (datasets are
 * stored grouped by node / boundary and ordered by |rt|; identity for
 * WFPT_DS_INPUT_ORDER). An identity order is answered from the host, also after
 * the dataset's context was closed; a stored permutation lives in device memory
 * and needs the context (WFPT_ERR_ARG once it is closed). The copy is serialised
 * with the context's calls. */
int wfpt_dataset_order(const wfpt_ds *ds, int64_t *perm);
/* Same on a host array (uploaded for this call). */
int wfpt_wiener_like_host(wfpt_ctx *ctx, const double *x, int64_t n, const wfpt_params *p,
                          const wfpt_knobs *k, double *out_logp);
/* Per-node sums for a dataset created with node ids: params[n_nodes] in,
 * out_logp[n_nodes] out (each = wiener_like of that node's trials). */
int wfpt_wiener_like_nodes(wfpt_ctx *ctx, const wfpt_ds *ds, const wfpt_params *per_node,
                           const wfpt_knobs *k, double *out_logp);
/* As wfpt_wiener_like_nodes; out_trial (nullable, ds size) also receives
 * each trial's log term, in the order the caller passed the trials to
 * wfpt_dataset_create: log of the node's mixture p (1 - p_outlier) +
 * w_outlier p_outlier, -inf for a zero mixture density or a p_outlier outside
 * [0, 1] (wfpt.pyx:63-72 per node). */
int wfpt_wiener_like_nodes_ex(wfpt_ctx *ctx, const wfpt_ds *ds, const wfpt_params *per_node,
                              const wfpt_knobs *k, double *out_logp, double *out_trial);
/* n_tables parameter tables over the same resident node dataset in ONE
 * launch: tables[t * n_nodes + j] is node j's row in table t, out_logp[t *
 * n_nodes + j] its sum. Replaces n_tables separate wfpt_like evaluations of
 * every node (hddm/likelihoods.py:52-73, reached once per node per slice
 * evaluation by the reference's samplers): several MCMC chains in lockstep
 * (HDDM's multi-chain usage, docs/source/howto.rst:267-291) or both probes of
 * a slice step's stepping-out. Table t's sums are bit for bit those of
 * wfpt_wiener_like_nodes on table t alone. out_trial (nullable, n_tables x
 * ds size): table t's per-trial terms at out_trial[t * n + i], caller order. */
int wfpt_wiener_like_nodes_multi(wfpt_ctx *ctx, const wfpt_ds *ds, const wfpt_params *tables,
                                 int32_t n_tables, const wfpt_knobs *k, double *out_logp);
int wfpt_wiener_like_nodes_multi_ex(wfpt_ctx *ctx, const wfpt_ds *ds, const wfpt_params *tables,
                                    int32_t n_tables, const wfpt_knobs *k, double *out_logp,
                                    double *out_trial);
/* Per-trial mixture density, or its log if logp != 0 (wfpt.pyx:32-48). */
int wfpt_pdf_array(wfpt_ctx *ctx, const double *x, int64_t n, const wfpt_params *p,
                   const wfpt_knobs *k, int logp, double *out);
/* Single full_pdf (no mixture) (pdf.pxi:104-146). */
int wfpt_full_pdf(wfpt_ctx *ctx, double x, const wfpt_params *p, const wfpt_knobs *k,
                  double *out);
/* Per-trial parameters (wfpt.pyx:244-274). arrays[j] (j = v,sv,a,z,sz,t,st)
 * is a host array of n values or NULL to use scalars[j]. |x| == 999 marks a
 * missing response scored by prob_ub (pdf.pxi:67-72). */
int wfpt_wiener_like_multi(wfpt_ctx *ctx, const double *x, int64_t n,
                           const double *const arrays[7], const double scalars[7],
                           const wfpt_knobs *k, double p_outlier, double *out_logp);
/* As wfpt_wiener_like_multi; out_trial (nullable, n values) also receives
 * each trial's term of the sum (wfpt.pyx:261-272), in trial order. */
int wfpt_wiener_like_multi_ex(wfpt_ctx *ctx, const double *x, int64_t n,
                              const double *const arrays[7], const double scalars[7],
                              const wfpt_knobs *k, double p_outlier, double *out_logp,
                              double *out_trial);
/* Same over a resident dataset created with WFPT_DS_INPUT_ORDER (the RTs of a
 * regression model stay fixed across MCMC; only the per-trial parameter
 * arrays, hddm_regression.py:26-36, go up per call). */
int wfpt_wiener_like_multi_resident(wfpt_ctx *ctx, const wfpt_ds *ds,
                                    const double *const arrays[7], const double scalars[7],
                                    const wfpt_knobs *k, double p_outlier, double *out_logp);
int wfpt_wiener_like_multi_resident_ex(wfpt_ctx *ctx, const wfpt_ds *ds,
                                       const double *const arrays[7], const double scalars[7],
                                       const wfpt_knobs *k, double p_outlier, double *out_logp,
                                       double *out_trial);

/* ---- DMAT / Tuerlinckx CDF ---------------------------------------------- */
/* Per-trial CDF of signed RTs with the outlier mixture, exactly
 * cdfdif_wrapper.dmat_cdf_array(x, v, sv, a, z, sz, t, st, p_outlier, w_outlier)
 * (src/cdfdif_wrapper.pyx:16-53 over cdfdif, src/cdfdif.c:59-221); p->p_outlier
 * is the mixture weight. Parameters outside the support return WFPT_ERR_ARG
 * (the reference raises ValueError, cdfdif_wrapper.pyx:23-25). */
int wfpt_dmat_cdf_array(wfpt_ctx *ctx, const double *x, int64_t n, const wfpt_params *p,
                        double w_outlier, double *out);

/* ---- multi-GPU: trials sharded over GPUs, RCCL all-reduce over xGMI ----- */
/* (The reference has no multi-device path; SURVEY.md §8(e). Every entry point
 * below is new, combining per-shard wiener_like sums, src/wfpt.pyx:66-76.) */
/* One process per GPU. The 128-byte RCCL unique id is created on rank 0 and
 * handed to every rank, either by the caller (wfpt_comm_init) or by the
 * library's own TCP rendezvous: rank 0 listens on host:port and sends the id
 * to each rank that connects (wfpt_comm_exchange_id; no GPU, no PyTorch). */
int wfpt_comm_unique_id(unsigned char id[128]);
int wfpt_comm_init(wfpt_ctx *ctx, int nranks, int rank, const unsigned char id[128]);
int wfpt_comm_exchange_id(int nranks, int rank, const char *host, int port, int timeout_ms,
                          unsigned char id[128]);
/* unique id on rank 0 + wfpt_comm_exchange_id + wfpt_comm_init */
int wfpt_comm_init_tcp(wfpt_ctx *ctx, int nranks, int rank, const char *host, int port,
                       int timeout_ms);
/* wiener_like over this rank's resident shard, combined across ranks with one
 * ncclAllReduce of 3 doubles {sum log p, #zero-density trials, encoded error
 * counts}; every rank receives the global total (-inf if any rank holds a
 * zero-density trial) or every rank fails: WFPT_ERR_UNSUPPORTED if some rank
 * exceeded the depth / evaluation limits; a rank whose call fails after its
 * communicator exists (bad dataset or pointer arguments, workspace allocation,
 * a kernel or timeout error in its local pass) returns its own error after
 * entering the exchange with a poisoned triple (wfpt_result_poison, written on
 * the device into a triple allocated at wfpt_open), and its peers return
 * WFPT_ERR_COMM — no rank is left waiting in the collective. Not covered: a
 * context without a communicator (no collective exists), and a broken device
 * stream (sticky fault), which cannot enqueue the exchange: that rank aborts
 * its communicator, and its peers' collective fails or times out in RCCL. A
 * failed call resets the dataset's call-sequence predictions. */
int wfpt_wiener_like_allreduce(wfpt_ctx *ctx, const wfpt_ds *ds, const wfpt_params *p,
                               const wfpt_knobs *k, double *out_logp);
/* One process driving n GPUs (e.g. a single PyMC sampler): ctxs[i] (distinct
 * devices) get one communicator each from ncclCommInitAll; dss[i] is the i-th
 * shard, resident on ctxs[i]. The group call overlaps the devices' level-0
 * passes and issues the n all-reduces inside one ncclGroupStart/End; a local
 * failure on any device ends the call before the collective. */
int wfpt_comm_init_all(wfpt_ctx *const *ctxs, int n);
int wfpt_wiener_like_allreduce_group(wfpt_ctx *const *ctxs, const wfpt_ds *const *dss, int n,
                                     const wfpt_params *p, const wfpt_knobs *k,
                                     double *out_logp);
/* This rank's local triple {sum log p, #zero-density trials, encoded error
 * counts} of its resident shard — exactly what wfpt_wiener_like_allreduce
 * contributes to its all-reduce — for a caller that combines shards with its
 * own collective (sum the triples, then wfpt_decode_result). A p_outlier
 * outside [0, 1] gives {0, 1, 0} (decodes to -inf). */
int wfpt_wiener_like_local(wfpt_ctx *ctx, const wfpt_ds *ds, const wfpt_params *p,
                           const wfpt_knobs *k, double triple[3]);
/* Hierarchical (batched) mode across ranks ("count =
 * n_nodes"): each rank holds a node dataset of its own trial shard with the
 * global node ids (a node may be split over ranks or absent); its per-node
 * partial sums plus the encoded error count (n_nodes + 1 doubles) are summed
 * with one ncclAllReduce, and every rank receives the per-node totals of all
 * trials in out_logp[n_nodes] (a node with a zero-density trial on any rank is
 * -inf). n_nodes is the length of per_node, the same on every rank; the
 * exchange's count is taken from it, never from the dataset, so a rank whose
 * dataset is bad (null, another context's, without node ids, or with another
 * node count: WFPT_ERR_ARG) still enters the same n_nodes + 1 exchange,
 * poisoned. Failure semantics otherwise as wfpt_wiener_like_allreduce;
 * n_nodes < 0 returns WFPT_ERR_ARG before any collective. */
int wfpt_wiener_like_nodes_allreduce(wfpt_ctx *ctx, const wfpt_ds *ds,
                                     const wfpt_params *per_node, int32_t n_nodes,
                                     const wfpt_knobs *k, double *out_logp);
/* This rank's part of that exchange, for a caller with its own collective:
 * out[n_nodes + 1] = the per-node partial sums of its shard and the encoded
 * error count (sum over ranks, then a nonzero last entry decodes as in
 * wfpt_decode_result's third word). */
int wfpt_wiener_like_nodes_local(wfpt_ctx *ctx, const wfpt_ds *ds, const wfpt_params *per_node,
                                 const wfpt_knobs *k, double *out);
/* The triple a rank that failed before the exchange contributes: {0, 0,
 * 2^40} (one "failed rank" unit; see wfpt_decode_result). */
int wfpt_result_poison(double r[3]);

/* Decodes a likelihood result triple {sum of log p over trials with nonzero
 * density, #zero-density trials, encoded error counts} — the 3 doubles that
 * wfpt_wiener_like_allreduce sums over ranks — into the reference's value:
 * -inf if any trial had zero density (wfpt.pyx:71-72), else the sum; a nonzero
 * error count returns an error naming each kind: WFPT_ERR_UNSUPPORTED for the
 * depth / budget limits, WFPT_ERR_COMM when only failed ranks are counted.
 * Error encoding: (#ranks past WFPT_MAX_DEPTH) + 2^20 * (#ranks past
 * WFPT_EVAL_BUDGET) + 2^40 * (#ranks failed before the exchange), so kinds
 * stay apart under the sum. */
int wfpt_decode_result(const double r[3], double *out_logp);

/* ---- measurement -------------------------------------------------------- */
/* flags & WFPT_PROF_EVENTS: bracket the main likelihood kernel of each call
 * with HIP events on the context's stream (per-launch device time);
 * flags & WFPT_PROF_EVALS: count pdf_sv evaluations (a separate kernel build
 * with one integer atomic per block; use it in an untimed pass). 0 = off. */
#define WFPT_PROF_EVENTS 1
#define WFPT_PROF_EVALS 2
int wfpt_profile_enable(wfpt_ctx *ctx, int flags);
/* Accumulated main-kernel milliseconds, launches and pdf_sv evaluations since
 * the last reset. */
int wfpt_profile_read(wfpt_ctx *ctx, double *kernel_ms, int64_t *launches, int64_t *n_evals,
                      int reset);
/* Refinement work of the adaptive calls made under WFPT_PROF_EVALS since the
 * last reset (synchronises the stream): counts[L] (L = 1, 2) t-node (or z
 * grid) evaluations of tree level L, counts[4] trials whose root interval was
 * refined, counts[5] trials settled on the exact path, counts[6] trials
 * continued on the per-lane walk, counts[7] z walks (counts[8 + L]: at tree
 * level L). counts[11..15]: per-phase engine time of diagnostic builds
 * (WFPT_PHASE_TIMING), kilo-cycles summed over waves. The per-node path
 * (wfpt_wiener_like_nodes, adaptive families) adds to the same counters, plus
 * counts[3] trials its level-0 pass left to the chunk engine and counts[0]
 * node segments the chunk engine ran (one per node present in a listed
 * chunk). */
int wfpt_profile_lists(wfpt_ctx *ctx, int64_t counts[16], int reset);
/* Diagnostic builds (WFPT_PHASE_TIMING): the last engine launch's per-wave
 * records, 8 words per 64-trial chunk {start, end (100 MHz real-time clock),
 * 5 phase cycle counts, z rounds | t rounds << 32}; zeros otherwise. */
int wfpt_debug_waves(wfpt_ctx *ctx, uint64_t *out, int64_t max_records);
/* The first n per-chunk partials {sum of the chunk's log terms, zero word}
 * the last summing call left on the device (64 stored trials per chunk for
 * the adaptive / direct families; synchronises the stream). Tests compare
 * them with the reference's per-chunk sums. */
int wfpt_debug_partials(wfpt_ctx *ctx, double *part, int32_t *zero, int64_t n);
/* Kernels the last likelihood call launched (OR of WFPT_PATH_*). */
#define WFPT_PATH_LEAN 1     /* lean level-0 pass (lean_kernel) */
#define WFPT_PATH_ENGINE 2   /* in-wave adaptive engine over every chunk */
#define WFPT_PATH_SMALL 4    /* one-block level 0 + finalize (small_kernel) */
#define WFPT_PATH_REDO 8     /* engine over the chunks the lean pass flagged */
#define WFPT_PATH_FOLD 16    /* deferred trials (exact path / deep trees) */
#define WFPT_PATH_DIRECT 32  /* simple-DDM level 0 (fast_kernel) */
#define WFPT_PATH_FIXED 64   /* fixed Simpson (trial_kernel) */
#define WFPT_PATH_SPLIT 128  /* heavy chunks split into one-wave units */
#define WFPT_PATH_SMALL_SPLIT 256 /* the full DDM's one-block call, three lanes per
                                     trial (small_split_kernel; with WFPT_PATH_SMALL) */
#define WFPT_PATH_NODE_SPLIT 512  /* per-node call: t-node split level 0
                                     (node_grid_kernel + node_split_kernel) */
#define WFPT_PATH_NODE_RARE 1024  /* per-node call: rare trials (exact path / deep trees)
                                     settled by node_rare_kernel, sums published again */
int wfpt_last_path(wfpt_ctx *ctx, int *path);
int wfpt_synchronize(wfpt_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* WFPT_AMD_H */
