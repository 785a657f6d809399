/* liboi -- MI355X-native per-grid-cell full-GP regression (C ABI).
 *
 * Drop-in boundary for the hot path of William-gregory/OptimalInterpolation,
 * 2021_paper_production/GPR_CS2S3.py (abbreviated GPR: below):
 *
 *   oi_gpr_batch        replaces the per-cell loops GPR:258-261 (pass 1,
 *                       GPR3D(index) with opt=True) and GPR:316-319 (pass 2,
 *                       GPR3D(index, opt=False)): one call fits / predicts a
 *                       ragged batch of cells.  Per cell it computes exactly
 *                       what GPR3D (GPR:143-191) returns.
 *   oi_nlml_grad_batch  replaces SMLII (GPR:107-141) for a batch of cells at
 *                       given log-hyper-parameters.
 *   oi_cg_*             the host optimiser on its own: scipy's
 *                       minimize(method='CG', jac=True) as called at GPR:166,
 *                       driven by caller-supplied objective values.
 *
 * Conventions: plain host pointers, row-major arrays, fp64 throughout.  The
 * library owns all device memory.  Functions return 0 on success or a
 * negative OI_E* code (API misuse / HIP failure; message via oi_last_error).
 * Per-cell numerical failure is NOT an error: as in GPR:139-140 and
 * GPR:187-191, a non-positive-definite covariance gives nlZ = +inf / gradient
 * +inf (objective) or NaN outputs (GPR3D), with status[c] = 1.
 * A cell with zero observations is valid (GPR3D returns (mean, sqrt(sf2), -0, ...)).
 */
#ifndef OI_H
#define OI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OI_VERSION 1

#define OI_E_ARG (-1)    /* invalid argument */
#define OI_E_HIP (-2)    /* HIP runtime / kernel launch failure */
#define OI_E_NOMEM (-3)  /* a single cell does not fit the device workspace */
#define OI_E_NODEV (-4)  /* no usable GPU */

typedef struct oi_options {
  int32_t device;      /* HIP device ordinal (default 0) */
  int32_t maxiter;     /* CG maxiter; <0 => len(x0)*200 = 1200 (scipy default) */
  double gtol;         /* CG gradient tolerance (scipy default 1e-5) */
  void* stream;        /* hipStream_t to launch on; NULL => the library's stream */
  int64_t pool_bytes;  /* device workspace budget; 0 => 60% of free HBM */
  int32_t max_pool;    /* max cells resident at once; 0 => automatic */
  int32_t profile;     /* 1 => record per-kernel HIP-event timings (oi_profile_json) */
  int32_t device_inputs; /* 1 => xyt / z / y / mX are DEVICE pointers already resident
                            in HBM on `device` (offs, xs, x0, hyp, h stay on the host) */
} oi_options;

/* Fill *o with defaults. */
void oi_options_default(oi_options* o);

/* Per-cell GP regression for a ragged batch (GPR3D semantics, GPR:143-191).
 *   xyt    [N x 3]  neighbour inputs (x [m], y [m], t [day]) of all cells,
 *                   cell c owning rows offs[c] .. offs[c+1]-1, in the order
 *                   the caller's neighbour query returned them (GPR:159-160)
 *   z      [N]      observations (GPR:161)
 *   offs   [ncell+1] row offsets, offs[0] = 0, non-decreasing
 *   xs     [ncell x 3] prediction targets (cx, cy, T_mid)  (GPR:164)
 *   mean   prior mean (GPR:212); mX = mean * ones(n)      (GPR:163)
 *   x0     [6] initial log-hyper-parameters (GPR:217); used when opt != 0
 *   opt    1: fit hypers by CG then predict (GPR:166-168)
 *          0: predict with given hypers hyp (GPR:170-172)
 *   hyp    [ncell x 5] (lx, ly, lt, sf2, sn2) when opt == 0, else NULL
 *   out    [ncell x 8] (fs, sd, lZ, lx, ly, lt, sf2, sn2); for opt == 0
 *                   only fs, sd, lZ are meaningful (hyp echoed in 3..7)
 *   status [ncell]   0 ok, 1 covariance not positive definite (NaN outputs)
 *   info   [ncell x 4] or NULL: (nit, cg_status, nfev, n_objective_evals)
 */
int oi_gpr_batch(const double* xyt, const double* z, const int64_t* offs, int64_t ncell,
                 const double* xs, double mean, const double* x0, int32_t opt,
                 const double* hyp, double* out, int32_t* status, int32_t* info,
                 const oi_options* opts);

/* Stream ordering (opts->device_inputs = 1): device inputs are read on
 * opts->stream when it is set; with stream == NULL the library's own stream
 * first waits for the legacy NULL stream (PyTorch's default stream), so any
 * producer of xyt / z / y / mX queued there has finished.  A producer on
 * another stream must pass that stream.  Host outputs are complete on return. */

/* ---- session: continuous batching across calls ------------------------
 * The per-cell loops GPR:258-261 / GPR:316-319 as a stream of batches: every
 * submitted batch (same arguments and semantics as oi_gpr_batch) joins one
 * queue; cells are admitted largest-n first within a batch and FIFO across
 * batches, so cells of the next batch fill the GPU while the previous one's
 * slowest cells finish.  Per-cell results are bitwise the same as one
 * oi_gpr_batch call's (they never depend on which cells share a round).
 *   oi_session_submit  returns a ticket >= 0 (or a negative OI_E* code).  Host
 *                      metadata (offs, xs, x0, hyp) and host inputs are copied
 *                      before it returns; DEVICE inputs and all outputs must
 *                      stay valid until the ticket completes.
 *   oi_session_wait    runs rounds until the ticket completes (ticket < 0: all
 *                      submitted work); it may return with later batches'
 *                      rounds still in flight on the device.
 *   oi_session_set_stream  the stream whose queued work later submissions'
 *                      DEVICE inputs are ordered after (default: opts->stream
 *                      at creation, NULL = the legacy NULL stream); the
 *                      session's rounds keep running on their own stream.
 *   oi_session_done    1 if the ticket has completed, else 0.
 *   oi_session_destroy waits for in-flight rounds and frees the session
 *                      (unfinished cells are dropped, outputs left unwritten).
 * A session is used from one thread at a time. */
typedef struct oi_session oi_session;
oi_session* oi_session_create(const oi_options* opts);
int64_t oi_session_submit(oi_session* s, const double* xyt, const double* z, const int64_t* offs,
                          int64_t ncell, const double* xs, double mean, const double* x0,
                          int32_t opt, const double* hyp, double* out, int32_t* status,
                          int32_t* info);
int oi_session_set_stream(oi_session* s, void* stream);
int oi_session_wait(oi_session* s, int64_t ticket);
int oi_session_done(oi_session* s, int64_t ticket);
void oi_session_destroy(oi_session* s);

/* SMLII (GPR:107-141) for a batch of cells at fixed log-hypers.
 *   xyt, offs as above; y [N] outputs; mX [N] prior mean per observation
 *   h   [ncell x 6] log-hypers (lx, ly, lt, sf2, sn2, unused)
 *   nlz [ncell] ; grad [ncell x 6] (reference gradient incl. its factor-2
 *   components 3 and 4 and the zero 6th component); status [ncell] or NULL
 */
int oi_nlml_grad_batch(const double* xyt, const double* y, const double* mX,
                       const int64_t* offs, int64_t ncell, const double* h, double* nlz,
                       double* grad, int32_t* status, const oi_options* opts);

/* ---- day pipeline: the steps either side of the per-cell loops ----------
 * With opts->device_inputs = 1 every array argument below is a DEVICE pointer
 * on opts->device except vmax, kern and offs, which are always host arrays. */

/* smooth() (GPR:65-76) of nf fields at once -- the five calls GPR:303-307.
 *   fields [nf x ny x nx]  (the reference's 2-D grids, row-major)
 *   vmax   [nf]            clip values (GPR:303-307: 2*radius*1000, .., T, 0.1, 0.05)
 *   mask   [ny x nx]       SIE grid; NaN entries are set to NaN in the output
 *   kern   [ks x ks] or NULL: the Gaussian2DKernel(x_stddev=std) array; NULL =>
 *                          built here from std (astropy's definition)
 *   out    [nf x ny x nx]
 * inf -> NaN, clip at vmax, astropy convolve() defaults (fill 0 boundary,
 * NaN-interpolating renormalised kernel), zeros -> np.nanmean, mask. */
int oi_smooth_fields(const double* fields, int32_t nf, int64_t ny, int64_t nx, const double* vmax,
                     const double* mask, double std, const double* kern, int32_t ks, double* out,
                     const oi_options* opts);

/* X_tree.query_ball_point(X[index], r) (GPR:159) for Q targets at once.
 *   pts [M x 2] training (x, y); q [Q x 2] targets; r radius (same units)
 *   offs [Q+1] (host) always written: target k owns idx[offs[k] .. offs[k+1])
 *   idx  [cap] written only when cap >= offs[Q] (call once with idx = NULL to
 *        size it).  Indices ascending within a target (sorted(ID)); the test
 *        is scipy cKDTree's p=2 one: (dx*dx + dy*dy) <= r*r. */
int oi_ball_query(const double* pts, int64_t M, const double* q, int64_t Q, double r,
                  int64_t* offs, int64_t* idx, int64_t cap, const oi_options* opts);

/* inputs = [x_train, y_train, t_train][ID], outputs = z[ID] (GPR:160-161) for a
 * ragged index list (e.g. oi_ball_query's idx): xyt [N x 3], zout [N].
 * Out-of-range indices are an OI_E_ARG error (host mode) or NaN rows (device). */
int oi_gather_rows(const double* x_train, const double* y_train, const double* t_train,
                   const double* z, int64_t M, const int64_t* idx, int64_t N, double* xyt,
                   double* zout, const oi_options* opts);

/* ---- Nystrom variant (GP_example.ipynb code cell 1: Nystroem, SMLII and GPR
 * with approx=True) -- the rank-M approximation of the notebook -----------
 * Per cell c (rows offs[c] .. offs[c+1]-1):
 *   xyt [N x 3] inputs, y [N] outputs minus the prior mean (NB1 passes
 *       outputs - mX to both SMLII and GPR; GPR adds `mean` back to fs)
 *   sel [soffs[ncell]] inducing rows of each cell, 0-based within the cell
 *       (NB1 Nystroem: sorted(np.random.choice(range(n), M, replace=False))
 *       after np.random.seed(20); the caller draws them)
 *   hyp [ncell x 5] LINEAR (ell_x, ell_y, ell_t, sf2, sn2) as GPR() takes them
 *       (SMLII's log-hypers exponentiated by the caller)
 *   xs  [ncell x 3] prediction targets (needed with pred)
 *   nlz [ncell], grad [ncell x 5]: SMLII(approx=True) (NULL both to skip)
 *   pred [ncell x 3]: (fs = mean + k*.A, sd, prior sd)  (NULL to skip)
 *   status [ncell]: 0 ok, 1 eigh / Cholesky failed (NB1 LinAlgError):
 *       nlZ = grad = +inf, fs = sd = NaN
 * 1 <= M <= n per cell.  With opts->device_inputs xyt and y are device pointers. */
int oi_nystrom_batch(const double* xyt, const double* y, const int64_t* offs, int64_t ncell,
                     const int64_t* sel, const int64_t* soffs, const double* hyp,
                     const double* xs, double mean, double* nlz, double* grad, double* pred,
                     int32_t* status, const oi_options* opts);

/* NB1 code cell 5 for a ragged batch: minimize(SMLII, x0, args=(x, y, True, M),
 * method='CG', jac=True) per cell (the restated scipy CG, maxiter <0 => 1000 =
 * len(x0)*200; gtol from opts), then GPR(approx=True, returnprior=True) at the
 * fitted hypers.
 *   x0  [5] initial log-hypers (NB1: log 25e3, log 25e3, 0, 0, log .1)
 *   out [ncell x 8] (fs, sd, prior sd, ell_x, ell_y, ell_t, sf2, sn2)
 *   status [ncell] as above at the fitted hypers; info [ncell x 4] or NULL:
 *   (nit, cg_status, nfev, n_objective_evals).  Other arguments as above. */
int oi_nystrom_fit_batch(const double* xyt, const double* y, const int64_t* offs, int64_t ncell,
                         const int64_t* sel, const int64_t* soffs, const double* x0,
                         const double* xs, double mean, double* out, int32_t* status,
                         int32_t* info, const oi_options* opts);

/* Nystrom fits as a stream of batches (continuous batching across calls, as
 * oi_session_* for the full GP): every submitted batch (oi_nystrom_fit_batch's
 * arguments; host copies of offs, sel, soffs, x0, xs are taken, DEVICE inputs
 * and all outputs must stay valid until the ticket completes) joins one queue;
 * up to OI_NYS_CAP (32) cells per stream group fit at once and finished cells
 * are replaced from the queue, so a batch's slowest cells overlap later
 * batches.  Per-cell results equal oi_nystrom_fit_batch's bit for bit.
 *   submit returns a ticket >= 0 (or a negative OI_E* code); wait runs rounds
 *   until the ticket completes (ticket < 0: all submitted work). */
typedef struct oi_nystrom_session oi_nystrom_session;
oi_nystrom_session* oi_nystrom_session_create(const oi_options* opts);
int64_t oi_nystrom_session_submit(oi_nystrom_session* s, const double* xyt, const double* y,
                                  const int64_t* offs, int64_t ncell, const int64_t* sel,
                                  const int64_t* soffs, const double* x0, const double* xs, double mean,
                                  double* out, int32_t* status, int32_t* info);
int oi_nystrom_session_wait(oi_nystrom_session* s, int64_t ticket);
void oi_nystrom_session_destroy(oi_nystrom_session* s);

/* ---- SVGP variant (dev/sparseGP_example.ipynb code cell 5: GPflow SVGP with a
 * Matern32 kernel, Gaussian likelihood, Constant mean, whitened q(u), trained
 * by TF2 Adam on minibatches, then predict_f) -- one workgroup per cell runs
 * the whole training in one launch --------------------------------------
 *   xyt [N x 3], y [N]: the cell's inputs and RAW outputs (the Constant mean
 *       function holds the prior mean, as in the notebook)
 *   Z0  [ncell x M x 3] initial inducing inputs (NB2: per-dimension linspace)
 *   init [ncell x 6]: lengthscales (3), kernel variance, noise variance, mean
 *   batch (<= 256) rows per minibatch, iterations Adam steps (TF2 Adam, lr),
 *   log_every: the notebook's training_loss() call after every log_every-th
 *       step (draws one extra minibatch; 0 = none); elbo [ncell x
 *       ceil(iterations/log_every)] receives those ELBO values (or NULL)
 *   seed: minibatch stream of cell c keyed by seed + c (a deterministic
 *       per-epoch permutation; tf.data's shuffle is not reproducible)
 *   xs [ncell x 3] targets; pred [ncell x 2] = predict_f mean, variance of f
 *   params [ncell x oi_svgp_param_count(M)] final unconstrained parameters
 *       (ls_raw[3], var_raw, lik_raw, c, Z[M x 3], q_mu[M], tril(q_sqrt)) or NULL
 *   status [ncell]: 1 if a K_uu Cholesky failed during training
 * 1 <= M <= 64. */
int32_t oi_svgp_param_count(int32_t M);
int oi_svgp_batch(const double* xyt, const double* y, const int64_t* offs, int64_t ncell,
                  const double* Z0, int32_t M, const double* init, int32_t batch,
                  int32_t iterations, int32_t log_every, uint64_t seed, double lr,
                  const double* xs, double* pred, double* params, double* elbo, int32_t* status,
                  const oi_options* opts);

/* ---- host optimiser (scipy 1.15 CG restated; see csrc/cg.hpp) ---- */
typedef struct oi_cg oi_cg;
/* x0: 6 log-hypers. gtol/maxiter as in oi_options (maxiter < 0 => 1200). */
oi_cg* oi_cg_create(const double* x0, double gtol, int32_t maxiter);
/* Advance until the optimiser needs an objective value: returns 1 and writes
 * the requested point to x_req[6]; returns 0 when finished; <0 on misuse. */
int oi_cg_step(oi_cg* h, double* x_req);
/* Supply f and g[6] at the last requested point. */
int oi_cg_feed(oi_cg* h, double f, const double* g);
/* Result after oi_cg_step returned 0: x[6], fun, nit, status (scipy codes),
 * nfev/njev (scipy counters) and nobj (objective evaluations made). */
int oi_cg_result(oi_cg* h, double* x, double* fun, int32_t* nit, int32_t* status,
                 int64_t* nfev, int64_t* njev, int64_t* nobj);
void oi_cg_destroy(oi_cg* h);

/* ---- diagnostics ---- */
const char* oi_last_error(void);  /* thread-local message of the last failure */
int32_t oi_version(void);
/* JSON with per-kernel {launches, total_ms, flops} since the last reset
 * (requires opts.profile=1 on the timed calls). Returns bytes needed. */
int64_t oi_profile_json(char* buf, int64_t len);
void oi_profile_reset(void);

#ifdef __cplusplus
}
#endif
#endif /* OI_H */
