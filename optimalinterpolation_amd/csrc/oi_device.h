// Device-side data layout shared by the HIP kernels (oi_kernels.hip) and the
// host engine (engine.cpp).  See DESIGN.md "Data layout in HBM".
//
// A cell with n observations is padded to T = ceil(n/64) blocks of 64.  Its
// covariance lives as the T(T+1)/2 lower 64x64 tiles of a packed tile array,
// tile (i, j), i >= j, at offset (i(i+1)/2 + j) * 4096 doubles.
//   L    : tiles of K + sn2 I, overwritten in place by its Cholesky factor;
//          each tile COLUMN-major (element (r, c) at c*64 + r).
//   W    : tiles of L^-1, each tile ROW-major (element (r, c) at r*64 + c),
//          i.e. the column-major image of L^-T.  Eval mode only.
//   Dinv : T tiles, inverse of each diagonal L tile, column-major.
// Padding rows/cols carry the identity, so the padded factor/inverse are
// block-diagonal [[L, 0], [0, I]] and padded vector entries stay 0.
#pragma once
#include <stdint.h>

#define OI_NB 64
#define OI_TILE (OI_NB * OI_NB)

enum OiMode { OI_MODE_EVAL = 0, OI_MODE_PREDICT = 1 };

// per-cell status bits (device-written)
enum OiStatus { OI_OK = 0, OI_NOT_PD = 1 };
// Duplicate sites and the reference's non-PD branch (GPR:126, :139-140): with
// repeated rows, numpy's n x n Cholesky of K + sn2 I loses the repeated row's
// pivot (exact value ~2 sn2) to rounding once sn2 / sf2 falls below a band that
// grows with n.  Measured on the reference's own cholesky (numpy 2.2.6 /
// OpenBLAS 0.3.29) over synthetic day cells and permutations of them: failure
// probability 50 % at sn2 / sf2 ~ 1e-18 n_obs (n = 500: 42 % at 5e-16;
// n = 1000: 83 % at 1e-15; n = 2000: 50 % at 2e-15), 100 % below a fifth of
// that and 0 % above 5x (tests/test_gpu_parity.py::test_duplicate_nonpd_band).
// The m x m site form stays PD, so k_diag_factor4w(0) flags the cell not-PD below the
// 50 % point (and whenever sf2 + sn2 rounds to sf2).
#define OI_DUP_NONPD_TAU 1e-18

// Duplicate sites.  Observations with identical (x, y, t) (several
// satellites binned into one grid cell on one day) give identical rows of K.
// With n observations at m distinct sites, incidence P (n x m), counts
// c = diag(P^T P), d = sqrt(c) and Kd the m x m kernel of the sites,
//   K + sn2 I = sn2 I + P Kd P^T,   M = D Kd D + sn2 I  (m x m, D = diag d)
// and exactly (no approximation):
//   log det(K + sn2 I) = (n - m) log sn2 + log det M
//   r^T (K + sn2 I)^-1 r = SSW / sn2 + v^T M^-1 v,   v = D^-1 P^T r,
//                          SSW = sum_a (r_a - mean of r over a's site)^2
//   P^T (K + sn2 I)^-1 P = D M^-1 D,   P^T alpha = u = D M^-1 v
//   tr((K + sn2 I)^-1) - alpha^T alpha = (n - m)/sn2 - SSW/sn2^2
//                                        + tr(M^-1) - |M^-1 v|^2
// so SMLII's nlZ and gradient (GPR:124-138) and the predict block
// (GPR:173-182, k* = P kd*) follow from an m x m problem: the kernels below
// run on the SITES (n = m, xyt = site coordinates, r = v, dw = d) and the
// (n - m), SSW terms are added at the end.  Without duplicates m = n, d = 1,
// v = r, SSW = 0 and every formula is the plain one.  k_dedup (once per cell,
// at submission) builds the sites.
struct OiCell {
  double* L;          // packed lower tiles (T(T+1)/2 * 4096)
  double* W;          // packed lower tiles of L^-1 (eval mode), else null
  double* Dinv;       // T * 4096
  double* vec;        // 4 * T * 64: z | alpha | kstar | v.  z = L^-1 r and (predict)
                      // v = L^-1 k* are built in place during the factorisation
  double* part;       // partial sums, see OI_PART_*
  const double* xyt;  // n x 3 site coordinates (device)
  const double* r;    // n site residuals v = D^-1 P^T (y - mX) (device)
  const double* dw;   // n site weights d = sqrt(count) (device)
  double* out;        // OI_OUT_N doubles of results
  int32_t* status;    // one int
  int32_t n, T, mode, n_obs;  // n = sites m; n_obs = observations
  double hyp[5];      // lx, ly, lt, sf2, sn2 (the values the objective uses)
  double xs[3];       // prediction target (predict mode)
  double mean;        // prior mean (predict mode)
  double ssw;         // within-site residual sum of squares SSW
  double pad2_;
};

// partial-sum layout inside OiCell::part (ntile = T(T+1)/2)
#define OI_PART_GRAD(ntile) 0              // 5 per tile: s0 s1 s2 sK2 trace
#define OI_PART_LOGDET(ntile, T) (5 * (ntile) + (T))  // T: sum log diag(L_kk) (T slots before it spare)
#define OI_PART_PRED(ntile, T) (5 * (ntile) + 2 * (T))  // 3 per block: z.z, z.v, v.v
#define OI_PART_SIZE(ntile, T) (5 * (ntile) + 5 * (T))

// results inside OiCell::out
//   eval   : [0] nlZ, [1..6] dnlZ
//   predict: [0] fs, [1] sd, [2] lZ
#define OI_OUT_N 8
#define OI_OUT_STATUS 7  // the cell's status after the round (k_finalize), as a double

#ifdef __cplusplus
extern "C" {
#endif
// kernel launchers (oi_kernels.hip); `cells` and `list` are device pointers,
// `list` holds indices into `cells` sorted by T descending.
int oi_launch_diag_factor(const OiCell* cells, const int32_t* list, int ncell, int j, void* stream);
// the panels stream the L tiles and apply Dinv_jj to the finished sum (post-form);
// fuse_diag: the look-ahead workgroup also factors diagonal tile j+1 (else
// oi_launch_diag_factor(j+1) follows)
int oi_launch_chol_panel(const OiCell* cells, const int32_t* list, int ncell, int maxT, int j,
                         int kbeg, int with_trtri, int fuse_diag, void* stream);
int oi_launch_panel4(const OiCell* cells, const int32_t* list, int ncell, int maxT, int j, int with_trtri,
                     int fuse_diag, void* stream);
int oi_launch_panel_even(const OiCell* cells, const int32_t* list, int ncell, int maxT, int j,
                         int with_trtri, int fuse_diag, void* stream);
int oi_launch_lauum_grad(const OiCell* cells, const int32_t* list, int ncell, int maxT,
                         void* stream);
// flag != nullptr: the last workgroup stores seq to *flag (pinned host) once all
// result rows are in host memory; *done (device, zero) counts finished cells
int oi_launch_finalize(const OiCell* cells, const int32_t* list, int ncell, unsigned* done,
                       unsigned long long* flag, unsigned long long seq, void* stream);
// r[a] = y[a] - (mX ? mX[a] : 1.0 * mean)
int oi_set_debug(int on);
// Sites of every cell of a batch (one workgroup per cell): offs (device,
// ncell+1) index xyt / r by observation; outputs at the same offsets: site
// coordinates (3 per site), v, d; per cell m and SSW.  nodup: every
// observation its own site (m = n, d = 1, v = r, SSW = 0).  maxn: the largest
// n of the batch (sizes the LDS).
int oi_launch_dedup(const double* xyt, const double* r, const int64_t* offs, int ncell, int maxn,
                    int nodup, double* sites, double* v, double* dw, int32_t* mcount, double* ssw,
                    void* stream);
int oi_launch_residual(const double* y, const double* mX, double mean, double* r, int64_t N,
                       void* stream);
#ifdef __cplusplus
}
#endif
