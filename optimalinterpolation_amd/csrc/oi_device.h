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

struct OiCell {
  double* L;          // packed lower tiles (T(T+1)/2 * 4096)
  double* W;          // packed lower tiles of L^-1 (eval mode), else null
  double* Dinv;       // T * 4096
  double* P;          // T * 4096: P_jk = -Dinv_jj L_jk of the current block column
  double* vec;        // 4 * T * 64: z | alpha | kstar | v
  double* part;       // partial sums, see OI_PART_*
  const double* xyt;  // n x 3 inputs (device)
  const double* r;    // n residuals y - mX (device)
  double* out;        // OI_OUT_N doubles of results
  int32_t* status;    // one int
  int32_t n, T, mode, pad_;
  double hyp[5];      // lx, ly, lt, sf2, sn2 (the values the objective uses)
  double xs[3];       // prediction target (predict mode)
  double mean;        // prior mean (predict mode)
  double pad2_[2];
};

// partial-sum layout inside OiCell::part (ntile = T(T+1)/2)
#define OI_PART_GRAD(ntile) 0              // 5 per tile: s0 s1 s2 sK2 trace
#define OI_PART_QUAD(ntile) (5 * (ntile))  // T: r_k . alpha_k
#define OI_PART_LOGDET(ntile, T) (5 * (ntile) + (T))  // T: sum log diag(L_kk)
#define OI_PART_SIZE(ntile, T) (5 * (ntile) + 2 * (T))

// results inside OiCell::out
//   eval   : [0] nlZ, [1..6] dnlZ
//   predict: [0] fs, [1] sd, [2] lZ
#define OI_OUT_N 8

#ifdef __cplusplus
extern "C" {
#endif
// kernel launchers (oi_kernels.hip); `cells` and `list` are device pointers,
// `list` holds indices into `cells` sorted by T descending.
int oi_launch_build(const OiCell* cells, const int32_t* list, int ncell, int maxT, void* stream);
int oi_launch_diag_factor(const OiCell* cells, const int32_t* list, int ncell, int j, void* stream);
int oi_launch_scale(const OiCell* cells, const int32_t* list, int ncell, int j, int kbeg,
                    void* stream);
int oi_launch_chol_panel(const OiCell* cells, const int32_t* list, int ncell, int maxT, int j,
                         int kbeg, int with_trtri, void* stream);
int oi_launch_panel_even(const OiCell* cells, const int32_t* list, int ncell, int maxT, int j,
                         int with_trtri, void* stream);
int oi_launch_zvec(const OiCell* cells, const int32_t* list, int ncell, int maxT, void* stream);
int oi_launch_avec(const OiCell* cells, const int32_t* list, int ncell, int maxT, void* stream);
int oi_launch_lauum_grad(const OiCell* cells, const int32_t* list, int ncell, int maxT,
                         void* stream);
int oi_launch_predict(const OiCell* cells, const int32_t* list, int ncell, void* stream);
int oi_launch_finalize(const OiCell* cells, const int32_t* list, int ncell, void* stream);
// r[a] = y[a] - (mX ? mX[a] : 1.0 * mean)
int oi_set_debug(int on);
int oi_launch_residual(const double* y, const double* mX, double mean, double* r, int64_t N,
                       void* stream);
#ifdef __cplusplus
}
#endif
