// HIP kernels (gfx950 / CDNA4, fp64) for the per-cell full-GP hot path:
// SMLII (GPR_CS2S3.py:107-141) and the GPR3D predict block (GPR_CS2S3.py:173-182)
// for a ragged batch of independent grid cells.  Data layout: oi_device.h.
//
// Per objective evaluation of a cell (T = ceil(n/64) tiles per side):
//   k_build        K + sn2 I (Matern-3/2, GPR:93-94)                    O(n^2)
//   k_chol_update  left-looking Cholesky, block column j: tile GEMMs on
//                  v_mfma_f64_16x16x4f64; the diagonal tile is then
//                  factored and inverted in LDS                          n^3/3
//   k_trsm_trtri   L_ij = A_ij L_jj^-T  and  row j of W = L^-1           n^3/3
//   k_zvec/k_avec  z = W r, alpha = W^T z (K^-1 r, GPR:127)              O(n^2)
//   k_lauum_grad   K^-1 = W^T W tile by tile, fused with the gradient
//                  traces sum((K^-1 - alpha alpha^T) o dK_j) with K, dK_j
//                  regenerated from coordinates (GPR:130-138)            n^3/3
//   k_finalize     nlZ and dnlZ (GPR:128, GPR:131-138), fixed-order sums
// Predict (GPR:173-182): k_build, Cholesky, then k_predict (two triangular
// solves per cell + fs / sd / lZ).
//
// Every reduction has a fixed order that depends only on the cell, so a
// cell's results are bitwise independent of the batch it runs in.
#include <hip/hip_runtime.h>
#include <math.h>

#include "oi_device.h"

typedef double d4 __attribute__((ext_vector_type(4)));

#define NB OI_NB
#define LDSS 80                 // LDS row stride (doubles): rows k and k+1 fall in
                                // opposite bank halves for ds_read_b64
#define KC 16                   // k-depth of one staged chunk
#define STAGE (KC * LDSS)       // doubles per staged operand chunk
#define GEMM_LDS (4 * STAGE)    // [2 buffers][A, B] = 40 KiB
#define SQRT3 1.7320508075688772
#define LOG2PI 1.8378770664093453  // np.log(2*np.pi)

__device__ __forceinline__ size_t tri(int i) { return (size_t)i * (i + 1) / 2; }
__device__ __forceinline__ double* tileL(const OiCell& c, int i, int j) {
  return c.L + (tri(i) + j) * OI_TILE;
}
__device__ __forceinline__ double* tileW(const OiCell& c, int i, int j) {
  return c.W + (tri(i) + j) * OI_TILE;
}
__device__ __forceinline__ double* tileD(const OiCell& c, int j) {
  return c.Dinv + (size_t)j * OI_TILE;
}

// ------------------------------------------------------------------ GEMM
// One 256-thread workgroup computes a 64x64 tile D. Wave w owns the 32x32
// quadrant (32*(w>>1), 32*(w&1)) as 2x2 blocks of the 16x16 fp64 MFMA.
// Lane l of block (mb, nb) holds D[16mb + (l>>4) + 4r][16nb + (l&15)], r=0..3.
struct Quad {
  d4 c[2][2];
};

__device__ __forceinline__ void quad_zero(Quad& q) {
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b) q.c[a][b] = (d4){0.0, 0.0, 0.0, 0.0};
}

// element coordinates of accumulator entry (mb, nb, r) for this lane
__device__ __forceinline__ int acc_row(int mb, int r) {
  int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  return 32 * (w >> 1) + 16 * mb + (lane >> 4) + 4 * r;
}
__device__ __forceinline__ int acc_col(int nb) {
  int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  return 32 * (w & 1) + 16 * nb + (lane & 15);
}

// D[m][n] += sum_p sum_k A_p[k*64 + m] * B_p[k*64 + n]
// ("k-major" 64x64 operand tiles: a column-major tile X used as X[m][k], or a
// row-major tile used as X^T).  `pair(p, a, b)` returns the p-th tile pair.
// Staging: global -> registers -> LDS, double-buffered in KC-deep chunks.
template <class PairFn>
__device__ __forceinline__ void gemm_kmajor(Quad& acc, double* lds, int npairs, PairFn pair) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1;
  const int nch = npairs * (NB / KC);
  if (nch == 0) return;
  // this thread stages 4 consecutive doubles (k = t/16, m = 4*(t%16)) per operand
  const int sk = t >> 4, sm = (t & 15) * 4;
  double2 ra0, ra1, rb0, rb1;
  auto load = [&](int ch) {
    const double *pa, *pb;
    pair(ch >> 2, pa, pb);
    const int off = (ch & 3) * KC * NB + t * 4;
    ra0 = *(const double2*)(pa + off);
    ra1 = *(const double2*)(pa + off + 2);
    rb0 = *(const double2*)(pb + off);
    rb1 = *(const double2*)(pb + off + 2);
  };
  auto store = [&](int buf) {
    double* As = lds + buf * 2 * STAGE;
    double* Bs = As + STAGE;
    *(double2*)(As + sk * LDSS + sm) = ra0;
    *(double2*)(As + sk * LDSS + sm + 2) = ra1;
    *(double2*)(Bs + sk * LDSS + sm) = rb0;
    *(double2*)(Bs + sk * LDSS + sm + 2) = rb1;
  };
  load(0);
  store(0);
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  for (int ch = 0; ch < nch; ++ch) {
    if (ch + 1 < nch) load(ch + 1);
    const double* As = lds + (ch & 1) * 2 * STAGE;
    const double* Bs = As + STAGE;
#pragma unroll
    for (int kk = 0; kk < KC / 4; ++kk) {
      const int k = kk * 4 + fk;
      double a0 = As[k * LDSS + 32 * wr + fr];
      double a1 = As[k * LDSS + 32 * wr + 16 + fr];
      double b0 = Bs[k * LDSS + 32 * wc + fr];
      double b1 = Bs[k * LDSS + 32 * wc + 16 + fr];
      acc.c[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc.c[0][0], 0, 0, 0);
      acc.c[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc.c[0][1], 0, 0, 0);
      acc.c[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc.c[1][0], 0, 0, 0);
      acc.c[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc.c[1][1], 0, 0, 0);
    }
    if (ch + 1 < nch) store((ch + 1) & 1);
    __syncthreads();
  }
}

// deterministic block reduction of NV values (256 threads), result valid in thread 0
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* red /* >= 4*NV */) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    double x = v[q];
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_down(x, o, 64);
    v[q] = x;
  }
  __syncthreads();
  if (lane == 0)
    for (int q = 0; q < NV; ++q) red[w * NV + q] = v[q];
  __syncthreads();
  if (t == 0)
    for (int q = 0; q < NV; ++q) v[q] = ((red[q] + red[NV + q]) + red[2 * NV + q]) + red[3 * NV + q];
}

__device__ __forceinline__ bool decode_tri(int x, int T, int& i, int& j) {
  if (x >= T * (T + 1) / 2) return false;
  int ii = (int)((sqrt(8.0 * x + 1.0) - 1.0) * 0.5);
  while ((ii + 1) * (ii + 2) / 2 <= x) ++ii;
  while (ii * (ii + 1) / 2 > x) --ii;
  i = ii;
  j = x - ii * (ii + 1) / 2;
  return true;
}

// ------------------------------------------------------------- k_build
// K + sn2*I for tile (i, j), GPR:93-94 and GPR:126; identity on padding.
__global__ __launch_bounds__(256) void k_build(const OiCell* __restrict__ cells,
                                               const int32_t* __restrict__ list) {
  const OiCell& c = cells[list[blockIdx.y]];
  int i, j;
  if (!decode_tri(blockIdx.x, c.T, i, j)) return;
  __shared__ double u[2][3][NB];
  const int t = threadIdx.x, n = c.n;
  if (t < 2 * NB) {
    int side = t >> 6, idx = t & 63, a = (side ? j : i) * NB + idx;
    for (int d = 0; d < 3; ++d) u[side][d][idx] = a < n ? (SQRT3 * c.xyt[3 * a + d]) / c.hyp[d] : 0.0;
  }
  __syncthreads();
  const double sf2 = c.hyp[3], sn2 = c.hyp[4];
  double* Y = tileL(c, i, j);
  for (int e = t; e < OI_TILE; e += 256) {
    int r = e & 63, cc = e >> 6, a = i * NB + r, b = j * NB + cc;
    double val;
    if (a >= n || b >= n) {
      val = (a == b) ? 1.0 : 0.0;
    } else {
      double d0 = u[0][0][r] - u[1][0][cc], d1 = u[0][1][r] - u[1][1][cc], d2 = u[0][2][r] - u[1][2][cc];
      double Q = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
      val = sf2 * ((1.0 + Q) * exp(-Q));
      if (a == b) val += sn2;
    }
    Y[e] = val;
  }
}

// --------------------------------------------------- diagonal tile: potrf
// In-place lower Cholesky of S (64x64, stride 65) with 256 threads.
// Fails exactly when a pivot is <= 0 (NaN pivots propagate, as with the
// reference's numpy/OpenBLAS cholesky).  Returns false on failure.
__device__ bool potrf_lds(double* S) {
  const int t = threadIdx.x;
  for (int cc = 0; cc < NB; ++cc) {
    __syncthreads();
    const double d = S[cc * 65 + cc];
    if (d <= 0.0) return false;  // uniform: every thread read the same value
    const double l = sqrt(d);
    __syncthreads();
    if (t == 0) S[cc * 65 + cc] = l;
    if (t > cc && t < NB) S[t * 65 + cc] /= l;
    __syncthreads();
    const int m = NB - 1 - cc;
    for (int e = t; e < m * m; e += 256) {
      int rr = e / m, ss = e - rr * m;
      if (ss <= rr) {
        int r = cc + 1 + rr, s = cc + 1 + ss;
        S[r * 65 + s] -= S[r * 65 + cc] * S[s * 65 + cc];
      }
    }
  }
  __syncthreads();
  return true;
}

// In-place inverse of the lower-triangular S (LAPACK trti2 order: last column first).
__device__ void trtri_lds(double* S, double* tmp) {
  const int t = threadIdx.x;
  for (int cc = NB - 1; cc >= 0; --cc) {
    __syncthreads();
    const double ajj = 1.0 / S[cc * 65 + cc];
    double x = 0.0;
    if (t > cc && t < NB) {
      // x_t = sum_{k=cc+1}^{t} Sinv[t][k] * S[k][cc]
      for (int k = cc + 1; k <= t; ++k) x += S[t * 65 + k] * S[k * 65 + cc];
    }
    __syncthreads();
    if (t == 0) S[cc * 65 + cc] = ajj;
    if (t > cc && t < NB) S[t * 65 + cc] = -ajj * x;
  }
  __syncthreads();
  (void)tmp;
}

// ------------------------------------------------------- k_chol_update(j)
// Tile (i, j), i >= j:  A_ij -= sum_{k<j} L_ik L_jk^T  (computed transposed so
// that loads and stores of the column-major tiles are coalesced).  The
// diagonal tile is then factored, inverted, and its log-determinant recorded.
__global__ __launch_bounds__(256) void k_chol_update(const OiCell* __restrict__ cells,
                                                     const int32_t* __restrict__ list, int j) {
  __shared__ __attribute__((aligned(16))) double lds[GEMM_LDS];
  const OiCell& c = cells[list[blockIdx.y]];
  const int i = j + blockIdx.x;
  if (i >= c.T || *c.status != OI_OK) return;
  Quad acc;
  quad_zero(acc);
  gemm_kmajor(acc, lds, j, [&](int p, const double*& a, const double*& b) {
    a = tileL(c, j, p);
    b = tileL(c, i, p);
  });
  double* Y = tileL(c, i, j);
  double val[2][2][4];
  for (int mb = 0; mb < 2; ++mb)
    for (int nb = 0; nb < 2; ++nb)
      for (int r = 0; r < 4; ++r) {
        int m = acc_row(mb, r), nn = acc_col(nb);
        val[mb][nb][r] = Y[m * NB + nn] - acc.c[mb][nb][r];  // (Y^T)[m][nn]
      }
  if (i != j) {
    for (int mb = 0; mb < 2; ++mb)
      for (int nb = 0; nb < 2; ++nb)
        for (int r = 0; r < 4; ++r) Y[acc_row(mb, r) * NB + acc_col(nb)] = val[mb][nb][r];
    return;
  }
  // ---- diagonal tile: factor + invert in LDS
  double* S = lds;  // 64 x 65
  __shared__ double red[16];
  __syncthreads();
  for (int mb = 0; mb < 2; ++mb)
    for (int nb = 0; nb < 2; ++nb)
      for (int r = 0; r < 4; ++r) S[acc_row(mb, r) * 65 + acc_col(nb)] = val[mb][nb][r];
  const bool ok = potrf_lds(S);
  const int t = threadIdx.x;
  if (!ok) {
    if (t == 0) *c.status = OI_NOT_PD;
    return;
  }
  // L_jj back to global (column-major, zero upper triangle)
  for (int e = t; e < OI_TILE; e += 256) {
    int r = e & 63, cc = e >> 6;
    Y[e] = r >= cc ? S[r * 65 + cc] : 0.0;
  }
  // log-determinant contribution of this diagonal tile
  {
    double v[1] = {0.0};
    if (t < NB && j * NB + t < c.n) v[0] = log(S[t * 65 + t]);
    block_sum<1>(v, red);
    if (t == 0) {
      const int ntile = c.T * (c.T + 1) / 2;
      c.part[OI_PART_LOGDET(ntile, c.T) + j] = v[0];
    }
  }
  trtri_lds(S, nullptr);
  double* Dj = tileD(c, j);
  for (int e = t; e < OI_TILE; e += 256) {
    int r = e & 63, cc = e >> 6;
    Dj[e] = r >= cc ? S[r * 65 + cc] : 0.0;  // column-major
  }
  if (c.mode == OI_MODE_EVAL) {
    double* Wj = tileW(c, j, j);
    for (int e = t; e < OI_TILE; e += 256) {
      int r = e >> 6, cc = e & 63;
      Wj[e] = r >= cc ? S[r * 65 + cc] : 0.0;  // row-major
    }
  }
}

// --------------------------------------------------- k_trsm_trtri(j)
// blockIdx.x <  T-1-j : L_ij = A_ij Dinv_jj^T for i = j+1+x      (trsm)
// blockIdx.x >= T-1-j : W_j,jj = -Dinv_jj sum_{k=jj}^{j-1} L_jk W_k,jj (row j of L^-1)
__global__ __launch_bounds__(256) void k_trsm_trtri(const OiCell* __restrict__ cells,
                                                    const int32_t* __restrict__ list, int j) {
  __shared__ __attribute__((aligned(16))) double lds[GEMM_LDS];
  const OiCell& c = cells[list[blockIdx.y]];
  const int T = c.T;
  if (j >= T || *c.status != OI_OK) return;
  const int ntrsm = T - 1 - j;
  const int x = blockIdx.x;
  Quad acc;
  quad_zero(acc);
  if (x < ntrsm) {
    const int i = j + 1 + x;
    double* Y = tileL(c, i, j);
    const double* Dj = tileD(c, j);
    gemm_kmajor(acc, lds, 1, [&](int, const double*& a, const double*& b) {
      a = Dj;
      b = Y;
    });
    // acc = L_ij^T ; all global reads of Y are complete
    for (int mb = 0; mb < 2; ++mb)
      for (int nb = 0; nb < 2; ++nb)
        for (int r = 0; r < 4; ++r) Y[acc_row(mb, r) * NB + acc_col(nb)] = acc.c[mb][nb][r];
    return;
  }
  const int jj = x - ntrsm;
  if (c.mode != OI_MODE_EVAL || jj >= j) return;
  // S = sum_{k=jj}^{j-1} L_jk W_k,jj
  gemm_kmajor(acc, lds, j - jj, [&](int p, const double*& a, const double*& b) {
    a = tileL(c, j, jj + p);
    b = tileW(c, jj + p, jj);
  });
  // S -> LDS as [k][n] (stride LDSS), then W_j,jj = -Dinv_jj S
  double* Ss = lds;
  for (int mb = 0; mb < 2; ++mb)
    for (int nb = 0; nb < 2; ++nb)
      for (int r = 0; r < 4; ++r) Ss[acc_row(mb, r) * LDSS + acc_col(nb)] = acc.c[mb][nb][r];
  __syncthreads();
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;
  const int fr = lane & 15, fk = lane >> 4;
  const double* Dj = tileD(c, j);
  Quad acc2;
  quad_zero(acc2);
#pragma unroll 4
  for (int kk = 0; kk < NB / 4; ++kk) {
    const int k = kk * 4 + fk;
    double a0 = Dj[k * NB + 32 * wr + fr];
    double a1 = Dj[k * NB + 32 * wr + 16 + fr];
    double b0 = Ss[k * LDSS + 32 * wc + fr];
    double b1 = Ss[k * LDSS + 32 * wc + 16 + fr];
    acc2.c[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc2.c[0][0], 0, 0, 0);
    acc2.c[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc2.c[0][1], 0, 0, 0);
    acc2.c[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc2.c[1][0], 0, 0, 0);
    acc2.c[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc2.c[1][1], 0, 0, 0);
  }
  double* Wt = tileW(c, j, jj);
  for (int mb = 0; mb < 2; ++mb)
    for (int nb = 0; nb < 2; ++nb)
      for (int r = 0; r < 4; ++r) Wt[acc_row(mb, r) * NB + acc_col(nb)] = -acc2.c[mb][nb][r];
}

// ------------------------------------------------------------- k_zvec
// z_i = sum_{k<=i} W_ik r_k   (one workgroup per (cell, block row i))
__global__ __launch_bounds__(256) void k_zvec(const OiCell* __restrict__ cells,
                                              const int32_t* __restrict__ list) {
  const OiCell& c = cells[list[blockIdx.y]];
  const int i = blockIdx.x;
  if (i >= c.T || *c.status != OI_OK) return;
  const int t = threadIdx.x, m = t >> 2, q = t & 3, n = c.n;
  double s = 0.0;
  for (int k = 0; k <= i; ++k) {
    const double* Wt = tileW(c, i, k) + m * NB + 16 * q;
    const int b0 = k * NB + 16 * q;
#pragma unroll
    for (int cc = 0; cc < 16; ++cc) {
      const int b = b0 + cc;
      s += Wt[cc] * (b < n ? c.r[b] : 0.0);
    }
  }
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  if (q == 0) c.vec[i * NB + m] = s;
}

// ------------------------------------------------------------- k_avec
// alpha_k = sum_{i>=k} W_ik^T z_i ; partial r_k . alpha_k
__global__ __launch_bounds__(256) void k_avec(const OiCell* __restrict__ cells,
                                              const int32_t* __restrict__ list) {
  const OiCell& c = cells[list[blockIdx.y]];
  const int k = blockIdx.x, T = c.T;
  if (k >= T || *c.status != OI_OK) return;
  __shared__ double red[4][NB + 1];
  const int t = threadIdx.x, cc = t & 63, mq = t >> 6, n = c.n;
  const double* z = c.vec;
  double s = 0.0;
  for (int i = k; i < T; ++i) {
    const double* Wt = tileW(c, i, k);
#pragma unroll 4
    for (int mm = 0; mm < 16; ++mm) {
      const int m = 16 * mq + mm;
      s += Wt[m * NB + cc] * z[i * NB + m];
    }
  }
  red[mq][cc] = s;
  __syncthreads();
  if (t < NB) {
    const double a = ((red[0][t] + red[1][t]) + red[2][t]) + red[3][t];
    double* alpha = c.vec + T * NB;
    alpha[k * NB + t] = a;
    const int b = k * NB + t;
    double p = b < n ? c.r[b] * a : 0.0;
    for (int o = 32; o >= 1; o >>= 1) p += __shfl_down(p, o, 64);
    if (t == 0) c.part[OI_PART_QUAD(T * (T + 1) / 2) + k] = p;
  }
}

// ------------------------------------------------------ k_lauum_grad
// Tile (i, j) of K^-1 = W^T W  (K^-1_ij = sum_{k>=i} W_ki^T W_kj), fused with
// sum over the tile of (K^-1 - alpha alpha^T) o {dK_0, dK_1, dK_2, 2K} and its
// trace (GPR:130-138).  Symmetry: strictly-lower entries count twice.
__global__ __launch_bounds__(256) void k_lauum_grad(const OiCell* __restrict__ cells,
                                                    const int32_t* __restrict__ list) {
  __shared__ __attribute__((aligned(16))) double lds[GEMM_LDS];
  __shared__ double red[4 * 5];
  const OiCell& c = cells[list[blockIdx.y]];
  const int T = c.T;
  int i, j;
  if (!decode_tri(blockIdx.x, T, i, j)) return;
  if (*c.status != OI_OK) return;
  Quad acc;
  quad_zero(acc);
  gemm_kmajor(acc, lds, T - i, [&](int p, const double*& a, const double*& b) {
    a = tileW(c, i + p, i);
    b = tileW(c, i + p, j);
  });
  // coordinates of the tile's rows (tile i) and columns (tile j), alpha
  double* uQ = lds;            // [2][3][64] (sqrt3*x)/ell
  double* uq = lds + 6 * NB;   // [2][3][64] sqrt3*(x/ell)
  double* al = lds + 12 * NB;  // [2][64]
  const int t = threadIdx.x, n = c.n;
  if (t < 2 * NB) {
    int side = t >> 6, idx = t & 63, a = (side ? j : i) * NB + idx;
    for (int d = 0; d < 3; ++d) {
      double xv = a < n ? c.xyt[3 * a + d] : 0.0;
      uQ[(side * 3 + d) * NB + idx] = (SQRT3 * xv) / c.hyp[d];
      uq[(side * 3 + d) * NB + idx] = SQRT3 * (xv / c.hyp[d]);
    }
    al[side * NB + idx] = c.vec[T * NB + a];
  }
  __syncthreads();
  const double sf2 = c.hyp[3];
  double s[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  for (int mb = 0; mb < 2; ++mb)
    for (int nb = 0; nb < 2; ++nb)
      for (int r = 0; r < 4; ++r) {
        const int m = acc_row(mb, r), nn = acc_col(nb);
        const int a = i * NB + m, b = j * NB + nn;
        if (a >= n || b >= n || (i == j && m < nn)) continue;
        const double wgt = (a == b) ? 1.0 : 2.0;
        const double w = acc.c[mb][nb][r] - al[m] * al[NB + nn];
        double d0 = uQ[0 * NB + m] - uQ[3 * NB + nn];
        double d1 = uQ[1 * NB + m] - uQ[4 * NB + nn];
        double d2 = uQ[2 * NB + m] - uQ[5 * NB + nn];
        const double Q = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
        const double e = exp(-Q);
        const double K = sf2 * ((1.0 + Q) * e);
        double q0 = uq[0 * NB + m] - uq[3 * NB + nn];
        double q1 = uq[1 * NB + m] - uq[4 * NB + nn];
        double q2 = uq[2 * NB + m] - uq[5 * NB + nn];
        s[0] += wgt * (w * (sf2 * ((q0 * q0) * e)));
        s[1] += wgt * (w * (sf2 * ((q1 * q1) * e)));
        s[2] += wgt * (w * (sf2 * ((q2 * q2) * e)));
        s[3] += wgt * (w * (2.0 * K));
        if (a == b) s[4] += w;
      }
  block_sum<5>(s, red);
  if (t == 0) {
    double* pp = c.part + OI_PART_GRAD(0) + 5 * (size_t)blockIdx.x;
    for (int q = 0; q < 5; ++q) pp[q] = s[q];
  }
}

// ---------------------------------------------------------- k_finalize
// nlZ = r.alpha/2 + sum log diag L + n log(2 pi)/2 (GPR:128); dnlZ (GPR:131-138)
__global__ __launch_bounds__(256) void k_finalize(const OiCell* __restrict__ cells,
                                                  const int32_t* __restrict__ list) {
  const OiCell& c = cells[list[blockIdx.x]];
  if (c.mode != OI_MODE_EVAL) return;
  __shared__ double red[4 * 7];
  const int t = threadIdx.x, T = c.T, ntile = T * (T + 1) / 2;
  if (*c.status != OI_OK) {
    if (t < 7) c.out[t] = INFINITY;
    return;
  }
  double v[7] = {0, 0, 0, 0, 0, 0, 0};
  for (int x = t; x < ntile; x += 256)
    for (int q = 0; q < 5; ++q) v[q] += c.part[OI_PART_GRAD(ntile) + 5 * x + q];
  for (int k = t; k < T; k += 256) {
    v[5] += c.part[OI_PART_QUAD(ntile) + k];
    v[6] += c.part[OI_PART_LOGDET(ntile, T) + k];
  }
  block_sum<7>(v, red);
  if (t == 0) {
    const double quad = v[5], logdet = v[6];
    c.out[0] = (quad / 2 + logdet) + (c.n * LOG2PI) / 2;
    c.out[1] = v[0] / 2;
    c.out[2] = v[1] / 2;
    c.out[3] = v[2] / 2;
    c.out[4] = v[3] / 2;
    c.out[5] = c.hyp[4] * v[4];
    c.out[6] = 0.0;
  }
}

// ----------------------------------------------------------- k_predict
// GPR:173-182 for one cell per workgroup, given L and Dinv:
//   z = L^-1 r, v = L^-1 k*, alpha = L^-T z,
//   fs = mean + k*.alpha, sd = sqrt(sf2 - v.v), lZ = -r.alpha/2 - sum log L_aa - n log(2pi)/2
__global__ __launch_bounds__(256) void k_predict(const OiCell* __restrict__ cells,
                                                 const int32_t* __restrict__ list) {
  const OiCell& c = cells[list[blockIdx.x]];
  if (c.mode != OI_MODE_PREDICT) return;
  const int t = threadIdx.x, T = c.T, n = c.n;
  if (*c.status != OI_OK) {
    if (t < 3) c.out[t] = NAN;
    return;
  }
  __shared__ double red2[4][2][NB + 1];
  __shared__ double tv[2][NB];
  __shared__ double red[4 * 5];
  double* z = c.vec;
  double* alpha = c.vec + T * NB;
  double* ks = c.vec + 2 * T * NB;
  double* v = c.vec + 3 * T * NB;
  const double sf2 = c.hyp[3];
  // k* (GPR:174): cdist of scaled coordinates
  {
    const double xs0 = (SQRT3 * c.xs[0]) / c.hyp[0], xs1 = (SQRT3 * c.xs[1]) / c.hyp[1],
                 xs2 = (SQRT3 * c.xs[2]) / c.hyp[2];
    for (int a = t; a < T * NB; a += 256) {
      double kv = 0.0;
      if (a < n) {
        double d0 = (SQRT3 * c.xyt[3 * a]) / c.hyp[0] - xs0;
        double d1 = (SQRT3 * c.xyt[3 * a + 1]) / c.hyp[1] - xs1;
        double d2 = (SQRT3 * c.xyt[3 * a + 2]) / c.hyp[2] - xs2;
        double Q = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
        kv = sf2 * ((1.0 + Q) * exp(-Q));
      }
      ks[a] = kv;
    }
  }
  __syncthreads();
  // forward: [z v]_i = Dinv_ii ([r ks]_i - sum_{k<i} L_ik [z v]_k)
  const int m = t & 63, cq = t >> 6;
  for (int i = 0; i < T; ++i) {
    double s0 = 0.0, s1 = 0.0;
    for (int k = 0; k < i; ++k) {
      const double* Lt = c.L + (((size_t)i * (i + 1) / 2) + k) * OI_TILE;
      for (int cc = 16 * cq; cc < 16 * cq + 16; ++cc) {
        const double l = Lt[cc * NB + m];
        s0 += l * z[k * NB + cc];
        s1 += l * v[k * NB + cc];
      }
    }
    red2[cq][0][m] = s0;
    red2[cq][1][m] = s1;
    __syncthreads();
    if (t < NB) {
      const int b = i * NB + t;
      const double rb = b < n ? c.r[b] : 0.0;
      tv[0][t] = rb - (((red2[0][0][t] + red2[1][0][t]) + red2[2][0][t]) + red2[3][0][t]);
      tv[1][t] = ks[b] - (((red2[0][1][t] + red2[1][1][t]) + red2[2][1][t]) + red2[3][1][t]);
    }
    __syncthreads();
    const double* Dt = c.Dinv + (size_t)i * OI_TILE;
    s0 = 0.0;
    s1 = 0.0;
    for (int cc = 16 * cq; cc < 16 * cq + 16; ++cc) {
      const double d = Dt[cc * NB + m];
      s0 += d * tv[0][cc];
      s1 += d * tv[1][cc];
    }
    red2[cq][0][m] = s0;
    red2[cq][1][m] = s1;
    __syncthreads();
    if (t < NB) {
      z[i * NB + t] = ((red2[0][0][t] + red2[1][0][t]) + red2[2][0][t]) + red2[3][0][t];
      v[i * NB + t] = ((red2[0][1][t] + red2[1][1][t]) + red2[2][1][t]) + red2[3][1][t];
    }
    __syncthreads();
  }
  // backward: alpha_i = Dinv_ii^T (z_i - sum_{k>i} L_ki^T alpha_k)
  const int mr = t >> 2, q = t & 3;
  for (int i = T - 1; i >= 0; --i) {
    double s0 = 0.0;
    for (int k = i + 1; k < T; ++k) {
      const double* Lt = c.L + (((size_t)k * (k + 1) / 2) + i) * OI_TILE;
      for (int cc = 16 * q; cc < 16 * q + 16; ++cc) s0 += Lt[mr * NB + cc] * alpha[k * NB + cc];
    }
    s0 += __shfl_xor(s0, 1, 64);
    s0 += __shfl_xor(s0, 2, 64);
    if (q == 0) tv[0][mr] = z[i * NB + mr] - s0;
    __syncthreads();
    const double* Dt = c.Dinv + (size_t)i * OI_TILE;
    double s1 = 0.0;
    for (int cc = 16 * q; cc < 16 * q + 16; ++cc) s1 += Dt[mr * NB + cc] * tv[0][cc];
    s1 += __shfl_xor(s1, 1, 64);
    s1 += __shfl_xor(s1, 2, 64);
    if (q == 0) alpha[i * NB + mr] = s1;
    __syncthreads();
  }
  // reductions: k*.alpha, v.v, r.alpha, sum log diag L
  double acc5[4] = {0.0, 0.0, 0.0, 0.0};
  for (int a = t; a < n; a += 256) {
    acc5[0] += ks[a] * alpha[a];
    acc5[1] += v[a] * v[a];
    acc5[2] += c.r[a] * alpha[a];
    const int bi = a >> 6, bm = a & 63;
    acc5[3] += log(c.L[(((size_t)bi * (bi + 1) / 2) + bi) * OI_TILE + bm * NB + bm]);
  }
  block_sum<4>(acc5, red);
  if (t == 0) {
    c.out[0] = c.mean + acc5[0];
    c.out[1] = sqrt(sf2 - acc5[1]);
    c.out[2] = ((-acc5[2]) / 2 - acc5[3]) - (n * LOG2PI) / 2;
  }
}

// ---------------------------------------------------------- k_residual
__global__ void k_residual(const double* __restrict__ y, const double* __restrict__ mX,
                           double mean, double* __restrict__ r, int64_t N) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a < N) r[a] = y[a] - (mX ? mX[a] : 1.0 * mean);
}

// ------------------------------------------------------------ launchers
static inline hipStream_t S(void* s) { return (hipStream_t)s; }
static inline int ret() { return hipGetLastError() == hipSuccess ? 0 : -1; }

#define FOR_CHUNKS(ncell, body)                         \
  for (int base = 0; base < (ncell); base += 65535) {    \
    const int cnt = (ncell) - base < 65535 ? (ncell) - base : 65535; \
    body                                                 \
  }

extern "C" int oi_launch_build(const OiCell* cells, const int32_t* list, int ncell, int maxT,
                               void* stream) {
  if (ncell <= 0 || maxT <= 0) return 0;
  FOR_CHUNKS(ncell, {
    hipLaunchKernelGGL(k_build, dim3(maxT * (maxT + 1) / 2, cnt), dim3(256), 0, S(stream), cells,
                       list + base);
  })
  return ret();
}

extern "C" int oi_launch_chol_update(const OiCell* cells, const int32_t* list, int ncell, int maxT,
                                     int j, void* stream) {
  if (ncell <= 0 || maxT - j <= 0) return 0;
  FOR_CHUNKS(ncell, {
    hipLaunchKernelGGL(k_chol_update, dim3(maxT - j, cnt), dim3(256), 0, S(stream), cells,
                       list + base, j);
  })
  return ret();
}

extern "C" int oi_launch_trsm_trtri(const OiCell* cells, const int32_t* list, int ncell, int maxT,
                                    int j, void* stream) {
  if (ncell <= 0 || maxT - 1 <= 0) return 0;
  FOR_CHUNKS(ncell, {
    hipLaunchKernelGGL(k_trsm_trtri, dim3(maxT - 1, cnt), dim3(256), 0, S(stream), cells,
                       list + base, j);
  })
  return ret();
}

extern "C" int oi_launch_zvec(const OiCell* cells, const int32_t* list, int ncell, int maxT,
                              void* stream) {
  if (ncell <= 0 || maxT <= 0) return 0;
  FOR_CHUNKS(ncell, {
    hipLaunchKernelGGL(k_zvec, dim3(maxT, cnt), dim3(256), 0, S(stream), cells, list + base);
  })
  return ret();
}

extern "C" int oi_launch_avec(const OiCell* cells, const int32_t* list, int ncell, int maxT,
                              void* stream) {
  if (ncell <= 0 || maxT <= 0) return 0;
  FOR_CHUNKS(ncell, {
    hipLaunchKernelGGL(k_avec, dim3(maxT, cnt), dim3(256), 0, S(stream), cells, list + base);
  })
  return ret();
}

extern "C" int oi_launch_lauum_grad(const OiCell* cells, const int32_t* list, int ncell, int maxT,
                                    void* stream) {
  if (ncell <= 0 || maxT <= 0) return 0;
  FOR_CHUNKS(ncell, {
    hipLaunchKernelGGL(k_lauum_grad, dim3(maxT * (maxT + 1) / 2, cnt), dim3(256), 0, S(stream),
                       cells, list + base);
  })
  return ret();
}

extern "C" int oi_launch_predict(const OiCell* cells, const int32_t* list, int ncell,
                                 void* stream) {
  if (ncell <= 0) return 0;
  hipLaunchKernelGGL(k_predict, dim3(ncell), dim3(256), 0, S(stream), cells, list);
  return ret();
}

extern "C" int oi_launch_finalize(const OiCell* cells, const int32_t* list, int ncell,
                                  void* stream) {
  if (ncell <= 0) return 0;
  hipLaunchKernelGGL(k_finalize, dim3(ncell), dim3(256), 0, S(stream), cells, list);
  return ret();
}

extern "C" int oi_launch_residual(const double* y, const double* mX, double mean, double* r,
                                  int64_t N, void* stream) {
  if (N <= 0) return 0;
  hipLaunchKernelGGL(k_residual, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, S(stream), y, mX,
                     mean, r, N);
  return ret();
}
