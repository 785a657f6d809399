// HIP kernels (gfx950 / CDNA4, fp64) for the per-cell full-GP hot path:
// SMLII (GPR_CS2S3.py:107-141) and the GPR3D predict block (GPR_CS2S3.py:173-182)
// for a ragged batch of independent grid cells.  Data layout: oi_device.h.
//
// Per objective evaluation of a cell (T = ceil(n/64) tiles per side):
//   k_build        K + sn2 I (Matern-3/2, GPR:93-94)                         O(n^2)
//   k_diag_factor(j) factor + invert diagonal tile j: one wave per cell, rows in
//                  registers (potrf + trti2, fully unrolled)             ~n^2 * 64
//   k_scale(j)     P_jk = -Dinv_jj L_jk (k < j; only k = j-1 at odd j)        ~n^2 * 64
//   k_panel_even(j), j even: left-looking Cholesky for the column pair (j, j+1)
//                  on one stream of block row i (64x128 blocks, 512 threads):
//                  L_ij = sum_{k<j} L_ik P_jk^T + A_ij Dinv_jj^T  (update and
//                  triangular solve in one GEMM loop), A_i,j+1 -= sum_{k<j}
//                  L_ik L_j+1,k^T, look-ahead of diagonal tile j+1; rows j and
//                  j+1 of W = L^-1 from one stream of W_k,jj
//   k_chol_panel(j, kbeg = j-1), j odd: finishes column j / W row j with two
//                  products per tile, look-ahead of tile j+1       (both) 2 n^3/3
//                  (kbeg = 0: the one-column scheme, OI_PANEL=1)
//   (forward substitution z = L^-1 r runs inside the factorisation: k_diag_factor
//                  applies Dinv_jj to block j, the panels subtract L_ij z_j; and
//                  alpha = W^T z = K^-1 r (GPR:127) is accumulated as each W tile
//                  is finished: alpha_jj += W_j,jj^T z_j; r^T alpha = z^T z)
//   k_lauum_grad1  K^-1 = W^T W, one tile per workgroup, fused with the
//                  gradient traces sum((K^-1 - alpha alpha^T) o dK_j); K and
//                  dK_j are regenerated from coordinates (GPR:130-138)         n^3/3
//   k_finalize     nlZ and dnlZ (GPR:128, GPR:131-138), fixed-order sums
// Predict (GPR:173-182): k_build (also k*), the Cholesky with the forward
// substitution of r and k* folded in, then k_finalize (fs = mean + v.z,
// sd = sqrt(sf2 - v.v), lZ from z.z): no separate triangular solves.
//
// Every reduction has a fixed order that depends only on the cell, so a
// cell's results are bitwise independent of the batch it runs in.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdlib.h>

#include "oi_device.h"
#include "oi_gemm.h"
#include "oi_masks.h"

// GEMM1(acc, lds, npairs, pair): the 64x64 tile-GEMM loop of the panel / lauum kernels
#define GEMM1(acc, lds, np, ...) gemm1_kmajor<false>(acc, lds, 4 * (np), 0u, __VA_ARGS__)

#define NB OI_NB
#define SQRT3 1.7320508075688772
#define LOG2PI 1.8378770664093453  // np.log(2*np.pi)

// structurally-zero operand tile (tiles above the block diagonal); device
// globals are zero-initialised by the loader and never written
__device__ double g_zero_tile[OI_TILE];
// OI_DEBUG=1 (oi_set_debug): diagnostic printf from the factorisation
__device__ int g_debug;

extern "C" int oi_set_debug(int on) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_debug), &on, sizeof(int)) == hipSuccess ? 0 : -1;
}

// Descriptor pointers are generic, so plain accesses through them compile to
// flat_* instructions, which count against lgkmcnt as well: every LDS wait and
// single-wave barrier then also waits for the tile stores still in flight.
// gst / gld access through the global address space (global_* instructions).
typedef __attribute__((address_space(1))) double gdouble;
__device__ __forceinline__ void gst(double* p, double v) { *(gdouble*)p = v; }
__device__ __forceinline__ double gld(const double* p) { return *(const gdouble*)p; }
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

// deterministic block reduction of NV values, result valid in thread 0;
// red must hold NWAVES*NV doubles
template <int NV, int NWAVES>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* red) {
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
    for (int q = 0; q < NV; ++q) {
      double s = red[q];
      for (int ww = 1; ww < NWAVES; ++ww) s += red[ww * NV + q];
      v[q] = s;
    }
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

// Blocks are dealt round-robin over the 8 XCDs (b, b+8, ... share one).  Deal
// whole CELLS round-robin instead: block b works on cell (b&7) + 8*((b>>3)/gx),
// slot (b>>3) % gx, so all tiles of a cell run on one XCD and share its L2,
// while neighbouring cells (similar sizes: the list is sorted by T) spread
// over all XCDs.  The grid is gx * roundup(ncell, 8) blocks.
__device__ __forceinline__ bool xcd_cell_slot(int gx, int ncell, int& cell, int& x) {
  const int b = blockIdx.x, t = b >> 3;
  cell = (b & 7) + 8 * (t / gx);
  x = t % gx;
  return cell < ncell;
}

// Same cell -> XCD dealing, but the slot-0 workgroups of every cell are
// dispatched first: in k_chol_panel slot 0 also runs the look-ahead of the
// next diagonal tile (j + 1 serial products), the launch's longest chain, so
// all of them start at once instead of trailing the short two-product rows.
__device__ __forceinline__ bool xcd_cell_slot_lead0(int gx, int ncell, int& cell, int& x) {
  const int b = blockIdx.x, t = b >> 3, g0 = (ncell + 7) >> 3;
  if (t < g0) {
    cell = (b & 7) + 8 * t;
    x = 0;
  } else {
    const int u = t - g0;
    cell = (b & 7) + 8 * (u / (gx - 1));
    x = 1 + u % (gx - 1);
  }
  return cell < ncell;
}

// ------------------------------------------------------------- k_build
// M = D Kd D + sn2 I for tile (i, j) (K + sn2 I of GPR:93-94 / GPR:126 on the
// sites, oi_device.h); identity on padding.
__global__ __launch_bounds__(256) void k_build(const OiCell* __restrict__ cells,
                                               const int32_t* __restrict__ list, int gx,
                                               int ncell) {
  int ci, x;
  if (!xcd_cell_slot(gx, ncell, ci, x)) return;
  const OiCell& c = cells[list[ci]];
  int i, j;
  if (!decode_tri(x, c.T, i, j)) return;
  __shared__ double u[2][3][NB];
  __shared__ double dws[2][NB];
  const int t = threadIdx.x, n = c.n;
  if (t < 2 * NB) {
    int side = t >> 6, idx = t & 63, a = (side ? j : i) * NB + idx;
    for (int d = 0; d < 3; ++d) u[side][d][idx] = a < n ? (SQRT3 * c.xyt[3 * a + d]) / c.hyp[d] : 0.0;
    dws[side][idx] = a < n ? c.dw[a] : 0.0;
  }
  __syncthreads();
  const double sf2 = c.hyp[3], sn2 = c.hyp[4];
  // Duplicate sites make K + sn2 I singular up to sn2: the reference's
  // n x n Cholesky loses the pivot of a repeated row, (sf2 + sn2) - sf2^2 /
  // (sf2 + sn2), to rounding (always once sf2 + sn2 rounds to sf2, sn2 = 0
  // included; with probability 1/2 at sn2 / sf2 = OI_DUP_NONPD_TAU n_obs) and
  // takes the LinAlgError branch (GPR:139-140); the m x m site form would not
  // notice (oi_device.h).
  if (x == 0 && t == 0 && c.n_obs > n && (sf2 + sn2 == sf2 || sn2 < OI_DUP_NONPD_TAU * c.n_obs * sf2))
    *c.status = OI_NOT_PD;
  if (i == j && t < NB) {
    // right-hand sides of the forward substitution run inside the
    // factorisation: z = r (site residuals), and for predict v = k* = D kd*
    // (GPR:174, cdist of scaled coordinates)
    const int a = i * NB + t;
    gst(c.vec + a, a < n ? c.r[a] : 0.0);
    if (c.mode == OI_MODE_PREDICT) {
      double kv = 0.0;
      if (a < n) {
        const double xs0 = (SQRT3 * c.xs[0]) / c.hyp[0], xs1 = (SQRT3 * c.xs[1]) / c.hyp[1],
                     xs2 = (SQRT3 * c.xs[2]) / c.hyp[2];
        const double d0 = (SQRT3 * c.xyt[3 * a]) / c.hyp[0] - xs0;
        const double d1 = (SQRT3 * c.xyt[3 * a + 1]) / c.hyp[1] - xs1;
        const double d2 = (SQRT3 * c.xyt[3 * a + 2]) / c.hyp[2] - xs2;
        const double Q = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
        kv = c.dw[a] * (sf2 * ((1.0 + Q) * exp(-Q)));
      }
      gst(c.vec + 3 * c.T * NB + a, kv);
    }
  }
  double* Y = tileL(c, i, j);
  // a diagonal tile is built on its lower triangle only (2080 entries, column-
  // packed so whole waves retire early): the factor kernels treat the upper
  // triangle as scratch and clear it (k_diag_factor*)
  const int ne = i == j ? NB * (NB + 1) / 2 : OI_TILE;
  for (int e = t; e < ne; e += 256) {
    int r, cc;
    if (i == j) {  // column cc starts at S(cc) = 64 cc - cc (cc - 1) / 2
      cc = (int)((129.0 - sqrt(16641.0 - 8.0 * e)) * 0.5);
      while (cc > 0 && NB * cc - cc * (cc - 1) / 2 > e) --cc;
      while (NB * (cc + 1) - (cc + 1) * cc / 2 <= e) ++cc;
      r = cc + (e - (NB * cc - cc * (cc - 1) / 2));
    } else {
      r = e & 63;
      cc = e >> 6;
    }
    const int a = i * NB + r, b = j * NB + cc;
    double val;
    if (a >= n || b >= n) {
      val = (a == b) ? 1.0 : 0.0;
    } else {
      double d0 = u[0][0][r] - u[1][0][cc], d1 = u[0][1][r] - u[1][1][cc], d2 = u[0][2][r] - u[1][2][cc];
      double Q = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
      val = (dws[0][r] * dws[1][cc]) * (sf2 * ((1.0 + Q) * exp(-Q)));  // M = D Kd D (+ sn2 I)
      if (a == b) val += sn2;
    }
    gst(Y + cc * NB + r, val);
  }
}

// --------------------------------------------- k_diag_factor(j)
// Factor + invert diagonal tile j of every cell: one 64-lane wave per cell,
// lane r holding row r of the tile in registers (fully unrolled loops, column
// values broadcast with v_readlane).  The tile already holds the updated
// A_jj - sum_{k<j} L_jk L_jk^T (k_chol_panel(j-1) wrote it; for j = 0 it is
// K + sn2 I from k_build).  Writes L_jj, its log-determinant, Dinv_jj and
// (eval mode) W_jj.  Pivot <= 0 -> status = not PD (GPR:139-140); NaN pivots
// propagate like the reference's numpy/OpenBLAS cholesky.
__device__ __forceinline__ double rdlane(double v, int lane) {
  const long long x = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane((int)(x & 0xffffffffLL), lane);
  const int hi = __builtin_amdgcn_readlane((int)(x >> 32), lane);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}

// One wave multiplies two 32x32 operands staged in LDS (row stride 33):
// D[m][n] = sum_k A(m, k) B(k, n) with A(m, k) = a[m*33 + k] (row-major) and
// B(k, n) = b[k*33 + n] (row-major) or b[n*33 + k] (b_rows_are_n), on 2x2
// v_mfma_f64_16x16x4f64 blocks; the result goes to d[m*33 + n].
__device__ __forceinline__ void wave_gemm32(const double* a, const double* b, bool b_rows_are_n,
                                            double* d, double sign) {
  const int l = threadIdx.x & 63, fr = l & 15, fk = l >> 4;
  d4 acc[2][2];
  for (int mb = 0; mb < 2; ++mb)
    for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    const int k = 4 * kk + fk;
    double av[2], bv[2];
    for (int q = 0; q < 2; ++q) {
      av[q] = a[(16 * q + fr) * 33 + k];
      bv[q] = b_rows_are_n ? b[(16 * q + fr) * 33 + k] : b[k * 33 + 16 * q + fr];
    }
    for (int mb = 0; mb < 2; ++mb)
      for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = MFMA64(av[mb], bv[nb], acc[mb][nb]);
  }
  for (int mb = 0; mb < 2; ++mb)
    for (int nb = 0; nb < 2; ++nb)
      for (int r = 0; r < 4; ++r) d[(16 * mb + fk + 4 * r) * 33 + 16 * nb + fr] = sign * acc[mb][nb][r];
}

// Factor + invert diagonal tile j: one 64-lane wave per cell, lane r holding
// row r of the tile in registers; blocked 2 x 2 over 32-column halves so the
// serial (v_readlane-broadcast) part is a quarter of the unblocked one:
//   potrf of columns 0..31 over all 64 rows  -> L00, L10
//   A11 -= L10 L10^T                          (MFMA, via LDS)
//   potrf of A11                              -> L11
//   trti2 of L11 and of L00 (LAPACK dtrti2 order within each)
//   Inv10 = -Inv11 (L10 Inv00)                (two MFMA products)
__global__ __launch_bounds__(64) void k_diag_factor(const OiCell* __restrict__ cells,
                                                   const int32_t* __restrict__ list, int j) {
  __shared__ double Tt[128 * 33];  // transpose buffer for the row-major W_jj (64 x 65); also the
                                  // 32x33 staging areas of the blocked steps
  const OiCell& c = cells[list[blockIdx.x]];
  if (j >= c.T || *c.status != OI_OK) return;
  const int r = threadIdx.x;
  const bool lo = r < 32;
  double* Y = tileL(c, j, j);
  double R[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) R[q] = gld(Y + q * NB + r);  // row r of the column-major tile
  double* S0 = Tt;             // 32 x 33
  double* S1 = Tt + 32 * 33;   // 32 x 33
  double* S2 = Tt + 64 * 33;   // 32 x 33
  bool ok = true;
  // ---- potrf, columns 0..31 (all 64 rows: rows 32..63 become L10)
#pragma unroll
  for (int cc = 0; cc < 32; ++cc) {
    const double d = rdlane(R[cc], cc);
    ok = ok && !(d <= 0.0);
    const double l = sqrt(d);
    const double lr = r > cc ? R[cc] / l : 0.0;
    R[cc] = r > cc ? lr : (r == cc ? l : R[cc]);
#pragma unroll
    for (int s2 = cc + 1; s2 < 32; ++s2) R[s2] -= lr * rdlane(R[cc], s2);
  }
  // ---- A11 -= L10 L10^T
  if (!lo)
#pragma unroll
    for (int k = 0; k < 32; ++k) S0[(r - 32) * 33 + k] = R[k];
  __syncthreads();
  wave_gemm32(S0, S0, true, S1, 1.0);
  __syncthreads();
  if (!lo)
#pragma unroll
    for (int n = 0; n < 32; ++n) R[32 + n] -= S1[(r - 32) * 33 + n];
  // ---- potrf of A11 (rows 32..63; rows 0..31 see lr = 0)
#pragma unroll
  for (int cc = 32; cc < NB; ++cc) {
    const double d = rdlane(R[cc], cc);
    ok = ok && !(d <= 0.0);
    const double l = sqrt(d);
    const double lr = r > cc ? R[cc] / l : 0.0;
    R[cc] = r > cc ? lr : (r == cc ? l : R[cc]);
#pragma unroll
    for (int s2 = cc + 1; s2 < NB; ++s2) R[s2] -= lr * rdlane(R[cc], s2);
  }
  if (!ok) {
    if (r == 0) {
      *c.status = OI_NOT_PD;
      if (g_debug)
        printf("oi debug: not PD: cell n=%d T=%d diagonal tile j=%d hyp %g %g %g %g %g\n", c.n, c.T,
               j, c.hyp[0], c.hyp[1], c.hyp[2], c.hyp[3], c.hyp[4]);
    }
    return;
  }
  double dg = 1.0;  // L_rr, picked out by selects: one log per lane, not one per q
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    if (q > r) R[q] = 0.0;  // clear the upper part
    dg = q == r ? R[q] : dg;
    gst(Y + q * NB + r, R[q]);  // L_jj, column-major
  }
  double lg = (j * NB + r < c.n) ? log(dg) : 0.0;  // log L_rr
  for (int o = 32; o >= 1; o >>= 1) lg += __shfl_down(lg, o, 64);
  if (r == 0) {
    const int ntile = c.T * (c.T + 1) / 2;
    c.part[OI_PART_LOGDET(ntile, c.T) + j] = lg;
  }
  // L10 stays staged in S0 (rows 32..63 of the factor, columns 0..31)
  // ---- trti2 of L11 (columns 63..32), then of L00 (columns 31..0, k <= 31)
#pragma unroll
  for (int cc = NB - 1; cc >= 32; --cc) {
    const double ajj = 1.0 / rdlane(R[cc], cc);
    double x = 0.0;
#pragma unroll
    for (int k = cc + 1; k < NB; ++k) x += R[k] * rdlane(R[cc], k);
    R[cc] = r > cc ? -ajj * x : (r == cc ? ajj : R[cc]);
  }
#pragma unroll
  for (int cc = 31; cc >= 0; --cc) {
    const double ajj = 1.0 / rdlane(R[cc], cc);
    double x = 0.0;
#pragma unroll
    for (int k = cc + 1; k < 32; ++k) x += R[k] * rdlane(R[cc], k);
    R[cc] = (lo && r > cc) ? -ajj * x : (r == cc ? ajj : R[cc]);
  }
  // ---- Inv10 = -Inv11 (L10 Inv00)
  if (lo) {
#pragma unroll
    for (int n = 0; n < 32; ++n) S1[r * 33 + n] = R[n];  // Inv00 rows
  } else {
#pragma unroll
    for (int k = 0; k < 32; ++k) S2[(r - 32) * 33 + k] = R[32 + k];  // Inv11 rows
  }
  __syncthreads();
  wave_gemm32(S0, S1, false, Tt + 96 * 33, 1.0);  // Y = L10 Inv00 -> scratch after S2
  __syncthreads();
  wave_gemm32(S2, Tt + 96 * 33, false, S0, -1.0);  // Inv10 = -Inv11 Y -> S0
  __syncthreads();
  if (!lo)
#pragma unroll
    for (int n = 0; n < 32; ++n) R[n] = S0[(r - 32) * 33 + n];
  __syncthreads();  // Tt is reused below
  double* Dj = tileD(c, j);
#pragma unroll
  for (int q = 0; q < NB; ++q) gst(Dj + q * NB + r, R[q]);  // column-major
  // forward substitution, block j: z_j = Dinv_jj (r_j - sum_{k<j} L_jk z_k) -- the
  // panels already subtracted the sum -- and v_j likewise for predict (k* rhs)
  double zn = 0.0;
  {
    const bool pred = c.mode == OI_MODE_PREDICT;
    double* zj = c.vec + j * NB;
    double* vj = c.vec + 3 * c.T * NB + j * NB;
    Tt[r] = zj[r];
    Tt[NB + r] = pred ? vj[r] : 0.0;
    __syncthreads();
    double vn = 0.0;
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      zn = fma(R[q], Tt[q], zn);
      vn = fma(R[q], Tt[NB + q], vn);
    }
    gst(zj + r, zn);
    if (pred) gst(vj + r, vn);
    double zz = zn * zn, zv = zn * vn, vv = vn * vn;
    for (int o = 32; o >= 1; o >>= 1) {
      zz += __shfl_down(zz, o, 64);
      zv += __shfl_down(zv, o, 64);
      vv += __shfl_down(vv, o, 64);
    }
    if (r == 0) {
      double* pp = c.part + OI_PART_PRED(c.T * (c.T + 1) / 2, c.T) + 3 * j;
      pp[0] = zz;
      pp[1] = zv;
      pp[2] = vv;
    }
    __syncthreads();  // Tt is reused below
  }
  if (c.mode == OI_MODE_EVAL) {
#pragma unroll
    for (int q = 0; q < NB; ++q) Tt[q * 65 + r] = R[q];  // Tt[c][r] = Inv[r][c]
    __syncthreads();
    Tt[NB * 65 + r] = zn;
    __syncthreads();
    double* Wj = tileW(c, j, j);
    double al = 0.0;  // alpha_j = W_jj^T z_j starts the alpha = W^T z accumulation
    for (int q = 0; q < NB; ++q) {
      const double wv = Tt[r * 65 + q];
      gst(Wj + q * NB + r, wv);  // W[q][r], row-major
      al = fma(wv, Tt[NB * 65 + q], al);
    }
    gst(c.vec + c.T * NB + j * NB + r, al);
  }
}

// ------------------------------------------ k_diag_factor16(j) (default)
// The same contract as k_diag_factor, blocked by 16 columns so the serial
// (v_readlane-broadcast) work shrinks and the MFMA unit -- idle in the
// 32-blocked kernel -- does the rest.  One 64-lane wave per cell, lane r
// holding row r of the tile in registers:
//   potrf: for each 16-column panel J, the panel is factored serially (<= 15
//          broadcasts per column instead of <= 63), then the trailing block
//          update A_IK -= P_I P_K^T (I >= K > J) runs on v_mfma_f64_16x16x4f64
//          through LDS;
//   inverse: the four 16x16 diagonal blocks are inverted at once (trti2 in
//          LAPACK dtrti2 order, broadcasts within 16-lane groups), then the
//          off-diagonal blocks Inv_IJ = -Inv_II sum_{K=J}^{I-1} L_IK Inv_KJ by
//          levels I - J = 1, 2, 3 on the MFMA unit.
// LDS: Ls (the factor, row-major, stride 65) and Iv (the inverse, column-major
// -- Iv[c*65 + r] = Inv[r][c] -- stride 65); the potrf panel (in Iv) and the
// trailing-update results (in Ls) alias them.
#define D16_LD 65
// packed block slots: L_IK (I > K) and Inv_IK (I >= K) of the 4 x 4 blocks of a tile
__device__ __forceinline__ int lb_index(int I, int K) { return I * (I - 1) / 2 + K; }
__device__ __forceinline__ int ib_index(int I, int K) { return I * (I + 1) / 2 + K; }
// acc (16x16, lane l holds rows (l>>4) + 4q, column l&15) += A B with
// A[m][k] = Am[m * la + k] (or Am[k * la + m] if a_km) and B[k][n] = Bt[n * lb + k]
__device__ __forceinline__ void mfma16x16(d4& acc, const double* Am, int la, bool a_km, const double* Bt,
                                          int lb) {
  const int l = threadIdx.x & 63, fr = l & 15, fk = l >> 4;
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const int k = 4 * kk + fk;
    const double a = a_km ? Am[k * la + fr] : Am[fr * la + k];
    acc = MFMA64(a, Bt[fr * lb + k], acc);
  }
}

// broadcast lane l (0..15, a constant after unrolling) of every 16-lane row to
// the whole row: DPP row_newbcast, a VALU move (no LDS round trip as __shfl)
__device__ __forceinline__ int bcast16_i(int v, int l) {
#define OI_RB(n) \
  case n:        \
    return __builtin_amdgcn_update_dpp(0, v, 0x150 + n, 0xF, 0xF, false);
  switch (l) {
    OI_RB(0) OI_RB(1) OI_RB(2) OI_RB(3) OI_RB(4) OI_RB(5) OI_RB(6) OI_RB(7)
    OI_RB(8) OI_RB(9) OI_RB(10) OI_RB(11) OI_RB(12) OI_RB(13) OI_RB(14)
    default: return __builtin_amdgcn_update_dpp(0, v, 0x15F, 0xF, 0xF, false);
  }
#undef OI_RB
}
__device__ __forceinline__ double bcast16(double v, int l) {
  const long long x = __builtin_bit_cast(long long, v);
  const int lo = bcast16_i((int)(x & 0xffffffffLL), l);
  const int hi = bcast16_i((int)(x >> 32), l);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}

#ifndef OI_LAUUM_EPI
#define OI_LAUUM_EPI 1
#endif
#ifndef OI_DIAG_RSQ
#define OI_DIAG_RSQ 1
#endif
// stage timestamps for tools/diag_engine_probe (compiled in only there)
#ifdef OI_DIAG_TIMING
__device__ long long g_diag_stamps[16];
#define DIAG_STAMP(k) \
  do { if (threadIdx.x == 0 && blockIdx.x == 0) g_diag_stamps[k] = clock64(); } while (0)
#else
#define DIAG_STAMP(k) do {} while (0)
#endif
__global__ __launch_bounds__(64) void k_diag_factor16(const OiCell* __restrict__ cells,
                                                     const int32_t* __restrict__ list, int j) {
  // packed 16x16 blocks (row stride 17): Lb holds L_IK (I > K, 6 blocks), Ib the
  // inverse's lower blocks Inv_IK (I >= K, 10 blocks) stored transposed (Ib[n*17 + m]
  // = Inv[16I + m][16K + n]); the potrf panel P and update results U alias them
  // (37 KB: four workgroups per CU)
  __shared__ double lds16[16 * 17 * 17 + 16 * 17];
  double* Lb = lds16;                 // 6 blocks
  double* Ib = lds16 + 6 * 272;       // 10 blocks
  double* Xs = lds16 + 16 * 272;      // 16 x 17
  const OiCell& c = cells[list[blockIdx.x]];
  if (j >= c.T || *c.status != OI_OK) return;
  DIAG_STAMP(0);
  const int r = threadIdx.x, fr = r & 15, fk = r >> 4, blk = r >> 4;
  double* Y = tileL(c, j, j);
  double R[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) R[q] = gld(Y + q * NB + r);  // row r of the column-major tile
  DIAG_STAMP(1);
  // smallest pivot (minNum: a NaN pivot is passed over, as !(d <= 0) passes it);
  // one v_min per column instead of a flag the compiler keeps 64 pivots for
  double dmin = __builtin_inf();
  // ---------------- potrf by 16-column panels
  // Entries above the diagonal are scratch until "clear the upper part" below:
  // every lane scales and updates its whole row, so no lane-dependent selects
  // guard the serial part (rows r < cc compute values nobody reads).
#pragma unroll
  for (int J = 0; J < 4; ++J) {
    const int c0 = 16 * J;
#pragma unroll
    for (int cc = c0; cc < c0 + 16; ++cc) {
      const double d = rdlane(R[cc], cc);
      dmin = fmin(dmin, d);
#if OI_DIAG_RSQ
      // 1/sqrt(d) by v_rsq_f64 + two Newton steps (<= 1 ulp); the column is
      // scaled by it (as LAPACK dpotf2 scales by 1/ajj) and L_cc = d/sqrt(d):
      // eight VALU ops per column where sqrt + an IEEE division take ~25
      double il = __builtin_amdgcn_rsq(d);
      il = fma(0.5 * il, fma(-d * il, il, 1.0), il);
      il = fma(0.5 * il, fma(-d * il, il, 1.0), il);
      const double l = d * il;
      const double qd = R[cc] * il;
#else
      const double l = sqrt(d);
      const double qd = R[cc] / l;  // on every lane: no exec-mask branch
#endif
      R[cc] = r == cc ? l : qd;
#pragma unroll
      for (int s2 = cc + 1; s2 < c0 + 16; ++s2) R[s2] -= qd * rdlane(R[cc], s2);
    }
    if (J == 3) break;
    // trailing update: A_IK -= P_I P_K^T for J < K <= I, P = rows of panel J
    double* P = lds16;              // 64 x 17
    double* U = lds16 + NB * 17;    // results: U[row * 49 + (s - c0 - 16)]
#pragma unroll
    for (int q = 0; q < 16; ++q) P[r * 17 + q] = r >= c0 + q ? R[c0 + q] : 0.0;
    __syncthreads();
#pragma unroll
    for (int I = J + 1; I < 4; ++I)
#pragma unroll
      for (int K = J + 1; K <= I; ++K) {
        d4 acc = (d4){0.0, 0.0, 0.0, 0.0};
        mfma16x16(acc, P + 16 * I * 17, 17, false, P + 16 * K * 17, 17);
#pragma unroll
        for (int q = 0; q < 4; ++q) U[(16 * I + fk + 4 * q) * 49 + 16 * (K - J - 1) + fr] = acc[q];
      }
    __syncthreads();
#pragma unroll
    for (int s2 = c0 + 16; s2 < NB; ++s2) {  // selected, not branched (unwritten U entries are dropped)
      const double u = U[r * 49 + (s2 - c0 - 16)];
      R[s2] -= (s2 >> 4) <= blk ? u : 0.0;
    }
    __syncthreads();  // P / U are rewritten by the next panel
  }
  DIAG_STAMP(2);
  if (dmin <= 0.0) {
    if (r == 0) {
      *c.status = OI_NOT_PD;
      if (g_debug)
        printf("oi debug: not PD: cell n=%d T=%d diagonal tile j=%d hyp %g %g %g %g %g\n", c.n, c.T,
               j, c.hyp[0], c.hyp[1], c.hyp[2], c.hyp[3], c.hyp[4]);
    }
    return;
  }
  double dg = 1.0;  // L_rr, picked out by selects: one log per lane, not one per q
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    if (q > r) R[q] = 0.0;  // clear the upper part
    dg = q == r ? R[q] : dg;
    gst(Y + q * NB + r, R[q]);  // L_jj, column-major
  }
  double lg = (j * NB + r < c.n) ? log(dg) : 0.0;  // log L_rr
  __syncthreads();  // lds16 held the potrf scratch
#pragma unroll
  for (int K = 0; K < 4; ++K)  // L_IK blocks (I = blk > K), row-major for the MFMA A operand
    if (K < blk) {
#pragma unroll
      for (int q = 0; q < 16; ++q) Lb[lb_index(blk, K) * 272 + fr * 17 + q] = R[16 * K + q];
    }
  for (int o = 32; o >= 1; o >>= 1) lg += __shfl_down(lg, o, 64);
  if (r == 0) {
    const int ntile = c.T * (c.T + 1) / 2;
    c.part[OI_PART_LOGDET(ntile, c.T) + j] = lg;
  }
  // ---------------- inverse: four diagonal 16x16 blocks at once (dtrti2 order)
  DIAG_STAMP(3);
  double D[16];
#pragma unroll
  for (int q = 0; q < 16; ++q)  // D[q] = L[r][16 blk + q]
    D[q] = blk == 0 ? R[q] : blk == 1 ? R[16 + q] : blk == 2 ? R[32 + q] : R[48 + q];
#pragma unroll
  for (int cc = 15; cc >= 0; --cc) {
    const double ajj = 1.0 / bcast16(D[cc], cc);
    double x = 0.0;
#pragma unroll
    for (int k = cc + 1; k < 16; ++k) x += D[k] * bcast16(D[cc], k);
    D[cc] = fr > cc ? -ajj * x : (fr == cc ? ajj : D[cc]);
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) Ib[ib_index(blk, blk) * 272 + q * 17 + fr] = D[q];  // Inv_II (transposed)
  __syncthreads();
  DIAG_STAMP(4);
  // ---------------- off-diagonal blocks by levels: Inv_IJ = -Inv_II X, X = sum_K L_IK Inv_KJ
#pragma unroll
  for (int lev = 1; lev < 4; ++lev) {
#pragma unroll
    for (int J = 0; J + lev < 4; ++J) {
      const int I = J + lev;
      d4 acc = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int K = J; K < I; ++K)  // A = L_IK (row-major), B = Inv_KJ: Bt[n][k] = Inv[16K + k][16J + n]
        mfma16x16(acc, Lb + lb_index(I, K) * 272, 17, false, Ib + ib_index(K, J) * 272, 17);
#pragma unroll
      for (int q = 0; q < 4; ++q) Xs[fr * 17 + fk + 4 * q] = acc[q];  // Xs[n][m] = X[m][n]
      __syncthreads();
      d4 y = (d4){0.0, 0.0, 0.0, 0.0};
      // A = Inv_II: A[m][k] = Inv[16I + m][16I + k] = Ib_II[k * 17 + m]  (k-major)
      mfma16x16(y, Ib + ib_index(I, I) * 272, 17, true, Xs, 17);
      __syncthreads();
#pragma unroll
      for (int q = 0; q < 4; ++q) Ib[ib_index(I, J) * 272 + fr * 17 + fk + 4 * q] = -y[q];
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < NB; ++q) {  // row r of the inverse: Inv[r][q] (zero above the diagonal blocks)
    const int K = q >> 4;
    R[q] = K <= blk ? Ib[ib_index(blk, K) * 272 + (q & 15) * 17 + fr] : 0.0;
  }
  double* Dj = tileD(c, j);
#pragma unroll
  for (int q = 0; q < NB; ++q) gst(Dj + q * NB + r, R[q]);  // column-major
  DIAG_STAMP(5);
  // forward substitution, block j (see k_diag_factor)
  double zn = 0.0;
  {
    const bool pred = c.mode == OI_MODE_PREDICT;
    double* zj = c.vec + j * NB;
    double* vj = c.vec + 3 * c.T * NB + j * NB;
    Xs[r] = zj[r];
    Xs[NB + r] = pred ? vj[r] : 0.0;  // Xs has room for 272 doubles
    __syncthreads();
    double vn = 0.0;
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      zn = fma(R[q], Xs[q], zn);
      vn = fma(R[q], Xs[NB + q], vn);
    }
    gst(zj + r, zn);
    if (pred) gst(vj + r, vn);
    double zz = zn * zn, zv = zn * vn, vv = vn * vn;
    for (int o = 32; o >= 1; o >>= 1) {
      zz += __shfl_down(zz, o, 64);
      zv += __shfl_down(zv, o, 64);
      vv += __shfl_down(vv, o, 64);
    }
    if (r == 0) {
      double* pp = c.part + OI_PART_PRED(c.T * (c.T + 1) / 2, c.T) + 3 * j;
      pp[0] = zz;
      pp[1] = zv;
      pp[2] = vv;
    }
  }
  DIAG_STAMP(6);
  if (c.mode == OI_MODE_EVAL) {
    double* Wj = tileW(c, j, j);  // row-major W = L^-1: W[q][r] = Inv[q][r]
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NB; ++q) lds16[q * D16_LD + r] = R[q];  // lds16[c*65 + r] = Inv[r][c]
    Xs[2 * NB + r] = zn;
    __syncthreads();
    double al = 0.0;  // alpha_j = W_jj^T z_j starts the alpha = W^T z accumulation
    for (int q = 0; q < NB; ++q) {
      const double wv = lds16[r * D16_LD + q];
      gst(Wj + q * NB + r, wv);
      al = fma(wv, Xs[2 * NB + q], al);
    }
    gst(c.vec + c.T * NB + j * NB + r, al);
  }
  DIAG_STAMP(7);
}

// ------------------------------------------ k_diag_factor4w(j) (default since round 3)
// The same contract as k_diag_factor16 on four waves with the tile in LDS, for
// latency (config 1's lone cell waits for four of these per evaluation; the
// single-wave kernel spent half its 60 k cycles outside the serial potrf, one
// wave issuing every store, the dtrti2 broadcasts and the inverse levels):
//   potrf: 16-column panels; wave 0 factors the panel (row per lane, column
//          values by v_readlane), all four waves then apply the trailing
//          update A_IK -= P_I P_K^T (I >= K > J) on v_mfma_f64_16x16x4f64;
//   inverse: wave b inverts diagonal block b by forward substitution, one
//          lane per column (L read by LDS broadcast), then the off-diagonal
//          blocks Inv_IJ = -Inv_II sum_{K=J}^{I-1} L_IK Inv_KJ by levels
//          I - J = 1, 2, 3, one block per wave;
//   stores of L, Dinv and W by all 256 threads (coalesced columns).
// LDS (77 KB, two workgroups per CU): As = the tile, then L (row-major, stride
// 65, zero above the diagonal); Is = Inv (row-major, zero above); per-wave
// 16 x 17 scratch; z_j / v_j.
#define DW_LD 65
// workgroup barrier that waits for this wave's LDS operations only: HIP's
// __syncthreads() is a workgroup-scope release, which also waits for every
// outstanding global store (vmcnt(0)) -- here the L / Dinv / W stores would
// stall each following phase on HBM write latency.  The workgroup shares only
// LDS data between phases; the "memory" clobber keeps the compiler from moving
// memory operations across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// potrf of the 64 x 64 tile in As (row-major, stride DW_LD, lower triangle; the
// upper triangle is scratch) on four waves, As <- L with zeros above the
// diagonal.  Returns the smallest pivot in wave 0 (+inf in the other waves;
// minNum passes a NaN pivot over, as the reference's cholesky does).
__device__ __forceinline__ double potrf4w(double* As) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, fr = lane & 15, fk = lane >> 4;
  double dmin = __builtin_inf();
#pragma unroll
  for (int J = 0; J < 4; ++J) {
    const int c0 = 16 * J;
    if (w == 0) {
      const int r = lane;
      double R[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) R[q] = As[r * DW_LD + c0 + q];
      // rows r < c0 + q compute values nobody reads (zeros are written back)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int cc = c0 + q;
        const double d = rdlane(R[q], cc);
        dmin = fmin(dmin, d);
        // 1/sqrt(d) by v_rsq_f64 + two Newton steps (<= 1 ulp), as k_diag_factor16
        double il = __builtin_amdgcn_rsq(d);
        il = fma(0.5 * il, fma(-d * il, il, 1.0), il);
        il = fma(0.5 * il, fma(-d * il, il, 1.0), il);
        const double l = d * il;
        const double qd = R[q] * il;
        R[q] = r == cc ? l : qd;
#pragma unroll
        for (int s2 = q + 1; s2 < 16; ++s2) R[s2] -= qd * rdlane(R[q], c0 + s2);
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) As[r * DW_LD + c0 + q] = r >= c0 + q ? R[q] : 0.0;
    }
    lds_barrier();
    if (J == 3) break;
    // trailing update A_IK -= P_I P_K^T for J < K <= I (P: the panel's rows),
    // 6 / 3 / 1 blocks of 16 x 16 over the four waves; the diagonal blocks'
    // upper halves are scratch until their panel writes zeros back
    const int nblk = (3 - J) * (4 - J) / 2;
    for (int b = w; b < nblk; b += 4) {
      int I = J + 1, rem = b;
      while (rem >= I - J) {
        rem -= I - J;
        ++I;
      }
      const int K = J + 1 + rem;
      d4 acc = (d4){0.0, 0.0, 0.0, 0.0};
      mfma16x16(acc, As + 16 * I * DW_LD + c0, DW_LD, false, As + 16 * K * DW_LD + c0, DW_LD);
#pragma unroll
      for (int q = 0; q < 4; ++q) As[(16 * I + fk + 4 * q) * DW_LD + 16 * K + fr] -= acc[q];
    }
    lds_barrier();
  }
  return dmin;
}

// Is <- L^-1 of the factored tile in As (row-major, stride DW_LD); Is must
// hold zeros in its blocks above the diagonal.  Xs: 4 x 16 x 17 scratch.
__device__ __forceinline__ void trtri4w(const double* As, double* Is, double* Xs) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, fr = lane & 15, fk = lane >> 4;
  {
    // column fr of Inv_ww: x = L_ww^-1 e_fr, right-looking (x_i final once the
    // columns before it are applied; the updates of later rows are independent),
    // x_i scaled by 1/L_ii as LAPACK's dtrti2 does (lane i holds 1/L_ii)
    const int o = 16 * w;
    const double rl = 1.0 / As[(o + fr) * DW_LD + o + fr];
    double x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = i == fr ? 1.0 : 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      x[i] *= rdlane(rl, i);  // rows above the column: exact zeros
#pragma unroll
      for (int k = i + 1; k < 16; ++k) x[k] -= As[(o + k) * DW_LD + o + i] * x[i];
    }
    if (fk == 0)
#pragma unroll
      for (int i = 0; i < 16; ++i) Is[(o + i) * DW_LD + o + fr] = x[i];
  }
  lds_barrier();
  DIAG_STAMP(4);
  // ---------------- off-diagonal blocks by levels (wave w: J = w, I = J + lev)
  double* Xw = Xs + w * 272;
#pragma unroll
  for (int lev = 1; lev < 4; ++lev) {
    const int Jb = w, Ib = w + lev;
    const bool act = Ib < 4;
    if (act) {
      d4 acc = (d4){0.0, 0.0, 0.0, 0.0};
      for (int K = Jb; K < Ib; ++K)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int k = 4 * kk + fk;
          acc = MFMA64(As[(16 * Ib + fr) * DW_LD + 16 * K + k], Is[(16 * K + k) * DW_LD + 16 * Jb + fr], acc);
        }
#pragma unroll
      for (int q = 0; q < 4; ++q) Xw[(fk + 4 * q) * 17 + fr] = acc[q];  // Xw[k][n] = X[k][n]
    }
    lds_barrier();
    if (act) {
      d4 y = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int k = 4 * kk + fk;
        y = MFMA64(Is[(16 * Ib + fr) * DW_LD + 16 * Ib + k], Xw[k * 17 + fr], y);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) Is[(16 * Ib + fk + 4 * q) * DW_LD + 16 * Jb + fr] = -y[q];
    }
    lds_barrier();
  }
}

__global__ __launch_bounds__(256) void k_diag_factor4w(const OiCell* __restrict__ cells,
                                                      const int32_t* __restrict__ list, int j) {
  __shared__ double As[NB * DW_LD];
  __shared__ double Is[NB * DW_LD];
  __shared__ double Xs[4 * 16 * 17];
  __shared__ double Vs[3 * NB];
  __shared__ int bad;
  const OiCell& c = cells[list[blockIdx.x]];
  if (j >= c.T || *c.status != OI_OK) return;
  DIAG_STAMP(0);
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const bool pred = c.mode == OI_MODE_PREDICT;
  double* Y = tileL(c, j, j);
  double* zj = c.vec + j * NB;
  double* vj = c.vec + 3 * c.T * NB + j * NB;
  // element (r, q) of the column-major tile at q*64 + r: 16 coalesced loads per
  // thread; the upper triangle (scratch of k_build) is replaced by zeros
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int e = t + 256 * u, q = e >> 6, r = e & 63;
    const double v = gld(Y + e);
    As[r * DW_LD + q] = r >= q ? v : 0.0;
    Is[r * DW_LD + q] = 0.0;
  }
  if (t < NB) {
    Vs[t] = zj[t];
    Vs[NB + t] = pred ? vj[t] : 0.0;
  }
  lds_barrier();
  DIAG_STAMP(1);
  const double dmin = potrf4w(As);  // smallest pivot (wave 0)
  DIAG_STAMP(2);
  if (t == 0) bad = dmin <= 0.0;
  lds_barrier();
  if (bad) {
    if (t == 0) {
      *c.status = OI_NOT_PD;
      if (g_debug)
        printf("oi debug: not PD: cell n=%d T=%d diagonal tile j=%d hyp %g %g %g %g %g\n", c.n, c.T,
               j, c.hyp[0], c.hyp[1], c.hyp[2], c.hyp[3], c.hyp[4]);
    }
    return;
  }
  // L_jj (column-major) and sum log L_rr
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int e = t + 256 * u, q = e >> 6, r = e & 63;
    gst(Y + e, As[r * DW_LD + q]);
  }
  if (w == 0) {
    double lg = (j * NB + lane < c.n) ? log(As[lane * (DW_LD + 1)]) : 0.0;
    for (int o = 32; o >= 1; o >>= 1) lg += __shfl_down(lg, o, 64);
    if (lane == 0) {
      const int ntile = c.T * (c.T + 1) / 2;
      c.part[OI_PART_LOGDET(ntile, c.T) + j] = lg;
    }
  }
  DIAG_STAMP(3);
  trtri4w(As, Is, Xs);
  DIAG_STAMP(5);
  // Dinv_jj column-major: D[q*64 + r] = Inv[r][q]
  double* Dj = tileD(c, j);
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int e = t + 256 * u, q = e >> 6, r = e & 63;
    gst(Dj + e, Is[r * DW_LD + q]);
  }
  // forward substitution, block j: z_j = Dinv_jj z_j (the panels subtracted the
  // sum over k < j), v_j likewise for predict; z^T z, z^T v, v^T v partials
  if (w == 0) {
    double zp[4] = {0.0, 0.0, 0.0, 0.0}, vp[4] = {0.0, 0.0, 0.0, 0.0};  // four chains
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const double a = Is[lane * DW_LD + q];
      zp[q & 3] = fma(a, Vs[q], zp[q & 3]);
      vp[q & 3] = fma(a, Vs[NB + q], vp[q & 3]);
    }
    const double zn = (zp[0] + zp[1]) + (zp[2] + zp[3]), vn = (vp[0] + vp[1]) + (vp[2] + vp[3]);
    gst(zj + lane, zn);
    if (pred) gst(vj + lane, vn);
    Vs[2 * NB + lane] = zn;
    double zz = zn * zn, zv = zn * vn, vv = vn * vn;
    for (int o = 32; o >= 1; o >>= 1) {
      zz += __shfl_down(zz, o, 64);
      zv += __shfl_down(zv, o, 64);
      vv += __shfl_down(vv, o, 64);
    }
    if (lane == 0) {
      double* pp = c.part + OI_PART_PRED(c.T * (c.T + 1) / 2, c.T) + 3 * j;
      pp[0] = zz;
      pp[1] = zv;
      pp[2] = vv;
    }
  }
  DIAG_STAMP(6);
  if (c.mode == OI_MODE_EVAL) {
    // W_jj row-major (W[q][r] = Inv[q][r]) and alpha_j = W_jj^T z_j
    double* Wj = tileW(c, j, j);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = t + 256 * u;
      gst(Wj + e, Is[(e >> 6) * DW_LD + (e & 63)]);
    }
    lds_barrier();  // z_j in Vs
    if (w == 0) {
      double ap[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int q = 0; q < NB; ++q) ap[q & 3] = fma(Is[q * DW_LD + lane], Vs[2 * NB + q], ap[q & 3]);
      gst(c.vec + c.T * NB + j * NB + lane, (ap[0] + ap[1]) + (ap[2] + ap[3]));
    }
  }
  DIAG_STAMP(7);
}

// ------------------------------------------------ k_diag_pair(j), j even
// Folded pair step (OI_FOLD=1, default): the 128 x 128 diagonal block
// JJ = (j, j+1) of a cell -- tile j alone when j + 1 = T -- is factored and
// inverted in one launch, so that k_panel_pair(j) finishes BOTH block columns of
// every row below it (no odd-column launch).  On entry the block holds
//   A_JJ - sum_{k<j-2} L_Jk L_Jk^T   (k_panel_pair(j-2)'s look-ahead slot, in place)
// and c.P tiles 0..2 hold E = sum_{k=j-2}^{j-1} L_Jk L_Jk^T for (j,j), (j+1,j),
// (j+1,j+1) (its first row-pair workgroup; j >= 2 only).  Steps:
//   L_jj = potrf(A'_jj - E_jj), Dinv_j = L_jj^-1        (potrf4w / trtri4w)
//   L_j+1,j = (A'_j+1,j - E_j+1,j) Dinv_j^T
//   L_j+1,j+1 = potrf(A'_j+1,j+1 - E_j+1,j+1 - L_j+1,j L_j+1,j^T), Dinv_j+1
//   W_j+1,j = -Dinv_j+1 (L_j+1,j Dinv_j)   (the off-diagonal block of Winv_JJ;
//            column-major copy in c.P tile 3 for the panel epilogue, row-major in W)
//   z_j = Dinv_j z_j, z_j+1 = Dinv_j+1 (z_j+1 - L_j+1,j z_j)  (v likewise, predict)
//   alpha_j = W_jj^T z_j + W_j+1,j^T z_j+1, alpha_j+1 = W_j+1,j+1^T z_j+1  (eval)
// Scratch X = L_j+1,j Dinv_j goes through c.P tile 3 (the workgroup's own
// global stores, ordered by __syncthreads): As / Is are the only tile buffers in
// LDS, so two workgroups still fit a CU.
__global__ __launch_bounds__(256) void k_diag_pair(const OiCell* __restrict__ cells,
                                                  const int32_t* __restrict__ list, int j) {
  __shared__ double As[NB * DW_LD];
  __shared__ double Is[NB * DW_LD];
  __shared__ double Xs[4 * 16 * 17];
  __shared__ double Vs[7 * NB];  // z_j v_j zf_j | z_j+1 v_j+1 vf_j zf_j+1
  __shared__ int bad;
  const OiCell& c = cells[list[blockIdx.x]];
  const int T = c.T;
  if (j >= T || *c.status != OI_OK) return;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63, fr = lane & 15, fk = lane >> 4;
  const bool pred = c.mode == OI_MODE_PREDICT, eval = c.mode == OI_MODE_EVAL;
  const bool pair = j + 1 < T, ext = j >= 2;
  const int ntile = T * (T + 1) / 2;
  double* z = c.vec;
  double* al = c.vec + T * NB;
  double* v = c.vec + 3 * T * NB;
  const double* E = c.P;
  double* W10c = c.P + 3 * OI_TILE;
  double* pp = c.part + OI_PART_PRED(ntile, T);
  double* lgd = c.part + OI_PART_LOGDET(ntile, T);
  auto fail = [&](int jt) {
    if (t == 0) {
      *c.status = OI_NOT_PD;
      if (g_debug)
        printf("oi debug: not PD: cell n=%d T=%d diagonal tile j=%d hyp %g %g %g %g %g\n", c.n, T, jt,
               c.hyp[0], c.hyp[1], c.hyp[2], c.hyp[3], c.hyp[4]);
    }
  };
  auto logdet = [&](int jt) {  // wave 0: sum log L_rr of the factored tile in As
    double lg = (jt * NB + lane < c.n) ? log(As[lane * (DW_LD + 1)]) : 0.0;
    for (int o = 32; o >= 1; o >>= 1) lg += __shfl_down(lg, o, 64);
    if (lane == 0) lgd[jt] = lg;
  };
  // ---- tile (j, j)
  {
    const double* Y = tileL(c, j, j);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = t + 256 * u, q = e >> 6, r = e & 63;
      const double x = gld(Y + e) - (ext ? gld(E + e) : 0.0);
      As[r * DW_LD + q] = r >= q ? x : 0.0;
      Is[r * DW_LD + q] = 0.0;
    }
  }
  if (t < NB) {
    Vs[t] = z[j * NB + t];
    Vs[NB + t] = pred ? v[j * NB + t] : 0.0;
    Vs[3 * NB + t] = pair ? z[(j + 1) * NB + t] : 0.0;
    Vs[4 * NB + t] = pair && pred ? v[(j + 1) * NB + t] : 0.0;
  }
  lds_barrier();
  double dmin = potrf4w(As);
  if (t == 0) bad = dmin <= 0.0;
  lds_barrier();
  if (bad) return fail(j);
  {
    double* Y = tileL(c, j, j);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = t + 256 * u, q = e >> 6, r = e & 63;
      gst(Y + e, As[r * DW_LD + q]);
    }
  }
  if (w == 0) logdet(j);
  trtri4w(As, Is, Xs);
  {
    double* Dj = tileD(c, j);
    double* Wj = eval ? tileW(c, j, j) : nullptr;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = t + 256 * u, q = e >> 6, r = e & 63;
      gst(Dj + e, Is[r * DW_LD + q]);                     // column-major
      if (eval) gst(Wj + e, Is[(e >> 6) * DW_LD + (e & 63)]);  // row-major
    }
  }
  // z_j = Dinv_j z_j (v_j likewise), partial dot products of block j
  if (w == 0) {
    double zp[4] = {0.0, 0.0, 0.0, 0.0}, vp[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const double a = Is[lane * DW_LD + q];
      zp[q & 3] = fma(a, Vs[q], zp[q & 3]);
      vp[q & 3] = fma(a, Vs[NB + q], vp[q & 3]);
    }
    const double zn = (zp[0] + zp[1]) + (zp[2] + zp[3]), vn = (vp[0] + vp[1]) + (vp[2] + vp[3]);
    gst(z + j * NB + lane, zn);
    if (pred) gst(v + j * NB + lane, vn);
    Vs[2 * NB + lane] = zn;
    Vs[5 * NB + lane] = vn;
    double zz = zn * zn, zv = zn * vn, vv = vn * vn;
    for (int o = 32; o >= 1; o >>= 1) {
      zz += __shfl_down(zz, o, 64);
      zv += __shfl_down(zv, o, 64);
      vv += __shfl_down(vv, o, 64);
    }
    if (lane == 0) {
      pp[3 * j] = zz;
      pp[3 * j + 1] = zv;
      pp[3 * j + 2] = vv;
    }
  }
  lds_barrier();
  double a_j = 0.0;  // wave 0: alpha_j[lane], W_jj^T z_j part
  if (eval && w == 0) {
    double ap[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < NB; ++q) ap[q & 3] = fma(Is[q * DW_LD + lane], Vs[2 * NB + q], ap[q & 3]);
    a_j = (ap[0] + ap[1]) + (ap[2] + ap[3]);
    if (!pair) gst(al + j * NB + lane, a_j);
  }
  if (!pair) return;
  // ---- L_j+1,j = A'_j+1,j Dinv_j^T (A' row-major in As; wave w: row block w)
  {
    const double* Y = tileL(c, j + 1, j);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = t + 256 * u, q = e >> 6, r = e & 63;
      As[r * DW_LD + q] = gld(Y + e) - (ext ? gld(E + OI_TILE + e) : 0.0);
    }
  }
  lds_barrier();
  {
    d4 o[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      o[nb] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < 16; ++kk)  // B(q, n) = Dinv_j[n][q]: zero for q > n
        if (kk <= 4 * nb + 3)
          o[nb] = MFMA64(As[(16 * w + fr) * DW_LD + 4 * kk + fk], Is[(16 * nb + fr) * DW_LD + 4 * kk + fk], o[nb]);
    }
    lds_barrier();
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) As[(16 * w + fk + 4 * r) * DW_LD + 16 * nb + fr] = o[nb][r];
  }
  lds_barrier();
  {
    double* Y = tileL(c, j + 1, j);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = t + 256 * u, q = e >> 6, r = e & 63;
      gst(Y + e, As[r * DW_LD + q]);
    }
  }
  // z_j+1 -= L_j+1,j z_j (wave 0), v_j+1 -= L_j+1,j v_j (wave 1, predict)
  if (w == 0 || (w == 1 && pred)) {
    const double* u = Vs + (w == 0 ? 2 : 5) * NB;
    double sp[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < NB; ++q) sp[q & 3] = fma(As[lane * DW_LD + q], u[q], sp[q & 3]);
    Vs[(w == 0 ? 3 : 4) * NB + lane] -= (sp[0] + sp[1]) + (sp[2] + sp[3]);
  }
  // syrk S = L_j+1,j L_j+1,j^T (lower 16x16 blocks w, w+4, w+8) and X = L_j+1,j Dinv_j
  d4 sb[3], xo[4];
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    sb[s] = (d4){0.0, 0.0, 0.0, 0.0};
    const int b = w + 4 * s;
    if (b < 10) {
      const int bm = b >= 6 ? 3 : b >= 3 ? 2 : b >= 1 ? 1 : 0, bn = b - bm * (bm + 1) / 2;
#pragma unroll
      for (int kk = 0; kk < 16; ++kk)
        sb[s] = MFMA64(As[(16 * bm + fr) * DW_LD + 4 * kk + fk], As[(16 * bn + fr) * DW_LD + 4 * kk + fk], sb[s]);
    }
  }
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    xo[nb] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)  // B(q, n) = Dinv_j[q][n]: zero for q < n
      if (kk >= 4 * nb)
        xo[nb] = MFMA64(As[(16 * w + fr) * DW_LD + 4 * kk + fk], Is[(4 * kk + fk) * DW_LD + 16 * nb + fr], xo[nb]);
  }
  // X row-major into c.P tile 3 (read back below as the B operand, then replaced by W_j+1,j)
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) gst(W10c + (16 * w + fk + 4 * r) * NB + 16 * nb + fr, xo[nb][r]);
  lds_barrier();  // As / Is reads done, Vs updates visible
  // ---- tile (j+1, j+1): A'_j+1,j+1 - E - S
  {
    const double* Y = tileL(c, j + 1, j + 1);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = t + 256 * u, q = e >> 6, r = e & 63;
      const double x = gld(Y + e) - (ext ? gld(E + 2 * OI_TILE + e) : 0.0);
      As[r * DW_LD + q] = r >= q ? x : 0.0;
      Is[r * DW_LD + q] = 0.0;
    }
  }
  lds_barrier();
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int b = w + 4 * s;
    if (b < 10) {
      const int bm = b >= 6 ? 3 : b >= 3 ? 2 : b >= 1 ? 1 : 0, bn = b - bm * (bm + 1) / 2;
#pragma unroll
      for (int r = 0; r < 4; ++r) As[(16 * bm + fk + 4 * r) * DW_LD + 16 * bn + fr] -= sb[s][r];
    }
  }
  lds_barrier();
  dmin = potrf4w(As);
  if (t == 0) bad = dmin <= 0.0;
  lds_barrier();
  if (bad) return fail(j + 1);
  {
    double* Y = tileL(c, j + 1, j + 1);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = t + 256 * u, q = e >> 6, r = e & 63;
      gst(Y + e, As[r * DW_LD + q]);
    }
  }
  if (w == 0) logdet(j + 1);
  trtri4w(As, Is, Xs);
  {
    double* Dj = tileD(c, j + 1);
    double* Wj = eval ? tileW(c, j + 1, j + 1) : nullptr;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = t + 256 * u, q = e >> 6, r = e & 63;
      gst(Dj + e, Is[r * DW_LD + q]);
      if (eval) gst(Wj + e, Is[(e >> 6) * DW_LD + (e & 63)]);
    }
  }
  // z_j+1 = Dinv_j+1 z_j+1 (v likewise), partial dot products of block j+1
  if (w == 0) {
    double zp[4] = {0.0, 0.0, 0.0, 0.0}, vp[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const double a = Is[lane * DW_LD + q];
      zp[q & 3] = fma(a, Vs[3 * NB + q], zp[q & 3]);
      vp[q & 3] = fma(a, Vs[4 * NB + q], vp[q & 3]);
    }
    const double zn = (zp[0] + zp[1]) + (zp[2] + zp[3]), vn = (vp[0] + vp[1]) + (vp[2] + vp[3]);
    gst(z + (j + 1) * NB + lane, zn);
    if (pred) gst(v + (j + 1) * NB + lane, vn);
    Vs[6 * NB + lane] = zn;
    double zz = zn * zn, zv = zn * vn, vv = vn * vn;
    for (int o = 32; o >= 1; o >>= 1) {
      zz += __shfl_down(zz, o, 64);
      zv += __shfl_down(zv, o, 64);
      vv += __shfl_down(vv, o, 64);
    }
    if (lane == 0) {
      pp[3 * j + 3] = zz;
      pp[3 * j + 4] = zv;
      pp[3 * j + 5] = vv;
    }
  }
  __syncthreads();  // X (global, this workgroup's stores) and z_j+1 complete
  // W_j+1,j = -Dinv_j+1 X: A(m, q) = Inv[m][q] (zero for q > m), B(q, n) = X[q][n]
  d4 wo[4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    wo[nb] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)
      if (kk <= 4 * w + 3)
        wo[nb] = MFMA64(Is[(16 * w + fr) * DW_LD + 4 * kk + fk], gld(W10c + (4 * kk + fk) * NB + 16 * nb + fr),
                        wo[nb]);
  }
  __syncthreads();  // every read of X is done; As (L_j+1,j+1, stored) is free
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) As[(16 * w + fk + 4 * r) * DW_LD + 16 * nb + fr] = -wo[nb][r];
  lds_barrier();
  {
    double* Wt = eval ? tileW(c, j + 1, j) : nullptr;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = t + 256 * u;
      gst(W10c + e, As[(e & 63) * DW_LD + (e >> 6)]);       // column-major: [n*64 + m] = W[m][n]
      if (eval) gst(Wt + e, As[(e >> 6) * DW_LD + (e & 63)]);  // row-major
    }
  }
  if (eval && w == 0) {
    double ap[4] = {0.0, 0.0, 0.0, 0.0}, bp[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const double zq = Vs[6 * NB + q];
      ap[q & 3] = fma(As[q * DW_LD + lane], zq, ap[q & 3]);
      bp[q & 3] = fma(Is[q * DW_LD + lane], zq, bp[q & 3]);
    }
    gst(al + j * NB + lane, a_j + ((ap[0] + ap[1]) + (ap[2] + ap[3])));
    gst(al + (j + 1) * NB + lane, (bp[0] + bp[1]) + (bp[2] + bp[3]));
  }
}

// ----------------------------------------------------------- k_scale(j)
// P_jk = -Dinv_jj L_jk for k < j (column-major), so that the panel tiles and
// the row of W become single GEMM loops (no separate Dinv product per tile).
// A 256-thread workgroup handles SCALE_KPW tiles k of one cell: the Dinv_jj
// operand stays in registers, each L_jk is staged transposed through LDS and
// D = P^T = -L_jk^T Dinv_jj^T is stored coalesced as P[n][m].
#define SCALE_KPW 4
__global__ __launch_bounds__(256) void k_scale(const OiCell* __restrict__ cells,
                                               const int32_t* __restrict__ list, int j, int kbeg,
                                               int gx, int ncell) {
  __shared__ __attribute__((aligned(16))) double As[NB * LDSA];  // As[q][m] = L_jk[q][m]
  int ci, g;
  if (!xcd_cell_slot(gx, ncell, ci, g)) return;
  const OiCell& c = cells[list[ci]];
  const int k0 = kbeg + g * SCALE_KPW;
  if (j >= c.T || k0 >= j || *c.status != OI_OK) return;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;
  const int fr = lane & 15, fk = lane >> 4;
  const double* D = tileD(c, j);
  double b0[NB / 4], b1[NB / 4];  // B[q][n] = Dinv[n][q] at q*64 + n
#pragma unroll
  for (int kk = 0; kk < NB / 4; ++kk) {
    const int q = kk * 4 + fk;
    b0[kk] = gld(D + q * NB + 32 * wc + fr);
    b1[kk] = gld(D + q * NB + 32 * wc + 16 + fr);
  }
  const int sm = t >> 2, sq = (t & 3) * 16;  // staging: column sm, rows sq..sq+15
  for (int k = k0; k < k0 + SCALE_KPW && k < j; ++k) {
    const double* L = tileL(c, j, k);
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; u += 2) {
      const dv2 x = gload2(L + sm * NB + sq + u);
      v[u] = x[0];
      v[u + 1] = x[1];
    }
    __syncthreads();  // previous tile's reads of As are done
#pragma unroll
    for (int u = 0; u < 16; ++u) As[(sq + u) * LDSA + sm] = v[u];
    __syncthreads();
    Quad acc;
    quad_zero(acc);
    // B(q, n) = Dinv[n][q] is 0 for q > n: k-steps past a block's last column are skipped
    const int nlast = __builtin_amdgcn_readfirstlane(32 * wc) + 15;
#pragma unroll
    for (int kk = 0; kk < NB / 4; ++kk) {
      const int q = kk * 4 + fk;
      const double a0 = As[q * LDSA + 32 * wr + fr], a1 = As[q * LDSA + 32 * wr + 16 + fr];
      if (4 * kk <= nlast) {
        acc.c[0][0] = MFMA64(a0, b0[kk], acc.c[0][0]);
        acc.c[1][0] = MFMA64(a1, b0[kk], acc.c[1][0]);
      }
      if (4 * kk <= nlast + 16) {
        acc.c[0][1] = MFMA64(a0, b1[kk], acc.c[0][1]);
        acc.c[1][1] = MFMA64(a1, b1[kk], acc.c[1][1]);
      }
    }
    double* P = c.P + (size_t)k * OI_TILE;
    for (int mb = 0; mb < 2; ++mb)
      for (int nb = 0; nb < 2; ++nb)
        for (int r = 0; r < 4; ++r) {
          const int m = 32 * wr + 16 * mb + (lane >> 4) + 4 * r, n = 32 * wc + 16 * nb + (lane & 15);
          gst(P + m * NB + n, -acc.c[mb][nb][r]);  // D[m][n] = (Dinv L)[n][m] -> P[n][m]
        }
  }
}

// wave masks of the GEMM cores (padding, triangular operands, syrk halves): oi_masks.h

#define XLD 65  // LDS row stride of a staged 64x64 tile (doubles)

// Forward substitution inside the factorisation: once tile L_ij (i > j) is
// final, z_i -= L_ij z_j (and v_i -= L_ij v_j for predict; z_j, v_j final since
// k_diag_factor(j)).  fwd_preload, issued before the tile's GEMM loop so its
// latency hides behind it, gives thread t one value: z_i[t] (t < 64), z_j
// (64..127), v_i (128..191), v_j (192..255).  fwd_update then stages z_j, v_j
// in LDS, forms L_ij [z_j v_j] from the tile staged as X[col * ld + row] with
// partial sums over NTHREADS/64 column groups combined in a fixed order, and
// writes z_i, v_i.  scratch (>= (2 * NTHREADS/64 + 2) * 64 doubles) must not
// alias X.  Launch order makes the updates of z_i sequential in j.
__device__ __forceinline__ double fwd_preload(const OiCell& c, int i, int j) {
  const int t = threadIdx.x;
  const bool pred = c.mode == OI_MODE_PREDICT;
  const double* z = c.vec;
  const double* v = c.vec + 3 * c.T * NB;
  if (t < 64) return z[i * NB + t];
  if (t < 128) return z[j * NB + t - 64];
  if (pred && t < 192) return v[i * NB + t - 128];
  if (pred && t < 256) return v[j * NB + t - 192];
  return 0.0;
}

template <int NTHREADS>
__device__ __forceinline__ void fwd_update(const OiCell& c, const double* X, int ld, int i, double pre,
                                           double* scratch) {
  constexpr int G = NTHREADS / 64, CW = NB / G;
  const bool pred = c.mode == OI_MODE_PREDICT;
  const int t = threadIdx.x, row = t & 63, grp = t >> 6;
  double* red = scratch;
  double* zj = scratch + 2 * G * NB;
  double* vj = zj + NB;
  if (t >= 64 && t < 128) zj[t - 64] = pre;
  if (t >= 192 && t < 256) vj[t - 192] = pre;
  __syncthreads();
  double sz = 0.0, sv = 0.0;
#pragma unroll 4
  for (int q = 0; q < CW; ++q) {
    const int col = grp * CW + q;
    const double l = X[col * ld + row];
    sz = fma(l, zj[col], sz);
    if (pred) sv = fma(l, vj[col], sv);
  }
  red[grp * NB + row] = sz;
  red[(G + grp) * NB + row] = sv;
  __syncthreads();
  if (t < 64 || (pred && t >= 128 && t < 192)) {
    const int h = t < 64 ? 0 : 1;
    double a = 0.0;
    for (int g = 0; g < G; ++g) a += red[(h * G + g) * NB + row];
    gst(c.vec + (h ? 3 * c.T * NB : 0) + i * NB + row, pre - a);
  }
}

// alpha = W^T z accumulated while W is built (round 2; replaces k_avec):
// once tile W_{j,jj} is final, alpha_jj += W_{j,jj}^T z_j (z_j final since
// k_diag_factor(j), which also starts alpha_j = W_jj^T z_j).  Same staging as
// fwd_update: the tile sits in LDS as X[col * ld + row] with the product's
// output index as `row`; thread t < 64 preloads alpha_jj[t], 64..127 z_j.
__device__ __forceinline__ double alpha_preload(const OiCell& c, int jj, int j) {
  const int t = threadIdx.x;
  if (t < 64) return c.vec[c.T * NB + jj * NB + t];
  if (t < 128) return c.vec[j * NB + t - 64];
  return 0.0;
}

template <int NTHREADS>
__device__ __forceinline__ void alpha_update(const OiCell& c, const double* X, int ld, int jj, double pre,
                                             double* scratch) {
  constexpr int G = NTHREADS / 64, CW = NB / G;
  const int t = threadIdx.x, row = t & 63, grp = t >> 6;
  double* red = scratch;
  double* zj = scratch + G * NB;
  if (t >= 64 && t < 128) zj[t - 64] = pre;
  __syncthreads();
  double sa = 0.0;
#pragma unroll 4
  for (int q = 0; q < CW; ++q) {
    const int col = grp * CW + q;
    sa = fma(X[col * ld + row], zj[col], sa);
  }
  red[grp * NB + row] = sa;
  __syncthreads();
  if (t < 64) {
    double a = 0.0;
    for (int g = 0; g < G; ++g) a += red[g * NB + row];
    gst(c.vec + c.T * NB + jj * NB + row, pre + a);
  }
}

// --------------------------------------------------- k_chol_panel(j)
// One 256-thread workgroup per output tile; logical slots of a cell:
//   x <  T-1-j : tile (i = j+1+x, j) of the factor, one GEMM loop:
//                  L_ij^T = sum_{k<j} P_jk L_ik^T + Dinv_jj A_ij^T
//                (= Dinv_jj (A_ij - sum_k L_ik L_jk^T)^T); slot 0 (i = j+1) then
//                applies the update of diagonal tile j+1 (look-ahead) for
//                k_diag_factor(j+1).
//   x >= T-1-j : (eval) tile (j, jj = x-(T-1-j)) of W = L^-1:
//                  W_j,jj = sum_{k=jj}^{j-1} P_jk W_k,jj
// Post-form (POST, default): the GEMM loop streams L_jk instead of P_jk and the
// Dinv_jj product is applied once to the finished sum (post_left), so no
// k_scale launch and no P tiles are needed:
//   L_ij^T  = Dinv_jj (A_ij^T - sum_{k=kbeg}^{j-1} L_jk L_ik^T)
//   W_j,jj  = Dinv_jj (Vneg - sum_{k=kfirst}^{j-1} L_jk W_k,jj)   (Vneg = 0 if kfirst = jj)
// out(m, n) = sum_q Dinv[m][q] S(q, n), S(m, n) = base[m*64 + n] - acc(m, n)
// (base null: S = -acc).  S is staged in LDS at row stride LDSA = 80 (B operand:
// rows k, k+1 of a 32-lane ds_read_b64 in opposite bank halves); Dinv_jj (column-major,
// lower triangular, zero above the diagonal) is read into registers once, all
// loads in flight together.  The 160 block-k-steps of the triangular product
// are split evenly: wave w owns row blocks {0, 3} (w even) or {1, 2} and column
// blocks 2(w>>1), 2(w>>1)+1 -- 40 MFMAs per wave.  The result is written to
// dst[m*64 + n] and staged in lds as X[m*XLD + n] (what fwd_update /
// alpha_update and the look-ahead read).
__device__ __forceinline__ void post_left(const Quad& acc, double* lds, const double* base, const double* Dj,
                                          double* dst) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int mA = (w & 1) ? 1 : 0, mB = 3 - mA, n0 = 2 * (w >> 1);
  double bv[16];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        bv[(2 * mb + nb) * 4 + r] = base ? gld(base + acc1_row(mb, r) * NB + acc1_col(nb)) : 0.0;
  __syncthreads();  // the GEMM's last LDS reads are done
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r)  // B(q, n) = S[q][n] at q*LDSA + n
        lds[acc1_row(mb, r) * LDSA + acc1_col(nb)] = bv[(2 * mb + nb) * 4 + r] - acc.c[mb][nb][r];
  // A(m, q) = Dinv[m][q] at Dj[q*64 + m]: row block mA needs k-steps kk <= 4 mA + 3, mB up to
  // 4 mB + 3; loaded once S is staged (acc, bv dead: the kernel stays at 4 waves per SIMD)
  double dA[8], dB[16];
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) dA[kk] = kk <= 4 * mA + 3 ? gld(Dj + (4 * kk + fk) * NB + 16 * mA + fr) : 0.0;
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) dB[kk] = kk <= 4 * mB + 3 ? gld(Dj + (4 * kk + fk) * NB + 16 * mB + fr) : 0.0;
  __syncthreads();
  d4 o[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) o[a][b] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) {
    const int k = 4 * kk + fk;
    const double b0 = lds[k * LDSA + 16 * n0 + fr], b1 = lds[k * LDSA + 16 * n0 + 16 + fr];
    if (kk <= 4 * mA + 3) {  // wave-uniform
      o[0][0] = MFMA64(dA[kk < 8 ? kk : 7], b0, o[0][0]);
      o[0][1] = MFMA64(dA[kk < 8 ? kk : 7], b1, o[0][1]);
    }
    if (kk <= 4 * mB + 3) {
      o[1][0] = MFMA64(dB[kk], b0, o[1][0]);
      o[1][1] = MFMA64(dB[kk], b1, o[1][1]);
    }
  }
  __syncthreads();  // S is read before the result replaces it
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * (a ? mB : mA) + (lane >> 4) + 4 * r, n = 16 * (n0 + b) + fr;
        gst(dst + m * NB + n, o[a][b][r]);
        lds[m * XLD + n] = o[a][b][r];
      }
  __syncthreads();
}

template <bool POST>
__global__ __launch_bounds__(256) void k_chol_panel(const OiCell* __restrict__ cells,
                                                   const int32_t* __restrict__ list, int j,
                                                   int kbeg, int gx, int ncell) {
  __shared__ __attribute__((aligned(16))) double lds[GEMM1_LDS];
  int ci, x;
  if (!xcd_cell_slot_lead0(gx, ncell, ci, x)) return;
  const OiCell& c = cells[list[ci]];
  const int T = c.T;
  if (j >= T || *c.status != OI_OK) return;
  const int ntrsm = T - 1 - j;
  const double* Pj = c.P;
  const double* Dj = tileD(c, j);
  Quad acc;
  quad_zero(acc);
  // padding rows of the last block (exact zeros) are skipped per 16x16 block
  const int rT = c.n - NB * (T - 1);
  const int wv = threadIdx.x >> 6, wr = wv >> 1, wc = wv & 1;
  if (x < ntrsm) {
    const int i = j + 1 + x;
    auto fpair = [=, &c](int p, const double*& a, const double*& b) {
      const int k = kbeg + p;
      a = k < j ? Pj + (size_t)k * OI_TILE : Dj;
      b = tileL(c, i, k);  // k == j: A_ij, already holding A_ij - sum_{k<kbeg} L_ik L_jk^T
    };
    const double pre = fwd_preload(c, i, j);
    // n = row of block row i: padding rows of the last block are skipped
    const unsigned psk = i == T - 1 ? pad_skip(32 * wr, 32 * wc, NB, rT) : 0u;
    double* Y = tileL(c, i, j);
    if constexpr (POST) {
      gemm1_kmajor<true>(acc, lds, 4 * (j - kbeg), psk, [=, &c](int p, const double*& a, const double*& b) {
        a = tileL(c, j, kbeg + p);
        b = tileL(c, i, kbeg + p);
      });
      post_left(acc, lds, Y, Dj, Y);  // L_ij^T = Dinv_jj (A_ij^T - acc), stored and staged
    } else {
      const int chD = 4 * (j - kbeg);  // first chunk of the Dinv_jj pair (A(m, k) = 0 for k > m)
      auto cm = [=](int ch) { return ch >= chD ? rows_above(ch - chD, 32 * wr) : 0u; };
      gemm1_kmajor<true>(acc, lds, 4 * (j + 1 - kbeg), psk, fpair, cm);
      for (int mb = 0; mb < 2; ++mb)
        for (int nb = 0; nb < 2; ++nb)
          for (int r = 0; r < 4; ++r) {
            gst(Y + acc1_row(mb, r) * NB + acc1_col(nb), acc.c[mb][nb][r]);  // L_ij, column-major
            lds[acc1_row(mb, r) * XLD + acc1_col(nb)] = acc.c[mb][nb][r];  // staged: X[col*XLD + row]
          }
      __syncthreads();
    }
    fwd_update<256>(c, lds, XLD, i, pre, lds + NB * XLD);
    if (x != 0) return;
    // ---- look-ahead: diagonal tile j+1 = i.
    // S_d = A_ii - L_ij L_ij^T - sum_{k<j} L_ik L_ik^T; the first product uses
    // this workgroup's own L_ij, staged k-major in lds (X[c*XLD + m] = L_ij[m][c])
    const double* Xs = lds;
    Quad accd;
    quad_zero(accd);
    {
      const int t = threadIdx.x, lane = t & 63, w = t >> 6;
      const int wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
#pragma unroll 4
      for (int kk = 0; kk < NB / 4; ++kk) {
        const int k = kk * 4 + fk;
        const double a0 = Xs[k * XLD + 32 * wr + fr], a1 = Xs[k * XLD + 32 * wr + 16 + fr];
        const double b0 = Xs[k * XLD + 32 * wc + fr], b1 = Xs[k * XLD + 32 * wc + 16 + fr];
        accd.c[0][0] = MFMA64(a0, b0, accd.c[0][0]);
        accd.c[0][1] = MFMA64(a0, b1, accd.c[0][1]);
        accd.c[1][0] = MFMA64(a1, b0, accd.c[1][0]);
        accd.c[1][1] = MFMA64(a1, b1, accd.c[1][1]);
      }
    }
    __syncthreads();
    // symmetric, and only its lower triangle is read (k_diag_factor): accd(m, n)
    // lands at row n, column m of the column-major tile, so the accumulator
    // blocks with m > n -- the tile's upper triangle -- are skipped
    gemm1_kmajor<true>(accd, lds, 4 * j, lower_blocks(32 * wr, 32 * wc), [=, &c](int p, const double*& a, const double*& b) {
      a = tileL(c, i, p);
      b = a;
    });
    double* Yd = tileL(c, i, i);
    for (int mb = 0; mb < 2; ++mb)
      for (int nb = 0; nb < 2; ++nb)
        for (int r = 0; r < 4; ++r) {
          const int m = acc1_row(mb, r), n = acc1_col(nb);
          gst(Yd + m * NB + n, gld(Yd + m * NB + n) - accd.c[mb][nb][r]);
        }
    return;
  }
  const int jj = x - ntrsm;
  if (c.mode != OI_MODE_EVAL || jj >= j) return;
  // kbeg > jj: W_j,jj holds Vneg = -sum_{k=jj}^{kbeg-1} L_jk W_k,jj (k_panel_even), so
  // W_j,jj = sum_{k=kbeg}^{j-1} P_jk W_k,jj + Dinv_jj Vneg
  const int kfirst = jj > kbeg ? jj : kbeg, extra = kbeg > jj ? 1 : 0;
  auto wpair = [=, &c](int p, const double*& a, const double*& b) {
    const int k = kfirst + p;
    a = k < j ? Pj + (size_t)k * OI_TILE : Dj;
    b = tileW(c, k, jj);  // k == j: Vneg
  };
  const double apre = alpha_preload(c, jj, j);
  // m = row of W block row j: padding rows of the last block are skipped
  const unsigned psk = j == T - 1 ? pad_skip(32 * wr, 32 * wc, rT, NB) : 0u;
  double* Wt = tileW(c, j, jj);
  if constexpr (POST) {
    // pair k = jj: B = W_jj,jj (B(k, n) = 0 for k < n)
    auto cm = [=](int ch) { return !extra && ch < 4 ? cols_below(ch, 32 * wc) : 0u; };
    gemm1_kmajor<true>(acc, lds, 4 * (j - kfirst), psk, [=, &c](int p, const double*& a, const double*& b) {
      a = tileL(c, j, kfirst + p);
      b = tileW(c, kfirst + p, jj);
    }, cm);
    post_left(acc, lds, extra ? Wt : nullptr, Dj, Wt);  // W_j,jj = Dinv_jj (Vneg - acc), stored and staged
  } else {
    // pair k = jj: B = W_jj,jj (B(k, n) = 0 for k < n); pair k = j: A = Dinv_jj
    const int chD = extra ? 4 * (j - kfirst) : 1 << 30;
    auto cm = [=](int ch) {
      return (!extra && ch < 4 ? cols_below(ch, 32 * wc) : 0u) | (ch >= chD ? rows_above(ch - chD, 32 * wr) : 0u);
    };
    gemm1_kmajor<true>(acc, lds, 4 * (j - kfirst + extra), psk, wpair, cm);
    for (int mb = 0; mb < 2; ++mb)
      for (int nb = 0; nb < 2; ++nb)
        for (int r = 0; r < 4; ++r) {
          gst(Wt + acc1_row(mb, r) * NB + acc1_col(nb), acc.c[mb][nb][r]);  // row-major
          lds[acc1_row(mb, r) * XLD + acc1_col(nb)] = acc.c[mb][nb][r];  // X[row of W * XLD + col]
        }
    __syncthreads();
  }
  alpha_update<256>(c, lds, XLD, jj, apre, lds + NB * XLD);  // alpha_jj += W_j,jj^T z_j
}

// --------------------------------------------------- k_panel_even(j), j even
// Shared-stream form of two consecutive block columns: every streamed tile
// feeds two outputs (64 x 128 block per 512-thread workgroup, gemm2 core), so
// the L / W streams of the left-looking factorisation are read from HBM once
// per PAIR of columns.  Slots of a cell:
//   x <  T-1-j : row i = j+1+x of the factor:
//                  L_ij      = sum_{k<j} L_ik P_jk^T + A_ij Dinv_jj^T
//                  A_i,j+1  -= sum_{k<j} L_ik L_j+1,k^T     (partial update of
//                              column j+1; k_chol_panel(j+1, kbeg=j) adds k = j)
//                i = j+1 (x = 0) instead completes A_j+1,j+1 (look-ahead):
//                  A_j+1,j+1 -= sum_{k<j} L_j+1,k L_j+1,k^T + L_j+1,j L_j+1,j^T
//   x >= T-1-j : (eval) jj = x-(T-1-j) < j, rows j and j+1 of W = L^-1:
//                  W_j,jj    = sum_{k=jj}^{j-1} P_jk W_k,jj
//                  W_j+1,jj  = Vneg := -sum_{k=jj}^{j-1} L_j+1,k W_k,jj  (finished
//                              by k_chol_panel(j+1, kbeg=j))
// Accumulators come out transposed with respect to the tile storage, so each
// 64x64 half goes through LDS and is written back with coalesced 16 B rows.
enum { EMIT_STORE = 0, EMIT_SUB = 1, EMIT_NEG = 2 };

// dst[n*64 + m] (op)= D_h[m][n] for the 64x64 half h of a gemm2 accumulator.
// Leaves the staged tile in X[n*XLD + m] (= dst's storage order) for reuse.
__device__ __forceinline__ void emit_half(const Quad& acc, int h, double* X, double* dst, int op) {
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if (((w & 3) >> 1) == h) {
    for (int mb = 0; mb < 2; ++mb)
      for (int nb = 0; nb < 2; ++nb)
        for (int r = 0; r < 4; ++r)
          X[(acc_col(nb) - 64 * h) * XLD + acc_row(mb, r)] = acc.c[mb][nb][r];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < OI_TILE; e += GEMM_THREADS) {
    const double v = X[(e >> 6) * XLD + (e & 63)];
    if (op == EMIT_STORE)
      gst(dst + e, v);
    else if (op == EMIT_SUB)
      gst(dst + e, gld(dst + e) - v);
    else
      gst(dst + e, -v);
  }
}

// dst[n*64 + m] (op)= X[n*XLD + m] for a tile staged in lds (second half of emit_half)
__device__ __forceinline__ void emit_copy(const double* X, double* dst, int op) {
  for (int e = threadIdx.x; e < OI_TILE; e += GEMM_THREADS) {
    const double v = X[(e >> 6) * XLD + (e & 63)];
    if (op == EMIT_STORE)
      gst(dst + e, v);
    else if (op == EMIT_SUB)
      gst(dst + e, gld(dst + e) - v);
    else
      gst(dst + e, -v);
  }
}

// Post-form (POST): half 0 accumulates sum_{k<j} L_ik L_jk^T (factor) or
// sum_k W_k,jj^T L_jk^T (W rows) and is finished by post_right:
//   L_ij = (A_ij - acc) Dinv_jj^T,   W_j,jj^T = -acc Dinv_jj^T.
// out(m, n) = sum_q S(m, q) Dinv[n][q], S(m, n) = base[n*64 + m] - acc(m, n)
// (base null: S = -acc).  S is staged in LDS row-major at S[m*SLD + q] (A
// operand, SLD = 66: the ds_read_b64 of rows k, k+1 by one 32-lane group land
// on disjoint banks, 4m + 2k mod 64, and the accumulator write-back is 16
// consecutive doubles per lane group) and Dinv_jj's ten lower 16x16 blocks
// next to it, packed (block (I, K) at (I(I+1)/2 + K) * 256, element (n, k) at
// (k & 15) * 16 + (n & 15): rows k, k+1 in opposite bank halves); both global
// reads are issued before the first barrier.  (Round 2 staged S as X[q*65 + m]
// and packed Dinv at stride 17: 2-way conflicts on every read, PMC
// SQ_LDS_BANK_CONFLICT 1.2e11 over the day.)  All eight waves share
// the 160 block-k-steps of the triangular product: wave w owns row block w & 3
// and column blocks {0, 3} (w < 4) or {1, 2} -- 20 MFMAs each.  The result is
// left staged as X[n*XLD + m] (emit_half's layout) for emit_copy.
#define SLD 66
#define DPK_OFF (NB * SLD)
static_assert(DPK_OFF + 10 * 256 <= GEMM2_LDS, "post_right staging must fit the GEMM LDS");
__device__ __forceinline__ void post_right(const Quad& acc, double* lds, const double* base, const double* Dj) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const bool mine = (w & 3) < 2;  // the waves holding half 0
  double dv[5];                   // 2560 packed Dinv entries, 5 per thread
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const int e = t + GEMM_THREADS * q, blk = e >> 8, kl = (e >> 4) & 15, nl = e & 15;
    const int I = blk >= 6 ? 3 : blk >= 3 ? 2 : blk >= 1 ? 1 : 0, K = blk - I * (I + 1) / 2;
    dv[q] = gld(Dj + (16 * K + kl) * NB + 16 * I + nl);
  }
  double bv[16];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        bv[(2 * mb + nb) * 4 + r] = (mine && base) ? gld(base + acc_col(nb) * NB + acc_row(mb, r)) : 0.0;
  __syncthreads();  // the GEMM's last LDS reads are done
  if (mine) {
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          lds[acc_row(mb, r) * SLD + acc_col(nb)] = bv[(2 * mb + nb) * 4 + r] - acc.c[mb][nb][r];
  }
  double* Dp = lds + DPK_OFF;
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const int e = t + GEMM_THREADS * q, blk = e >> 8, kl = (e >> 4) & 15, nl = e & 15;
    Dp[blk * 256 + kl * 16 + nl] = dv[q];
  }
  __syncthreads();
  const int mb = w & 3, nA = (w >> 2) ? 1 : 0, nB = 3 - nA;
  d4 o0 = (d4){0.0, 0.0, 0.0, 0.0}, o1 = o0;
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) {
    const int k = 4 * kk + fk, K = kk >> 2;
    const double a = lds[(16 * mb + fr) * SLD + k];
    // B(k, n) = Dinv[n][k]: block (nX, K), zero for K > nX (wave-uniform skip)
    if (kk <= 4 * nA + 3) o0 = MFMA64(a, Dp[(nA * (nA + 1) / 2 + K) * 256 + (k & 15) * 16 + fr], o0);
    if (kk <= 4 * nB + 3) o1 = MFMA64(a, Dp[(nB * (nB + 1) / 2 + K) * 256 + (k & 15) * 16 + fr], o1);
  }
  __syncthreads();  // S and Dinv are read before the result replaces S
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = 16 * mb + (lane >> 4) + 4 * r;
    lds[(16 * nA + fr) * XLD + m] = o0[r];
    lds[(16 * nB + fr) * XLD + m] = o1[r];
  }
  __syncthreads();
}

template <bool POST>
__global__ __launch_bounds__(GEMM_THREADS) void k_panel_even(const OiCell* __restrict__ cells,
                                                            const int32_t* __restrict__ list,
                                                            int j, int gx, int ncell) {
  __shared__ __attribute__((aligned(16))) double lds[GEMM2_LDS];
  static_assert(NB * XLD <= GEMM2_LDS, "staging tile must fit the GEMM LDS");
  int ci, x;
  if (!xcd_cell_slot(gx, ncell, ci, x)) return;
  const OiCell& c = cells[list[ci]];
  const int T = c.T;
  if (j >= T || *c.status != OI_OK) return;
  const int ntrsm = T - 1 - j;
  const bool has_next = j + 1 < T;
  const double* Pj = c.P;
  const double* Dj = tileD(c, j);
  Quad acc;
  quad_zero(acc);
  // rows / columns of the last block beyond n are padding: their products are
  // exact zeros (identity padding), so those accumulator blocks are skipped
  const int rT = c.n - NB * (T - 1);
  const int w = threadIdx.x >> 6, wr = (w >> 2) & 1, wc = w & 3;
  if (x < ntrsm) {
    const int i = j + 1 + x;
    auto fpair = [=, &c](int p, const double*& a, const double*& b0, const double*& b1) {
      if (p < j) {
        a = tileL(c, i, p);
        b0 = Pj + (size_t)p * OI_TILE;
        b1 = tileL(c, j + 1, p);
      } else {
        a = tileL(c, i, j);  // A_ij
        b0 = Dj;
        b1 = g_zero_tile;
      }
    };
    // m = row of block row i; half 1's n = column of block column j+1
    const int mlim = i == T - 1 ? rT : NB, nlim = (wc >= 2 && j + 1 == T - 1) ? rT : NB;
    const double pre = fwd_preload(c, i, j);
    // last pair: half 0 multiplies by Dinv_jj^T (B(k, n) = 0 for k > n), half 1 by
    // the zero tile; the first row's half 1 (x = 0) is the diagonal tile j+1,
    // symmetric: its blocks above the diagonal are never read
    const int chD = 4 * j;
    const unsigned sk = pad_skip(32 * wr, 32 * (wc & 1), mlim, nlim) |
                        (x == 0 && wc >= 2 ? upper_blocks(32 * wr, 32 * (wc - 2)) : 0u);
    if constexpr (POST) {
      gemm2_kmajor<true>(acc, lds, j, [=, &c](int p, const double*& a, const double*& b0, const double*& b1) {
        a = tileL(c, i, p);
        b0 = tileL(c, j, p);
        b1 = tileL(c, j + 1, p);
      }, sk);
      post_right(acc, lds, tileL(c, i, j), Dj);  // L_ij = (A_ij - acc) Dinv_jj^T, staged
      emit_copy(lds, tileL(c, i, j), EMIT_STORE);
    } else {
      auto cm = [=](int ch) { return ch < chD ? 0u : wc >= 2 ? 0xFu : cols_above(ch - chD, 32 * wc); };
      gemm2_kmajor<true>(acc, lds, j + 1, fpair, sk, cm);
      emit_half(acc, 0, lds, tileL(c, i, j), EMIT_STORE);  // L_ij (staged in lds as X[col*XLD+row])
    }
    fwd_update<GEMM_THREADS>(c, lds, XLD, i, pre, lds + NB * XLD);
    if (x != 0) {
      if (j > 0) emit_half(acc, 1, lds, tileL(c, i, j + 1), EMIT_SUB);  // partial update of A_i,j+1 (empty at j = 0)
      return;
    }
    // i = j+1: add the fresh L_j+1,j L_j+1,j^T (staged in lds as X[q*XLD + m] =
    // L[m][q]) to the half-1 accumulator, then complete A_j+1,j+1.
    __syncthreads();
    {
      const int t = threadIdx.x, lane = t & 63, w = t >> 6;
      const int wr = (w >> 2) & 1, wc = w & 3, fr = lane & 15, fk = lane >> 4;
      if ((wc >> 1) == 1) {
        const int c0 = 32 * (wc - 2);
#pragma unroll 4
        for (int kk = 0; kk < NB / 4; ++kk) {
          const int q = kk * 4 + fk;
          const double a0 = lds[q * XLD + 32 * wr + fr], a1 = lds[q * XLD + 32 * wr + 16 + fr];
          const double b0 = lds[q * XLD + c0 + fr], b1 = lds[q * XLD + c0 + 16 + fr];
          acc.c[0][0] = MFMA64(a0, b0, acc.c[0][0]);
          acc.c[0][1] = MFMA64(a0, b1, acc.c[0][1]);
          acc.c[1][0] = MFMA64(a1, b0, acc.c[1][0]);
          acc.c[1][1] = MFMA64(a1, b1, acc.c[1][1]);
        }
      }
    }
    emit_half(acc, 1, lds, tileL(c, i, i), EMIT_SUB);
    return;
  }
  const int jj = x - ntrsm;
  if (c.mode != OI_MODE_EVAL || jj >= j) return;
  auto wpair = [=, &c](int p, const double*& a, const double*& b0, const double*& b1) {
    const int k = jj + p;
    a = tileW(c, k, jj);
    b0 = POST ? tileL(c, j, k) : Pj + (size_t)k * OI_TILE;
    b1 = has_next ? tileL(c, j + 1, k) : g_zero_tile;
  };
  // n = row of W block row j (half 0) or j+1 (half 1)
  const int nlim = ((wc < 2 && j == T - 1) || (wc >= 2 && j + 1 == T - 1)) ? rT : NB;
  const double apre = alpha_preload(c, jj, j);
  // pair k = jj: A = W_jj,jj^T (A(m, k) = 0 for k < m); no row j+1: half 1 idle
  const unsigned sk = pad_skip(0, 32 * (wc & 1), NB, nlim) | (!has_next && wc >= 2 ? 0xFu : 0u);
  auto cm = [=](int ch) { return ch < 4 ? rows_below(ch, 32 * wr) : 0u; };
  gemm2_kmajor<true>(acc, lds, j - jj, wpair, sk, cm);
  if constexpr (POST) {
    post_right(acc, lds, nullptr, Dj);  // W_j,jj^T = -acc Dinv_jj^T, staged
    emit_copy(lds, tileW(c, j, jj), EMIT_STORE);
  } else {
    emit_half(acc, 0, lds, tileW(c, j, jj), EMIT_STORE);  // W_j,jj (row-major), staged X[n*XLD+m]
  }
  alpha_update<GEMM_THREADS>(c, lds, XLD, jj, apre, lds + NB * XLD);  // alpha_jj += W_j,jj^T z_j
  if (has_next) emit_half(acc, 1, lds, tileW(c, j + 1, jj), EMIT_NEG);  // Vneg
}

// --------------------------------------------------- k_panel4(j), j even
// k_panel_even on the 128 x 128 gemm4 core (OI_PANEL4=1): a workgroup owns TWO
// block rows, so every streamed tile feeds four outputs instead of two -- half
// the operand traffic per flop of the 64 x 128 core, whose in-kernel rate
// (53.9 TF/s executed on the day) sits at its own streaming limit (52.5 TF/s,
// tools/gemm4_probe.hip; the 128 x 128 core streams at 61).  Slots of a cell:
//   x <  nfp = ceil((T-1-j)/2) : rows i1 = j+1+2x, i2 = i1+1 (absent past T-1):
//        quadrant (r, 0) = L_{i_r, j} (post-form: (A - sum_k L L^T) Dinv_jj^T),
//        quadrant (r, 1) = partial update of A_{i_r, j+1}; x = 0 completes the
//        diagonal tile A_{j+1, j+1} (look-ahead) with the fresh L_{j+1,j} L^T
//   x >= nfp (eval): W columns jj1 = 2y, jj2 = 2y+1 (y = x - nfp, j even):
//        quadrant (r, 0) = W_{j, jj_r}, quadrant (r, 1) = Vneg of W_{j+1, jj_r}
// Nothing but the accumulators is live across the GEMM (the core takes all 128
// VGPRs at 4 waves per SIMD; even loading A_ij into the accumulators before it
// spills), and the epilogue
// empties the accumulators into LDS first: the column-(j+1) quadrants go out
// as partial updates, then both S tiles are staged (row-major, stride SLD) and
// the two triangular products S_r Dinv_jj^T run together, each wave holding
// its Dinv_jj operand fragments in registers.
__host__ __device__ inline int nslot4_factor(int T, int j) { return (T - j) >> 1; }  // ceil((T-1-j)/2)

// quadrant (qr, 1) of a gemm4 accumulator staged as X[n*XLD + m] (dst's storage order)
__device__ __forceinline__ void stage4_q1(const Quad8& acc, int qr, double* X) {
  const int w = threadIdx.x >> 6;
  if ((w >> 2) == qr && (w & 1) == 1) {
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int r = 0; r < 4; ++r) X[(acc4_col(nb) - 64) * XLD + (acc4_row(mb, r) - 64 * qr)] = acc.c[mb][nb][r];
  }
}

// Both triangular products out_r(m, n) = sum_q S_r(m, q) Dinv[n][q], S_r = A_r - acc
// of quadrant (r, 0) (A_r column-major, null: S_r = -acc), r = 0, 1 (`two`):
// stages S_r at lds + r * 64 * SLD (row-major; A_r added with coalesced reads),
// wave w computes row block w & 3 of both tiles against column blocks {0, 3}
// (w < 4) or {1, 2} (20 + 20 MFMAs); returns with the products in o[r][0..1].
__device__ __forceinline__ void post_right4x2(const Quad8& acc, double* lds, const double* Dj, bool two,
                                              const double* A0, const double* A1, d4 (&o)[2][2]) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int mb = w & 3, nA = (w >> 2) ? 1 : 0, nB = 3 - nA;
  if ((w & 1) == 0) {
    const int qr = w >> 2;
    if (qr == 0 || two) {
      double* S = lds + qr * NB * SLD;
#pragma unroll
      for (int m2 = 0; m2 < 2; ++m2)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
#pragma unroll
          for (int r = 0; r < 4; ++r) S[(acc4_row(m2, r) - 64 * qr) * SLD + acc4_col(nb)] = -acc.c[m2][nb][r];
    }
  }
  // (the accumulators are dead from here on)
  // B(k, n) = Dinv[n][k] at Dj[k*64 + n]: this wave's column blocks nA, nB, k-steps kk <= 4 nX + 3
  double bA[8], bB[16];
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) bA[kk] = kk <= 4 * nA + 3 ? gld(Dj + (4 * kk + fk) * NB + 16 * nA + fr) : 0.0;
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) bB[kk] = kk <= 4 * nB + 3 ? gld(Dj + (4 * kk + fk) * NB + 16 * nB + fr) : 0.0;
  if (A0) {  // S_r += A_r: element (m, q) at q*64 + m, 8 per thread and tile.  A wave-
    // instruction covers 32 rows m x 2 columns q (lane l: m = m0 + l/2, q = q0 + l%2):
    // the global reads are two 256-B runs, and S[m*SLD + q] (bank 4m + 2q) hits 64
    // distinct banks per 32-lane read and 32 per 16-lane write (2m + q distinct mod 16)
    double av[8], bv[8];
    int ix[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int g = t + GEMM_THREADS * u, b = g >> 6, l = g & 63;
      const int m = 32 * (b & 1) + (l >> 1), q = 2 * (b >> 1) + (l & 1);
      ix[u] = m * SLD + q;
      av[u] = gld(A0 + q * NB + m);
      bv[u] = two ? gld(A1 + q * NB + m) : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      lds[ix[u]] += av[u];
      if (two) lds[NB * SLD + ix[u]] += bv[u];
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    o[r][0] = (d4){0.0, 0.0, 0.0, 0.0};
    o[r][1] = o[r][0];
    if (r == 1 && !two) break;
    const double* S = lds + r * NB * SLD;
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const double a = S[(16 * mb + fr) * SLD + 4 * kk + fk];
      if (kk <= 4 * nA + 3) o[r][0] = MFMA64(a, bA[kk < 8 ? kk : 7], o[r][0]);
      if (kk <= 4 * nB + 3) o[r][1] = MFMA64(a, bB[kk], o[r][1]);
    }
  }
}

// out tile r (o[r]) staged as X[n*XLD + m] (emit_copy / fwd_update / alpha_update layout)
__device__ __forceinline__ void stage_post4(const d4 (&o)[2][2], int r, double* X) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int fr = lane & 15, mb = w & 3, nA = (w >> 2) ? 1 : 0, nB = 3 - nA;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int m = 16 * mb + (lane >> 4) + 4 * q;
    X[(16 * nA + fr) * XLD + m] = o[r][0][q];
    X[(16 * nB + fr) * XLD + m] = o[r][1][q];
  }
}

__global__ __launch_bounds__(GEMM_THREADS) __attribute__((amdgpu_waves_per_eu(4, 4)))
void k_panel4(const OiCell* __restrict__ cells, const int32_t* __restrict__ list, int j, int gx, int ncell) {
  __shared__ __attribute__((aligned(16))) double lds[GEMM4_LDS];
  static_assert(2 * NB * SLD <= GEMM4_LDS && 2 * NB * XLD <= GEMM4_LDS, "panel4 staging must fit");
  int ci, x;
  if (!xcd_cell_slot(gx, ncell, ci, x)) return;
  const OiCell& c = cells[list[ci]];
  const int T = c.T;
  if (j >= T || *c.status != OI_OK) return;
  const int nfp = nslot4_factor(T, j);
  const bool has_next = j + 1 < T;
  const double* Dj = tileD(c, j);
  const int rT = c.n - NB * (T - 1);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;
  Quad8 acc;
  quad8_zero(acc);
  d4 o[2][2];
  if (x < nfp) {
    const int i1 = j + 1 + 2 * x, i2 = i1 + 1;
    const bool two = i2 < T;
    const int ti = wr >= 2 ? i2 : i1, tj = wc ? j + 1 : j;
    unsigned skip = 0;
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const int m0 = 32 * (wr & 1) + 16 * mb, n0 = 16 * nb;
        const bool off = ti >= T || (ti == T - 1 && m0 >= rT) || (tj == T - 1 && n0 >= rT) ||
                         (x == 0 && wr < 2 && wc == 1 && m0 + 15 < n0);
        if (off) skip |= 1u << (4 * mb + nb);
      }
    auto fpair = [=, &c](int p, const double*& a0, const double*& a1, const double*& b0, const double*& b1) {
      a0 = tileL(c, i1, p);
      a1 = two ? tileL(c, i2, p) : g_zero_tile;
      b0 = tileL(c, j, p);
      b1 = tileL(c, j + 1, p);
    };
    const bool masked = x == 0 || i2 >= T - 1 || j + 1 == T - 1;
    if (masked)
      gemm4_kmajor<true>(acc, lds, 4 * j, skip, fpair);
    else
      gemm4_kmajor<false>(acc, lds, 4 * j, 0u, fpair);
    __syncthreads();  // the GEMM's last LDS reads are done
    // column j+1: partial updates of A_{i_r, j+1} (x = 0: the diagonal tile, whose
    // L_{j+1,j} L_{j+1,j}^T part follows once that tile is final); at j = 0 the
    // sums are empty and A - 0 is A bit for bit: no round trip through HBM
    if (j > 0) {
      stage4_q1(acc, 0, lds);
      if (two) stage4_q1(acc, 1, lds + NB * XLD);
      __syncthreads();
      emit_copy(lds, tileL(c, i1, j + 1), EMIT_SUB);
      if (two) emit_copy(lds + NB * XLD, tileL(c, i2, j + 1), EMIT_SUB);
      __syncthreads();
    }
    post_right4x2(acc, lds, Dj, two, tileL(c, i1, j), two ? tileL(c, i2, j) : nullptr, o);
    const double pre1 = fwd_preload(c, i1, j);
    const double pre2 = two ? fwd_preload(c, i2, j) : 0.0;
    __syncthreads();
    stage_post4(o, 0, lds);  // L_{i1,j}
    __syncthreads();
    emit_copy(lds, tileL(c, i1, j), EMIT_STORE);
    fwd_update<GEMM_THREADS>(c, lds, XLD, i1, pre1, lds + NB * XLD);
    if (x == 0) {
      // A_{j+1,j+1} -= L_{j+1,j} L_{j+1,j}^T: the fresh tile is staged as X[q*XLD + m]
      // = L[m][q]; its 10 lower 16x16 blocks go to the 8 waves (blocks w, w + 8)
      double* Y = lds + NB * XLD;
      __syncthreads();  // fwd_update's scratch (= Y) is free
      for (int e = t; e < OI_TILE; e += GEMM_THREADS) Y[(e >> 6) * XLD + (e & 63)] = 0.0;
      __syncthreads();
      const int fr = lane & 15, fk = lane >> 4;
      for (int bidx = w; bidx < 10; bidx += 8) {
        const int bm = bidx >= 6 ? 3 : bidx >= 3 ? 2 : bidx >= 1 ? 1 : 0, bn = bidx - bm * (bm + 1) / 2;
        d4 s = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
        for (int kk = 0; kk < NB / 4; ++kk) {
          const int q = 4 * kk + fk;
          s = MFMA64(lds[q * XLD + 16 * bm + fr], lds[q * XLD + 16 * bn + fr], s);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) Y[(16 * bn + fr) * XLD + 16 * bm + (lane >> 4) + 4 * r] = s[r];
      }
      __syncthreads();
      emit_copy(Y, tileL(c, i1, i1), EMIT_SUB);
    }
    if (!two) return;
    __syncthreads();
    stage_post4(o, 1, lds);  // L_{i2,j}
    __syncthreads();
    emit_copy(lds, tileL(c, i2, j), EMIT_STORE);
    fwd_update<GEMM_THREADS>(c, lds, XLD, i2, pre2, lds + NB * XLD);
    return;
  }
  const int y = x - nfp;
  if (c.mode != OI_MODE_EVAL || 2 * y >= j) return;
  const int jj1 = 2 * y, jj2 = jj1 + 1;
  const int tj = wc ? j + 1 : j;
  unsigned skip = 0;
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const int n0 = 16 * nb;
      if ((wc == 1 && !has_next) || (tj == T - 1 && n0 >= rT)) skip |= 1u << (4 * mb + nb);
    }
  auto wpair = [=, &c](int p, const double*& a0, const double*& a1, const double*& b0, const double*& b1) {
    const int k = jj1 + p;
    a0 = tileW(c, k, jj1);
    a1 = k >= jj2 ? tileW(c, k, jj2) : g_zero_tile;
    b0 = tileL(c, j, k);
    b1 = has_next ? tileL(c, j + 1, k) : g_zero_tile;
  };
  if (j >= T - 2)
    gemm4_kmajor<true>(acc, lds, 4 * (j - jj1), skip, wpair);
  else
    gemm4_kmajor<false>(acc, lds, 4 * (j - jj1), 0u, wpair);
  __syncthreads();
  if (has_next) {  // Vneg of W_{j+1, jj_r}
    stage4_q1(acc, 0, lds);
    stage4_q1(acc, 1, lds + NB * XLD);
    __syncthreads();
    emit_copy(lds, tileW(c, j + 1, jj1), EMIT_NEG);
    emit_copy(lds + NB * XLD, tileW(c, j + 1, jj2), EMIT_NEG);
    __syncthreads();
  }
  post_right4x2(acc, lds, Dj, true, nullptr, nullptr, o);
  const double apre1 = alpha_preload(c, jj1, j);
  const double apre2 = alpha_preload(c, jj2, j);
  __syncthreads();
  stage_post4(o, 0, lds);  // W_{j,jj1}^T
  __syncthreads();
  emit_copy(lds, tileW(c, j, jj1), EMIT_STORE);
  alpha_update<GEMM_THREADS>(c, lds, XLD, jj1, apre1, lds + NB * XLD);
  __syncthreads();
  stage_post4(o, 1, lds);  // W_{j,jj2}^T
  __syncthreads();
  emit_copy(lds, tileW(c, j, jj2), EMIT_STORE);
  alpha_update<GEMM_THREADS>(c, lds, XLD, jj2, apre2, lds + NB * XLD);
}

// --------------------------------------------------- k_panel_pair(j), j even
// Folded pair step (OI_FOLD=1, default): with the whole 128 x 128 diagonal
// block JJ = (j, j+1) factored and inverted by k_diag_pair(j), Winv_JJ =
// [[Dinv_j, 0], [W_j+1,j, Dinv_j+1]], one stream per row pair finishes BOTH
// block columns -- there is no odd-column launch (k_chol_panel) and no partial
// update of column j+1 goes through HBM:
//   [L_ij  L_i,j+1] = (A_iJ - sum_{k<j} L_ik L_Jk^T) Winv_JJ^T          (i >= j+2)
//   [W_j,jj  ; W_j+1,jj] = -Winv_JJ sum_{k<j} L_Jk W_k,jj                 (jj < j)
// Slots of a cell (gemm4 core, 512 threads, two 64-row outputs per workgroup):
//   x < lead (= 1 if j >= 2): look-ahead of the next diagonal block J' = (j+2, j+3):
//        A_J'J' -= sum_{k<j} L_J'k L_J'k^T (lower quadrants, in place)
//   next nrp = ceil((T-2-j)/2): rows i1 = j+2+2y, i2 = i1+1; the first pair
//        (rows J') then also forms E = sum_{k=j}^{j+1} L_J'k L_J'k^T into c.P
//        tiles 0..2 for k_diag_pair(j+2) -- the two products the look-ahead
//        slot cannot see, as their tiles are made in this launch
//   then (eval) W column pairs jj1 = 2y', jj2 = jj1+1 < j.
// Epilogue per output row r (64 x 128): S_r = A - acc staged row-major in LDS
// (stride SLD2), out = S_r Winv_JJ^T on the MFMA unit, B fragments of Winv read
// from L2 (Dinv tiles and W_j+1,j's column-major copy in c.P tile 3); the
// accumulators of row 1 leave through their destination tiles in HBM (A - acc)
// while row 0 is processed, since LDS holds one staged row and the registers
// one accumulator set.
#define SLD2 130  // (4m + 2q) mod 64: the 32-lane halves of a ds_read_b64 hit distinct banks
static_assert(NB * SLD2 <= GEMM4_LDS && 2 * NB * XLD + 768 <= GEMM4_LDS, "panel-pair staging must fit");
__host__ __device__ inline int npair_rows(int T, int j) { return T - 1 - j > 0 ? (T - 1 - j) >> 1 : 0; }

// column blocks of a wave's share of the 128-wide triangular product: rows
// 16 (w & 3) .. +16 against {0, 7, 2, 5} (w < 4) or {1, 6, 3, 4}: 72 k-steps each
__device__ __forceinline__ int pair_nb(int h, int u) {
  return h ? (u == 0 ? 1 : u == 1 ? 6 : u == 2 ? 3 : 4) : (u == 0 ? 0 : u == 1 ? 7 : u == 2 ? 2 : 5);
}

// B(q, n) = Winv_JJ[n][q], every part column-major ([q*64 + n]); callers ask only q <= n|15
__device__ __forceinline__ double winv_frag(const double* D0, const double* W10, const double* D1, int n, int q) {
  if (n < NB) return gld(D0 + q * NB + n);
  if (q < NB) return gld(W10 + q * NB + (n - NB));
  return gld(D1 + (q - NB) * NB + (n - NB));
}

// o[u] = (S Winv^T) block (w & 3, pair_nb(w >> 2, u)), S staged at S[m*SLD2 + q]; two = false:
// the second block column is absent (columns 64..127 not formed).  The B
// fragments come from L2 in groups of four k-steps, the next group in flight
// while the current one's MFMAs run (the loop is kept rolled: register budget).
__device__ __forceinline__ void post_pair(const double* S, const double* D0, const double* W10, const double* D1,
                                          bool two, d4 (&o)[4]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fk = lane >> 4;
  const int mb = w & 3, h = w >> 2;
  const double* Srow = S + (16 * mb + fr) * SLD2 + fk;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    o[u] = (d4){0.0, 0.0, 0.0, 0.0};
    const int nb = pair_nb(h, u);
#ifdef OI_PP_NOEPI  // timing experiment only (scripts/build_exp_lib.sh): no triangular product
    continue;
#endif
    if (!two && nb >= 4) continue;
    const int ng = nb + 1, n = 16 * nb + fr;  // groups of 4 k-steps: q < 16 nb + 16
    double b[4], bn[4];
#pragma unroll
    for (int kq = 0; kq < 4; ++kq) b[kq] = winv_frag(D0, W10, D1, n, 4 * kq + fk);
#pragma unroll 1
    for (int g = 0; g < ng; ++g) {
      const int gn = g + 1 < ng ? g + 1 : g;  // the last prefetch re-reads the group
#pragma unroll
      for (int kq = 0; kq < 4; ++kq) bn[kq] = winv_frag(D0, W10, D1, n, 16 * gn + 4 * kq + fk);
#pragma unroll
      for (int kq = 0; kq < 4; ++kq) o[u] = MFMA64(Srow[16 * g + 4 * kq], b[kq], o[u]);
#pragma unroll
      for (int kq = 0; kq < 4; ++kq) b[kq] = bn[kq];
    }
  }
}

// S[m*SLD2 + q] (op)= tile[q*64 + m] for a column-major 64 x 64 tile into columns
// c0 .. c0+63 of the staged row (coalesced 256 B runs; add = false: assign)
__device__ __forceinline__ void stage_tile_rm(double* S, int c0, const double* tile, bool add) {
  const int t = threadIdx.x;
  double av[8];
  int ix[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int g = t + GEMM_THREADS * u, b = g >> 6, l = g & 63;
    const int m = 32 * (b & 1) + (l >> 1), q = 2 * (b >> 1) + (l & 1);
    ix[u] = m * SLD2 + c0 + q;
    av[u] = gld(tile + q * NB + m);
  }
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    if (add)
      S[ix[u]] += av[u];
    else
      S[ix[u]] = av[u];
  }
}

// quadrant (qr, qc) of a gemm4 accumulator staged as X[n*XLD + m] (emit_copy's layout)
__device__ __forceinline__ void stage4_q(const Quad8& acc, int qr, int qc, double* X) {
  const int w = threadIdx.x >> 6;
  if ((w >> 2) == qr && (w & 1) == qc) {
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          X[(acc4_col(nb) - 64 * qc) * XLD + (acc4_row(mb, r) - 64 * qr)] = acc.c[mb][nb][r];
  }
}

// y_d[m] = pre_d + sign * sum_{n<ncol} X[n*XLD + m] u_d[n] for d = 0 and (two) d = 1:
// the forward substitution z_i -= L_iJ z_J (v likewise) of a finished factor
// row, or alpha_jj += W_J,jj^T z_J of a finished W row.  Threads t < 256: row
// m = t & 63, column group t >> 6; partial sums combined in a fixed order.
// vec_preload (issued before the epilogue's products) gives thread t: u = u0[t]
// (t < 128) / u1[t - 128], y = y0[t] (t < 64) / y1[t - 64] (t < 128).
struct VecPre {
  double u, y;
};
__device__ __forceinline__ VecPre vec_preload(const double* u0, const double* u1, const double* y0, const double* y1,
                                              int ncol) {
  const int t = threadIdx.x;
  VecPre p = {0.0, 0.0};
  if (t < ncol) p.u = u0[t];
  else if (u1 && t >= 128 && t - 128 < ncol) p.u = u1[t - 128];
  if (t < 64) p.y = y0[t];
  else if (y1 && t < 128) p.y = y1[t - 64];
  return p;
}
__device__ __forceinline__ void vec_update(const double* X, int ncol, bool two, VecPre p, double* y0, double* y1,
                                           double sign, double* scratch) {
  double* uu = scratch;         // 2 x 128
  double* red = scratch + 256;  // 2 x 4 x 64
  const int t = threadIdx.x;
  if (t < 256) uu[t] = p.u;
  __syncthreads();
  if (t < 256) {
    const int m = t & 63, g = t >> 6, cw = ncol >> 2;
    double s0 = 0.0, s1 = 0.0;
#pragma unroll 4
    for (int q = 0; q < cw; ++q) {
      const int n = g * cw + q;
      const double x = X[n * XLD + m];
      s0 = fma(x, uu[n], s0);
      if (two) s1 = fma(x, uu[128 + n], s1);
    }
    red[g * 64 + m] = s0;
    red[256 + g * 64 + m] = s1;
  }
  __syncthreads();
  if (t < 64 || (two && t < 128)) {
    const int m = t & 63, d = t >> 6;
    const double* rd = red + 256 * d;
    const double a = (rd[m] + rd[64 + m]) + (rd[128 + m] + rd[192 + m]);
    gst((d ? y1 : y0) + m, p.y + sign * a);
  }
}

// One output row of a pair workgroup: S (staged) -> out = S Winv^T -> dst0 (columns of
// block j) / dst1 (block j+1, if two) and the vector update.  Leaves LDS free.
__device__ __forceinline__ void pair_row_out(double* lds, const double* D0, const double* W10, const double* D1,
                                             bool two, double* dst0, double* dst1, VecPre p, bool two_vec,
                                             double* y0, double* y1, double sign) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15;
  const int mb = w & 3, h = w >> 2;
  d4 o[4];
  post_pair(lds, D0, W10, D1, two, o);
  __syncthreads();  // S is read; its space takes the result
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int nb = pair_nb(h, u);
#pragma unroll
    for (int r = 0; r < 4; ++r) lds[(16 * nb + fr) * XLD + 16 * mb + (lane >> 4) + 4 * r] = o[u][r];
  }
  __syncthreads();
  emit_copy(lds, dst0, EMIT_STORE);
  if (two) emit_copy(lds + NB * XLD, dst1, EMIT_STORE);
  vec_update(lds, two ? 2 * NB : NB, two_vec, p, y0, y1, sign, lds + 2 * NB * XLD);
  __syncthreads();
}

__global__ __launch_bounds__(GEMM_THREADS) __attribute__((amdgpu_waves_per_eu(4, 4)))
void k_panel_pair(const OiCell* __restrict__ cells, const int32_t* __restrict__ list, int j, int gx, int ncell) {
  __shared__ __attribute__((aligned(16))) double lds[GEMM4_LDS];
  int ci, x;
  if (!xcd_cell_slot(gx, ncell, ci, x)) return;
  const OiCell& c = cells[list[ci]];
  const int T = c.T;
  if (j >= T || *c.status != OI_OK) return;
  const int lead = j >= 2 ? 1 : 0, nrp = npair_rows(T, j);
  const bool has_next = j + 1 < T, pred = c.mode == OI_MODE_PREDICT;
  const int rT = c.n - NB * (T - 1);
  const int t = threadIdx.x, w = t >> 6, wr = w >> 1, wc = w & 1;
  const double* D0 = tileD(c, j);
  const double* D1 = has_next ? tileD(c, j + 1) : nullptr;
  const double* W10 = c.P + 3 * OI_TILE;
  double* z = c.vec;
  double* v = c.vec + 3 * T * NB;
  Quad8 acc;
  quad8_zero(acc);
  if (x < lead) {
    // ---- look-ahead: A_J'J' -= sum_{k<j} L_J'k L_J'k^T, J' = (j+2, j+3)
    const int a = j + 2, b = j + 3;
    if (a >= T) return;
#ifdef OI_PP_NOLA  // timing experiment only: no look-ahead workgroup
    return;
#endif
    const bool two = b < T;
    unsigned skip = 0;
    const int qr = wr >> 1;
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const int m0 = 32 * (wr & 1) + 16 * mb, n0 = 16 * nb, ti = qr ? b : a, tj = wc ? b : a;
        const bool off = (qr == 0 && wc == 1) || ti >= T || tj >= T || (qr == wc && m0 + 15 < n0) ||
                         (ti == T - 1 && m0 >= rT) || (tj == T - 1 && n0 >= rT);
        if (off) skip |= 1u << (4 * mb + nb);
      }
    gemm4_kmajor<true>(acc, lds, 4 * j, skip, [=, &c](int p, const double*& a0, const double*& a1,
                                                       const double*& b0, const double*& b1) {
      a0 = tileL(c, a, p);
      a1 = two ? tileL(c, b, p) : g_zero_tile;
      b0 = a0;
      b1 = a1;
    });
    __syncthreads();
    stage4_q(acc, 0, 0, lds);
    if (two) stage4_q(acc, 1, 0, lds + NB * XLD);
    __syncthreads();
    emit_copy(lds, tileL(c, a, a), EMIT_SUB);
    if (!two) return;
    emit_copy(lds + NB * XLD, tileL(c, b, a), EMIT_SUB);
    __syncthreads();
    stage4_q(acc, 1, 1, lds);
    __syncthreads();
    emit_copy(lds, tileL(c, b, b), EMIT_SUB);
    return;
  }
  if (x < lead + nrp) {
    // ---- rows i1, i2 of both block columns j, j+1 (j+1 < T here)
    const int y = x - lead, i1 = j + 2 + 2 * y, i2 = i1 + 1;
    const bool two = i2 < T;
    unsigned skip = 0;
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const int m0 = 32 * (wr & 1) + 16 * mb, n0 = 16 * nb, ti = wr >= 2 ? i2 : i1, tj = wc ? j + 1 : j;
        if (ti >= T || (ti == T - 1 && m0 >= rT) || (tj == T - 1 && n0 >= rT)) skip |= 1u << (4 * mb + nb);
      }
    auto fpair = [=, &c](int p, const double*& a0, const double*& a1, const double*& b0, const double*& b1) {
      a0 = tileL(c, i1, p);
      a1 = two ? tileL(c, i2, p) : g_zero_tile;
      b0 = tileL(c, j, p);
      b1 = tileL(c, j + 1, p);
    };
    if (i2 >= T - 1 || j + 1 == T - 1)
      gemm4_kmajor<true>(acc, lds, 4 * j, skip, fpair);
    else
      gemm4_kmajor<false>(acc, lds, 4 * j, 0u, fpair);
    __syncthreads();  // the GEMM's last LDS reads are done
    if (two) {  // row i2 leaves through its tiles: A - acc
      stage4_q(acc, 1, 0, lds);
      stage4_q(acc, 1, 1, lds + NB * XLD);
      __syncthreads();
      emit_copy(lds, tileL(c, i2, j), EMIT_SUB);
      emit_copy(lds + NB * XLD, tileL(c, i2, j + 1), EMIT_SUB);
      __syncthreads();
    }
    if ((w >> 2) == 0) {  // S_1 = -acc of row i1, then + A
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
#pragma unroll
          for (int r = 0; r < 4; ++r) lds[acc4_row(mb, r) * SLD2 + acc4_col(nb)] = -acc.c[mb][nb][r];
    }
    __syncthreads();
    stage_tile_rm(lds, 0, tileL(c, i1, j), true);
    stage_tile_rm(lds, NB, tileL(c, i1, j + 1), true);
    VecPre p = vec_preload(z + j * NB, pred ? v + j * NB : nullptr, z + i1 * NB, pred ? v + i1 * NB : nullptr, 2 * NB);
    __syncthreads();
    pair_row_out(lds, D0, W10, D1, true, tileL(c, i1, j), tileL(c, i1, j + 1), p, pred, z + i1 * NB,
                 pred ? v + i1 * NB : nullptr, -1.0);
    if (two) {
      stage_tile_rm(lds, 0, tileL(c, i2, j), false);
      stage_tile_rm(lds, NB, tileL(c, i2, j + 1), false);
      p = vec_preload(z + j * NB, pred ? v + j * NB : nullptr, z + i2 * NB, pred ? v + i2 * NB : nullptr, 2 * NB);
      __syncthreads();
      pair_row_out(lds, D0, W10, D1, true, tileL(c, i2, j), tileL(c, i2, j + 1), p, pred, z + i2 * NB,
                   pred ? v + i2 * NB : nullptr, -1.0);
    }
    if (y != 0) return;
    // ---- E = sum_{k=j}^{j+1} L_J'k L_J'k^T for k_diag_pair(j+2), J' = (i1, i2), from the
    // tiles just stored (this workgroup's own global stores, ordered by __syncthreads)
    quad8_zero(acc);
    gemm4_kmajor<false>(acc, lds, 8, 0u, [=, &c](int p, const double*& a0, const double*& a1, const double*& b0,
                                                 const double*& b1) {
      a0 = tileL(c, i1, j + p);
      a1 = two ? tileL(c, i2, j + p) : g_zero_tile;
      b0 = a0;
      b1 = a1;
    });
    __syncthreads();
    double* E = c.P;
    stage4_q(acc, 0, 0, lds);
    if (two) stage4_q(acc, 1, 0, lds + NB * XLD);
    __syncthreads();
    emit_copy(lds, E, EMIT_STORE);
    if (!two) return;
    emit_copy(lds + NB * XLD, E + OI_TILE, EMIT_STORE);
    __syncthreads();
    stage4_q(acc, 1, 1, lds);
    __syncthreads();
    emit_copy(lds, E + 2 * OI_TILE, EMIT_STORE);
    return;
  }
  // ---- rows j, j+1 of W for the column pair jj1, jj2 (eval)
  const int yw = x - lead - nrp;
  if (c.mode != OI_MODE_EVAL || 2 * yw >= j) return;
  const int jj1 = 2 * yw, jj2 = jj1 + 1;
  unsigned skip = 0;
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const int tj = wc ? j + 1 : j;
      if ((wc == 1 && !has_next) || (tj == T - 1 && 16 * nb >= rT)) skip |= 1u << (4 * mb + nb);
    }
  auto wpair = [=, &c](int p, const double*& a0, const double*& a1, const double*& b0, const double*& b1) {
    const int k = jj1 + p;
    a0 = tileW(c, k, jj1);
    a1 = k >= jj2 ? tileW(c, k, jj2) : g_zero_tile;
    b0 = tileL(c, j, k);
    b1 = has_next ? tileL(c, j + 1, k) : g_zero_tile;
  };
  if (j >= T - 2)
    gemm4_kmajor<true>(acc, lds, 4 * (j - jj1), skip, wpair);
  else
    gemm4_kmajor<false>(acc, lds, 4 * (j - jj1), 0u, wpair);
  __syncthreads();
  // row jj2 leaves through its tiles: -acc
  stage4_q(acc, 1, 0, lds);
  if (has_next) stage4_q(acc, 1, 1, lds + NB * XLD);
  __syncthreads();
  emit_copy(lds, tileW(c, j, jj2), EMIT_NEG);
  if (has_next) emit_copy(lds + NB * XLD, tileW(c, j + 1, jj2), EMIT_NEG);
  __syncthreads();
  if ((w >> 2) == 0) {
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int r = 0; r < 4; ++r) lds[acc4_row(mb, r) * SLD2 + acc4_col(nb)] = -acc.c[mb][nb][r];
  }
  double* al = c.vec + T * NB;
  const int ncol = has_next ? 2 * NB : NB;
  VecPre p = vec_preload(z + j * NB, nullptr, al + jj1 * NB, nullptr, ncol);
  __syncthreads();
  pair_row_out(lds, D0, W10, D1, has_next, tileW(c, j, jj1), has_next ? tileW(c, j + 1, jj1) : nullptr, p, false,
               al + jj1 * NB, nullptr, 1.0);
  stage_tile_rm(lds, 0, tileW(c, j, jj2), false);
  if (has_next) stage_tile_rm(lds, NB, tileW(c, j + 1, jj2), false);
  p = vec_preload(z + j * NB, nullptr, al + jj2 * NB, nullptr, ncol);
  __syncthreads();
  pair_row_out(lds, D0, W10, D1, has_next, tileW(c, j, jj2), has_next ? tileW(c, j + 1, jj2) : nullptr, p, false,
               al + jj2 * NB, nullptr, 1.0);
}

// ------------------------------------------------------ k_lauum_grad
// Tile (i, j) of K^-1 = W^T W (K^-1_ij = sum_{k>=i} W_ki^T W_kj), one 256-thread
// workgroup per lower tile (40 KiB LDS -> 4 workgroups per CU), fused with
// sum over the tile of (K^-1 - alpha alpha^T) o {dK_0, dK_1, dK_2, 2K} and the
// trace (GPR:130-138); K and dK are regenerated from the coordinates.
// Strictly-lower entries count twice.
__global__ __launch_bounds__(256) void k_lauum_grad1(const OiCell* __restrict__ cells,
                                                    const int32_t* __restrict__ list, int gx,
                                                    int ncell) {
  __shared__ __attribute__((aligned(16))) double lds[GEMM1_LDS];
  int ci, tile;
  if (!xcd_cell_slot(gx, ncell, ci, tile)) return;
  const OiCell& c = cells[list[ci]];
  const int T = c.T;
  int i, j;
  if (!decode_tri(tile, T, i, j)) return;
  if (*c.status != OI_OK || c.mode != OI_MODE_EVAL) return;
  Quad acc;
  quad_zero(acc);
  // k rows of the last tile beyond n are padding (exact zeros of W off the
  // padded identity): the last pair's chunks stop at the cell's last row
  const int n = c.n, rT = n - NB * (T - 1);
  const int nch = 4 * (T - i - 1) + (rT + KC - 1) / KC;
  // 16x16 accumulator blocks this wave may drop: the upper triangle of a
  // diagonal tile (never read below) and padding rows / columns
  const int w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
  unsigned skip = 0;
  for (int mb = 0; mb < 2; ++mb)
    for (int nb = 0; nb < 2; ++nb) {
      const int m0 = 32 * wr + 16 * mb, n0 = 32 * wc + 16 * nb;
      const bool upper = i == j && m0 + 15 < n0;
      const bool pad = (i == T - 1 && m0 >= rT) || (j == T - 1 && n0 >= rT);
      if (upper || pad) skip |= 1u << (2 * mb + nb);
    }
  auto wpair = [=, &c](int p, const double*& a, const double*& b) {
    a = tileW(c, i + p, i);
    b = tileW(c, i + p, j);
  };
  // pair k = i: A = W_ii^T (A(m, k) = 0 for k < m), and B = W_ii too on the diagonal
  auto cm = [=](int ch) { return ch < 4 ? rows_below(ch, 32 * wr) | (i == j ? cols_below(ch, 32 * wc) : 0u) : 0u; };
  gemm1_kmajor<true>(acc, lds, nch, skip, wpair, cm);
  double* uQ = lds;            // [3][128]: rows 0..63, columns 64..127
  double* uq = lds + 3 * 128;  // [3][128]
  double* al = lds + 6 * 128;  // [128]
  double* dl = lds + 7 * 128;  // [128] site weights d
  double* red = lds + 8 * 128;
  const int t = threadIdx.x;
  __syncthreads();  // the GEMM's last LDS reads are done before the epilogue reuses lds
  if (t < 128) {
    const int a = t < 64 ? i * NB + t : j * NB + (t - 64);
    for (int d = 0; d < 3; ++d) {
      const double xv = a < n ? c.xyt[3 * a + d] : 0.0;
      uQ[d * 128 + t] = (SQRT3 * xv) / c.hyp[d];
      uq[d * 128 + t] = SQRT3 * (xv / c.hyp[d]);
    }
    al[t] = c.vec[T * NB + a];
    dl[t] = a < n ? c.dw[a] : 0.0;
  }
  __syncthreads();
  const double sf2 = c.hyp[3];
  double s[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  for (int mb = 0; mb < 2; ++mb)
    for (int nb = 0; nb < 2; ++nb)
      for (int r = 0; r < 4; ++r) {
        const int m = acc1_row(mb, r), nn = acc1_col(nb);
        const int a = i * NB + m, b = j * NB + nn;
        if (a >= n || b >= n || (i == j && m < nn)) continue;
#if OI_LAUUM_EPI == 0  // timing experiments only (tools): no epilogue
        s[3] += acc.c[mb][nb][r];
        continue;
#endif
        const double wgt = (a == b) ? 1.0 : 2.0;
        const double w0 = acc.c[mb][nb][r] - al[m] * al[64 + nn];  // (M^-1 - aa^T)_st
        const double w = (dl[m] * dl[64 + nn]) * w0;                // (D M^-1 D - uu^T)_st
        const double d0 = uQ[0 * 128 + m] - uQ[0 * 128 + 64 + nn];
        const double d1 = uQ[1 * 128 + m] - uQ[1 * 128 + 64 + nn];
        const double d2 = uQ[2 * 128 + m] - uQ[2 * 128 + 64 + nn];
        const double Q = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
#if OI_LAUUM_EPI == 2  // timing experiments only (tools): no exp
        const double e = 1.0 - Q;
#else
        const double e = exp(-Q);
#endif
        const double K = sf2 * ((1.0 + Q) * e);
        const double q0 = uq[0 * 128 + m] - uq[0 * 128 + 64 + nn];
        const double q1 = uq[1 * 128 + m] - uq[1 * 128 + 64 + nn];
        const double q2 = uq[2 * 128 + m] - uq[2 * 128 + 64 + nn];
        s[0] += wgt * (w * (sf2 * ((q0 * q0) * e)));
        s[1] += wgt * (w * (sf2 * ((q1 * q1) * e)));
        s[2] += wgt * (w * (sf2 * ((q2 * q2) * e)));
        s[3] += wgt * (w * (2.0 * K));
        if (a == b) s[4] += w0;
      }
  block_sum<5, 4>(s, red);
  if (t == 0) {
    double* pp = c.part + OI_PART_GRAD(0) + 5 * (size_t)tile;
    for (int q = 0; q < 5; ++q) pp[q] = s[q];
  }
}

// ------------------------------------------------------ k_lauum_grad4 (OI_LAUUM=4)
// The same sums on 2 x 2 blocks of output tiles: workgroup (I2, J2), I2 >= J2,
// covers tile rows i0 = 2 I2, i1 = i0 + 1 and columns j0 = 2 J2, j1 = j0 + 1
// (512 threads, the 128 x 128 gemm4 core: every streamed W tile feeds two
// outputs).  K^-1_{i,j} = sum_{k >= max(i, j)} W_ki^T W_kj: the block streams
// k = i0 .. T-1 with W_{i0, i1} (k = i0) and W_{j0, j1} (k = j0 = i0 on a
// diagonal block) the structural zero tile; k rows of the last tile beyond n
// are skipped.  A wave's 32 x 64 accumulator lies in one output tile, so the
// epilogue reduces per tile (two waves each, fixed order) and writes the
// tile's partials at its usual slot.  Tiles beyond T, the block (i0, j1) of a
// diagonal block and the upper triangles of diagonal tiles are masked out.
__global__ __launch_bounds__(GEMM_THREADS) __attribute__((amdgpu_waves_per_eu(4, 4)))
void k_lauum_grad4(const OiCell* __restrict__ cells,
                                                             const int32_t* __restrict__ list,
                                                             int gx, int ncell) {
  __shared__ __attribute__((aligned(16))) double lds[GEMM4_LDS];
  int ci, blk;
  if (!xcd_cell_slot(gx, ncell, ci, blk)) return;
  const OiCell& c = cells[list[ci]];
  const int T = c.T, T2 = (T + 1) >> 1;
  int I2, J2;
  if (!decode_tri(blk, T2, I2, J2)) return;
  if (*c.status != OI_OK || c.mode != OI_MODE_EVAL) return;
  const int i0 = 2 * I2, i1 = i0 + 1, j0 = 2 * J2, j1 = j0 + 1;
  const int n = c.n, rT = n - NB * (T - 1);
  const int nch = 4 * (T - i0 - 1) + (rT + KC - 1) / KC;
  const int w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
  // this wave's output tile and its 16x16 blocks that are never used
  const int ti = wr >= 2 ? i1 : i0, tj = wc ? j1 : j0;
  const bool tile_ok = ti < T && tj < T && ti >= tj;
  unsigned skip = 0;
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const int m0 = 32 * (wr & 1) + 16 * mb, n0 = 16 * nb;
      const bool upper = ti == tj && m0 + 15 < n0;
      const bool pad = (ti == T - 1 && m0 >= rT) || (tj == T - 1 && n0 >= rT);
      if (!tile_ok || upper || pad) skip |= 1u << (4 * mb + nb);
    }
  const bool masked = I2 == J2 || i1 >= T - 1;  // diagonal block or the last block row
  auto wpair = [=, &c](int p, const double*& a0, const double*& a1, const double*& b0, const double*& b1) {
    const int k = i0 + p;
    a0 = tileW(c, k, i0);
    a1 = (i1 < T && k >= i1) ? tileW(c, k, i1) : g_zero_tile;
    b0 = tileW(c, k, j0);
    b1 = (j1 < T && k >= j1) ? tileW(c, k, j1) : g_zero_tile;
  };
  Quad8 acc;
  quad8_zero(acc);
  if (masked)
    gemm4_kmajor<true>(acc, lds, nch, skip, wpair);
  else
    gemm4_kmajor<false>(acc, lds, nch, 0u, wpair);
  // epilogue data: rows of tiles i0, i1 (entries 0..127), columns of j0, j1 (128..255)
  double* uQ = lds;            // [3][256]
  double* uq = lds + 3 * 256;  // [3][256]
  double* al = lds + 6 * 256;  // [256]
  double* dl = lds + 7 * 256;  // [256]
  double* red = lds + 8 * 256; // [8 waves][5]
  const int t = threadIdx.x;
  __syncthreads();
  if (t < 256) {
    const int tt = t & 127;
    const int a = t < 128 ? (tt < 64 ? i0 : i1) * NB + (tt & 63) : (tt < 64 ? j0 : j1) * NB + (tt & 63);
    const bool in = a < n && (t < 128 ? (tt < 64 || i1 < T) : (tt < 64 || j1 < T));
    for (int d = 0; d < 3; ++d) {
      const double xv = in ? c.xyt[3 * a + d] : 0.0;
      uQ[d * 256 + t] = (SQRT3 * xv) / c.hyp[d];
      uq[d * 256 + t] = SQRT3 * (xv / c.hyp[d]);
    }
    al[t] = in ? c.vec[T * NB + a] : 0.0;
    dl[t] = in ? c.dw[a] : 0.0;
  }
  __syncthreads();
  const double sf2 = c.hyp[3];
  double s[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  if (tile_ok) {
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int mr = acc4_row(mb, r), nc = acc4_col(nb);  // 0..127 within the block
          const int m = mr & 63, nn = nc & 63;
          const int a = ti * NB + m, b = tj * NB + nn;
          if (a >= n || b >= n || (ti == tj && m < nn)) continue;
          const double wgt = (a == b) ? 1.0 : 2.0;
          const double w0 = acc.c[mb][nb][r] - al[mr] * al[128 + nc];  // (M^-1 - aa^T)_st
          const double ww = (dl[mr] * dl[128 + nc]) * w0;               // (D M^-1 D - uu^T)_st
          const double d0 = uQ[0 * 256 + mr] - uQ[0 * 256 + 128 + nc];
          const double d1 = uQ[1 * 256 + mr] - uQ[1 * 256 + 128 + nc];
          const double d2 = uQ[2 * 256 + mr] - uQ[2 * 256 + 128 + nc];
          const double Q = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
          const double e = exp(-Q);
          const double K = sf2 * ((1.0 + Q) * e);
          const double q0 = uq[0 * 256 + mr] - uq[0 * 256 + 128 + nc];
          const double q1 = uq[1 * 256 + mr] - uq[1 * 256 + 128 + nc];
          const double q2 = uq[2 * 256 + mr] - uq[2 * 256 + 128 + nc];
          s[0] += wgt * (ww * (sf2 * ((q0 * q0) * e)));
          s[1] += wgt * (ww * (sf2 * ((q1 * q1) * e)));
          s[2] += wgt * (ww * (sf2 * ((q2 * q2) * e)));
          s[3] += wgt * (ww * (2.0 * K));
          if (a == b) s[4] += w0;
        }
  }
#pragma unroll
  for (int q = 0; q < 5; ++q)
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s[q] += __shfl_down(s[q], o, 64);
  if ((t & 63) == 0)
#pragma unroll
    for (int q = 0; q < 5; ++q) red[w * 5 + q] = s[q];
  __syncthreads();
  if (t < 4) {  // tile slot t = (row half, column half); its waves are (2 rh) * 2 + ch and (2 rh + 1) * 2 + ch
    const int rh = t >> 1, ch = t & 1;
    const int ti2 = rh ? i1 : i0, tj2 = ch ? j1 : j0;
    if (ti2 < T && tj2 < T && ti2 >= tj2) {
      const int wa = (2 * rh) * 2 + ch, wb = (2 * rh + 1) * 2 + ch;
      double* pp = c.part + OI_PART_GRAD(0) + 5 * ((size_t)ti2 * (ti2 + 1) / 2 + tj2);
      for (int q = 0; q < 5; ++q) pp[q] = red[wa * 5 + q] + red[wb * 5 + q];
    }
  }
}

// ---------------------------------------------------------- k_finalize
// nlZ = r.alpha/2 + sum log diag L + n log(2 pi)/2 (GPR:128); dnlZ (GPR:131-138)
__device__ __forceinline__ void finalize_cell(const OiCell& c) {
  __shared__ double red[4 * 7];
  const int t = threadIdx.x, T = c.T, ntile = T * (T + 1) / 2;
  // the round's status rides home in the result row (one D2H copy per round)
  if (t == 0) c.out[OI_OUT_STATUS] = (double)*c.status;
  if (c.mode == OI_MODE_PREDICT) {
    // GPR:178-182 from the forward substitution run inside the factorisation:
    // z = L^-1 r, v = L^-1 k*: k*^T K^-1 r = v.z, k*^T K^-1 k* = v.v, r^T K^-1 r = z.z
    if (*c.status != OI_OK) {
      if (t < 3) c.out[t] = NAN;
      return;
    }
    double p[4] = {0.0, 0.0, 0.0, 0.0};
    for (int k = t; k < T; k += 256) {
      const double* pp = c.part + OI_PART_PRED(ntile, T) + 3 * k;
      p[0] += pp[0];
      p[1] += pp[1];
      p[2] += pp[2];
      p[3] += c.part[OI_PART_LOGDET(ntile, T) + k];
    }
    block_sum<4, 4>(p, red);
    if (t == 0) {
      const double sf2 = c.hyp[3], sn2 = c.hyp[4], nm = (double)(c.n_obs - c.n);
      c.out[0] = c.mean + p[1];
      c.out[1] = sqrt(sf2 - p[2]);
      c.out[2] = ((-(p[0] + c.ssw / sn2)) / 2 - (p[3] + (nm / 2) * log(sn2))) - (c.n_obs * LOG2PI) / 2;
    }
    return;
  }
  const int nslot = ntile;
  if (*c.status != OI_OK) {
    if (t < 7) c.out[t] = INFINITY;
    return;
  }
  double v[7] = {0, 0, 0, 0, 0, 0, 0};
  for (int x = t; x < nslot; x += 256)
    for (int q = 0; q < 5; ++q) v[q] += c.part[OI_PART_GRAD(ntile) + 5 * x + q];
  for (int k = t; k < T; k += 256) {
    v[5] += c.part[OI_PART_PRED(ntile, T) + 3 * k];  // r^T alpha = z^T z, z = L^-1 r
    v[6] += c.part[OI_PART_LOGDET(ntile, T) + k];
  }
  block_sum<7, 4>(v, red);
  if (t == 0) {
    // site form (oi_device.h): r^T alpha = SSW/sn2 + v^T M^-1 v,
    // sum log diag L = log det M / 2 + (n - m)/2 log sn2, tr Q += (n - m)/sn2 - SSW/sn2^2
    const double quad = v[5], logdet = v[6], sn2 = c.hyp[4];
    const double nm = (double)(c.n_obs - c.n);
    c.out[0] = ((quad + c.ssw / sn2) / 2 + (logdet + (nm / 2) * log(sn2))) + (c.n_obs * LOG2PI) / 2;
    c.out[1] = v[0] / 2;
    c.out[2] = v[1] / 2;
    c.out[3] = v[2] / 2;
    c.out[4] = v[3] / 2;
    c.out[5] = sn2 * ((v[4] + nm / sn2) - c.ssw / (sn2 * sn2));
    c.out[6] = 0.0;
  }
}

// The result rows live in fine-grained pinned host memory (no D2H copy per
// round).  With `flag` set, the workgroup that finishes last stores `seq` to
// the group's host flag after every row has reached host memory, and the host
// spins on that word instead of a stream synchronise (config 1's lone cell
// waits for ~90 of these round trips: 7 us spinning vs 12 us synchronising,
// + 3 us for the copy, tools/sync_probe.hip).
__global__ __launch_bounds__(256) void k_finalize(const OiCell* __restrict__ cells,
                                                  const int32_t* __restrict__ list, unsigned* done,
                                                  unsigned long long* flag, unsigned long long seq,
                                                  int ncell) {
  finalize_cell(cells[list[blockIdx.x]]);
  if (flag == nullptr) return;
  __threadfence_system();  // this thread's result stores are in host memory
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(done, 1u) == (unsigned)(ncell - 1)) {
    *done = 0u;  // for the group's next round (stream order)
    __threadfence_system();
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ------------------------------------------------------------- k_dedup
// Distinct observation sites of each cell (oi_device.h, "Duplicate sites"),
// one workgroup per cell, once per submitted batch.  Site s = the s-th first
// occurrence in observation order; prev[a] = the latest earlier observation
// with bitwise-equal (x, y, t), nxt the reverse link, so every site's
// observations are walked in observation order: fixed-order sums, results
// independent of the batch.  Coordinates are staged in LDS for n <= 4096
// (36 B per observation with the links), read from global memory above.
#define DEDUP_LDS_N 4096
#define DEDUP_MAX_N 13000  // 8 B x 13000 <= 36 B x 4096
__global__ __launch_bounds__(256) void k_dedup(const double* __restrict__ xyt,
                                               const double* __restrict__ r,
                                               const int64_t* __restrict__ offs, int nodup,
                                               double* __restrict__ sites, double* __restrict__ v,
                                               double* __restrict__ dw, int32_t* __restrict__ mcount,
                                               double* __restrict__ ssw) {
  extern __shared__ double sh[];
  __shared__ int scan[256];
  __shared__ double red[4];
  const int c = blockIdx.x, t = threadIdx.x;
  const int64_t a0 = offs[c];
  const int n = (int)(offs[c + 1] - a0);
  const double* X = xyt + 3 * a0;
  const double* R = r + a0;
  const bool single = nodup || n > DEDUP_MAX_N;  // every observation its own site
  const bool in_lds = !single && n <= DEDUP_LDS_N;
  double* cx = sh;
  double* cy = sh + n;
  double* ct = sh + 2 * n;
  int* prev = (int*)(sh + (in_lds ? 3 * n : 0));
  int* nxt = prev + n;
  if (in_lds)
    for (int b = t; b < n; b += 256) {
      cx[b] = X[3 * b];
      cy[b] = X[3 * b + 1];
      ct[b] = X[3 * b + 2];
    }
  if (!single)
    for (int a = t; a < n; a += 256) nxt[a] = -1;
  __syncthreads();
  if (!single) {
    for (int a = t; a < n; a += 256) {
      int p = -1;
      if (in_lds) {
        const double xa = cx[a], ya = cy[a], ta = ct[a];
        for (int b = a - 1; b >= 0; --b)
          if (cx[b] == xa && cy[b] == ya && ct[b] == ta) {
            p = b;
            break;
          }
      } else {
        const double xa = X[3 * a], ya = X[3 * a + 1], ta = X[3 * a + 2];
        for (int b = a - 1; b >= 0; --b)
          if (X[3 * b] == xa && X[3 * b + 1] == ya && X[3 * b + 2] == ta) {
            p = b;
            break;
          }
      }
      prev[a] = p;
    }
    __syncthreads();
    for (int a = t; a < n; a += 256)
      if (prev[a] >= 0) nxt[prev[a]] = a;
  }
  // exclusive scan of first-occurrence flags over contiguous segments
  const int seg = (n + 255) / 256, s0 = min(n, t * seg), s1 = min(n, s0 + seg);
  int cnt = 0;
  for (int a = s0; a < s1; ++a) cnt += (single || prev[a] < 0) ? 1 : 0;
  scan[t] = cnt;
  __syncthreads();
  if (t == 0) {
    int acc = 0;
    for (int q = 0; q < 256; ++q) {
      const int x = scan[q];
      scan[q] = acc;
      acc += x;
    }
    mcount[c] = acc;
  }
  __syncthreads();
  int s = scan[t];
  double part = 0.0;
  for (int a = s0; a < s1; ++a) {
    if (!(single || prev[a] < 0)) continue;
    double rs = 0.0, cntd = 0.0;
    if (single) {
      rs = R[a];
      cntd = 1.0;
    } else {
      for (int b = a; b >= 0; b = nxt[b]) {
        rs += R[b];
        cntd += 1.0;
      }
      const double rbar = rs / cntd;
      for (int b = a; b >= 0; b = nxt[b]) {
        const double e = R[b] - rbar;
        part += e * e;
      }
    }
    const double d = sqrt(cntd);
    const int64_t o = a0 + s;
    sites[3 * o] = X[3 * a];
    sites[3 * o + 1] = X[3 * a + 1];
    sites[3 * o + 2] = X[3 * a + 2];
    v[o] = rs / d;
    dw[o] = d;
    ++s;
  }
  for (int o = 32; o >= 1; o >>= 1) part += __shfl_down(part, o, 64);
  if ((t & 63) == 0) red[t >> 6] = part;
  __syncthreads();
  if (t == 0) ssw[c] = ((red[0] + red[1]) + red[2]) + red[3];
}

extern "C" int oi_launch_dedup(const double* xyt, const double* r, const int64_t* offs, int ncell,
                               int maxn, int nodup, double* sites, double* v, double* dw,
                               int32_t* mcount, double* ssw, void* stream) {
  if (ncell <= 0) return 0;
  // LDS: coordinates + links (36 B per observation) for n <= DEDUP_LDS_N,
  // links only (8 B) above; cells beyond DEDUP_MAX_N run without deduplication
  size_t lds = 0;
  if (!nodup && maxn > 0)
    lds = maxn <= DEDUP_LDS_N ? (size_t)36 * maxn
                              : (size_t)36 * DEDUP_LDS_N;  // >= 8 * DEDUP_MAX_N
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_dedup, hipFuncAttributeMaxDynamicSharedMemorySize,
                              36 * DEDUP_LDS_N);
    attr = true;
  }
  hipLaunchKernelGGL(k_dedup, dim3(ncell), dim3(256), lds, (hipStream_t)stream, xyt, r, offs, nodup,
                     sites, v, dw, mcount, ssw);
  return hipGetLastError() == hipSuccess ? 0 : -1;
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
static inline unsigned grid1(int gx, int ncell) { return (unsigned)gx * (unsigned)((ncell + 7) & ~7); }

extern "C" int oi_launch_build(const OiCell* cells, const int32_t* list, int ncell, int maxT,
                               void* stream) {
  if (ncell <= 0 || maxT <= 0) return 0;
  const int gx = maxT * (maxT + 1) / 2;
  hipLaunchKernelGGL(k_build, dim3(grid1(gx, ncell)), dim3(256), 0, S(stream), cells, list, gx,
                     ncell);
  return ret();
}

extern "C" int oi_launch_diag_factor(const OiCell* cells, const int32_t* list, int ncell, int j,
                                     void* stream) {
  if (ncell <= 0) return 0;
  const char* ev = getenv("OI_DIAG");  // read per launch (tests switch it): ~0.1 us
  const int variant = ev ? atoi(ev) : 4;
  if (variant == 32)  // the round-1 32-blocked kernel (A/B)
    hipLaunchKernelGGL(k_diag_factor, dim3(ncell), dim3(64), 0, S(stream), cells, list, j);
  else if (variant == 16)  // round 2's single-wave 16-blocked kernel (A/B)
    hipLaunchKernelGGL(k_diag_factor16, dim3(ncell), dim3(64), 0, S(stream), cells, list, j);
  else
    hipLaunchKernelGGL(k_diag_factor4w, dim3(ncell), dim3(256), 0, S(stream), cells, list, j);
  return ret();
}

extern "C" int oi_launch_scale(const OiCell* cells, const int32_t* list, int ncell, int j,
                               int kbeg, void* stream) {
  if (ncell <= 0 || j - kbeg <= 0) return 0;
  const int gx = (j - kbeg + SCALE_KPW - 1) / SCALE_KPW;
  hipLaunchKernelGGL(k_scale, dim3(grid1(gx, ncell)), dim3(256), 0, S(stream), cells, list, j,
                     kbeg, gx, ncell);
  return ret();
}

extern "C" int oi_launch_chol_panel(const OiCell* cells, const int32_t* list, int ncell, int maxT,
                                    int j, int kbeg, int with_trtri, int pform, void* stream) {
  const int gx = (maxT - 1 - j) + (with_trtri ? j : 0);
  if (ncell <= 0 || gx <= 0) return 0;
  if (pform)
    hipLaunchKernelGGL(k_chol_panel<false>, dim3(grid1(gx, ncell)), dim3(256), 0, S(stream), cells, list, j,
                       kbeg, gx, ncell);
  else
    hipLaunchKernelGGL(k_chol_panel<true>, dim3(grid1(gx, ncell)), dim3(256), 0, S(stream), cells, list, j,
                       kbeg, gx, ncell);
  return ret();
}

extern "C" int oi_launch_panel_even(const OiCell* cells, const int32_t* list, int ncell, int maxT,
                                    int j, int with_trtri, int pform, void* stream) {
  const int gx = (maxT - 1 - j) + (with_trtri ? j : 0);
  if (ncell <= 0 || gx <= 0) return 0;
  if (pform)
    hipLaunchKernelGGL(k_panel_even<false>, dim3(grid1(gx, ncell)), dim3(GEMM_THREADS), 0, S(stream), cells,
                       list, j, gx, ncell);
  else
    hipLaunchKernelGGL(k_panel_even<true>, dim3(grid1(gx, ncell)), dim3(GEMM_THREADS), 0, S(stream), cells,
                       list, j, gx, ncell);
  return ret();
}

extern "C" int oi_launch_panel4(const OiCell* cells, const int32_t* list, int ncell, int maxT, int j,
                                int with_trtri, void* stream) {
  const int gx = nslot4_factor(maxT, j) + (with_trtri ? j / 2 : 0);
  if (ncell <= 0 || gx <= 0) return 0;
  hipLaunchKernelGGL(k_panel4, dim3(grid1(gx, ncell)), dim3(GEMM_THREADS), 0, S(stream), cells, list, j, gx,
                     ncell);
  return ret();
}

extern "C" int oi_launch_diag_pair(const OiCell* cells, const int32_t* list, int ncell, int j, void* stream) {
  if (ncell <= 0) return 0;
  hipLaunchKernelGGL(k_diag_pair, dim3(ncell), dim3(256), 0, S(stream), cells, list, j);
  return ret();
}

extern "C" int oi_launch_panel_pair(const OiCell* cells, const int32_t* list, int ncell, int maxT, int j,
                                    int with_trtri, void* stream) {
  const int gx = (j >= 2 ? 1 : 0) + npair_rows(maxT, j) + (with_trtri ? j / 2 : 0);
  if (ncell <= 0 || gx <= 0) return 0;
  hipLaunchKernelGGL(k_panel_pair, dim3(grid1(gx, ncell)), dim3(GEMM_THREADS), 0, S(stream), cells, list, j, gx,
                     ncell);
  return ret();
}

extern "C" int oi_launch_lauum_grad(const OiCell* cells, const int32_t* list, int ncell, int maxT,
                                    void* stream) {
  if (ncell <= 0 || maxT <= 0) return 0;
  const char* ev = getenv("OI_LAUUM");  // read per launch (tests switch it)
  const int variant = ev ? atoi(ev) : 1;
  if (variant != 4) {  // one 64x64 tile per 256-thread workgroup (default: measured faster)
    const int gx = maxT * (maxT + 1) / 2;
    hipLaunchKernelGGL(k_lauum_grad1, dim3(grid1(gx, ncell)), dim3(256), 0, S(stream), cells, list, gx,
                       ncell);
  } else {
    const int T2 = (maxT + 1) / 2, gx = T2 * (T2 + 1) / 2;
    hipLaunchKernelGGL(k_lauum_grad4, dim3(grid1(gx, ncell)), dim3(GEMM_THREADS), 0, S(stream), cells,
                       list, gx, ncell);
  }
  return ret();
}

extern "C" int oi_launch_finalize(const OiCell* cells, const int32_t* list, int ncell, unsigned* done,
                                  unsigned long long* flag, unsigned long long seq, void* stream) {
  if (ncell <= 0) return 0;
  hipLaunchKernelGGL(k_finalize, dim3(ncell), dim3(256), 0, S(stream), cells, list, done, flag, seq, ncell);
  return ret();
}

extern "C" int oi_launch_residual(const double* y, const double* mX, double mean, double* r,
                                  int64_t N, void* stream) {
  if (N <= 0) return 0;
  hipLaunchKernelGGL(k_residual, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, S(stream), y, mX,
                     mean, r, N);
  return ret();
}
