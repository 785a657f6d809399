// Hand-written batched dense fp64 linear algebra for the Nystrom variant
// (GP_example.ipynb, "NB1": Nystroem's np.linalg.eigh(Kmm), SMLII's
// np.linalg.cholesky and the n x M matrix products) on gfx950 -- no LAPACK,
// rocSOLVER or rocBLAS.  Interface: oi_linalg.h.
//
//   k_gemm        C = alpha op(A) op(B) + beta C, 64 x 64 output tile per
//                 256-thread workgroup on v_mfma_f64_16x16x4f64 (the oi_gemm.h
//                 quadrant layout), operands staged global -> registers -> LDS
//                 in 16-deep chunks, results staged through LDS for coalesced
//                 column stores; one launch covers a batch of differently
//                 sized products (grid.y = product)
//   k_gemv_t/_n   y = alpha op(A) x + beta y
//   k_potrf_tile  Cholesky + inverse of one 64 x 64 diagonal block per matrix
//                 (the blocked right-looking factorisation: potrf_tile ->
//                 panel product with the block inverse -> lower-tile update)
//   k_sy_symv / k_sy_w
//                 Householder tridiagonalisation (LAPACK dsytrd / dlatrd,
//                 lower), two launches per column over the batch: the
//                 column's reflector and the symmetric product over the
//                 trailing lower triangle on OI_SY_S workgroups per matrix,
//                 then the w vector and the next column's update by rows;
//                 per 32-column panel the rank-64 trailing update on k_gemm;
//                 V (unit lower, clean copy) and T (dlarft, forward
//                 columnwise) kept per panel
//   k_stebz       eigenvalues of the tridiagonal by bisection on Sturm counts
//                 (dstebz), one thread per eigenvalue
//   k_stein       eigenvectors by inverse iteration with partial pivoting
//                 (dlagtf / dlagts; dstein), one thread per eigenvalue,
//                 pseudo-random start per eigenvalue; k_stein_out transposes
//                 them into Z
//   k_orth_panel  Cholesky QR twice inside a 32-vector panel (Gram-Schmidt
//                 in column order; G = Z'Z on MFMA); where a column
//                 collapses (repeated eigenvalues) classical Gram-Schmidt
//                 twice column by column with fresh start vectors
//                 (k_mgs_panel); between panels block Gram-Schmidt twice
//                 (BCGS2) on k_gemm
//   back-transform U = Q Z, one block reflector I - V T V' per panel (k_gemm)
// The algorithm is modelled step for step in tools/eigh_model.py.
//
// Reductions run in a fixed order, so a matrix's results do not depend on the
// batch it is in.
#include "oi_linalg.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>

#include "oi_gemm.h"

namespace oila {

#define LC(expr)                                                                                \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess) throw LinalgErr{std::string(#expr) + ": " + hipGetErrorString(e_)}; \
  } while (0)

// Global-address-space views of the descriptors' pointers: plain accesses
// through generic pointers compile to flat_* instructions, which count
// against lgkmcnt too, so every LDS wait would also wait for the loads in
// flight (the prefetch of the next chunk, the symv's batch) -- G() makes them
// global_* instructions, counted by vmcnt only.
typedef __attribute__((address_space(1))) double gdouble;
__device__ __forceinline__ gdouble* G(double* p) { return (gdouble*)p; }
__device__ __forceinline__ const gdouble* G(const double* p) { return (const gdouble*)p; }

// Masked loads without branches: a raw buffer load whose offset is pushed
// past the descriptor's range returns 0 (hardware bounds check) -- a plain
// load under a condition becomes an exec-masked branch per load with a
// vmcnt(0) wait in it, which serialises the batch.  Descriptors are built
// from wave-uniform base pointers; offsets are in bytes from that base and
// must stay below 2 GiB (one matrix / panel per descriptor).
typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc rsrc(const double* p) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, 0x7FFFFFF0, 0x00020000);
}
__device__ __forceinline__ double bload(Rsrc r, bool ok, size_t idx) {
  const unsigned off = ok ? (unsigned)(idx * 8) : 0xFFFFFFF0u;
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}

// ------------------------------------------------------------------ k_gemm
#define GT 64
#define GKC 16
#define GLD 80  // LDS row stride of a staged 16 x 64 chunk (rows k, k+1 in opposite bank halves)
// Operands are staged as element pairs along their contiguous dimension (one
// 16-byte buffer load per pair on interior chunks, two masked 8-byte loads at
// the matrix edges).  A k-contiguous operand (A with TA, B without TB) is
// stored transposed: a half-wave holds 8 k-pairs of 4 rows, and plain
// placement would put its even rows on two banks (8-way conflicts), so element
// (k, m) sits at column m ^ 4 (k >> 1) -- a permutation inside m's aligned
// 32-block; the compute reads apply the same XOR and stay conflict-free
// (k >> 1 is uniform across a half-wave's lanes).

// elements idx, idx + 1: one 16-byte load when `full` (uniform), else two
// masked 8-byte loads
__device__ __forceinline__ dv2 pair_load(Rsrc r, bool full, bool ok0, bool ok1, size_t idx) {
  if (full) return __builtin_bit_cast(dv2, __builtin_amdgcn_raw_buffer_load_b128(r, (unsigned)(idx * 8), 0, 0));
  return dv2{bload(r, ok0, idx), bload(r, ok1, idx + 1)};
}

template <bool TA, bool TB>
__global__ __launch_bounds__(256) void k_gemm(const Gemm* __restrict__ gs) {
  __shared__ __attribute__((aligned(16))) double lds[2 * 2 * GKC * GLD];
  const Gemm g = gs[blockIdx.y];
  const int tm = (g.m + GT - 1) / GT, tn = (g.n + GT - 1) / GT;
  if ((int)blockIdx.x >= tm * tn) return;
  const int it = blockIdx.x % tm, jt = blockIdx.x / tm;
  if (g.tri == 1 && it < jt) return;
  int kmax = g.k;
  if (g.tri == 2) kmax = min(kmax, GT * (jt + 1));
  const int m0 = GT * it, n0 = GT * jt;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;
  const int fr = lane & 15, fk = lane >> 4;
  Quad acc;
  quad_zero(acc);
  const int nch = (kmax + GKC - 1) / GKC;
  const bool edge_mn = m0 + GT > g.m || n0 + GT > g.n;
  // pair p = t + 256 q of a 64 x 16 chunk: k-contiguous k = 2 (p & 7), row
  // p >> 3; otherwise k = p >> 5, rows 2 (p & 31), +1
  dv2 pa[2], pb[2];
  const Rsrc rA = rsrc(g.A), rB = rsrc(g.B);
  auto load = [&](int ch) __attribute__((always_inline)) {
    const int k0 = ch * GKC;
    const bool full = !edge_mn && k0 + GKC <= kmax;  // uniform
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int pp = t + 256 * q;
      if (TA) {
        const int gk = k0 + 2 * (pp & 7), gm = m0 + (pp >> 3);
        pa[q] = pair_load(rA, full, gm < g.m && gk < kmax, gm < g.m && gk + 1 < kmax, gk + (size_t)g.lda * gm);
      } else {
        const int gm = m0 + 2 * (pp & 31), gk = k0 + (pp >> 5);
        pa[q] = pair_load(rA, full, gm < g.m && gk < kmax, gm + 1 < g.m && gk < kmax, gm + (size_t)g.lda * gk);
      }
      if (TB) {
        const int gn = n0 + 2 * (pp & 31), gk = k0 + (pp >> 5);
        pb[q] = pair_load(rB, full, gn < g.n && gk < kmax, gn + 1 < g.n && gk < kmax, gn + (size_t)g.ldb * gk);
      } else {
        const int gk = k0 + 2 * (pp & 7), gn = n0 + (pp >> 3);
        pb[q] = pair_load(rB, full, gn < g.n && gk < kmax, gn < g.n && gk + 1 < kmax, gk + (size_t)g.ldb * gn);
      }
    }
  };
  auto store = [&](int buf) __attribute__((always_inline)) {
    double* As = lds + buf * 2 * GKC * GLD;
    double* Bs = As + GKC * GLD;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int pp = t + 256 * q;
      if (TA) {
        const int k = 2 * (pp & 7), m = (pp >> 3) ^ ((k >> 1) << 2);
        As[k * GLD + m] = pa[q].x;
        As[(k + 1) * GLD + m] = pa[q].y;
      } else {
        *(dv2*)(As + (pp >> 5) * GLD + 2 * (pp & 31)) = pa[q];
      }
      if (TB) {
        *(dv2*)(Bs + (pp >> 5) * GLD + 2 * (pp & 31)) = pb[q];
      } else {
        const int k = 2 * (pp & 7), n = (pp >> 3) ^ ((k >> 1) << 2);
        Bs[k * GLD + n] = pb[q].x;
        Bs[(k + 1) * GLD + n] = pb[q].y;
      }
    }
  };
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const double* As = lds + buf * 2 * GKC * GLD;
    const double* Bs = As + GKC * GLD;
#pragma unroll
    for (int kk = 0; kk < GKC / 4; ++kk) {
      const int k = kk * 4 + fk, sa = TA ? (k >> 1) << 2 : 0, sb = TB ? 0 : (k >> 1) << 2;
      const double a0 = As[k * GLD + ((32 * wr + fr) ^ sa)], a1 = As[k * GLD + ((32 * wr + 16 + fr) ^ sa)];
      const double b0 = Bs[k * GLD + ((32 * wc + fr) ^ sb)], b1 = Bs[k * GLD + ((32 * wc + 16 + fr) ^ sb)];
      acc.c[0][0] = MFMA64(a0, b0, acc.c[0][0]);
      acc.c[0][1] = MFMA64(a0, b1, acc.c[0][1]);
      acc.c[1][0] = MFMA64(a1, b0, acc.c[1][0]);
      acc.c[1][1] = MFMA64(a1, b1, acc.c[1][1]);
    }
  };
  if (nch > 0) {
    load(0);
    store(0);
    __syncthreads();
    for (int ch = 0; ch < nch; ++ch) {
      if (ch + 1 < nch) load(ch + 1);
      compute(ch & 1);
      if (ch + 1 < nch) store((ch + 1) & 1);
      __syncthreads();
    }
  }
  // stage the tile column-major in LDS (X[n * 65 + m]) for coalesced stores
  double* X = lds;
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) X[acc1_col(nb) * 65 + acc1_row(mb, r)] = acc.c[mb][nb][r];
  __syncthreads();
  for (int e = t; e < GT * GT; e += 256) {
    const int m = e & 63, n = e >> 6, gm = m0 + m, gn = n0 + n;
    if (gm >= g.m || gn >= g.n) continue;
    gdouble* c = G(g.C) + gm + (size_t)g.ldc * gn;
    const double v = g.alpha * X[n * 65 + m];
    *c = g.beta == 0.0 ? v : v + g.beta * *c;
  }
}

// ------------------------------------------------------------------ k_gemm128
// The same product on 128 x 128 output tiles, 512 threads (wave w: rows
// 32 (w >> 1) .., columns 64 (w & 1) .. as 2 x 4 MFMA blocks, the gemm4 core
// of oi_gemm.h): a streamed 16-deep chunk feeds twice the outputs of k_gemm's,
// half the operand traffic per flop.  Every output is accumulated by the same
// MFMA sequence over k as in k_gemm (chunks of 16, MFMA k-steps of 4 in
// order), so the two kernels are bitwise equal and the wrapper may pick either
// by shape.  tri == 0 only.  LDS: two (A, B) buffers of 16 x 128 chunks, row
// stride 144 (rows k, k+1 in opposite bank halves); the epilogue stages the
// tile 64 columns at a time.
#define GT2 128
#define GLD2 144
template <bool TA, bool TB>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_gemm128(const Gemm* __restrict__ gs) {
  __shared__ __attribute__((aligned(16))) double lds[2 * 2 * GKC * GLD2];
  const Gemm g = gs[blockIdx.y];
  const int tm = (g.m + GT2 - 1) / GT2, tn = (g.n + GT2 - 1) / GT2;
  if ((int)blockIdx.x >= tm * tn) return;
  const int it = blockIdx.x % tm, jt = blockIdx.x / tm;
  const int kmax = g.k;
  const int m0 = GT2 * it, n0 = GT2 * jt;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;
  const int fr = lane & 15, fk = lane >> 4;
  Quad8 acc;
  quad8_zero(acc);
  const int nch = (kmax + GKC - 1) / GKC;
  const bool edge_mn = m0 + GT2 > g.m || n0 + GT2 > g.n;
  // staged as element pairs along each operand's contiguous dimension: pair
  // p = t + 512 q of a 128 x 16 chunk -- k-contiguous (A with TA, B without
  // TB): k = 2 (p & 7), row p >> 3; otherwise k = p >> 6, rows 2 (p & 63), +1.
  // Interior chunks load a pair with one 16-byte buffer load; chunks at the
  // matrix edges load its two elements masked.
  dv2 pa[2], pb[2];
  const Rsrc rA = rsrc(g.A), rB = rsrc(g.B);
  auto load = [&](int ch) __attribute__((always_inline)) {
    const int k0 = ch * GKC;
    const bool full = !edge_mn && k0 + GKC <= kmax;  // uniform
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int pp = t + 512 * q;
      if (TA) {
        const int gk = k0 + 2 * (pp & 7), gm = m0 + (pp >> 3);
        pa[q] = pair_load(rA, full, gm < g.m && gk < kmax, gm < g.m && gk + 1 < kmax, gk + (size_t)g.lda * gm);
      } else {
        const int gm = m0 + 2 * (pp & 63), gk = k0 + (pp >> 6);
        pa[q] = pair_load(rA, full, gm < g.m && gk < kmax, gm + 1 < g.m && gk < kmax, gm + (size_t)g.lda * gk);
      }
      if (TB) {
        const int gn = n0 + 2 * (pp & 63), gk = k0 + (pp >> 6);
        pb[q] = pair_load(rB, full, gn < g.n && gk < kmax, gn + 1 < g.n && gk < kmax, gn + (size_t)g.ldb * gk);
      } else {
        const int gk = k0 + 2 * (pp & 7), gn = n0 + (pp >> 3);
        pb[q] = pair_load(rB, full, gn < g.n && gk < kmax, gn < g.n && gk + 1 < kmax, gk + (size_t)g.ldb * gn);
      }
    }
  };
  // k-contiguous operands sit at column m ^ 4 (k >> 1): the pair stores of a
  // half-wave (8 k-pairs x 4 rows) and the compute reads stay conflict-free
  auto store = [&](int buf) __attribute__((always_inline)) {
    double* As = lds + buf * 2 * GKC * GLD2;
    double* Bs = As + GKC * GLD2;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int pp = t + 512 * q;
      if (TA) {
        const int k = 2 * (pp & 7), m = (pp >> 3) ^ ((k >> 1) << 2);
        As[k * GLD2 + m] = pa[q].x;
        As[(k + 1) * GLD2 + m] = pa[q].y;
      } else {
        *(dv2*)(As + (pp >> 6) * GLD2 + 2 * (pp & 63)) = pa[q];
      }
      if (TB) {
        *(dv2*)(Bs + (pp >> 6) * GLD2 + 2 * (pp & 63)) = pb[q];
      } else {
        const int k = 2 * (pp & 7), n = (pp >> 3) ^ ((k >> 1) << 2);
        Bs[k * GLD2 + n] = pb[q].x;
        Bs[(k + 1) * GLD2 + n] = pb[q].y;
      }
    }
  };
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const double* As = lds + buf * 2 * GKC * GLD2;
    const double* Bs = As + GKC * GLD2;
#pragma unroll
    for (int kk = 0; kk < GKC / 4; ++kk) {
      const int k = kk * 4 + fk, sa = TA ? (k >> 1) << 2 : 0, sb = TB ? 0 : (k >> 1) << 2;
      const double a0 = As[k * GLD2 + ((32 * wr + fr) ^ sa)], a1 = As[k * GLD2 + ((32 * wr + 16 + fr) ^ sa)];
      double b[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) b[q] = Bs[k * GLD2 + ((64 * wc + 16 * q + fr) ^ sb)];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc.c[0][q] = MFMA64(a0, b[q], acc.c[0][q]);
        acc.c[1][q] = MFMA64(a1, b[q], acc.c[1][q]);
      }
    }
  };
  if (nch > 0) {
    load(0);
    store(0);
    __syncthreads();
    for (int ch = 0; ch < nch; ++ch) {
      if (ch + 1 < nch) load(ch + 1);
      compute(ch & 1);
      if (ch + 1 < nch) store((ch + 1) & 1);
      __syncthreads();
    }
  }
  // stage 64 columns at a time column-major in LDS (X[n * 129 + m]) for
  // coalesced stores; waves with wc == h own columns 64 h .. 64 h + 63
  double* X = lds;
  for (int h = 0; h < 2; ++h) {
    if (wc == h) {
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
#pragma unroll
          for (int r = 0; r < 4; ++r) X[(acc4_col(nb) - 64 * h) * 129 + acc4_row(mb, r)] = acc.c[mb][nb][r];
    }
    __syncthreads();
    for (int e = t; e < GT2 * 64; e += 512) {
      const int m = e & 127, n = e >> 7, gm = m0 + m, gn = n0 + 64 * h + n;
      if (gm < g.m && gn < g.n) {
        gdouble* c = G(g.C) + gm + (size_t)g.ldc * gn;
        const double v = g.alpha * X[n * 129 + m];
        *c = g.beta == 0.0 ? v : v + g.beta * *c;
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ k_gemv
// trans: y_j = alpha sum_i A(i, j) x_i + beta y_j, one wave per output.
__global__ __launch_bounds__(256) void k_gemv_t(const Gemv* __restrict__ gs) {
  const Gemv g = gs[blockIdx.y];
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (j >= g.n) return;
  const double* a = g.A + (size_t)g.lda * j;
  double s = 0.0;
  for (int i = lane; i < g.m; i += 64) s += a[i] * g.x[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
  if (lane == 0) g.y[j] = g.beta == 0.0 ? g.alpha * s : g.alpha * s + g.beta * g.y[j];
}

// else y_i = alpha sum_j A(i, j) x_j + beta y_i: 64 rows per workgroup (lane =
// row, coalesced column reads), its GV_W waves take contiguous column ranges
// and their partial sums are added in wave order (one thread per row over
// all columns left the chip ~70 waves for an n x M = 4600 x 928 product)
#define GV_W 16
__global__ __launch_bounds__(64 * GV_W) void k_gemv_n(const Gemv* __restrict__ gs) {
  __shared__ double part[GV_W][64];
  const Gemv g = gs[blockIdx.y];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  if (blockIdx.x * 64 >= g.m) return;  // uniform
  const int per = (g.n + GV_W - 1) / GV_W, j0 = w * per, j1 = min(g.n, j0 + per);
  double s = 0.0;
  if (i < g.m)
#pragma unroll 8
    for (int j = j0; j < j1; ++j) s += g.A[i + (size_t)g.lda * j] * g.x[j];
  part[w][lane] = s;
  __syncthreads();
  if (w == 0 && i < g.m) {
    double t = part[0][lane];
    for (int ww = 1; ww < GV_W; ++ww) t += part[ww][lane];
    g.y[i] = g.beta == 0.0 ? g.alpha * t : g.alpha * t + g.beta * g.y[i];
  }
}

// ------------------------------------------------------------ k_potrf_tile
// Block jb of a blocked right-looking Cholesky: factor the (updated) diagonal
// block A(jb:jb+nb, jb:jb+nb) in place (lower, nb = min(64, M - jb)) and write
// its inverse to dinv[jb/64] (64 x 64, column-major, identity beyond nb).
// Pivot <= 0 or NaN -> info = 1 (LAPACK dpotrf's info > 0; NB1's LinAlgError).
// One 64-thread wave per matrix, the block in LDS (row r = lane).
__global__ __launch_bounds__(64) void k_potrf_tile(const Chol* __restrict__ cs, int jb) {
  __shared__ double L[64 * 65];
  const Chol c = cs[blockIdx.x];
  if (jb >= c.M) return;
  const int nb = min(64, c.M - jb), r = threadIdx.x;
  gdouble* A = G(c.A) + jb + (size_t)c.lda * jb;
  for (int j = 0; j < 64; ++j)
    L[r * 65 + j] = (r < nb && j < nb) ? (j <= r ? A[r + (size_t)c.lda * j] : 0.0) : (r == j ? 1.0 : 0.0);
  __syncthreads();
  bool bad = false;
  for (int j = 0; j < nb; ++j) {
    const double p = L[j * 65 + j];
    if (p <= 0.0) bad = true;  // a NaN pivot propagates (numpy + OpenBLAS's dpotrf do not flag it)
    const double ljj = sqrt(p);
    __syncthreads();
    if (r == j) L[j * 65 + j] = ljj;
    if (r > j) L[r * 65 + j] = L[r * 65 + j] / ljj;
    __syncthreads();
    if (r > j) {
      const double lrj = L[r * 65 + j];
      for (int k = j + 1; k <= r; ++k) L[r * 65 + k] -= lrj * L[k * 65 + j];
    }
    __syncthreads();
  }
  if (bad && r == 0) *c.info = 1;
  // inverse: lane j forms column j of L^-1 by forward substitution
  gdouble* D = G(c.dinv) + (size_t)(jb / 64) * 4096;
  {
    const int j = r;
    double x[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) x[i] = 0.0;
    // x_i = (delta_ij - sum_{k<i} L_ik x_k) / L_ii with compile-time indices
    // (x stays in registers; a loop starting at k = j put x in scratch).  For
    // i < j every term is +0 and x_i = +0; for i >= j the k < j terms subtract
    // L_ik (+0) = +-0 from +0 or 1, which leaves s unchanged, so the sum is
    // the one from k = j exactly.
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      double s = i == j ? 1.0 : 0.0;
#pragma unroll
      for (int k = 0; k < i; ++k) s -= L[i * 65 + k] * x[k];
      x[i] = s / L[i * 65 + i];
    }
#pragma unroll
    for (int i = 0; i < 64; ++i) D[i + 64 * j] = x[i];
  }
  __syncthreads();
  for (int j = 0; j < nb; ++j)
    if (r >= j && r < nb) A[r + (size_t)c.lda * j] = L[r * 65 + j];
}

// ------------------------------------------------------------------ k_sytrd
#define TNB 32   // panel width
#define SY_T 512 // threads
#define SY_W (SY_T / 64)
#define SY_C 8   // symv: columns per wave group
#define SY_R 4   // symv: 64-row chunks per load batch (8: 190 VGPRs, one workgroup per CU)

struct EighWs {  // per-matrix workspace carve-up (eigh_workspace_doubles)
  double *Vc, *Ws, *T, *d, *e, *tau, *scr, *H, *X, *Y, *flag;
};
__host__ __device__ inline EighWs carve(double* w, int M) {
  EighWs s;
  const size_t MM = (size_t)M * M;
  s.Vc = w;
  s.scr = s.Vc + MM;               // 6 M^2: stein's LU factors and iterate
  s.Ws = s.scr + 6 * MM;           // M x 32
  s.H = s.Ws + (size_t)M * TNB;    // M x 32
  s.X = s.H + (size_t)M * TNB;     // 32 x M
  s.Y = s.X + (size_t)M * TNB;     // 32 x M
  s.T = s.Y + (size_t)M * TNB;     // panels x 32 x 32
  s.d = s.T + ((size_t)(M + TNB - 1) / TNB + 1) * TNB * TNB;
  s.e = s.d + M + 1;
  s.tau = s.e + M + 1;
  s.flag = s.tau + M + 1;  // k_orth_panel -> k_mgs_panel: the panel collapsed
  return s;
}
struct EighWsG {  // carve() as global-address-space pointers (device side)
  gdouble *Vc, *Ws, *T, *d, *e, *tau, *scr, *H, *X, *Y, *flag;
};
__device__ inline EighWsG carveG(double* w, int M) {
  const EighWs s = carve(w, M);
  return EighWsG{G(s.Vc), G(s.Ws), G(s.T), G(s.d), G(s.e), G(s.tau), G(s.scr), G(s.H), G(s.X), G(s.Y), G(s.flag)};
}
size_t eigh_workspace_doubles(int M) {
  const size_t MM = (size_t)M * M;
  return 7 * MM + 4 * (size_t)M * TNB + ((size_t)(M + TNB - 1) / TNB + 1) * TNB * TNB + 3 * (size_t)M + 16;
}

template <int NV>
__device__ __forceinline__ void wg_sum(double (&v)[NV], double* red) {
  // fixed-order block reduction over SY_T threads; every thread gets the sums
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < NV; ++q)
    for (int o = 32; o > 0; o >>= 1) v[q] += __shfl_down(v[q], o, 64);
  __syncthreads();
  if (lane == 0)
#pragma unroll
    for (int q = 0; q < NV; ++q) red[w * NV + q] = v[q];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    double s = red[q];
    for (int ww = 1; ww < (int)(blockDim.x >> 6); ++ww) s += red[ww * NV + q];
    v[q] = s;
  }
  __syncthreads();
}

__device__ __forceinline__ void ws_d0(const Eigh& E) { carve(E.work, E.M).d[0] = E.A[0]; }

// The tridiagonalisation runs column by column as two launches per column
// g = p + i (panel p, i < 32) over the whole batch -- the symmetric product
// y = A22 v streams the trailing lower triangle once per column, and one
// workgroup per matrix could pull it only at ~40 GB/s (a CU's outstanding
// misses bound it; measured round 4), so it is spread over ns workgroups per
// matrix, and so is everything else that streams the panel:
//   k_sy_symv(p, i)  every workgroup forms the reflector v_g of column g
//                    (dlarfg; identical fixed-order reductions, workgroup 0
//                    publishes v, d, e, tau), then its partial y (its waves
//                    own groups of SY_C consecutive columns), its share of the
//                    panel dots V'v, W'v and its partial y'v
//   k_sy_w(p, i)     SW_T rows per workgroup: w = tau (y - V(W'v) - W(V'v))
//                    - tau/2 (w'v) v with w'v = tau (y'v - 2 (W'v).(V'v)) from
//                    the dots, column i of the panel's T (dlarft, forward
//                    columnwise), and column g + 1 brought up to date with the
//                    panel's reflectors 0 .. i (dlatrd's column update)
// then, per panel, the trailing update A22 -= V W' + W V' on oila::gemm.
// symv workgroups per matrix: gridDim.y of k_sy_symv (OI_SY_S, default below)
#define SY_S_DEFAULT 8
#define SY_S_MAX TNB  // the partials live in the M x 32 H block
#define SW_T 128      // k_sy_w: rows (threads) per workgroup

// partial y of workgroup s into H[s M + r] (rows g+1 .. M-1); the panel dots
// pan[q] = W(:,q)'v, pan[TNB + q] = V(:,q)'v (rows > g) into X[0 .. 2 TNB);
// the partial y'v into X[2 TNB + s].  dynamic LDS: yw[SY_W][M] | v[M] | red[64]
// at most 128 VGPRs: two 512-thread workgroups per CU (their LDS fits too)
__global__ __launch_bounds__(SY_T) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_sy_symv(const Eigh* __restrict__ es, int p, int i) {
  extern __shared__ double sm[];
  const Eigh E = es[blockIdx.x];
  const int M = E.M, ld = E.lda, t = threadIdx.x, lane = t & 63, g = p + i, sgrp = blockIdx.y;
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);  // provably wave-uniform (buffer descriptors)
  if (p >= M - 1) {
    if (p == 0 && i == 0 && t == 0 && sgrp == 0) ws_d0(E);  // M == 1
    return;
  }
  if (g >= M - 1) return;  // this matrix's last panel is shorter
  EighWsG ws = carveG(E.work, M);
  double* yw = sm;
  double* v = yw + (size_t)SY_W * M;
  double* red = v + M;
  // (2) the reflector annihilating A(g+2:M, g) (dlarfg); column g is up to
  // date (k_sy_w(i - 1), or the trailing update for i = 0)
  const gdouble* A = G(E.A);
  {
    double xs[1] = {0.0};
    for (int r = g + 2 + t; r < M; r += SY_T) {
      const double a = A[r + (size_t)ld * g];
      xs[0] += a * a;
    }
    wg_sum<1>(xs, red);
    const double alpha = A[g + 1 + (size_t)ld * g];
    const double xn = sqrt(xs[0]);
    double tau, beta, scal;
    if (xn == 0.0) {
      tau = 0.0;
      beta = alpha;
      scal = 0.0;
    } else {
      beta = -copysign(sqrt(alpha * alpha + xn * xn), alpha);
      tau = (beta - alpha) / beta;
      scal = 1.0 / (alpha - beta);
    }
    gdouble* vg = ws.Vc + (size_t)M * g;
    for (int r = t; r < M; r += SY_T) {
      const double x = r < g + 1 ? 0.0 : r == g + 1 ? 1.0 : A[r + (size_t)ld * g] * scal;
      v[r] = x;
      if (sgrp == 0) vg[r] = x;
    }
    if (sgrp == 0 && t == 0) {
      ws.d[g] = A[g + (size_t)ld * g];
      ws.e[g] = beta;
      ws.tau[g] = tau;
    }
  }
  for (int r = t; r < SY_W * M; r += SY_T) yw[r] = 0.0;
  __syncthreads();
  // (3) y = A22 v over the lower triangle of A(g+1:M, g+1:M): global wave
  // gw = s SY_W + wv owns groups of SY_C consecutive columns (dealt below)
  // and streams their rows in batches of
  // SY_R x 64; per row one v[r] read and one yw[wv][r] read-modify-write (the
  // transposed half) serve the whole group; the group's column dots are
  // reduced once at its end
  double* myw = yw + (size_t)wv * M;
  const int gw = sgrp * SY_W + wv;
  const int ns = gridDim.y, nw = SY_W * ns;
  // groups dealt in snake order (k = j nw + gw, then j nw + nw - 1 - gw, ...):
  // a wave's long early group pairs with a short late one (round-robin left
  // the first waves ~1.6x the mean rows)
  for (int jg = 0;; ++jg) {
    const int c0 = g + 1 + SY_C * (jg * nw + ((jg & 1) ? nw - 1 - gw : gw));
    if (c0 >= M) break;
    const Rsrc rcol = rsrc(E.A + (size_t)ld * c0);
    double vc[SY_C], dot[SY_C];
#pragma unroll
    for (int j = 0; j < SY_C; ++j) {
      vc[j] = c0 + j < M ? v[c0 + j] : 0.0;
      dot[j] = 0.0;
    }
    for (int r0 = c0; r0 < M; r0 += SY_R * 64) {
      double a[SY_R][SY_C];
#pragma unroll
      for (int u = 0; u < SY_R; ++u)
#pragma unroll
        for (int j = 0; j < SY_C; ++j) {
          const int r = r0 + lane + 64 * u;
          a[u][j] = bload(rcol, r < M && r >= c0 + j, r + (size_t)ld * j);
        }
#pragma unroll
      for (int u = 0; u < SY_R; ++u) {
        const int r = r0 + lane + 64 * u;
        if (r < M) {
          const double vr = v[r];
          double tr = 0.0;
#pragma unroll
          for (int j = 0; j < SY_C; ++j) {
            dot[j] += a[u][j] * vr;
            if (r > c0 + j) tr += a[u][j] * vc[j];
          }
          myw[r] += tr;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < SY_C; ++j)
      for (int o = 32; o > 0; o >>= 1) dot[j] += __shfl_down(dot[j], o, 64);
    if (lane == 0)
#pragma unroll
      for (int j = 0; j < SY_C; ++j)
        if (c0 + j < M) myw[c0 + j] += dot[j];
  }
  // panel dots, one per global wave (rows > g, 4 row chunks per load batch)
  for (int jq = gw; jq < 2 * i; jq += SY_W * ns) {
    const int q = jq % i;
    const Rsrc rc = rsrc(jq < i ? carve(E.work, M).Ws + (size_t)M * q : carve(E.work, M).Vc + (size_t)M * (p + q));
    double s4[4] = {0.0, 0.0, 0.0, 0.0};
    for (int r = g + 1 + lane; r < M; r += 256) {
      double a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] = bload(rc, r + 64 * u < M, r + 64 * u);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (r + 64 * u < M) s4[u] += a[u] * v[r + 64 * u];
    }
    double sd = (s4[0] + s4[1]) + (s4[2] + s4[3]);
    for (int o = 32; o > 0; o >>= 1) sd += __shfl_down(sd, o, 64);
    if (lane == 0) ws.X[(jq < i ? 0 : TNB) + q] = sd;
  }
  __syncthreads();
  gdouble* yp = ws.H + (size_t)sgrp * M;
  double yv[1] = {0.0};
  for (int r = g + 1 + t; r < M; r += SY_T) {
    double sy = 0.0;
#pragma unroll
    for (int ww = 0; ww < SY_W; ++ww) sy += yw[(size_t)ww * M + r];
    yp[r] = sy;
    yv[0] += sy * v[r];
  }
  wg_sum<1>(yv, red);
  if (t == 0) ws.X[2 * TNB + sgrp] = yv[0];
}

// grid (matrices, ceil(Mmax / SW_T)): thread t of workgroup b owns row
// g + 1 + SW_T b + t
__global__ __launch_bounds__(SW_T) void k_sy_w(const Eigh* __restrict__ es, int p, int i, int ns, int next) {
  __shared__ double pan[2 * TNB];
  __shared__ double rowg1[2 * TNB + 1];  // W(g+1, q), V(g+1, q) for q < i; w_i(g+1)
  const Eigh E = es[blockIdx.x];
  const int M = E.M, ld = E.lda, t = threadIdx.x, g = p + i, g1 = g + 1;
  if (g >= M - 1) return;
  const int r = g + 1 + SW_T * blockIdx.y + t;
  if (g + 1 + SW_T * blockIdx.y >= M) return;  // no rows for this workgroup (uniform)
  EighWsG ws = carveG(E.work, M);
  const Rsrc rV = rsrc(carve(E.work, M).Vc + (size_t)M * p), rW = rsrc(carve(E.work, M).Ws);
  const bool upd = next && g1 < M - 1;
  // this thread's row of the panel's V and W, loaded once for w and for the
  // next column's update (all TNB columns in flight; q >= i loads 0, and the
  // sums below subtract exactly +0 there, so they equal the q < i sums)
  double vr[TNB], wr[TNB];
#pragma unroll
  for (int q = 0; q < TNB; ++q) {
    vr[q] = bload(rV, q < i && r < M, (size_t)M * q + r);
    wr[q] = bload(rW, q < i && r < M, (size_t)M * q + r);
  }
  const double tau = ws.tau[g];
  if (t < 2 * TNB) pan[t] = t % TNB < i ? ws.X[t] : 0.0;
  if (upd && t < TNB) {  // zeros from i on
    rowg1[t] = t < i ? ws.Ws[(size_t)M * t + g1] : 0.0;
    rowg1[TNB + t] = t < i ? ws.Vc[(size_t)M * (p + t) + g1] : 0.0;
  }
  __syncthreads();
  // w'v = tau (y'v - 2 (W'v).(V'v)), fixed order
  double yv = 0.0, dd = 0.0;
  for (int s = 0; s < ns; ++s) yv += ws.X[2 * TNB + s];
  for (int q = 0; q < i; ++q) dd += pan[q] * pan[TNB + q];
  const double a2 = -0.5 * tau * (tau * (yv - 2.0 * dd));
  const gdouble* vgc = ws.Vc + (size_t)M * g;
  // w_i(row) = tau (y - V(row,:) W'v - W(row,:) V'v) + a2 v(row)
  gdouble* wcol = ws.Ws + (size_t)M * i;
  if (blockIdx.y == 0) {
    // column i of the block reflector's T (dlarft, forward columnwise), in the
    // workspace: T(i,i) = tau, T(a,i) = -tau sum_{a<=k<i} T(a,k) (V_k'v)
    gdouble* Tp = ws.T + (size_t)(p / TNB) * TNB * TNB;
    if (i == 0)
      for (int e = t; e < TNB * TNB; e += SW_T) Tp[e] = 0.0;
    __syncthreads();
    if (t <= i) {
      double x = tau;
      if (t < i) {
        x = 0.0;
        for (int k = t; k < i; ++k) x += Tp[t + TNB * k] * pan[TNB + k];
        x *= -tau;
      }
      Tp[t + TNB * i] = x;
    }
    for (int rr = t; rr <= g && rr < M; rr += SW_T) wcol[rr] = 0.0;
  }
  if (upd && t == 0) {  // w_i(g1), for this workgroup's update (as the row formula below)
    double sa = 0.0;
    for (int s = 0; s < ns; ++s) sa += ws.H[(size_t)s * M + g1];
    for (int q = 0; q < i; ++q) sa -= ws.Vc[(size_t)M * (p + q) + g1] * pan[q] + ws.Ws[(size_t)M * q + g1] * pan[TNB + q];
    rowg1[2 * TNB] = tau * sa + a2 * vgc[g1];
  }
  double w = 0.0;
  if (r < M) {
    double sa = 0.0;
    for (int s = 0; s < ns; ++s) sa += ws.H[(size_t)s * M + r];
#pragma unroll
    for (int q = 0; q < TNB; ++q) sa -= vr[q] * pan[q] + wr[q] * pan[TNB + q];
    w = tau * sa + a2 * vgc[r];
    wcol[r] = w;
  }
  if (!upd) return;
  __syncthreads();
  // column g1, rows >= g1: A(r,g1) -= V(r,q) W(g1,q) + W(r,q) V(g1,q), q <= i
  if (r < M) {
    gdouble* A = G(E.A);
    double sa = A[r + (size_t)ld * g1];
#pragma unroll
    for (int q = 0; q < TNB; ++q) sa -= vr[q] * rowg1[q] + wr[q] * rowg1[TNB + q];
    sa -= vgc[r] * rowg1[2 * TNB] + w * vgc[g1];  // q = i: W(g1, i), V(g1, i) = v_g(g1)
    A[r + (size_t)ld * g1] = sa;
  }
}

// d[M-1] once the last panel's trailing update has run
__global__ __launch_bounds__(64) void k_sytrd_last(const Eigh* __restrict__ es) {
  const Eigh E = es[blockIdx.x];
  if (threadIdx.x == 0 && E.M > 1) carve(E.work, E.M).d[E.M - 1] = E.A[(E.M - 1) + (size_t)E.lda * (E.M - 1)];
}

// ------------------------------------------------- k_stebz / k_stein
__device__ __forceinline__ double start_value(int k, int i) {
  // deterministic pseudo-random start (splitmix64 of (k, i)) in [-1, 1)
  unsigned long long h = (unsigned long long)i * 0x9E3779B97F4A7C15ull + (unsigned long long)(k + 1) * 0xBF58476D1CE4E5B9ull;
  h ^= h >> 31;
  h *= 0x94D049BB133111EBull;
  h ^= h >> 29;
  return (double)(h >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
}

// Eigenpairs of the tridiagonal, ST_T eigenvalues per workgroup (grid
// matrices x ceil(M / ST_T)): the bisections and inverse iterations are long
// serial chains per thread, so the batch is spread over the whole chip.
// dynamic LDS: d[M] | e2[M] | red[64]
#define ST_T 64
__device__ __forceinline__ void tri_setup(const Eigh& E, const EighWsG& ws, double* d, double* e2, double* red,
                                          double* el = nullptr) {
  const int M = E.M, t = threadIdx.x;
  for (int i = t; i < M; i += ST_T) {
    d[i] = ws.d[i];
    e2[i] = i < M - 1 ? ws.e[i] * ws.e[i] : 0.0;
    if (el) el[i] = i < M - 1 ? ws.e[i] : 0.0;
  }
  __syncthreads();
  if (t == 0) {  // Gershgorin interval, ||T||, pivmin (dstebz)
    double gl = d[0], gu = d[0], emax2 = 0.0;
    for (int i = 0; i < M; ++i) {
      const double ae = (i > 0 ? fabs(ws.e[i - 1]) : 0.0) + (i < M - 1 ? fabs(ws.e[i]) : 0.0);
      gl = fmin(gl, d[i] - ae);
      gu = fmax(gu, d[i] + ae);
      emax2 = fmax(emax2, e2[i]);
    }
    const double tnorm = fmax(fabs(gl), fabs(gu));
    const double eps = 2.220446049250313e-16, pivmin = 2.2250738585072014e-308 * fmax(1.0, emax2);
    red[0] = gl - 2.1 * tnorm * eps * M - 2.1 * pivmin;
    red[1] = gu + 2.1 * tnorm * eps * M + 2.1 * pivmin;
    red[2] = tnorm;
    red[3] = pivmin;
  }
  __syncthreads();
}

__global__ __launch_bounds__(ST_T) void k_stebz(const Eigh* __restrict__ es) {
  extern __shared__ double sm[];
  const Eigh E = es[blockIdx.x];
  const int M = E.M, t = threadIdx.x;
  if ((int)blockIdx.y * ST_T >= M) return;
  EighWsG ws = carveG(E.work, M);
  double* d = sm;
  double* e2 = d + M;
  double* red = e2 + M;
  tri_setup(E, ws, d, e2, red);
  const double GL = red[0], GU = red[1], pivmin = red[3];
  const double eps = 2.220446049250313e-16;
  {
    const int k = (int)blockIdx.y * ST_T + t;
    if (k >= M) return;
    // eigenvalue k (ascending): count(x) = #eigenvalues < x; lambda_k = sup{x : count(x) <= k}
    // (bisection; multisection with 2 / 4 / 8 interleaved Sturm counts per
    // sweep, also with v_rcp_f64 + Newton in place of the division, measured
    // 8.2 - 11.6 vs 8.8 ms for stebz + stein on 64 matrices of M = 928: the
    // sweep is VALU-issue-bound at one wave per SIMD, profiles/r05/stebz/)
    double lo = GL, hi = GU;
    for (int it = 0; it < 128; ++it) {
      const double mid = 0.5 * (lo + hi);
      if (hi - lo <= 2.0 * eps * fmax(fabs(lo), fabs(hi)) + pivmin || mid == lo || mid == hi) break;
      int cnt = 0;
      double q = d[0] - mid;
      if (fabs(q) < pivmin) q = -pivmin;
      cnt += q < 0.0;
      // unrolled so that the LDS reads of d, e2 for 8 steps issue ahead of
      // the division chain (one wave per SIMD here: nothing else hides them)
#pragma unroll 8
      for (int i = 1; i < M; ++i) {
        q = d[i] - mid - e2[i - 1] / q;
        if (fabs(q) < pivmin) q = -pivmin;
        cnt += q < 0.0;
      }
      if (cnt <= k) lo = mid;
      else hi = mid;
    }
    G(E.w)[k] = 0.5 * (lo + hi);
  }
}

// eigenvector k of the tridiagonal into the stein iterate (element i at
// [i M + k], lanes over k: coalesced), its inverse norm into Ws[k]
__global__ __launch_bounds__(ST_T) void k_stein(const Eigh* __restrict__ es) {
  extern __shared__ double sm[];
  const Eigh E = es[blockIdx.x];
  const int M = E.M, t = threadIdx.x;
  if ((int)blockIdx.y * ST_T >= M) return;
  EighWsG ws = carveG(E.work, M);
  const gdouble* w = G(E.w);
  double* d = sm;
  double* e2 = d + M;
  double* red = e2 + M;
  double* el = red + 64;  // e, for the factorisation's loads
  tri_setup(E, ws, d, e2, red, el);
  const double tnorm = red[2];
  const double eps = 2.220446049250313e-16;
  const size_t MM = (size_t)M * M;
  gdouble* sa = ws.scr;          // U diagonal
  gdouble* sb = sa + MM;         // U first superdiagonal
  gdouble* sc = sb + MM;         // U second superdiagonal
  gdouble* sl = sc + MM;         // L multipliers
  gdouble* sp = sl + MM;         // row interchange flags
  gdouble* sx = sp + MM;         // iterate
  // The bottom cluster: eigenvalues 0 .. nb0-1 whose consecutive gaps are all
  // <= 1e3 eps ||T|| -- the numerical null space of a rank-deficient K_mm
  // (duplicated sites) and the noise band below it.  Inverse iteration cannot
  // separate vectors whose eigenvalues differ by less than its own accuracy
  // (they collapse onto the same few directions), so those vectors start
  // from independent random vectors instead, and the orthogonalisation, which
  // runs in DESCENDING eigenvalue order (eigenvector k is column M-1-k of Z
  // until the final reversal), makes them an orthonormal basis of the
  // complement of every other eigenvector -- the cluster's invariant subspace.
  if (t == 0) {
    const double gtol = 1e3 * eps * tnorm;
    int nb0 = 1;
    while (nb0 < M && w[nb0] - w[nb0 - 1] <= gtol) ++nb0;
    red[4] = nb0 >= 2 ? (double)nb0 : 0.0;
  }
  __syncthreads();
  const int nb0 = (int)red[4];
  {
    const int k = (int)blockIdx.y * ST_T + t;
    if (k >= M) return;
    const double lam = w[k];
    if (k < nb0) {
      double nrm = 0.0;
      for (int i = 0; i < M; ++i) {
        const double x = start_value(k, i);
        nrm += x * x;
      }
      for (int i = 0; i < M; ++i) sx[(size_t)i * M + k] = start_value(k, i);
      ws.Ws[k] = 1.0 / sqrt(nrm);
      return;
    }
    // T - lam I = P L U (dlagtf), factors at [i * M + k]
    {
      double ak = d[0] - lam, bk = M > 1 ? el[0] : 0.0;
#pragma unroll 4
      for (int i = 0; i < M - 1; ++i) {
        const double sub = el[i];
        const double an = d[i + 1] - lam, bn = i + 1 < M - 1 ? el[i + 1] : 0.0;
        double m, cnew = 0.0, a_i, b_i, a_next, b_next, piv = 0.0;
        if (fabs(ak) >= fabs(sub)) {
          m = ak != 0.0 ? sub / ak : 0.0;
          a_i = ak;
          b_i = bk;
          a_next = an - m * bk;
          b_next = bn;
        } else {
          m = ak / sub;
          piv = 1.0;
          a_i = sub;
          b_i = an;
          a_next = bk - m * an;
          if (i < M - 2) {
            cnew = bn;
            b_next = -m * cnew;
          } else {
            b_next = bn;
          }
        }
        const size_t o = (size_t)i * M + k;
        sa[o] = a_i;
        sb[o] = b_i;
        sc[o] = cnew;
        sl[o] = m;
        sp[o] = piv;
        ak = a_next;
        bk = b_next;
      }
      const size_t o = (size_t)(M - 1) * M + k;
      sa[o] = ak;
      sb[o] = 0.0;
      sc[o] = 0.0;
      sl[o] = 0.0;
      sp[o] = 0.0;
    }
    for (int i = 0; i < M; ++i) sx[(size_t)i * M + k] = start_value(k, i);
    const double tol = eps * tnorm;
    for (int iter = 0; iter < 2; ++iter) {
      // forward: apply P and L
      double prev = sx[k];
#pragma unroll 4
      for (int i = 0; i < M - 1; ++i) {
        const size_t o = (size_t)i * M + k;
        const double nx = sx[o + M];
        if (sp[o] != 0.0) {
          sx[o] = nx;
          prev = prev - sl[o] * nx;
        } else {
          sx[o] = prev;
          prev = nx - sl[o] * prev;
        }
      }
      sx[(size_t)(M - 1) * M + k] = prev;
      // backward with U, tiny pivots perturbed (dlagts, job = -1)
      double x1 = 0.0, x2 = 0.0, amax = 0.0;
#pragma unroll 4
      for (int i = M - 1; i >= 0; --i) {
        const size_t o = (size_t)i * M + k;
        double s = sx[o] - sb[o] * x1 - sc[o] * x2;
        double a = sa[o];
        if (fabs(a) < tol) a = a >= 0.0 ? tol : -tol;
        const double xi = s / a;
        sx[o] = xi;
        x2 = x1;
        x1 = xi;
        amax = fmax(amax, fabs(xi));
      }
      const double inv = 1.0 / amax;
      for (int i = 0; i < M; ++i) sx[(size_t)i * M + k] *= inv;
    }
    double nrm = 0.0;
    for (int i = 0; i < M; ++i) {
      const double x = sx[(size_t)i * M + k];
      nrm += x * x;
    }
    ws.Ws[k] = 1.0 / sqrt(nrm);
  }
}


// Z(:, M-1-k) = iterate k * Ws[k]: the iterate transposed through 64 x 64 LDS tiles
__global__ __launch_bounds__(256) void k_stein_out(const Eigh* __restrict__ es) {
  __shared__ double tile[64][65];
  const Eigh E = es[blockIdx.x];
  const int M = E.M, nt = (M + 63) / 64;
  if ((int)blockIdx.y >= nt * nt) return;
  const EighWsG ws = carveG(E.work, M);
  const gdouble* sx = ws.scr + 5 * (size_t)M * M;
  const int i0 = 64 * ((int)blockIdx.y % nt), k0 = 64 * ((int)blockIdx.y / nt), t = threadIdx.x;
  for (int e = t; e < 64 * 64; e += 256) {
    const int i = i0 + e / 64, k = k0 + e % 64;
    tile[e / 64][e % 64] = (i < M && k < M) ? sx[(size_t)i * M + k] * ws.Ws[k] : 0.0;
  }
  __syncthreads();
  for (int e = t; e < 64 * 64; e += 256) {
    const int i = i0 + e % 64, k = k0 + e / 64;
    if (i < M && k < M) G(E.A)[i + (size_t)E.lda * (M - 1 - k)] = tile[e % 64][e / 64];
  }
}

// column c <-> M-1-c (the eigenvectors back in ascending eigenvalue order)
__global__ __launch_bounds__(256) void k_reverse_cols(const Eigh* __restrict__ es) {
  const Eigh E = es[blockIdx.x];
  const int M = E.M;
  for (int c = blockIdx.y; c < M / 2; c += gridDim.y) {
    double* a = E.A + (size_t)E.lda * c;
    double* b = E.A + (size_t)E.lda * (M - 1 - c);
    for (int i = threadIdx.x; i < M; i += 256) {
      const double x = a[i];
      a[i] = b[i];
      b[i] = x;
    }
  }
}

// ------------------------------------------------------------ k_mgs_panel
// Columns [p, q) of Z (already orthogonal to columns < p): classical
// Gram-Schmidt twice against the panel's earlier columns, normalise; a column
// that collapses (repeated eigenvalue) is replaced by a fresh start vector
// projected out of every earlier column.
#define MG_T 256
__global__ __launch_bounds__(MG_T) void k_mgs_panel(const Eigh* __restrict__ es, int p) {
  __shared__ double red[4 * 33];
  const Eigh E = es[blockIdx.x];
  const int M = E.M;
  if (p >= M || carve(E.work, M).flag[0] == 0.0) return;  // k_orth_panel's Cholesky QR held
  const int q = min(M, p + TNB), t = threadIdx.x, lane = t & 63, w = t >> 6;
  gdouble* Z = G(E.A);
  const size_t ld = E.lda;
  auto reduce = [&](double (&v)[33]) {  // fixed-order sums of 33 values
#pragma unroll
    for (int a = 0; a < 33; ++a)
      for (int o = 32; o > 0; o >>= 1) v[a] += __shfl_down(v[a], o, 64);
    __syncthreads();
    if (lane == 0)
#pragma unroll
      for (int a = 0; a < 33; ++a) red[w * 33 + a] = v[a];
    __syncthreads();
#pragma unroll
    for (int a = 0; a < 33; ++a) v[a] = ((red[a] + red[33 + a]) + red[66 + a]) + red[99 + a];
    __syncthreads();
  };
  for (int j = p; j < q; ++j) {
    gdouble* zj = Z + ld * j;
    bool done = false, nan = false;
    for (int attempt = 0; attempt < 4; ++attempt) {
      const int lo = attempt == 0 ? p : 0;  // a fresh vector is projected out of everything
      double dv[33];
#pragma unroll
      for (int a = 0; a < 33; ++a) dv[a] = 0.0;
      for (int i = t; i < M; i += MG_T) dv[32] += zj[i] * zj[i];
      reduce(dv);
      const double n0 = dv[32];
      for (int pass = 0; pass < 2; ++pass) {
        for (int b0 = lo; b0 < j; b0 += 32) {
          const int nb = min(32, j - b0);
#pragma unroll
          for (int a = 0; a < 33; ++a) dv[a] = 0.0;
          for (int i = t; i < M; i += MG_T) {
            const double x = zj[i];
#pragma unroll
            for (int a = 0; a < 32; ++a)
              if (a < nb) dv[a] += Z[ld * (b0 + a) + i] * x;
          }
          reduce(dv);
          for (int i = t; i < M; i += MG_T) {
            double x = zj[i];
#pragma unroll
            for (int a = 0; a < 32; ++a)
              if (a < nb) x -= dv[a] * Z[ld * (b0 + a) + i];
            zj[i] = x;
          }
          __syncthreads();
        }
      }
#pragma unroll
      for (int a = 0; a < 33; ++a) dv[a] = 0.0;
      for (int i = t; i < M; i += MG_T) dv[32] += zj[i] * zj[i];
      reduce(dv);
      const double n1 = dv[32];
      nan = nan || !(n0 == n0) || !(n1 == n1);
      if (n1 > 1e-4 * n0 && n1 > 0.0) {
        const double inv = 1.0 / sqrt(n1);
        for (int i = t; i < M; i += MG_T) zj[i] *= inv;
        __syncthreads();
        done = true;
        break;
      }
      for (int i = t; i < M; i += MG_T) zj[i] = start_value(j + 7919 * (attempt + 1), i);
      __syncthreads();
    }
    // four collapses in a row of a finite column: it is not an orthonormal
    // vector (reported like a non-converged syevd).  NaN input
    // propagates instead, as numpy's eigh does when LAPACK returns NaNs.
    if (!done && !nan && t == 0 && E.info) *E.info = 1;
  }
}


// Columns [p, q) of Z (already orthogonal to columns < p): Cholesky QR twice --
// G = Z_p' Z_p on the MFMA core, G = R'R, Z_p <- Z_p R^-1 -- the same
// Gram-Schmidt in column order as mgs_panel in 2 block reductions per pass
// instead of 4 per column.  A pivot that keeps no more than 1e-4 of its
// column's squared norm (mgs_panel's collapse rule: numerically repeated
// eigenvalues) hands the panel to k_mgs_panel and its fresh start vectors.
#define RL (TNB + 1)  // LDS row stride of R and R^-1
__global__ __launch_bounds__(MG_T) void k_orth_panel(const Eigh* __restrict__ es, int p) {
  __shared__ double Gw[MG_T / 64][TNB * TNB];
  __shared__ double R[TNB * RL];
  __shared__ double Ri[TNB * RL];
  __shared__ double gd[TNB];
  __shared__ int bad;
  const Eigh E = es[blockIdx.x];
  const int M = E.M;
  if (p >= M) return;
  const int nb = min(TNB, M - p), t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int fr = lane & 15, fk = lane >> 4;
  const size_t ld = E.lda;
  gdouble* Z = G(E.A) + ld * p;
  const Rsrc rz = rsrc(E.A + ld * p);
  if (t == 0) carve(E.work, M).flag[0] = 0.0;
  for (int pass = 0; pass < 2; ++pass) {
    // (1) G = Z_p' Z_p: wave w sums the 16-row blocks 16 (w + 4 j), 4 k-steps per batch
    Quad acc;
    quad_zero(acc);
    // two row blocks per step: 16 loads per lane in flight
    auto gload = [&](int i0, double (&a0)[4], double (&a1)[4]) __attribute__((always_inline)) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + 4 * u + fk;
        a0[u] = bload(rz, i < M && fr < nb, i + ld * fr);
        a1[u] = bload(rz, i < M && 16 + fr < nb, i + ld * (16 + fr));
      }
    };
    auto gmfma = [&](const double (&a0)[4], const double (&a1)[4]) __attribute__((always_inline)) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc.c[0][0] = MFMA64(a0[u], a0[u], acc.c[0][0]);
        acc.c[0][1] = MFMA64(a0[u], a1[u], acc.c[0][1]);
        acc.c[1][0] = MFMA64(a1[u], a0[u], acc.c[1][0]);
        acc.c[1][1] = MFMA64(a1[u], a1[u], acc.c[1][1]);
      }
    };
    for (int i0 = 16 * w; i0 < M; i0 += 2 * 16 * (MG_T / 64)) {
      double a0[4], a1[4], b0[4], b1[4];
      gload(i0, a0, a1);
      gload(i0 + 16 * (MG_T / 64), b0, b1);  // past M: masked, loads 0 (adds +0 products)
      gmfma(a0, a1);
      gmfma(b0, b1);
    }
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int nbk = 0; nbk < 2; ++nbk)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          Gw[w][(16 * mb + (lane >> 4) + 4 * rr) + TNB * (16 * nbk + (lane & 15))] = acc.c[mb][nbk][rr];
    if (t == 0) bad = 0;
    __syncthreads();
    for (int e = t; e < TNB * TNB; e += MG_T) {
      const int a = e % TNB, b = e / TNB;
      double g = 0.0;
      if (a <= b && b < nb) {
        g = Gw[0][e];
        for (int ww = 1; ww < MG_T / 64; ++ww) g += Gw[ww][e];
      }
      R[a + RL * b] = g;
      if (a == b) gd[a] = g;
    }
    __syncthreads();
    // (2) G = R'R (upper R, right-looking, row j scaled by its pivot) and
    // (3) R^-1, both in wave 0's registers: lane c holds column c (g[k] = row
    // k), rows of R broadcast by lane reads -- the same operations in the same
    // order as the LDS form with three block barriers per column it replaces
    if (w == 0) {
      const int c = lane;
      double g[TNB];
#pragma unroll
      for (int k = 0; k < TNB; ++k) g[k] = c < TNB ? R[k + RL * c] : 0.0;
      bool badl = false;
#pragma unroll
      for (int j = 0; j < TNB; ++j) {
        if (j < nb) {  // uniform
          const double dj = __shfl(g[j], j, 64);
          if (!(dj > 1e-4 * gd[j])) badl = true;
          const double rjj = sqrt(fmax(dj, 1e-300));
          const double inv = 1.0 / rjj;
          if (c == j) g[j] = rjj;
          else if (c > j && c < nb) g[j] *= inv;
#pragma unroll
          for (int b = j + 1; b < TNB; ++b) {
            const double rjb = __shfl(g[j], b, 64);  // R(j, b)
            if (b < nb && c >= b && c < nb) g[b] -= rjb * g[j];
          }
        }
      }
      if (c < TNB)
#pragma unroll
        for (int k = 0; k < TNB; ++k) R[k + RL * c] = g[k];
      if (lane == 0) bad = badl;
      // R^-1 (upper), lane l = column l: x_a = (delta_al - sum_{k>a} R(a,k) x_k) / R(a,a);
      // x_k = +0 for k > l and past nb, so the sums are the k <= l ones exactly
      if (!badl && c < TNB) {
        double x[TNB];
#pragma unroll
        for (int aa = TNB - 1; aa >= 0; --aa) {
          double sx = aa == c ? 1.0 : 0.0;
#pragma unroll
          for (int k = aa + 1; k < TNB; ++k) sx -= R[aa + RL * k] * x[k];
          x[aa] = (aa < nb && c < nb) ? sx / R[aa + RL * aa] : 0.0;
        }
#pragma unroll
        for (int aa = 0; aa < TNB; ++aa) Ri[aa + RL * c] = x[aa];
      }
    }
    __syncthreads();
    if (bad) {  // k_mgs_panel takes the panel over
      if (t == 0) carve(E.work, M).flag[0] = 1.0;
      return;
    }
    // (4) Z_p <- Z_p R^-1 on the MFMA core, wave w over the 16-row blocks 16 (w + 4 j)
    double rb[2][TNB / 4];
#pragma unroll
    for (int kk = 0; kk < TNB / 4; ++kk)
#pragma unroll
      for (int nbk = 0; nbk < 2; ++nbk) rb[nbk][kk] = Ri[(4 * kk + fk) + RL * (16 * nbk + fr)];
    // the next row block's loads are issued before this block's stores (the
    // compiler cannot move them past stores into the same buffer itself)
    double za[TNB / 4];
    auto zload = [&](int i0, double (&z)[TNB / 4]) __attribute__((always_inline)) {
#pragma unroll
      for (int kk = 0; kk < TNB / 4; ++kk) {
        const int i = i0 + fr, a = 4 * kk + fk;
        z[kk] = bload(rz, i < M && a < nb, i + ld * a);
      }
    };
    zload(16 * w, za);
    for (int i0 = 16 * w; i0 < M; i0 += 16 * (MG_T / 64)) {
      double zn[TNB / 4];
      zload(i0 + 16 * (MG_T / 64), zn);  // past M: masked, loads 0
      d4 o0 = (d4){0.0, 0.0, 0.0, 0.0}, o1 = o0;
#pragma unroll
      for (int kk = 0; kk < TNB / 4; ++kk) {
        o0 = MFMA64(za[kk], rb[0][kk], o0);
        o1 = MFMA64(za[kk], rb[1][kk], o1);
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int i = i0 + (lane >> 4) + 4 * rr, c = lane & 15;
        if (i < M) {
          if (c < nb) Z[i + ld * c] = o0[rr];
          if (16 + c < nb) Z[i + ld * (16 + c)] = o1[rr];
        }
      }
#pragma unroll
      for (int kk = 0; kk < TNB / 4; ++kk) za[kk] = zn[kk];
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------- host --
Stager::~Stager() {
  if (host_) (void)hipHostFree(host_);
  if (dev_) (void)hipFree(dev_);
  for (auto& pr : retired_) {
    (void)hipHostFree(pr.first);
    (void)hipFree(pr.second);
  }
}

const void* Stager::put_bytes(const void* p, size_t bytes) {
  const size_t need = (off_ + bytes + 255) & ~(size_t)255;
  if (need > cap_) {
    if (host_) retired_.push_back({host_, dev_});  // still referenced by queued copies / launches
    size_t nc = std::max<size_t>(1 << 20, 2 * need);
    LC(hipHostMalloc((void**)&host_, nc, hipHostMallocDefault));
    LC(hipMalloc((void**)&dev_, nc));
    cap_ = nc;
    off_ = 0;
  }
  char* h = host_ + off_;
  char* d = dev_ + off_;
  std::memcpy(h, p, bytes);
  LC(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st_));
  off_ = (off_ + bytes + 255) & ~(size_t)255;
  return d;
}

// bload's descriptors cover 0x7FFFFFF0 bytes from an operand's base and take
// 32-bit byte offsets: an operand whose stored extent reaches past that would
// wrap or read zeros instead of failing, so the wrappers refuse it
static void check_extent(int64_t ld, int64_t rows, int64_t cols, const char* what) {
  if (rows <= 0 || cols <= 0) return;
  if ((ld * (cols - 1) + rows) * 8 >= (int64_t)0x7FFFFFF0)
    throw LinalgErr{std::string(what) + ": operand extent >= 2 GiB (32-bit buffer offsets)"};
}

// OI_GEMM128=0 keeps every product on the 64 x 64 kernel (A/B switch, read
// per call so a test can flip it)
static bool gemm128_ok() {
  const char* e = std::getenv("OI_GEMM128");
  return !(e && e[0] == '0');
}

void gemm(Stager& S, hipStream_t st, bool ta, bool tb, const std::vector<Gemm>& g) {
  std::vector<Gemm> live;
  int tiles = 0, tiles2 = 0;
  bool wide = gemm128_ok();
  for (const Gemm& x : g) {
    if (x.m > 0 && x.n > 0 && x.k > 0) {
      check_extent(x.lda, ta ? x.k : x.m, ta ? x.m : x.k, "gemm A");
      check_extent(x.ldb, tb ? x.n : x.k, tb ? x.k : x.n, "gemm B");
      check_extent(x.ldc, x.m, x.n, "gemm C");
    }
    if (x.m > 0 && x.n > 0) {
      live.push_back(x);
      tiles = std::max(tiles, ((x.m + GT - 1) / GT) * ((x.n + GT - 1) / GT));
      tiles2 = std::max(tiles2, ((x.m + GT2 - 1) / GT2) * ((x.n + GT2 - 1) / GT2));
      wide = wide && x.tri == 0 && x.m >= GT2 && x.n >= GT2 && x.k >= 4 * GKC;
    }
  }
  if (live.empty()) return;
  const Gemm* dg = S.put(live);
  if (wide) {  // bitwise equal to k_gemm (see k_gemm128)
    dim3 grid2((unsigned)tiles2, (unsigned)live.size());
    if (ta && tb) hipLaunchKernelGGL((k_gemm128<true, true>), grid2, dim3(512), 0, st, dg);
    else if (ta) hipLaunchKernelGGL((k_gemm128<true, false>), grid2, dim3(512), 0, st, dg);
    else if (tb) hipLaunchKernelGGL((k_gemm128<false, true>), grid2, dim3(512), 0, st, dg);
    else hipLaunchKernelGGL((k_gemm128<false, false>), grid2, dim3(512), 0, st, dg);
    LC(hipGetLastError());
    return;
  }
  dim3 grid((unsigned)tiles, (unsigned)live.size());
  if (ta && tb) hipLaunchKernelGGL((k_gemm<true, true>), grid, dim3(256), 0, st, dg);
  else if (ta) hipLaunchKernelGGL((k_gemm<true, false>), grid, dim3(256), 0, st, dg);
  else if (tb) hipLaunchKernelGGL((k_gemm<false, true>), grid, dim3(256), 0, st, dg);
  else hipLaunchKernelGGL((k_gemm<false, false>), grid, dim3(256), 0, st, dg);
  LC(hipGetLastError());
}

void gemv(Stager& S, hipStream_t st, bool trans, const std::vector<Gemv>& g) {
  std::vector<Gemv> live;
  int outs = 0;
  for (const Gemv& x : g)
    if (x.m > 0 && x.n > 0) {
      check_extent(x.lda, x.m, x.n, "gemv A");
      live.push_back(x);
      outs = std::max(outs, trans ? x.n : x.m);
    }
  if (live.empty()) return;
  const Gemv* dg = S.put(live);
  if (trans)
    hipLaunchKernelGGL(k_gemv_t, dim3((unsigned)((outs + 3) / 4), (unsigned)live.size()), dim3(256), 0, st, dg);
  else
    hipLaunchKernelGGL(k_gemv_n, dim3((unsigned)((outs + 63) / 64), (unsigned)live.size()), dim3(64 * GV_W), 0,
                       st, dg);
  LC(hipGetLastError());
}

void cholesky(Stager& S, hipStream_t st, const std::vector<Chol>& cs) {
  if (cs.empty()) return;
  int Mmax = 0;
  for (const Chol& c : cs) {
    Mmax = std::max(Mmax, c.M);
    check_extent(c.lda, c.M, c.M, "cholesky A");
  }
  const Chol* dc = S.put(cs);
  for (int jb = 0; jb < Mmax; jb += 64) {
    hipLaunchKernelGGL(k_potrf_tile, dim3((unsigned)cs.size()), dim3(64), 0, st, dc, jb);
    LC(hipGetLastError());
    std::vector<Gemm> pan, upd;
    for (const Chol& c : cs) {
      if (c.M <= jb + 64) continue;
      const int rest = c.M - jb - 64;
      double* colj = c.A + (jb + 64) + (size_t)c.lda * jb;
      // L(jb+64:, jb) = A(jb+64:, jb) Dinv_jj^T (in place: each output tile reads only its own rows)
      pan.push_back(Gemm{colj, c.dinv + (size_t)(jb / 64) * 4096, colj, rest, 64, 64, c.lda, 64, c.lda, 1.0, 0.0, 0});
      // A(jb+64:, jb+64:) -= L L^T, lower tiles
      upd.push_back(Gemm{colj, colj, c.A + (jb + 64) + (size_t)c.lda * (jb + 64), rest, rest, 64, c.lda, c.lda,
                         c.lda, -1.0, 1.0, 1});
    }
    gemm(S, st, false, true, pan);
    gemm(S, st, false, true, upd);
  }
}

void trsm_right_lt(Stager& S, hipStream_t st, const std::vector<TrsmRLT>& ts) {
  int Mmax = 0;
  for (const TrsmRLT& x : ts) Mmax = std::max(Mmax, x.M);
  for (int jb = 0; jb < Mmax; jb += 64) {
    std::vector<Gemm> sc, up;
    for (const TrsmRLT& x : ts) {
      if (x.M <= jb) continue;
      const int nbj = std::min(64, x.M - jb);
      double* Xj = x.X + (size_t)x.ldx * jb;
      // X(:, jb) <- X(:, jb) Dinv_jj^T (in place)
      sc.push_back(Gemm{Xj, x.dinv + (size_t)(jb / 64) * 4096, Xj, x.m, nbj, nbj, x.ldx, 64, x.ldx, 1.0, 0.0, 0});
      if (x.M > jb + 64)  // X(:, jb+64:) -= X(:, jb) L(jb+64:, jb)^T
        up.push_back(Gemm{Xj, x.L + (jb + 64) + (size_t)x.ldl * jb, x.X + (size_t)x.ldx * (jb + 64), x.m,
                          x.M - jb - 64, 64, x.ldx, x.ldl, x.ldx, -1.0, 1.0, 0});
    }
    gemm(S, st, false, true, sc);
    gemm(S, st, false, true, up);
  }
}

void eigh(Stager& S, hipStream_t st, const std::vector<Eigh>& es, const std::function<void(int)>& mark) {
  if (es.empty()) return;
  auto phase = [&](int k) {
    if (mark) mark(k);
  };
  int Mmax = 0;
  for (const Eigh& e : es) {
    Mmax = std::max(Mmax, e.M);
    check_extent(e.lda, e.M, e.M, "eigh A");
  }
  if (Mmax > 4096) throw LinalgErr{"eigh: M > 4096 not supported"};
  const Eigh* de = S.put(es);
  const unsigned n = (unsigned)es.size();
  const size_t lds_sy = ((size_t)(SY_W + 1) * Mmax + 64) * sizeof(double);
  const unsigned nsw = (unsigned)((Mmax + SW_T - 1) / SW_T);
  if (lds_sy > 160 * 1024) throw LinalgErr{"eigh: matrix too large for the tridiagonalisation's LDS"};
  static const int ns = [] {
    const char* e = getenv("OI_SY_S");
    const int v = e ? atoi(e) : SY_S_DEFAULT;
    return v < 1 ? 1 : v > SY_S_MAX ? SY_S_MAX : v;
  }();
  phase(0);
  // panel by panel: the panel's 32 reflectors on one workgroup per matrix,
  // then its trailing update A22 -= V W' + W V' (lower 64 x 64 tiles) as two
  // batched GEMMs over the whole chip
  for (int p = 0; p < std::max(Mmax - 1, 1); p += TNB) {
    for (int i = 0; i < TNB && (i == 0 || p + i < Mmax - 1); ++i) {
      // k_sy_symv forms column g's reflector; k_sy_w(i) brings column g + 1 up to date
      hipLaunchKernelGGL(k_sy_symv, dim3(n, ns), dim3(SY_T), lds_sy, st, de, p, i);
      const int next = i + 1 < TNB && p + i + 1 < Mmax - 1;
      hipLaunchKernelGGL(k_sy_w, dim3(n, nsw), dim3(SW_T), 0, st, de, p, i, ns, next);
    }
    LC(hipGetLastError());
    std::vector<Gemm> g1, g2;
    for (const Eigh& e : es) {
      const int nb = std::min(TNB, e.M - 1 - p), q0 = p + nb, L = e.M - q0;
      if (nb <= 0 || L <= 0) continue;
      EighWs w = carve(e.work, e.M);
      double* C = e.A + q0 + (size_t)e.lda * q0;
      const double* V = w.Vc + (size_t)e.M * p + q0;
      const double* W = w.Ws + q0;
      g1.push_back(Gemm{V, W, C, L, L, nb, e.M, e.M, e.lda, -1.0, 1.0, 1});
      g2.push_back(Gemm{W, V, C, L, L, nb, e.M, e.M, e.lda, -1.0, 1.0, 1});
    }
    gemm(S, st, false, true, g1);
    gemm(S, st, false, true, g2);
  }
  hipLaunchKernelGGL(k_sytrd_last, dim3(n), dim3(64), 0, st, de);
  LC(hipGetLastError());
  phase(1);
  const size_t lds_st = (3 * (size_t)Mmax + 64) * sizeof(double);  // d | e2 | red[64] | e (k_stein)
  const unsigned nst = (unsigned)((Mmax + ST_T - 1) / ST_T), nto = (unsigned)((Mmax + 63) / 64);
  hipLaunchKernelGGL(k_stebz, dim3(n, nst), dim3(ST_T), lds_st, st, de);
  LC(hipGetLastError());
  hipLaunchKernelGGL(k_stein, dim3(n, nst), dim3(ST_T), lds_st, st, de);
  LC(hipGetLastError());
  hipLaunchKernelGGL(k_stein_out, dim3(n, nto * nto), dim3(256), 0, st, de);
  LC(hipGetLastError());
  phase(2);
  // BCGS2 over blocks of `ob` eigenvectors (columns of Z = E.A): a block is
  // projected out of every earlier block twice (two wide products per pass,
  // k_gemm128 where the shapes allow), then orthogonalised inside as BCGS2
  // over its TNB-column panels (k_orth_panel / k_mgs_panel).  ob = TNB is
  // plain panel-wise BCGS2 (rounds 4-5); wider blocks do the same projections
  // in a quarter of the launches on full 128-column tiles.  H lives in stein's
  // scratch (free once k_stein_out has written Z).
  static const int ob = [] {
    const char* e = getenv("OI_ORTH_BLOCK");
    const int v = e ? atoi(e) : 4 * TNB;
    return v <= TNB ? TNB : v >= 8 * TNB ? 8 * TNB : (v / TNB) * TNB;
  }();
  auto project = [&](int lo, int p, int nbmax) {  // Z(:, p:p+nb) -= Z(:, lo:p) Z(:, lo:p)' Z(:, p:p+nb), twice
    for (int pass = 0; pass < 2; ++pass) {
      std::vector<Gemm> h, u;
      for (const Eigh& e : es) {
        if (e.M <= p) continue;
        EighWs w = carve(e.work, e.M);
        const int nb = std::min(nbmax, e.M - p), k = p - lo;
        const double* Zlo = e.A + (size_t)e.lda * lo;
        // H = Z(:, lo:p)' Z(:, p:p+nb)   (k x nb, ld M)
        h.push_back(Gemm{Zlo, e.A + (size_t)e.lda * p, w.scr, k, nb, e.M, e.lda, e.lda, e.M, 1.0, 0.0, 0});
        // Z(:, p:p+nb) -= Z(:, lo:p) H
        u.push_back(Gemm{Zlo, w.scr, e.A + (size_t)e.lda * p, e.M, nb, k, e.lda, e.M, e.lda, -1.0, 1.0, 0});
      }
      gemm(S, st, true, false, h);
      gemm(S, st, false, false, u);
    }
  };
  for (int P = 0; P < Mmax; P += ob) {
    if (P > 0) project(0, P, ob);
    for (int p = P; p < std::min(P + ob, Mmax); p += TNB) {
      if (p > P) project(P, p, TNB);
      hipLaunchKernelGGL(k_orth_panel, dim3(n), dim3(MG_T), 0, st, de, p);
      LC(hipGetLastError());
      hipLaunchKernelGGL(k_mgs_panel, dim3(n), dim3(MG_T), 0, st, de, p);
      LC(hipGetLastError());
    }
  }
  // back-transform: Z <- (I - V_p T_p V_p') Z for the panels in reverse order
  phase(3);
  const int npan = (Mmax - 1 + TNB - 1) / TNB;
  for (int pi = npan - 1; pi >= 0; --pi) {
    const int p = pi * TNB;
    std::vector<Gemm> g1, g2, g3;
    for (const Eigh& e : es) {
      if (e.M - 1 <= p) continue;
      EighWs w = carve(e.work, e.M);
      const int nb = std::min(TNB, e.M - 1 - p), rows = e.M - p - 1;  // v rows p+1 .. M-1
      const double* Vp = w.Vc + (size_t)e.M * p + (p + 1);
      // X = V_p' Z(p+1:, :)   (nb x M)
      g1.push_back(Gemm{Vp, e.A + (p + 1), w.X, nb, e.M, rows, e.M, e.lda, TNB, 1.0, 0.0, 0});
      // Y = T_p X
      g2.push_back(Gemm{w.T + (size_t)pi * TNB * TNB, w.X, w.Y, nb, e.M, nb, TNB, TNB, TNB, 1.0, 0.0, 0});
      // Z(p+1:, :) -= V_p Y
      g3.push_back(Gemm{Vp, w.Y, e.A + (p + 1), rows, e.M, nb, e.M, TNB, e.lda, -1.0, 1.0, 0});
    }
    gemm(S, st, true, false, g1);
    gemm(S, st, false, false, g2);
    gemm(S, st, false, false, g3);
  }
  hipLaunchKernelGGL(k_reverse_cols, dim3(n, 64), dim3(256), 0, st, de);
  LC(hipGetLastError());
  phase(4);
}

}  // namespace oila
