// Sparse variational GP of the dev notebook (dev/sparseGP_example.ipynb code
// cell 5 -- abbreviated NB2): GPflow SVGP (Matern32, Gaussian likelihood,
// Constant mean, whitened, full lower-triangular q_sqrt, trainable inducing
// inputs) trained by TF2 Adam on minibatches, then predict_f at the target.
// SURVEY.md §8f row 4 (second half).  Restated algorithm and its deviations:
// oracle/svgp_oracle.py (the CPU checker this kernel is tested against).
//
// MI355X shape of the problem: per cell M ~ 50 inducing points and B ~ 100
// rows per minibatch, 10 000 dependent Adam steps.  Every step is a chain of
// M x M x B products, an M x M Cholesky and its reverse-mode adjoint -- far too
// small to fill a GPU per cell and far too many steps to launch one kernel per
// step.  So ONE workgroup owns ONE cell for its WHOLE training run: a single
// launch covers all cells and all iterations (grid = cells, dealt round-robin
// over the 8 XCDs by the hardware), the M x M factors live in LDS, the M x B
// panels in a per-cell global scratch that stays in L2, and the parameters and
// Adam moments in global memory touched once per step.  No host round trips.
//
// Per step (A = L^-1 K_uf, L = chol(K_uu + 1e-6 I), S = q_sqrt, B rows):
//   forward : mu = c + A'q,  SA = S'A,  fvar = kvar - |A|^2 + |SA|^2
//   loss    : -(n/B) sum_b [-log(2pi)/2 - log(s2)/2 - ((y-mu)^2 + fvar)/(2 s2)] + KL
//   reverse : Abar = q gmu' - 2 A gv + 2 S SA gv;  Sbar = tril(2 (A gv) SA' + S - diag(1/S_ii))
//             Kfbar = L^-T Abar;  Lbar = tril(-Kfbar A');  P = Phi(L' Lbar)
//             Kbar = L^-T (P + P') L^-1 / 2  (Cholesky adjoint)
//             dk/dr2 = -(3/2) var e^{-sqrt3 r} -> lengthscales, Z, var
//   Adam on the unconstrained parameters (softplus transforms).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/oi.h"

extern "C" int oi_set_last_error(int code, const char* msg);  // oi_engine.cpp
extern "C" void oi_profile_add(const char* name, int64_t launches, double ms, double flops,
                               double bytes);  // oi_engine.cpp

namespace {

constexpr int NT_MAX = 1024;  // threads per workgroup (one cell); launched with OI_SVGP_THREADS
constexpr int MMAX = 64;      // inducing points per cell
constexpr int BMAX = 256;     // minibatch rows
constexpr double SQRT3 = 1.7320508075688772;
constexpr double JITTER = 1e-6;
constexpr double LIK_LOWER = 1e-6;
constexpr double LOG2PI = 1.8378770664093453;

// ------------------------------------------------------------ minibatches
__device__ __host__ inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  uint64_t z = x;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// keyed bijection of [0, n): 4-round Feistel on 2h bits, cycle-walked
// (oracle/svgp_oracle.py permute)
__device__ inline int64_t permute(uint64_t i, uint64_t n, uint64_t seed, uint64_t epoch) {
  int h = 1;
  while ((1ull << (2 * h)) < n) ++h;
  const uint64_t mask = (1ull << h) - 1;
  uint64_t key[4];
  for (int j = 0; j < 4; ++j) key[j] = splitmix64(seed * 0x9E3779B97F4A7C15ull + (epoch * 4 + j + 1));
  uint64_t x = i;
  for (;;) {  // terminates: a bijection of [0, 4^h) with 4^h < 4n
    uint64_t L = x >> h, R = x & mask;
    for (int j = 0; j < 4; ++j) {
      const uint64_t t = L ^ (splitmix64(R ^ key[j]) & mask);
      L = R;
      R = t;
    }
    x = (L << h) | R;
    if (x < n) return (int64_t)x;
  }
}

__device__ inline double softplus(double x) {  // np.logaddexp(0, x)
  return fmax(x, 0.0) + log1p(exp(-fabs(x)));
}
__device__ inline double sigmoid(double x) { return 0.5 * (1.0 + tanh(0.5 * x)); }

// ------------------------------------------------------------ block helpers
// sum over the workgroup (fixed order: lanes by shuffle tree, then waves in
// index order); every thread gets the total.  red holds >= waves * NV doubles
template <int NV>
__device__ inline void block_sum(double (&v)[NV], double* red) {
  for (int q = 0; q < NV; ++q)
    for (int o = 32; o > 0; o >>= 1) v[q] += __shfl_down(v[q], o, 64);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0)
    for (int q = 0; q < NV; ++q) red[w * NV + q] = v[q];
  __syncthreads();
  for (int q = 0; q < NV; ++q) {
    double t = red[q];
    for (int k = 1; k < nw; ++k) t += red[k * NV + q];
    v[q] = t;
  }
  __syncthreads();
}

// GPflow Matern32 pieces for one pair of 3-vectors (already divided by ls):
// r2 = |a|^2 + |b|^2 - 2 a.b clamped at 0 (GPflow's square_distance),
// r = sqrt(max(r2, 1e-36)); returns k/var = (1 + sqrt3 r) e, writes e
__device__ inline double m32(const double* a, const double* b, double& e) {
  const double sa = a[0] * a[0] + a[1] * a[1] + a[2] * a[2];
  const double sb = b[0] * b[0] + b[1] * b[1] + b[2] * b[2];
  const double ab = a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
  double r2 = (sa + sb) - 2.0 * ab;
  r2 = r2 > 0.0 ? r2 : 0.0;
  const double r = sqrt(r2 > 1e-36 ? r2 : 1e-36);
  e = exp(-SQRT3 * r);
  return (1.0 + SQRT3 * r) * e;
}

// L = chol(W) for the symmetric M x M matrix W (row-major, LDS; its lower
// triangle is overwritten).  Right-looking, one barrier per column: in step j
// every thread reads column j of W (final for this step) and scales it on the
// fly by 1/sqrt(a_jj) (as LAPACK dpotf2 does), writing L's column j and the
// trailing lower triangle.  Returns false if a pivot is not positive.
// (A one-wave variant with lane-owned rows and no block barriers measured 3x
// slower: each of its ~M^2/2 shuffle + LDS read-modify-write steps is exposed
// latency.)
__device__ bool chol_lds(double* W, double* L, int M, int* flag) {
  const int nt = (int)blockDim.x;
  for (int e = threadIdx.x; e < M * M; e += nt) L[e] = 0.0;
  if (threadIdx.x == 0) *flag = 0;
  __syncthreads();
  for (int j = 0; j < M; ++j) {
    const double d = W[j * M + j];
    const double ljj = sqrt(d), rj = 1.0 / ljj;
    if (threadIdx.x == 0 && !(d > 0.0)) *flag = 1;
    const int rem = M - j - 1;
    for (int e = threadIdx.x; e < rem * rem + rem + 1; e += nt) {
      if (e < rem * rem) {  // W[i][k] -= l_ij l_kj, j < k <= i
        const int i = j + 1 + e / rem, k = j + 1 + e % rem;
        if (k <= i) W[i * M + k] -= (W[i * M + j] * rj) * (W[k * M + j] * rj);
      } else {  // column j of L
        const int i = j + (e - rem * rem);
        L[i * M + j] = i == j ? ljj : W[i * M + j] * rj;
      }
    }
    __syncthreads();
  }
  return *flag == 0;
}

// Li = L^-1 (lower): one wave per column c, lane i holding x_i of the forward
// substitution L x = e_c (M <= 64); U (M x M scratch) receives L' so the
// column reads L[i][k] (fixed k, lanes over i) are contiguous
__device__ void trinv_lds(const double* L, double* Li, double* U, int M) {
  const int nt = (int)blockDim.x;
  for (int e = threadIdx.x; e < M * M; e += nt) {
    U[(e % M) * M + e / M] = L[e];
    Li[e] = 0.0;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = nt >> 6;
  for (int c = w; c < M; c += nw) {
    double x = lane == c ? 1.0 : 0.0;
    for (int k = c; k < M; ++k) {
      const double xk = __shfl(x, k, 64) / U[k * M + k];
      if (lane == k) x = xk;
      if (lane > k && lane < M) x -= U[k * M + lane] * xk;
    }
    if (lane >= c && lane < M) Li[lane * M + c] = x;
  }
  __syncthreads();
}

// Lower-triangle panel product, 4 outputs of one row per thread (one load of
// P[i][.] feeds 4 independent FMA chains): for j <= i,
//   f(i, j, sum_b P[i][b] Q[j][b])
template <class F>
__device__ inline void tri_pq(const double* P, const double* Q, int M, int B, int LB, F f) {
  int items = 0;
  for (int i = 0; i < M; ++i) items += i / 4 + 1;
  for (int it = threadIdx.x; it < items; it += (int)blockDim.x) {
    int i = 0, r = it;
    while (r >= i / 4 + 1) {
      r -= i / 4 + 1;
      ++i;
    }
    const int j0 = 4 * r, nj = (i - j0 + 1) < 4 ? (i - j0 + 1) : 4;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    const double* pi = P + i * LB;
    const double* q0 = Q + j0 * LB;
    for (int b = 0; b < B; ++b) {
      const double pv = pi[b];
      a0 += pv * q0[b];
      if (nj > 1) a1 += pv * q0[LB + b];
      if (nj > 2) a2 += pv * q0[2 * LB + b];
      if (nj > 3) a3 += pv * q0[3 * LB + b];
    }
    f(i, j0, a0);
    if (nj > 1) f(i, j0 + 1, a1);
    if (nj > 2) f(i, j0 + 2, a2);
    if (nj > 3) f(i, j0 + 3, a3);
  }
}

struct Shape {
  int M, B, P, nlog, LB;  // LB: panel row stride (B rounded up to odd: fewer LDS bank conflicts)
};

// parameter vector layout (oracle Params.flat): ls_raw[3], var_raw, lik_raw, c,
// Z[M*3], q_mu[M], tril(S) row-major [M(M+1)/2]
__device__ inline int tri_index(int i, int j) { return i * (i + 1) / 2 + j; }  // i >= j

// LDS layout (doubles): L, Li, T2, T3 (M*M each); Xb (B*3), yb, mu, gmu (B each);
// Zs (M*3, scaled), q, gq (M), gZ (M*3), gzp (4*M*3), red[128].
// Panel mode (host-chosen when it fits the 160 KB LDS): the M x B panels A
// and SA/Kfbar live in LDS too (PA, P3), and T3 -- used only after A is dead --
// aliases PA.  Otherwise they live in the per-cell global scratch.
struct Lds {
  double *L, *Li, *T2, *T3, *PA, *P3, *Xb, *yb, *mu, *gmu, *Zs, *q, *gq, *gZ, *gzp, *red;
  int* flag;
  unsigned long long* tacc;  // OI_SVGP_TIMING: per-phase clock64 sums (thread 0), [16] + last
};

// phase clock (diagnostics only: OI_SVGP_TIMING=1 prints block 0's per-phase cycles)
__device__ inline void tmark(Lds& s, int k) {
  if (threadIdx.x == 0) {
    const unsigned long long t = clock64();
    s.tacc[k] += t - s.tacc[16];
    s.tacc[16] = t;
  }
}

// mode 1: panels in LDS (T3 aliases PA); mode 0: panels in global scratch, T3 in
// LDS; mode 2 ("lean"): panels and T3 in global scratch (T3 aliases the Abar
// panel, dead by then) -- the smallest LDS footprint, so two cells share a CU
__host__ __device__ inline int panel_ld(int B) { return B % 2 ? B : B + 1; }

__host__ __device__ inline size_t carve_doubles(int M, int B, int mode) {
  const int LB = panel_ld(B);
  const size_t mats = mode == 1 ? 3 * M * M + 2 * M * LB : (mode == 0 ? 4 * M * M : 3 * M * M);
  return mats + 6 * B + 21 * M + 128 + 17;
}

__device__ inline Lds carve(double* base, int M, int B, int mode) {
  const bool panels = mode == 1;
  Lds s;
  double* p = base;
  s.L = p; p += M * M;
  s.Li = p; p += M * M;
  s.T2 = p; p += M * M;
  if (panels) {
    s.PA = p; p += M * panel_ld(B);
    s.P3 = p; p += M * panel_ld(B);
    s.T3 = s.PA;  // M <= B guaranteed by the host
  } else if (mode == 0) {
    s.PA = s.P3 = nullptr;
    s.T3 = p; p += M * M;
  } else {
    s.PA = s.P3 = nullptr;
    s.T3 = nullptr;  // set to the Abar panel by the kernel
  }
  s.Xb = p; p += B * 3;
  s.yb = p; p += B;
  s.mu = p; p += B;
  s.gmu = p; p += B;
  s.Zs = p; p += M * 3;
  s.q = p; p += M;
  s.gq = p; p += M;
  s.gZ = p; p += M * 3;
  s.gzp = p; p += 12 * M;  // 4 parts x M x 3
  s.red = p; p += 128;
  s.tacc = (unsigned long long*)p; p += 17;
  s.flag = (int*)p;
  return s;
}

inline size_t lds_bytes(int M, int B, int mode) { return carve_doubles(M, B, mode) * 8 + 16; }
constexpr size_t LDS_MAX = 160 * 1024;

// One minibatch: loss (always) and, if grad, the gradient into g[P].
// th: parameters; X/Y: the cell's rows; rows: stream batch number.
// Scratch (global, per cell): X1, X3 [M*B].  Returns the loss.
__device__ double step(const double* __restrict__ th, const double* __restrict__ X,
                       const double* __restrict__ Y, int64_t n, uint64_t seed, int64_t batchno,
                       const Shape& sh, Lds& s, double* __restrict__ X1, double* __restrict__ X2,
                       double* __restrict__ X3, double* __restrict__ g, bool grad, bool* ok) {
  const int M = sh.M, B = sh.B, LB = sh.LB, tid = threadIdx.x;
  const double ls[3] = {softplus(th[0]), softplus(th[1]), softplus(th[2])};
  const double var = softplus(th[3]), s2 = softplus(th[4]) + LIK_LOWER, c = th[5];
  const double* Z = th + 6;
  const double* qg = th + 6 + 3 * M;
  const double* St = th + 6 + 4 * M;  // tril(S), row-major
  // gather the minibatch; scaled inducing inputs; q
  for (int b = tid; b < B; b += (int)blockDim.x) {
    const uint64_t pos = (uint64_t)batchno * B + b;
    const int64_t r = permute(pos % (uint64_t)n, (uint64_t)n, seed, pos / (uint64_t)n);
    for (int d = 0; d < 3; ++d) s.Xb[b * 3 + d] = X[r * 3 + d] / ls[d];
    s.yb[b] = Y[r];
  }
  for (int m = tid; m < M; m += (int)blockDim.x) {
    for (int d = 0; d < 3; ++d) s.Zs[m * 3 + d] = Z[m * 3 + d] / ls[d];
    s.q[m] = qg[m];
  }
  __syncthreads();
  tmark(s, 0);
  // K_uu + jitter -> T2 (working copy), L = chol, Li = L^-1, then S dense -> T2
  for (int e = tid; e < M * M; e += (int)blockDim.x) {
    const int i = e / M, j = e % M;
    double ee;
    s.T2[e] = var * m32(s.Zs + i * 3, s.Zs + j * 3, ee) + (i == j ? JITTER : 0.0);
  }
  __syncthreads();
  tmark(s, 1);
  if (!chol_lds(s.T2, s.L, M, s.flag)) *ok = false;
  tmark(s, 2);
  trinv_lds(s.L, s.Li, s.T2, M);
  double* Sd = s.T2;  // S (lower, dense) until Lbar overwrites T2
  for (int e = tid; e < M * M; e += (int)blockDim.x) {
    const int i = e / M, j = e % M;
    Sd[e] = j <= i ? St[tri_index(i, j)] : 0.0;
  }
  __syncthreads();
  tmark(s, 3);
  // K_uf -> X1 ; A = Li K_uf -> X2  (row-major M x B, row stride LB)
  for (int e = tid; e < M * B; e += (int)blockDim.x) {
    const int m = e / B, b = e % B;
    double ee;
    X1[m * LB + b] = var * m32(s.Zs + m * 3, s.Xb + b * 3, ee);
  }
  __syncthreads();
  for (int e = tid; e < M * B; e += (int)blockDim.x) {
    const int m = e / B, b = e % B;
    double a = 0.0;
    for (int k = 0; k <= m; ++k) a += s.Li[m * M + k] * X1[k * LB + b];
    X2[m * LB + b] = a;
  }
  __syncthreads();
  tmark(s, 4);
  // SA = S' A -> X3 : SA[k][b] = sum_{m >= k} S[m][k] A[m][b]
  for (int e = tid; e < M * B; e += (int)blockDim.x) {
    const int k = e / B, b = e % B;
    double a = 0.0;
    for (int m = k; m < M; ++m) a += Sd[m * M + k] * X2[m * LB + b];
    X3[k * LB + b] = a;
  }
  __syncthreads();
  // per row: mu, fvar, residual terms
  const double scale = (double)n / (double)B;
  double part[3] = {0.0, 0.0, 0.0};  // sum ve, g_s2 partial, unused
  for (int b = tid; b < B; b += (int)blockDim.x) {
    double mu = 0.0, aa = 0.0, ss = 0.0;
    for (int m = 0; m < M; ++m) {
      const double a = X2[m * LB + b], sa = X3[m * LB + b];
      mu += a * s.q[m];
      aa += a * a;
      ss += sa * sa;
    }
    mu = c + mu;
    const double fv = (var - aa) + ss;
    const double res = s.yb[b] - mu;
    part[0] += -0.5 * LOG2PI - 0.5 * log(s2) - 0.5 * (res * res + fv) / s2;
    part[1] += -0.5 / s2 + 0.5 * (res * res + fv) / (s2 * s2);
    s.mu[b] = mu;
    s.gmu[b] = -scale * res / s2;
  }
  // KL = (q.q + |S|^2 - M - sum log S_ii^2) / 2
  double kl[1] = {0.0};
  const int ntri = M * (M + 1) / 2;
  for (int e = tid; e < ntri; e += (int)blockDim.x) kl[0] += St[e] * St[e];
  for (int m = tid; m < M; m += (int)blockDim.x) {
    const double d = St[tri_index(m, m)];
    kl[0] += s.q[m] * s.q[m] - log(d * d) - 1.0;
  }
  block_sum<3>(part, s.red);
  block_sum<1>(kl, s.red);
  const double loss = -(part[0] * scale - 0.5 * kl[0]);
  tmark(s, 5);
  if (!grad) return loss;
  const double gv = scale / (2.0 * s2);
  const double g_s2 = -scale * part[1];
  // Abar -> X1 (K_uf no longer needed) ; gq
  for (int e = tid; e < M * B; e += (int)blockDim.x) {
    const int m = e / B, b = e % B;
    double ssa = 0.0;  // (S SA)[m][b] = sum_{k <= m} S[m][k] SA[k][b]
    for (int k = 0; k <= m; ++k) ssa += Sd[m * M + k] * X3[k * LB + b];
    X1[m * LB + b] = s.q[m] * s.gmu[b] - 2.0 * X2[m * LB + b] * gv + 2.0 * ssa * gv;
  }
  // gq[m] = A[m][.] . gmu + q[m]: 16 lanes per m, shuffle-reduced in fixed order
  for (int m0 = tid >> 4; m0 < ((M + 3) / 4) * 4; m0 += (int)blockDim.x >> 4) {
    const int m = m0, part = tid & 15;
    double a = 0.0;
    if (m < M)
      for (int b = part; b < B; b += 16) a += X2[m * LB + b] * s.gmu[b];
    for (int o = 8; o > 0; o >>= 1) a += __shfl_down(a, o, 16);
    if (part == 0 && m < M) s.gq[m] = a + s.q[m];
  }
  // Sbar (lower) straight into the gradient: 2 sum_b A[m][b] gv SA[k][b] + S - diag(1/S)
  double* gS = g + 6 + 4 * M;
  tri_pq(X2, X3, M, B, LB, [&](int i, int j, double a) {
    const int e = tri_index(i, j);
    double v = 2.0 * gv * a + St[e];
    if (i == j) v -= 1.0 / St[e];
    gS[e] = v;
  });
  __syncthreads();
  tmark(s, 6);
  // Kfbar = Li' Abar -> X3 : Kfbar[m][b] = sum_{k >= m} Li[k][m] Abar[k][b]
  for (int e = tid; e < M * B; e += (int)blockDim.x) {
    const int m = e / B, b = e % B;
    double a = 0.0;
    for (int k = m; k < M; ++k) a += s.Li[k * M + m] * X1[k * LB + b];
    X3[m * LB + b] = a;
  }
  __syncthreads();
  tmark(s, 7);
  // Lbar = tril(-Kfbar A') -> T2
  for (int e = tid; e < M * M; e += (int)blockDim.x)
    if (e % M > e / M) s.T2[e] = 0.0;
  tri_pq(X3, X2, M, B, LB, [&](int i, int j, double a) { s.T2[i * M + j] = -a; });
  __syncthreads();
  tmark(s, 8);
  // P = Phi(L' Lbar) -> T3 : P[i][j] = sum_{k >= i} L[k][i] Lbar[k][j], i >= j, diag / 2
  for (int e = tid; e < M * M; e += (int)blockDim.x) {
    const int i = e / M, j = e % M;
    double a = 0.0;
    if (j <= i)
      for (int k = i; k < M; ++k) a += s.L[k * M + i] * s.T2[k * M + j];
    s.T3[e] = j < i ? a : (j == i ? 0.5 * a : 0.0);
  }
  __syncthreads();
  // Ps = P + P' -> T2
  for (int e = tid; e < M * M; e += (int)blockDim.x) {
    const int i = e / M, j = e % M;
    s.T2[e] = s.T3[i * M + j] + s.T3[j * M + i];
  }
  __syncthreads();
  // T3 = Ps Li : sum_{k >= j} Ps[i][k] Li[k][j]
  for (int e = tid; e < M * M; e += (int)blockDim.x) {
    const int i = e / M, j = e % M;
    double a = 0.0;
    for (int k = j; k < M; ++k) a += s.T2[i * M + k] * s.Li[k * M + j];
    s.T3[e] = a;
  }
  __syncthreads();
  // Kbar = Li' T3 / 2 -> T2 : sum_{k >= i} Li[k][i] T3[k][j]
  for (int e = tid; e < M * M; e += (int)blockDim.x) {
    const int i = e / M, j = e % M;
    double a = 0.0;
    for (int k = i; k < M; ++k) a += s.Li[k * M + i] * s.T3[k * M + j];
    s.T2[e] = 0.5 * a;
  }
  __syncthreads();
  tmark(s, 9);
  // kernel derivatives: 4 threads per inducing row m (quarter of b's and j's each)
  double acc[4] = {0.0, 0.0, 0.0, 0.0};  // g_var, g_ls[3] (before the -2/ls^3 factor)
  {
    const int m = tid & 63, part4 = tid >> 6, nparts = 4;
    double gz[3] = {0.0, 0.0, 0.0};
    if (m < M && part4 < nparts) {
      const double* zm = s.Zs + m * 3;
      for (int b = part4; b < B; b += nparts) {
        double e;
        const double kk = var * m32(zm, s.Xb + b * 3, e);
        const double kb = X3[m * LB + b];
        const double W = kb * (-1.5 * var) * e;
        acc[0] += kb * kk / var;
        for (int d = 0; d < 3; ++d) {
          const double diff = (zm[d] - s.Xb[b * 3 + d]) * ls[d];  // unscaled Z - X
          acc[1 + d] += W * diff * diff;
          gz[d] += W * diff;
        }
      }
      for (int j = part4; j < M; j += nparts) {
        double e;
        const double kk = var * m32(zm, s.Zs + j * 3, e);
        const double kb = s.T2[m * M + j];
        const double W = kb * (-1.5 * var) * e;
        acc[0] += kb * kk / var;
        for (int d = 0; d < 3; ++d) {
          const double diff = (zm[d] - s.Zs[j * 3 + d]) * ls[d];
          acc[1 + d] += W * diff * diff;
          gz[d] += 2.0 * W * diff;
        }
      }
    }
    // gZ[m][d] = sum of the 4 parts * 2 / ls^2, fixed order
    if (m < M && part4 < nparts)
      for (int d = 0; d < 3; ++d) s.gzp[(part4 * M + m) * 3 + d] = gz[d];
    __syncthreads();
    if (tid < M)
      for (int d = 0; d < 3; ++d) {
        double t = s.gzp[tid * 3 + d];
        for (int k = 1; k < nparts; ++k) t += s.gzp[(k * M + tid) * 3 + d];
        s.gZ[tid * 3 + d] = t * (2.0 / (ls[d] * ls[d]));
      }
  }
  double gvsum[1] = {0.0};
  for (int b = tid; b < B; b += (int)blockDim.x) gvsum[0] += gv;
  block_sum<4>(acc, s.red);
  block_sum<1>(gvsum, s.red);
  if (tid == 0) {
    for (int d = 0; d < 3; ++d) g[d] = acc[1 + d] * (-2.0 / (ls[d] * ls[d] * ls[d])) * sigmoid(th[d]);
    g[3] = (gvsum[0] + acc[0]) * sigmoid(th[3]);
    g[4] = g_s2 * sigmoid(th[4]);
  }
  // g_c = sum gmu
  double gc[1] = {0.0};
  for (int b = tid; b < B; b += (int)blockDim.x) gc[0] += s.gmu[b];
  block_sum<1>(gc, s.red);
  if (tid == 0) g[5] = gc[0];
  for (int e = tid; e < 3 * M; e += (int)blockDim.x) g[6 + e] = s.gZ[e];
  for (int m = tid; m < M; m += (int)blockDim.x) g[6 + 3 * M + m] = s.gq[m];
  __syncthreads();
  tmark(s, 10);
  return loss;
}

// GPflow SVGP.predict_f at one target with the final parameters
__device__ void predict(const double* __restrict__ th, const double* xs, const Shape& sh, Lds& s,
                        double* out, bool* ok) {
  const int M = sh.M, tid = threadIdx.x;
  const double ls[3] = {softplus(th[0]), softplus(th[1]), softplus(th[2])};
  const double var = softplus(th[3]), c = th[5];
  const double* Z = th + 6;
  const double* St = th + 6 + 4 * M;
  for (int m = tid; m < M; m += (int)blockDim.x)
    for (int d = 0; d < 3; ++d) s.Zs[m * 3 + d] = Z[m * 3 + d] / ls[d];
  if (tid < 3) s.Xb[tid] = xs[tid] / ls[tid];
  __syncthreads();
  for (int e = tid; e < M * M; e += (int)blockDim.x) {
    const int i = e / M, j = e % M;
    double ee;
    s.T2[e] = var * m32(s.Zs + i * 3, s.Zs + j * 3, ee) + (i == j ? JITTER : 0.0);
  }
  __syncthreads();
  if (!chol_lds(s.T2, s.L, M, s.flag)) *ok = false;
  __syncthreads();
  // k_us -> T2[0..M) ; a = L^-1 k_us -> T3[0..M) by forward substitution (thread 0; M small)
  double* ku = s.T2;
  double* av = s.Li;
  for (int m = tid; m < M; m += (int)blockDim.x) {
    double ee;
    ku[m] = var * m32(s.Zs + m * 3, s.Xb, ee);
  }
  __syncthreads();
  if (tid == 0) {
    for (int i = 0; i < M; ++i) {
      double a = ku[i];
      for (int k = 0; k < i; ++k) a -= s.L[i * M + k] * av[k];
      av[i] = a / s.L[i * M + i];
    }
    double mean = 0.0, aa = 0.0, ss = 0.0;
    for (int m = 0; m < M; ++m) {
      mean += av[m] * th[6 + 3 * M + m];
      aa += av[m] * av[m];
    }
    for (int k = 0; k < M; ++k) {
      double sa = 0.0;
      for (int m = k; m < M; ++m) sa += St[tri_index(m, k)] * av[m];
      ss += sa * sa;
    }
    out[0] = c + mean;
    out[1] = (var - aa) + ss;
  }
  __syncthreads();
}

// One workgroup = one cell, the whole training run.
__global__ void __launch_bounds__(NT_MAX) k_svgp_train(
    const double* __restrict__ xyt, const double* __restrict__ y, const int64_t* __restrict__ offs,
    Shape sh, int iters, int log_every, uint64_t seed, double lr, double* __restrict__ theta,
    double* __restrict__ mom, double* __restrict__ grad, double* __restrict__ scratch,
    const double* __restrict__ xs, double* __restrict__ pred, double* __restrict__ elbo,
    int32_t* __restrict__ status, int panels, unsigned long long* __restrict__ tdbg) {
  extern __shared__ double lds[];
  const int64_t c = blockIdx.x;
  const int M = sh.M, B = sh.B, P = sh.P, tid = threadIdx.x;
  Lds s = carve(lds, M, B, panels);
  const int64_t n = offs[c + 1] - offs[c];
  const double* X = xyt + offs[c] * 3;
  const double* Y = y + offs[c];
  double* th = theta + c * P;
  double* m1 = mom + c * 2 * P;
  double* m2 = m1 + P;
  double* g = grad + c * P;
  const int64_t pan = (int64_t)M * sh.LB;
  double* X1 = scratch + c * 3 * pan;
  double* X2 = panels == 1 ? s.PA : X1 + pan;
  double* X3 = panels == 1 ? s.P3 : X1 + 2 * pan;
  if (panels == 2) s.T3 = X1;  // M <= B guaranteed by the host
  const uint64_t cseed = seed + (uint64_t)c;
  bool ok = true;
  if (tid < 17) s.tacc[tid] = 0;
  __syncthreads();
  if (tid == 0) s.tacc[16] = clock64();
  const double b1 = 0.9, b2 = 0.999, eps = 1e-7;
  double b1t = 1.0, b2t = 1.0;
  int64_t used = 0, nl = 0;
  for (int k = 0; k < iters; ++k) {
    step(th, X, Y, n, cseed, used, sh, s, X1, X2, X3, g, true, &ok);
    ++used;
    // TF2 Adam
    b1t *= b1;
    b2t *= b2;
    const double lr_t = lr * sqrt(1.0 - b2t) / (1.0 - b1t);
    for (int p = tid; p < P; p += (int)blockDim.x) {
      const double gp = g[p];
      const double mm = b1 * m1[p] + (1.0 - b1) * gp;
      const double vv = b2 * m2[p] + (1.0 - b2) * gp * gp;
      m1[p] = mm;
      m2[p] = vv;
      th[p] = th[p] - lr_t * mm / (sqrt(vv) + eps);
    }
    __syncthreads();
    tmark(s, 11);
    if (log_every > 0 && k % log_every == 0) {  // the notebook's -training_loss() on the next batch
      const double l = step(th, X, Y, n, cseed, used, sh, s, X1, X2, X3, g, false, &ok);
      ++used;
      if (tid == 0 && elbo) elbo[c * sh.nlog + nl] = -l;
      ++nl;
      __syncthreads();
    }
  }
  tmark(s, 12);
  predict(th, xs + c * 3, sh, s, pred + c * 2, &ok);
  if (tid == 0) status[c] = ok ? 0 : 1;
  if (tdbg && c == 0 && tid < 16) tdbg[tid] = s.tacc[tid];
}

struct HipErr {
  std::string msg;
};
#define HC(expr)                                                                            \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) throw HipErr{std::string(#expr) + ": " + hipGetErrorString(e_)}; \
  } while (0)

struct Buf {
  void* p = nullptr;
  explicit Buf(size_t bytes) {
    if (bytes) HC(hipMalloc(&p, bytes));
  }
  ~Buf() {
    if (p) (void)hipFree(p);
  }
  Buf(const Buf&) = delete;
  Buf& operator=(const Buf&) = delete;
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

double inv_softplus(double v) { return v + std::log(-std::expm1(-v)); }

}  // namespace

extern "C" int32_t oi_svgp_param_count(int32_t M) { return 6 + 4 * M + M * (M + 1) / 2; }

extern "C" int oi_svgp_batch(const double* xyt, const double* y, const int64_t* offs,
                             int64_t ncell, const double* Z0, int32_t M, const double* init,
                             int32_t batch, int32_t iterations, int32_t log_every, uint64_t seed,
                             double lr, const double* xs, double* pred, double* params,
                             double* elbo, int32_t* status, const oi_options* opts) {
  if (ncell < 0) return oi_set_last_error(OI_E_ARG, "negative ncell");
  if (ncell == 0) return 0;
  if (!xyt || !y || !offs || !Z0 || !init || !xs || !pred || !status)
    return oi_set_last_error(OI_E_ARG, "null pointer");
  if (M < 1 || M > MMAX) return oi_set_last_error(OI_E_ARG, "M must be in [1, 64]");
  if (batch < 1 || batch > BMAX) return oi_set_last_error(OI_E_ARG, "batch must be in [1, 256]");
  if (iterations < 0 || log_every < 0) return oi_set_last_error(OI_E_ARG, "negative count");
  if (!(lr > 0.0)) return oi_set_last_error(OI_E_ARG, "lr must be > 0");
  if (offs[0] != 0) return oi_set_last_error(OI_E_ARG, "offs[0] must be 0");
  for (int64_t c = 0; c < ncell; ++c) {
    if (offs[c + 1] - offs[c] < 1) return oi_set_last_error(OI_E_ARG, "every cell needs n >= 1");
    for (int q = 0; q < 5; ++q)
      if (!(init[c * 6 + q] > (q == 4 ? 1e-6 : 0.0)))
        return oi_set_last_error(OI_E_ARG, "lengthscales / variances must be > 0 (noise > 1e-6)");
  }
  oi_options o;
  oi_options_default(&o);
  if (opts) o = *opts;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return oi_set_last_error(OI_E_NODEV, "no HIP device available");
  if (o.device < 0 || o.device >= ndev) return oi_set_last_error(OI_E_ARG, "bad device ordinal");
  if (hipSetDevice(o.device) != hipSuccess) return oi_set_last_error(OI_E_HIP, "hipSetDevice failed");
  hipStream_t st = (hipStream_t)o.stream;
  try {
    const int P = oi_svgp_param_count(M);
    const int nlog = log_every > 0 ? (iterations + log_every - 1) / log_every : 0;
    const int64_t N = offs[ncell];
    // initial unconstrained parameters (GPflow: softplus transforms, q_mu = 0, q_sqrt = I)
    std::vector<double> th0((size_t)ncell * P, 0.0);
    for (int64_t c = 0; c < ncell; ++c) {
      double* t = th0.data() + c * P;
      const double* in = init + c * 6;
      for (int d = 0; d < 3; ++d) t[d] = inv_softplus(in[d]);
      t[3] = inv_softplus(in[3]);
      t[4] = inv_softplus(in[4] - LIK_LOWER);
      t[5] = in[5];
      for (int e = 0; e < 3 * M; ++e) t[6 + e] = Z0[c * 3 * M + e];
      for (int i = 0; i < M; ++i) t[6 + 4 * M + i * (i + 1) / 2 + i] = 1.0;
    }
    Buf dth((size_t)ncell * P * 8), dmom((size_t)ncell * 2 * P * 8), dg((size_t)ncell * P * 8),
        dsc((size_t)ncell * 3 * M * panel_ld(batch) * 8), dxs((size_t)ncell * 3 * 8), dpred((size_t)ncell * 2 * 8),
        delbo((size_t)ncell * (nlog ? nlog : 1) * 8), dst((size_t)ncell * 4), doffs((ncell + 1) * 8);
    Buf hx(o.device_inputs ? 0 : N * 3 * 8), hy(o.device_inputs ? 0 : N * 8);
    const double* dx = xyt;
    const double* dy = y;
    if (!o.device_inputs) {
      HC(hipMemcpyAsync(hx.p, xyt, N * 3 * 8, hipMemcpyHostToDevice, st));
      HC(hipMemcpyAsync(hy.p, y, N * 8, hipMemcpyHostToDevice, st));
      dx = hx.as<double>();
      dy = hy.as<double>();
    }
    HC(hipMemcpyAsync(dth.p, th0.data(), th0.size() * 8, hipMemcpyHostToDevice, st));
    HC(hipMemsetAsync(dmom.p, 0, (size_t)ncell * 2 * P * 8, st));
    HC(hipMemcpyAsync(dxs.p, xs, ncell * 3 * 8, hipMemcpyHostToDevice, st));
    HC(hipMemcpyAsync(doffs.p, offs, (ncell + 1) * 8, hipMemcpyHostToDevice, st));
    Shape sh{M, batch, P, nlog, panel_ld(batch)};
    const bool timing = getenv("OI_SVGP_TIMING") && atoi(getenv("OI_SVGP_TIMING")) != 0;
    Buf dtd(timing ? 16 * 8 : 0);
    if (timing) HC(hipMemsetAsync(dtd.p, 0, 16 * 8, st));
    // LDS layout mode (see carve): 1 when the panels fit, else 0; OI_SVGP_PANELS
    // overrides (0 / 1 / 2), falling back to 0 where the request cannot hold
    int panels = (M <= batch && lds_bytes(M, batch, 1) <= LDS_MAX) ? 1 : 0;
    if (const char* e = getenv("OI_SVGP_PANELS")) {
      const int want = atoi(e);
      panels = (want == 1 && panels == 1) ? 1 : ((want == 2 && M <= batch) ? 2 : 0);
    }
    const size_t lb = lds_bytes(M, batch, panels);
    HC(hipFuncSetAttribute((const void*)k_svgp_train, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)lb));
    // threads per cell (OI_SVGP_THREADS: 64..1024, multiple of 64); 1024 measured
    // fastest (more waves to hide the latency of the per-step dependency chains)
    int nt = 1024;
    if (const char* e = getenv("OI_SVGP_THREADS")) nt = atoi(e);
    nt = std::max(64, std::min(NT_MAX, nt / 64 * 64));
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    if (o.profile) {
      HC(hipEventCreate(&ev0));
      HC(hipEventCreate(&ev1));
      HC(hipEventRecord(ev0, st));
    }
    hipLaunchKernelGGL(k_svgp_train, dim3((unsigned)ncell), dim3(nt), lb, st, dx, dy,
                       doffs.as<int64_t>(), sh, iterations, log_every, seed, lr, dth.as<double>(),
                       dmom.as<double>(), dg.as<double>(), dsc.as<double>(), dxs.as<double>(),
                       dpred.as<double>(), nlog ? delbo.as<double>() : nullptr, dst.as<int32_t>(),
                       panels, dtd.as<unsigned long long>());
    HC(hipGetLastError());
    if (o.profile) {
      HC(hipEventRecord(ev1, st));
      HC(hipEventSynchronize(ev1));
      float ms = 0.f;
      HC(hipEventElapsedTime(&ms, ev0, ev1));
      (void)hipEventDestroy(ev0);
      (void)hipEventDestroy(ev1);
      // algorithmic flops per Adam step: the M x M x B products (A, S'A, S SA,
      // Sbar, Kfbar, Lbar: 4.5 x 2 M^2 B) and M^3 terms (chol, inverse, adjoint:
      // 5/3 x 2 M^3); logging passes are forward-only (~1/3 of a step)
      const double dM = M, dB = batch;
      const double fstep = 9.0 * dM * dM * dB + 10.0 / 3.0 * dM * dM * dM;
      const double nsteps = iterations + (double)nlog / 3.0;
      oi_profile_add("k_svgp_train", 1, ms, fstep * nsteps * (double)ncell, 0.0);
    }
    if (timing) {
      unsigned long long t[16];
      HC(hipMemcpyAsync(t, dtd.p, sizeof(t), hipMemcpyDeviceToHost, st));
      HC(hipStreamSynchronize(st));
      fprintf(stderr, "svgp phase cycles (cell 0, threads %d, mode %d):", nt, panels);
      for (int k = 0; k < 13; ++k) fprintf(stderr, " %d:%llu", k, t[k]);
      fprintf(stderr, "\n");
    }
    HC(hipMemcpyAsync(pred, dpred.p, ncell * 2 * 8, hipMemcpyDeviceToHost, st));
    HC(hipMemcpyAsync(status, dst.p, ncell * 4, hipMemcpyDeviceToHost, st));
    if (params) HC(hipMemcpyAsync(params, dth.p, (size_t)ncell * P * 8, hipMemcpyDeviceToHost, st));
    if (elbo && nlog)
      HC(hipMemcpyAsync(elbo, delbo.p, (size_t)ncell * nlog * 8, hipMemcpyDeviceToHost, st));
    HC(hipStreamSynchronize(st));
    return 0;
  } catch (const HipErr& e) {
    return oi_set_last_error(OI_E_HIP, e.msg.c_str());
  } catch (const std::bad_alloc&) {
    return oi_set_last_error(OI_E_NOMEM, "allocation failed");
  }
}
