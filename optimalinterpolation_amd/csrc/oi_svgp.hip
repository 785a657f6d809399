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

// Cholesky (lower, in place) of the M x M matrix A (ld M) in LDS; false if not PD
__device__ bool chol_lds(double* A, int M, int* flag) {
  if (threadIdx.x == 0) *flag = 0;
  __syncthreads();
  for (int j = 0; j < M; ++j) {
    if (threadIdx.x == 0) {
      const double d = A[j * M + j];
      if (!(d > 0.0)) *flag = 1;
      A[j * M + j] = sqrt(d);
    }
    __syncthreads();
    const double ljj = A[j * M + j];
    for (int i = j + 1 + threadIdx.x; i < M; i += (int)blockDim.x) A[i * M + j] /= ljj;
    __syncthreads();
    // trailing update of the lower triangle: A[i][k] -= L[i][j] L[k][j], j < k <= i
    const int rem = M - j - 1;
    for (int e = threadIdx.x; e < rem * rem; e += (int)blockDim.x) {
      const int i = j + 1 + e / rem, k = j + 1 + e % rem;
      if (k <= i) A[i * M + k] -= A[i * M + j] * A[k * M + j];
    }
    __syncthreads();
  }
  // zero the strict upper triangle
  for (int e = threadIdx.x; e < M * M; e += (int)blockDim.x)
    if (e % M > e / M) A[e] = 0.0;
  __syncthreads();
  return *flag == 0;
}

// Li = L^-1 (lower), one column per thread (forward substitution)
__device__ void trinv_lds(const double* L, double* Li, int M) {
  for (int e = threadIdx.x; e < M * M; e += (int)blockDim.x) Li[e] = 0.0;
  __syncthreads();
  for (int c = threadIdx.x; c < M; c += (int)blockDim.x) {
    Li[c * M + c] = 1.0 / L[c * M + c];
    for (int i = c + 1; i < M; ++i) {
      double s = 0.0;
      for (int k = c; k < i; ++k) s += L[i * M + k] * Li[k * M + c];
      Li[i * M + c] = -s / L[i * M + i];
    }
  }
  __syncthreads();
}

struct Shape {
  int M, B, P, nlog;
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

__host__ __device__ inline size_t carve_doubles(int M, int B, bool panels) {
  return (size_t)(panels ? 3 * M * M + 2 * M * B : 4 * M * M) + 6 * B + 21 * M + 128 + 17;
}

__device__ inline Lds carve(double* base, int M, int B, bool panels) {
  Lds s;
  double* p = base;
  s.L = p; p += M * M;
  s.Li = p; p += M * M;
  s.T2 = p; p += M * M;
  if (panels) {
    s.PA = p; p += M * B;
    s.P3 = p; p += M * B;
    s.T3 = s.PA;  // M <= B guaranteed by the host
  } else {
    s.PA = s.P3 = nullptr;
    s.T3 = p; p += M * M;
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

inline size_t lds_bytes(int M, int B, bool panels) { return carve_doubles(M, B, panels) * 8 + 16; }
constexpr size_t LDS_MAX = 160 * 1024;

// One minibatch: loss (always) and, if grad, the gradient into g[P].
// th: parameters; X/Y: the cell's rows; rows: stream batch number.
// Scratch (global, per cell): X1, X3 [M*B].  Returns the loss.
__device__ double step(const double* __restrict__ th, const double* __restrict__ X,
                       const double* __restrict__ Y, int64_t n, uint64_t seed, int64_t batchno,
                       const Shape& sh, Lds& s, double* __restrict__ X1, double* __restrict__ X2,
                       double* __restrict__ X3, double* __restrict__ g, bool grad, bool* ok) {
  const int M = sh.M, B = sh.B, tid = threadIdx.x;
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
  // K_uu + jitter -> L, Cholesky, L^-1
  for (int e = tid; e < M * M; e += (int)blockDim.x) {
    const int i = e / M, j = e % M;
    double ee;
    s.L[e] = var * m32(s.Zs + i * 3, s.Zs + j * 3, ee) + (i == j ? JITTER : 0.0);
  }
  __syncthreads();
  tmark(s, 1);
  if (!chol_lds(s.L, M, s.flag)) *ok = false;
  tmark(s, 2);
  trinv_lds(s.L, s.Li, M);
  tmark(s, 3);
  // K_uf -> X1 ; A = Li K_uf -> X2  (row-major M x B)
  for (int e = tid; e < M * B; e += (int)blockDim.x) {
    const int m = e / B, b = e % B;
    double ee;
    X1[e] = var * m32(s.Zs + m * 3, s.Xb + b * 3, ee);
  }
  __syncthreads();
  for (int e = tid; e < M * B; e += (int)blockDim.x) {
    const int m = e / B, b = e % B;
    double a = 0.0;
    for (int k = 0; k <= m; ++k) a += s.Li[m * M + k] * X1[k * B + b];
    X2[e] = a;
  }
  __syncthreads();
  tmark(s, 4);
  // SA = S' A -> X3 : SA[k][b] = sum_{m >= k} S[m][k] A[m][b]
  for (int e = tid; e < M * B; e += (int)blockDim.x) {
    const int k = e / B, b = e % B;
    double a = 0.0;
    for (int m = k; m < M; ++m) a += St[tri_index(m, k)] * X2[m * B + b];
    X3[e] = a;
  }
  __syncthreads();
  // per row: mu, fvar, residual terms
  const double scale = (double)n / (double)B;
  double part[3] = {0.0, 0.0, 0.0};  // sum ve, g_s2 partial, unused
  for (int b = tid; b < B; b += (int)blockDim.x) {
    double mu = 0.0, aa = 0.0, ss = 0.0;
    for (int m = 0; m < M; ++m) {
      const double a = X2[m * B + b], sa = X3[m * B + b];
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
    for (int k = 0; k <= m; ++k) ssa += St[tri_index(m, k)] * X3[k * B + b];
    X1[e] = s.q[m] * s.gmu[b] - 2.0 * X2[e] * gv + 2.0 * ssa * gv;
  }
  for (int m = tid; m < M; m += (int)blockDim.x) {
    double a = 0.0;
    for (int b = 0; b < B; ++b) a += X2[m * B + b] * s.gmu[b];
    s.gq[m] = a + s.q[m];
  }
  // Sbar (lower) straight into the gradient: 2 sum_b A[m][b] gv SA[k][b] + S - diag(1/S)
  double* gS = g + 6 + 4 * M;
  for (int e = tid; e < ntri; e += (int)blockDim.x) {
    int i = (int)((sqrt(8.0 * e + 1.0) - 1.0) / 2.0);
    while (tri_index(i, 0) > e) --i;
    while (tri_index(i + 1, 0) <= e) ++i;
    const int j = e - tri_index(i, 0);
    double a = 0.0;
    for (int b = 0; b < B; ++b) a += X2[i * B + b] * X3[j * B + b];
    double v = 2.0 * gv * a + St[e];
    if (i == j) v -= 1.0 / St[e];
    gS[e] = v;
  }
  __syncthreads();
  tmark(s, 6);
  // Kfbar = Li' Abar -> X3 : Kfbar[m][b] = sum_{k >= m} Li[k][m] Abar[k][b]
  for (int e = tid; e < M * B; e += (int)blockDim.x) {
    const int m = e / B, b = e % B;
    double a = 0.0;
    for (int k = m; k < M; ++k) a += s.Li[k * M + m] * X1[k * B + b];
    X3[e] = a;
  }
  __syncthreads();
  tmark(s, 7);
  // Lbar = tril(-Kfbar A') -> T2
  for (int e = tid; e < M * M; e += (int)blockDim.x) {
    const int i = e / M, j = e % M;
    double a = 0.0;
    if (j <= i)
      for (int b = 0; b < B; ++b) a += X3[i * B + b] * X2[j * B + b];
    s.T2[e] = j <= i ? -a : 0.0;
  }
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
        const double kb = X3[m * B + b];
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
    s.L[e] = var * m32(s.Zs + i * 3, s.Zs + j * 3, ee) + (i == j ? JITTER : 0.0);
  }
  __syncthreads();
  if (!chol_lds(s.L, M, s.flag)) *ok = false;
  // k_us -> T2[0..M) ; a = L^-1 k_us -> T3[0..M) by forward substitution (thread 0; M small)
  double* ku = s.T2;
  double* av = s.T3;
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
  Lds s = carve(lds, M, B, panels != 0);
  const int64_t n = offs[c + 1] - offs[c];
  const double* X = xyt + offs[c] * 3;
  const double* Y = y + offs[c];
  double* th = theta + c * P;
  double* m1 = mom + c * 2 * P;
  double* m2 = m1 + P;
  double* g = grad + c * P;
  double* X1 = scratch + c * 3 * (int64_t)M * B;
  double* X2 = panels ? s.PA : X1 + (int64_t)M * B;
  double* X3 = panels ? s.P3 : X1 + 2 * (int64_t)M * B;
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
        dsc((size_t)ncell * 3 * M * batch * 8), dxs((size_t)ncell * 3 * 8), dpred((size_t)ncell * 2 * 8),
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
    Shape sh{M, batch, P, nlog};
    const bool timing = getenv("OI_SVGP_TIMING") && atoi(getenv("OI_SVGP_TIMING")) != 0;
    Buf dtd(timing ? 16 * 8 : 0);
    if (timing) HC(hipMemsetAsync(dtd.p, 0, 16 * 8, st));
    // panels in LDS when they fit (OI_SVGP_PANELS=0 forces the global scratch)
    bool panels = M <= batch && lds_bytes(M, batch, true) <= LDS_MAX;
    if (const char* e = getenv("OI_SVGP_PANELS")) panels = panels && atoi(e) != 0;
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
                       panels ? 1 : 0, dtd.as<unsigned long long>());
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
      fprintf(stderr, "svgp phase cycles (cell 0, threads %d, panels %d):", nt, (int)panels);
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
