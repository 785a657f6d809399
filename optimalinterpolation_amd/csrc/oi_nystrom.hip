// Nystrom-approximated GP of the reference notebook (GP_example.ipynb, code
// cell 1 -- abbreviated NB1): Nystroem, SMLII(approx=True, M) and
// GPR(approx=True, M) for a ragged batch of cells.
//
// Per cell, with n observations, M inducing rows sel (NB1 Nystroem draws them
// with np.random.seed(20); the caller passes them), Matern-3/2 kernel:
//
//   Kmm = K(x_sel, x_sel)            Knm = K(x, x_sel)            (kernels below)
//   s, u = eigh(Kmm); s[s<=0] = 1e-12; st = n s / M               (oila::eigh)
//   ut = sqrt(M/n) Knm u / s;  C = Vi ut = ut / sn2                (oila::gemm + kernel)
//   B = diag(1/st) + ut' C;  L = chol(B)                           (oila::gemm + cholesky)
//
// NB1 then forms alpha = L'^-1 L^-1 C' and Ki = Vi - C alpha (n x n).  Here
// the same quantities come from W' = C L^-T (n x M: a right-looking block
// triangular solve with the Cholesky's diagonal-block inverses):
//   C alpha = W'W,  A = Ki r = r/sn2 - W'(W r),  k*'Ki k* = |k*|^2/sn2 - |W k*|^2
// and, because D B D = H / sn2 for D = diag(sqrt(st)) and NB1's
// H = sn2 I + (sqrt(st) ut)'(sqrt(st) ut),
//   slogdet(H) = M log sn2 + sum log st + 2 sum log diag(L)
// -- no second Cholesky.  Only the objective needs the n x n Ki = Vi - W'W
// (one n x n x M GEMM), its lower triangle swept once by the fused kernel k_nys_grad, which
// regenerates K and dK_d from the 3-D inputs in registers and reduces
// (Ki - A A') against them, so the n x n x 3 dK array the notebook
// materialises never exists:
//   nlZ = r.A/2 + slogdet(H)/2 + n log(2 pi)/2
//   dnlZ_d = sum((Ki - A A') * dK_d)/2, dnlZ_3 = sum(Q * 2K)/2, dnlZ_4 = sn2 tr(Q)
//   (exact K, dK: NB1 SMLII quirks kept)
//   predict: fs = mean + k*.A;  sd = sqrt(sf2 - k*'Ki k*);  prior sd = sqrt(sf2)
//
// Every dense step -- the eigendecomposition, the Cholesky, the products --
// is a hand-written gfx950 kernel of oi_linalg.hip (no LAPACK / rocSOLVER /
// rocBLAS): the eigensolver is one workgroup per matrix for the Householder
// tridiagonalisation and the tridiagonal eigenpairs, batched MFMA products for
// the orthogonalisation and the back-transform.  Cells of a call are dealt
// over LANES (own stream and workspace); per-cell status comes back in one
// copy at the end.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <memory>
#include <cstdint>
#include <deque>
#include <string>
#include <vector>

#include "../../include/oi.h"
#include "oi_gemm.h"
#include "oi_linalg.h"

#pragma clang fp contract(off)

extern "C" int oi_set_last_error(int code, const char* msg);  // oi_engine.cpp
extern "C" void oi_profile_add(const char* name, int64_t launches, double ms, double flops,
                               double bytes);  // oi_engine.cpp

namespace {

constexpr double SQRT3 = 1.7320508075688772;  // np.sqrt(3.)

// ---------------------------------------------------------------- kernels --

// scaled coordinates as SGPkernel forms them (GPR:83, :93):
//   sc = np.sqrt(3.) * x / ell      (the 3-D distance Q)
//   sq = np.sqrt(3.) * (x / ell)    (the per-dimension q_d of dK)
__global__ void k_nys_scale(const double* __restrict__ x, int64_t n, double l0, double l1,
                            double l2, double* __restrict__ sc, double* __restrict__ sq) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double ell[3] = {l0, l1, l2};
  for (int d = 0; d < 3; ++d) {
    const double v = x[i * 3 + d];
    sc[i * 3 + d] = (SQRT3 * v) / ell[d];
    if (sq) sq[i * 3 + d] = SQRT3 * (v / ell[d]);
  }
}

__device__ inline double dist3(const double* a, const double* b) {
  const double d0 = a[0] - b[0], d1 = a[1] - b[1], d2 = a[2] - b[2];
  return sqrt(d0 * d0 + d1 * d1 + d2 * d2);  // scipy pdist/cdist 'euclidean'
}

// out[i + ld j] = sf2 (1 + Q) exp(-Q), Q = |sa[ia[i]] - sb[ib[j]]| (column-major)
__global__ void k_nys_cross(const double* __restrict__ sa, const int64_t* __restrict__ ia,
                            int64_t na, const double* __restrict__ sb,
                            const int64_t* __restrict__ ib, double sf2, double* __restrict__ out,
                            int64_t ld) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t j = blockIdx.y;
  if (i >= na) return;
  const int64_t ra = ia ? ia[i] : i, rb = ib ? ib[j] : j;
  const double Q = dist3(sa + ra * 3, sb + rb * 3);
  out[i + ld * j] = sf2 * ((1.0 + Q) * exp(-Q));
}

// s[s <= 0] = 1e-12; st = n * s / M  for the M real eigenvalues; st = 1 on a
// padded tail (so the pad contributes log 1 = 0 to the batched log-determinant)
__global__ void k_nys_eigpost(double* __restrict__ s, int64_t M, int64_t Mp, int64_t n,
                              double* __restrict__ st) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= Mp) return;
  if (k >= M) {
    st[k] = 1.0;
    return;
  }
  double v = s[k];
  if (v <= 0.0) v = 1e-12;
  s[k] = v;
  st[k] = ((double)n * v) / (double)M;
}

// ut = sqrt(M/n) * U1 / s  (column k divided by s[k]);  C = ut / sn2 (= Vi ut)
// (ut may alias U1: each element is read before it is written, by one thread)
__global__ void k_nys_ut(const double* U1, int64_t n, int64_t M,
                         const double* __restrict__ s, double c, double isn2,
                         double* ut, double* __restrict__ C) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * M) return;
  const int64_t k = e / n;
  const double u = (c * U1[e]) / s[k];
  ut[e] = u;
  C[e] = isn2 * u;
}

// A = r / sn2 (Vi r; the W'(W r) part is subtracted by a gemv)
__global__ void k_nys_vi(const double* __restrict__ r, int64_t n, double isn2,
                         double* __restrict__ A) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) A[i] = isn2 * r[i];
}

// A[i + ld i] = d + A[i + ld i]  (d = dv[i] if dv, else 1/dv-free scalar; inv => 1/dv[i])
__global__ void k_nys_diag(double* __restrict__ A, int64_t m, int64_t ld,
                           const double* __restrict__ dv, int inv, double d) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const double a = dv ? (inv ? 1.0 / dv[i] : dv[i]) : d;
  A[i + ld * i] = a + A[i + ld * i];
}

template <int NV>
__device__ inline void block_sum(double (&v)[NV], double* red) {
  // 256 threads: wave reduction then the 4 wave partials in fixed order
  for (int q = 0; q < NV; ++q)
    for (int o = 32; o > 0; o >>= 1) v[q] += __shfl_down(v[q], o, 64);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0)
    for (int q = 0; q < NV; ++q) red[w * NV + q] = v[q];
  __syncthreads();
  if (threadIdx.x == 0)
    for (int q = 0; q < NV; ++q) v[q] = ((red[q] + red[NV + q]) + red[2 * NV + q]) + red[3 * NV + q];
}

// out[0] = a . b   (one 256-thread block, fixed order)
__global__ void __launch_bounds__(256) k_nys_dot(const double* __restrict__ a,
                                                 const double* __restrict__ b, int64_t n,
                                                 double* __restrict__ out) {
  __shared__ double red[4];
  double v[1] = {0.0};
  for (int64_t i = threadIdx.x; i < n; i += 256) v[0] += a[i] * b[i];
  block_sum<1>(v, red);
  if (threadIdx.x == 0) out[0] = v[0];
}

// per matrix b of a strided batch of Cholesky factors:
//   res[b * NRES_ + 1] = sum_k log L_b[k + M k] + (sum_k log st_b[k]) / 2
// (slogdet(H)/2 minus M log(sn2)/2; one block per matrix)
__global__ void __launch_bounds__(256) k_nys_logdet(const double* __restrict__ L, int64_t M,
                                                    int64_t ld, int64_t strideL,
                                                    const double* __restrict__ st,
                                                    int64_t strideS, double* __restrict__ res,
                                                    int64_t strideR) {
  __shared__ double red[8];
  const int64_t b = blockIdx.x;
  L += b * strideL;
  st += b * strideS;
  double v[2] = {0.0, 0.0};
  for (int64_t i = threadIdx.x; i < M; i += 256) {
    v[0] += log(L[i + ld * i]);
    v[1] += log(st[i]);
  }
  block_sum<2>(v, red);
  if (threadIdx.x == 0) res[b * strideR + 1] = v[0] + v[1] / 2.0;
}

// pad the M x M matrix in the top-left of an Mp x Mp column-major buffer to a
// block-diagonal diag(A, d I): rows / columns M..Mp-1 zero except d on the
// diagonal.  Householder tridiagonalisation and Cholesky never mix the two
// blocks (the reflectors' entries in the pad rows are exactly 0), so the
// leading block's factors and eigenpairs are those of A itself.
__global__ void k_nys_pad(double* __restrict__ A, int64_t M, int64_t Mp, double d) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, j = blockIdx.y;
  if (i >= Mp || (i < M && j < M)) return;
  A[i + Mp * j] = i == j ? d : 0.0;
}

// The objective's n x n pass (NB1 SMLII, approx branch): the five sums
// sum Q dK_0, sum Q dK_1, sum Q dK_2, sum Q (2 K), tr Q over Q = Ki - A A',
// K = sf2 (1+D) e^-D, dK_d = sf2 q_d^2 e^-D regenerated from the scaled
// inputs (no n x n x 3 array).  Q and dK are symmetric and Ki is stored as its
// lower triangle only (syrk), so the sweep covers 64 x 64 tiles on or below
// the diagonal, weighting i > j by 2; one partial row of 5 per tile (zeros
// above the diagonal), Ki read once, coalesced along its columns.
__global__ void __launch_bounds__(256) k_nys_grad(const double* __restrict__ Ki,
                                                  const double* __restrict__ A,
                                                  const double* __restrict__ sc,
                                                  const double* __restrict__ sq, int64_t n,
                                                  double sf2, double* __restrict__ part) {
  __shared__ double red[4 * 5];
  double v[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  if (blockIdx.x >= blockIdx.y) {
    const int64_t i = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
    const int64_t j0 = (int64_t)blockIdx.y * 64 + (threadIdx.x >> 6) * 16;
    if (i < n) {
      const double ci[3] = {sc[i * 3], sc[i * 3 + 1], sc[i * 3 + 2]};
      const double qi[3] = {sq[i * 3], sq[i * 3 + 1], sq[i * 3 + 2]};
      const double Ai = A[i];
      int64_t jend = j0 + 16 < n ? j0 + 16 : n;
      jend = jend < i + 1 ? jend : i + 1;  // j <= i
      for (int64_t j = j0; j < jend; ++j) {
        const double Q = Ki[i + n * j] - Ai * A[j];
        const double D = dist3(ci, sc + j * 3);
        const double e = exp(-D);
        const double K = sf2 * ((1.0 + D) * e);
        const double w = j == i ? 1.0 : 2.0;
        for (int d = 0; d < 3; ++d) {
          // SGPkernel's q_d = pdist of one coordinate = sqrt(t*t) = |t| exactly
          // (binary64, round-to-nearest), so q_d^2 = fl(t*t): no sqrt needed
          const double t = qi[d] - sq[j * 3 + d];
          v[d] += w * (Q * (sf2 * ((t * t) * e)));
        }
        v[3] += w * (Q * (2.0 * K));
        if (j == i) v[4] += Q;
      }
    }
  }
  block_sum<5>(v, red);
  if (threadIdx.x == 0) {
    const int64_t b = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
    for (int q = 0; q < 5; ++q) part[b * 5 + q] = v[q];
  }
}

// out[q] = sum_b part[b*5 + q]  (fixed order)
__global__ void __launch_bounds__(256) k_nys_partsum(const double* __restrict__ part,
                                                     int64_t nb, double* __restrict__ out) {
  __shared__ double red[4 * 5];
  double v[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  for (int64_t b = threadIdx.x; b < nb; b += 256)
    for (int q = 0; q < 5; ++q) v[q] += part[b * 5 + q];
  block_sum<5>(v, red);
  if (threadIdx.x == 0)
    for (int q = 0; q < 5; ++q) out[q] = v[q];
}

// W' (n x M, column-major) -> 64 x 64 k-major tiles Wp[kt][it] (element
// kk*64 + mm = W'[64 it + mm][64 kt + kk], zero beyond n / M): the operand
// layout of the MFMA tile GEMM core (oi_gemm.h)
__global__ void __launch_bounds__(256) k_nys_pack(const double* __restrict__ Wt, int64_t n,
                                                  int64_t M, int Tn, double* __restrict__ Wp) {
  const int it = blockIdx.x % Tn, kt = blockIdx.x / Tn;
  double* dst = Wp + (size_t)blockIdx.x * 4096;
  for (int e = threadIdx.x; e < 4096; e += 256) {
    const int64_t a = (int64_t)it * 64 + (e & 63), k = (int64_t)kt * 64 + (e >> 6);
    dst[e] = (a < n && k < M) ? Wt[a + n * k] : 0.0;
  }
}

// The objective's n x n pass without materialising Ki: per lower 64 x 64 tile
// (i >= j) the MFMA core forms (W'W)_ij = sum_k Wp[k][i]^T Wp[k][j] in
// registers, then Ki = [a == b]/sn2 - (W'W)_ab, Q = Ki - A_a A_b and the five
// sums against K, dK regenerated from the scaled inputs (as k_nys_grad),
// off-diagonal entries weighted 2.  One partial row of 5 per tile.
__global__ void __launch_bounds__(256) k_nys_grad_mfma(const double* __restrict__ Wp, int Tn,
                                                       int Tk, const double* __restrict__ A,
                                                       const double* __restrict__ sc,
                                                       const double* __restrict__ sq, int64_t n,
                                                       double sf2, double isn2,
                                                       double* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) double lds[GEMM1_LDS];
  const int tile = blockIdx.x;
  int i = (int)((sqrt(8.0 * tile + 1.0) - 1.0) * 0.5);
  while ((i + 1) * (i + 2) / 2 <= tile) ++i;
  while (i * (i + 1) / 2 > tile) --i;
  const int j = tile - i * (i + 1) / 2;
  Quad acc;
  quad_zero(acc);
  gemm1_kmajor<false>(acc, lds, 4 * Tk, 0u, [=](int p, const double*& a, const double*& b) {
    a = Wp + ((size_t)p * Tn + i) * 4096;
    b = Wp + ((size_t)p * Tn + j) * 4096;
  });
  double* cQ = lds;            // [3][128] scaled inputs (distance), rows i | columns j
  double* cq = lds + 3 * 128;  // [3][128] per-dimension scaled inputs
  double* al = lds + 6 * 128;  // [128] A
  double* red = lds + 7 * 128;
  const int t = threadIdx.x;
  if (t < 128) {
    const int64_t a = t < 64 ? (int64_t)i * 64 + t : (int64_t)j * 64 + (t - 64);
    for (int d = 0; d < 3; ++d) {
      cQ[d * 128 + t] = a < n ? sc[3 * a + d] : 0.0;
      cq[d * 128 + t] = a < n ? sq[3 * a + d] : 0.0;
    }
    al[t] = a < n ? A[a] : 0.0;
  }
  __syncthreads();
  double v[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  for (int mb = 0; mb < 2; ++mb)
    for (int nb = 0; nb < 2; ++nb)
      for (int r = 0; r < 4; ++r) {
        const int m = acc1_row(mb, r), nn = acc1_col(nb);
        const int64_t a = (int64_t)i * 64 + m, b = (int64_t)j * 64 + nn;
        if (a >= n || b >= n || (i == j && m < nn)) continue;
        const double x = acc.c[mb][nb][r];
        const double Ki = a == b ? isn2 - x : -x;
        const double Q = Ki - al[m] * al[64 + nn];
        const double d0 = cQ[m] - cQ[64 + nn], d1 = cQ[128 + m] - cQ[128 + 64 + nn],
                     d2 = cQ[256 + m] - cQ[256 + 64 + nn];
        const double D = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
        const double e = exp(-D);
        const double K = sf2 * ((1.0 + D) * e);
        const double w = a == b ? 1.0 : 2.0;
        for (int d = 0; d < 3; ++d) {
          const double tt = cq[d * 128 + m] - cq[d * 128 + 64 + nn];
          v[d] += w * (Q * (sf2 * ((tt * tt) * e)));
        }
        v[3] += w * (Q * (2.0 * K));
        if (a == b) v[4] += Q;
      }
  block_sum<5>(v, red);
  if (t == 0)
    for (int q = 0; q < 5; ++q) part[(size_t)tile * 5 + q] = v[q];
}

// ------------------------------------------------------------------- host --

struct HipErr {
  std::string msg;
};

#define HC(expr)                                                                              \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess) throw HipErr{std::string(#expr) + ": " + hipGetErrorString(e_)};    \
  } while (0)
#define KCHK() HC(hipGetLastError())

// opts.profile: HIP events around each stage of each cell, summed per stage
// into oi_profile_json (algorithmic flops / bytes per stage alongside)
enum { S_BUILD, S_EIGH, S_EIGH_VEC, S_EIGH_ORTH, S_EIGH_BACK, S_PANEL, S_KI, S_APPLY, S_LOGDET, S_GRAD,
       S_PRED, S_COUNT };
// nys_eigh = the Householder tridiagonalisation; the eigensolver's other phases
// are timed as their own stages
const char* kStage[S_COUNT] = {"nys_build",  "nys_eigh",   "nys_eigh_vectors", "nys_eigh_orth",
                               "nys_eigh_back", "nys_panels", "nys_ki_gemm", "nys_apply",
                               "nys_logdet", "nys_grad",   "nys_predict"};
struct Stager {
  bool on = false;
  hipStream_t st = nullptr;
  std::vector<hipEvent_t> ev;
  std::vector<int> kind;
  std::vector<double> fl, by;
  void begin(int k, double flops, double bytes) {
    if (!on) return;
    kind.push_back(k);
    fl.push_back(flops);
    by.push_back(bytes);
    rec();
  }
  void end() {
    if (on) rec();
  }
  void rec() {
    hipEvent_t e;
    HC(hipEventCreate(&e));
    ev.push_back(e);
    HC(hipEventRecord(e, st));
  }
  void flush() {  // after the stream has been synchronised
    if (!on) return;
    double ms[S_COUNT] = {}, f[S_COUNT] = {}, b[S_COUNT] = {};
    int64_t n[S_COUNT] = {};
    for (size_t q = 0; q < kind.size(); ++q) {
      float t = 0.f;
      HC(hipEventElapsedTime(&t, ev[2 * q], ev[2 * q + 1]));
      ms[kind[q]] += t;
      f[kind[q]] += fl[q];
      b[kind[q]] += by[q];
      n[kind[q]] += 1;
    }
    for (int k = 0; k < S_COUNT; ++k)
      if (n[k]) oi_profile_add(kStage[k], n[k], ms[k], f[k], b[k]);
    for (auto e : ev) (void)hipEventDestroy(e);
    ev.clear();
    kind.clear();
    fl.clear();
    by.clear();
  }
  ~Stager() {
    for (auto e : ev) (void)hipEventDestroy(e);
  }
};

inline unsigned blocks(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

// per-cell device results: [r.A, sum log diag(L) + sum log st / 2, g0..g4 raw
// sums, k*.A, |k*|^2, |W k*|^2]
constexpr int NRES = 10;
// per-cell infos: [eigh, potrf(B)] (LAPACK's info semantics)
constexpr int NINFO = 2;

}  // namespace

namespace {

// Validated ragged batch + the device-side state of one liboi call.
struct Batch {
  const double* xyt;
  const double* y;
  const int64_t* offs;
  int64_t ncell;
  const int64_t* sel;
  const int64_t* soffs;
  int64_t nmax = 0, mmax = 0;
};

int check_batch(Batch& b) {
  if (b.ncell < 0) return oi_set_last_error(OI_E_ARG, "negative ncell");
  if (b.ncell == 0) return 0;
  if (!b.offs || !b.soffs || !b.sel || !b.xyt || !b.y) return oi_set_last_error(OI_E_ARG, "null pointer");
  if (b.offs[0] != 0 || b.soffs[0] != 0) return oi_set_last_error(OI_E_ARG, "offs[0] must be 0");
  for (int64_t c = 0; c < b.ncell; ++c) {
    const int64_t n = b.offs[c + 1] - b.offs[c], M = b.soffs[c + 1] - b.soffs[c];
    if (n < 1 || M < 1 || M > n) return oi_set_last_error(OI_E_ARG, "each cell needs 1 <= M <= n");
    for (int64_t k = b.soffs[c]; k < b.soffs[c + 1]; ++k)
      if (b.sel[k] < 0 || b.sel[k] >= n)
        return oi_set_last_error(OI_E_ARG, "inducing index out of range");
    b.nmax = n > b.nmax ? n : b.nmax;
    b.mmax = M > b.mmax ? M : b.mmax;
  }
  if (b.nmax > INT32_MAX / 2) return oi_set_last_error(OI_E_ARG, "cell too large");
  return 0;
}

int setup(const oi_options* opts, oi_options& o) {
  oi_options_default(&o);
  if (opts) o = *opts;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return oi_set_last_error(OI_E_NODEV, "no HIP device available");
  if (o.device < 0 || o.device >= ndev) return oi_set_last_error(OI_E_ARG, "bad device ordinal");
  if (hipSetDevice(o.device) != hipSuccess) return oi_set_last_error(OI_E_HIP, "hipSetDevice failed");
  return 0;
}

// One cell's inputs on the device: the row of the cell table a Runner reads.
struct CellSrc {
  const double* x;     // n x 3
  const double* y;     // n (outputs minus the prior mean, as NB1 passes them)
  const int64_t* sel;  // M inducing rows, 0-based within the cell
  const double* xs;    // 3 (prediction target) or null
  int64_t n, M;
};

struct Buf;
// Outcome of one cell at one hyper point (host side).
struct CellOut {
  double nlz, grad[5], fs, sd, sprior;
  int status;
};

// Device buffer; stream-ordered (hipMallocAsync / hipFreeAsync on `st`) when
// given a stream, so freeing it never waits for the whole device.
struct Buf {
  void* p = nullptr;
  hipStream_t st = nullptr;
  bool async = false;
  Buf() = default;
  Buf(const Buf&) = delete;
  Buf& operator=(const Buf&) = delete;
  void alloc(size_t bytes) {
    if (bytes) HC(hipMalloc(&p, bytes));
  }
  void alloc_async(size_t bytes, hipStream_t s) {
    st = s;
    async = true;
    if (bytes) HC(hipMallocAsync(&p, bytes, s));
  }
  ~Buf() {
    if (p) (void)(async ? hipFreeAsync(p, st) : hipFree(p));
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

// Device copy of one validated batch (inputs when they came from the host,
// inducing rows, targets) and its rows of the cell table.
// Allocated and filled on stream `st` (stream-ordered; the constructor
// returns once the copies are done) and freed on it: a session orders `st`
// after every group's last use before dropping a batch.
struct BatchDev {
  Buf hx, hy, dsel, dxs;
  std::vector<CellSrc> rows;
  BatchDev(const Batch& b, const double* xs, bool device_inputs, hipStream_t st) {
    const int64_t N = b.offs[b.ncell], S = b.soffs[b.ncell];
    const double* dx = b.xyt;
    const double* dy = b.y;
    if (!device_inputs) {
      hx.alloc_async(N * 3 * 8, st);
      hy.alloc_async(N * 8, st);
      HC(hipMemcpyAsync(hx.p, b.xyt, N * 3 * 8, hipMemcpyHostToDevice, st));
      HC(hipMemcpyAsync(hy.p, b.y, N * 8, hipMemcpyHostToDevice, st));
      dx = hx.as<double>();
      dy = hy.as<double>();
    }
    dsel.alloc_async(S * 8, st);
    HC(hipMemcpyAsync(dsel.p, b.sel, S * 8, hipMemcpyHostToDevice, st));
    if (xs) {
      dxs.alloc_async(b.ncell * 3 * 8, st);
      HC(hipMemcpyAsync(dxs.p, xs, b.ncell * 3 * 8, hipMemcpyHostToDevice, st));
    }
    HC(hipStreamSynchronize(st));  // host arrays may go away once submit returns
    rows.resize(b.ncell);
    for (int64_t c = 0; c < b.ncell; ++c)
      rows[c] = CellSrc{dx + b.offs[c] * 3, dy + b.offs[c], dsel.as<int64_t>() + b.soffs[c],
                        xs ? dxs.as<double>() + c * 3 : nullptr, b.offs[c + 1] - b.offs[c],
                        b.soffs[c + 1] - b.soffs[c]};
  }
};

// objective pass: fused MFMA kernel (default) or, with OI_NYS_FUSED=0, the
// n x n product forming Ki (oila::gemm) followed by k_nys_grad
inline bool fused_objective() {
  const char* e = getenv("OI_NYS_FUSED");
  return !(e && atoi(e) == 0);
}

struct Lane {
  hipStream_t st = nullptr;
  oila::Stager la;  // launch descriptors of the oila kernels on this lane's stream
  Buf Knm, U1, ut, Ki, Wp, Av, tv, ks, kv, xsc, part;
  Stager sg;
  hipEvent_t done = nullptr;
  Lane(int64_t nmax, int64_t mmax, bool obj, bool pred, bool profile) {
    HC(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    HC(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    la.bind(st);
    const int64_t nM = nmax * mmax, nt = blocks(nmax, 64);
    Knm.alloc(nM * 8);
    U1.alloc(nM * 8);
    ut.alloc(nM * 8);
    Av.alloc(nmax * 8);
    tv.alloc(mmax * 8);
    if (obj) {
      if (fused_objective()) {
        Wp.alloc((size_t)blocks(mmax, 64) * nt * 4096 * 8);
      } else {
        Ki.alloc(nmax * nmax * 8);
      }
      part.alloc(nt * nt * 5 * 8);
    }
    if (pred) {
      ks.alloc(nmax * 8);
      kv.alloc(mmax * 8);
      xsc.alloc(3 * 8);
    }
    sg.on = profile;
    sg.st = st;
  }
  ~Lane() {
    if (done) (void)hipEventDestroy(done);
    if (st) (void)hipStreamDestroy(st);
  }
};

// Evaluates any subset of a validated batch's cells at given LINEAR hypers.
//
// The eigensolver runs one workgroup per matrix and the blocked Cholesky one
// launch sequence for many matrices, so a run is phase-major over CHUNKS of
// cells (sorted by M): (1) K_mm of every cell, (2) one batched eigh per
// equal-padded-M group, (3) the n x M panels and B of every cell, (4) one
// batched Cholesky per group, (5) the triangular solve, objective and
// prediction of every cell.
// Per-cell phases are dealt round-robin over LANES (OI_NYS_LANES, default 1:
// stream + oila::gemm descriptor ring + scratch each; more lanes measured no faster with
// the box's 4 hardware queues); per-slot state (scaled inputs,
// K_mm -> u, s, st, C, B -> L) lives in chunk-sized slot arrays.
class Runner {
 public:
  // Reads cells from *tab (rows indexed by cell id; the table may grow between
  // calls); every cell has n <= nmax, M <= mmax; at most `cap` cells per
  // evaluation.  own_stream: work on a private stream (several Runners then
  // overlap); otherwise on the caller's opts.stream
  Runner(const std::vector<CellSrc>* tab, int64_t nmax, int64_t mmax, int64_t cap, const oi_options& o,
         bool want_obj, bool want_pred, bool own_stream = false)
      : tab_(tab), nmax_(nmax), cap_(cap), st_((hipStream_t)o.stream), alloc_obj_(want_obj),
        alloc_pred_(want_pred) {
    if (own_stream) {
      HC(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
      own_ = true;
    }
    res_.alloc(cap * NRES * 8);
    info_.alloc(cap * NINFO * sizeof(int32_t));
    HC(hipHostMalloc((void**)&hr_, cap * NRES * 8, hipHostMallocDefault));
    HC(hipHostMalloc((void**)&hi_, cap * NINFO * sizeof(int32_t), hipHostMallocDefault));
    la_.bind(st_);
    sg_.on = o.profile != 0;
    sg_.st = st_;
    int nl = 1;
    if (const char* e = getenv("OI_NYS_LANES")) nl = atoi(e);
    nl = nl < 1 ? 1 : nl;
    nl = nl > cap ? (int)cap : nl;
    for (int l = 0; l < nl; ++l)
      lanes_.emplace_back(new Lane(nmax, mmax, want_obj, want_pred, o.profile != 0));
    // padding quantum (OI_NYS_PAD, default 32; 0 = no padding): K_mm and B of a
    // cell are factored as diag(A, d I) of size Mp = M rounded up (the slot
    // strides of the chunk arrays; results equal the unpadded path to rounding)
    if (const char* e = getenv("OI_NYS_PAD")) padq_ = std::max(0, atoi(e));
    mpmax_ = Mp(mmax);
    // slot arrays: sc, sq (n x 3), Kmm (Mp^2), s, st (Mp), C (n x M), B (Mp^2),
    // the eigensolver's workspace, the Cholesky's diagonal-block inverses;
    // chunk <= 64 cells and <= 1/4 of the free HBM
    const int64_t mmaxp = mpmax_;
    ewd_ = oila::eigh_workspace_doubles((int)mmaxp);
    nd64_ = (mmaxp + 63) / 64;
    // OI_NYS_B3 (default 1): phase 3's two n x M products batched over the
    // chunk (per-slot K_nm and U1 / ut) instead of one cell at a time per lane
    if (const char* e = getenv("OI_NYS_B3")) b3_ = atoi(e) != 0;
    const size_t per = (size_t)(6 * nmax + 2 * mmaxp * mmaxp + 2 * mmaxp + (b3_ ? 3 : 1) * nmax * mmaxp) * 8 +
                       (ewd_ + (size_t)nd64_ * 4096) * 8;
    size_t fr = 0, tot = 0;
    HC(hipMemGetInfo(&fr, &tot));
    int64_t ch = std::min<int64_t>(64, cap);
    ch = std::min<int64_t>(ch, std::max<int64_t>(1, (int64_t)(fr / 4 / per)));
    chunk_ = ch;
    sc_.alloc(ch * nmax * 3 * 8);
    sq_.alloc(ch * nmax * 3 * 8);
    Kmm_.alloc(ch * mmaxp * mmaxp * 8);
    eval_.alloc(ch * mmaxp * 8);
    stl_.alloc(ch * mmaxp * 8);
    C_.alloc(ch * nmax * mmaxp * 8);
    if (b3_) {
      Knm_.alloc(ch * nmax * mmaxp * 8);
      U1_.alloc(ch * nmax * mmaxp * 8);
    }
    B_.alloc(ch * mmaxp * mmaxp * 8);
    EW_.alloc(ch * ewd_ * 8);
    Dinv_.alloc(ch * nd64_ * 4096 * 8);
    HC(hipEventCreateWithFlags(&ready_, hipEventDisableTiming));
  }
  ~Runner() {
    if (own_ && st_) (void)hipStreamSynchronize(st_);
    for (Lane* l : lanes_) delete l;
    if (ready_) (void)hipEventDestroy(ready_);
    if (hr_) (void)hipHostFree(hr_);
    if (hi_) (void)hipHostFree(hi_);
    if (own_ && st_) (void)hipStreamDestroy(st_);
  }

  // cells[k] at LINEAR hypers hyp[k*5 ..]; results into out[k]
  void run(const std::vector<int64_t>& cells, const double* hyp, double mean, CellOut* out,
           bool want_obj, bool want_pred) {
    enqueue(cells, hyp, mean, want_obj, want_pred);
    collect(out);
  }

  // queue one evaluation of cells[k] at hyp[k*5 ..] (copied) without waiting
  void enqueue(const std::vector<int64_t>& cells, const double* hyp, double mean, bool want_obj,
               bool want_pred) {
    const int64_t nc = (int64_t)cells.size();
    ncq_ = nc;
    if (!nc) return;
    if (nc > cap_) throw HipErr{"Runner: more cells than its capacity"};
    if ((want_obj && !alloc_obj_) || (want_pred && !alloc_pred_))
      throw HipErr{"Runner: stage not allocated"};
    obj_ = want_obj;
    pred_ = want_pred;
    mean_ = mean;
    cellv_ = cells;
    hypv_.assign(hyp, hyp + nc * 5);
    cells_ = &cellv_;
    hyp_ = hypv_.data();
    // positions sorted by M (equal-M cells adjacent for the batched factorisations)
    order_.resize(nc);
    for (int64_t k = 0; k < nc; ++k) order_[k] = k;
    std::stable_sort(order_.begin(), order_.end(), [&](int64_t a, int64_t c) {
      return Mof(cells[a]) < Mof(cells[c]);
    });
    HC(hipMemsetAsync(res_.p, 0, nc * NRES * 8, st_));
    HC(hipMemsetAsync(info_.p, 0, nc * NINFO * sizeof(int32_t), st_));
    for (int64_t p0 = 0; p0 < nc; p0 += chunk_) {
      const int64_t p1 = std::min(nc, p0 + chunk_);
      lanes_phase(p0, p1, 1);
      batched(p0, p1, 0);
      if (b3_)
        batched3(p0, p1);
      else
        lanes_phase(p0, p1, 3);
      batched(p0, p1, 1);
      lanes_phase(p0, p1, 5);
    }
    HC(hipMemcpyAsync(hr_, res_.p, nc * NRES * 8, hipMemcpyDeviceToHost, st_));
    HC(hipMemcpyAsync(hi_, info_.p, nc * NINFO * sizeof(int32_t), hipMemcpyDeviceToHost, st_));
  }

  // wait for the queued evaluation; out[k] for the enqueued cells[k]
  void collect(CellOut* out) {
    const int64_t nc = ncq_;
    if (!nc) return;
    const std::vector<int64_t>& cells = cellv_;
    const double* hyp = hyp_;
    const double mean = mean_;
    HC(hipStreamSynchronize(st_));
    sg_.flush();
    for (Lane* l : lanes_) l->sg.flush();
    la_.reset();  // every launch that read the staged descriptors has completed
    for (Lane* l : lanes_) l->la.reset();
    const double inf = INFINITY, nan = NAN;
    for (int64_t p = 0; p < nc; ++p) {
      const int64_t k = order_[p], c = cells[k];
      const int64_t n = (*tab_)[c].n, M = Mof(c);
      const double sf2 = hyp[k * 5 + 3], sn2 = hyp[k * 5 + 4];
      const double* rr = hr_ + p * NRES;
      const int32_t* ii = hi_ + p * NINFO;
      const bool bad = ii[0] != 0 || ii[1] != 0;  // NB1's LinAlgError (eigh / cholesky)
      CellOut& r = out[k];
      r.status = bad ? 1 : 0;
      if (obj_) {
        if (bad) {
          r.nlz = inf;
          for (int q = 0; q < 5; ++q) r.grad[q] = inf;
        } else {
          // det = slogdet(H)/2 = (M log sn2 + sum log st + 2 sum log diag L) / 2
          const double det = (double)M * std::log(sn2) / 2.0 + rr[1];
          r.nlz = (rr[0] / 2.0 + det) + (double)n * std::log(2.0 * M_PI) / 2.0;
          r.grad[0] = rr[2] / 2.0;
          r.grad[1] = rr[3] / 2.0;
          r.grad[2] = rr[4] / 2.0;
          r.grad[3] = rr[5] / 2.0;
          r.grad[4] = sn2 * rr[6];
        }
      }
      if (pred_) {
        const double err = rr[8] / sn2 - rr[9];  // k*'Ki k* = |k*|^2/sn2 - |W k*|^2
        r.fs = bad ? nan : mean + rr[7];
        r.sd = bad ? nan : std::sqrt(sf2 - err);
        r.sprior = std::sqrt(sf2);
      }
    }
  }

 private:
  int64_t Mof(int64_t c) const { return (*tab_)[c].M; }
  int64_t Mp(int64_t M) const { return padq_ > 0 ? (M + padq_ - 1) / padq_ * padq_ : M; }

  // per-cell phase `ph` for positions [p0, p1) dealt over the lanes, fenced
  // against the main stream on both sides
  void lanes_phase(int64_t p0, int64_t p1, int ph) {
    const int64_t nl = std::min<int64_t>((int64_t)lanes_.size(), p1 - p0);
    HC(hipEventRecord(ready_, st_));
    for (int64_t l = 0; l < nl; ++l) HC(hipStreamWaitEvent(lanes_[l]->st, ready_, 0));
    for (int64_t p = p0; p < p1; ++p) {
      Lane& L = *lanes_[(p - p0) % nl];
      if (ph == 1) phase1(L, p, p - p0);
      else if (ph == 3) phase3(L, p, p - p0);
      else phase5(L, p, p - p0);
    }
    for (int64_t l = 0; l < nl; ++l) {
      HC(hipEventRecord(lanes_[l]->done, lanes_[l]->st));
      HC(hipStreamWaitEvent(st_, lanes_[l]->done, 0));
    }
  }

  // which = 0: s, u = eigh(Kmm) (oila::eigh; u overwrites Kmm); 1: L = chol(B)
  // (oila::cholesky, in place, with the diagonal-block inverses kept for the
  // triangular solve) -- one batched call per run of slots with equal padded
  // size, on the main stream
  void batched(int64_t p0, int64_t p1, int which) {
    const int64_t mm = mpmax_ * mpmax_;
    for (int64_t g0 = p0; g0 < p1;) {
      const int64_t M = Mp(Mof((*cells_)[order_[g0]]));  // padded size of the group
      int64_t g1 = g0 + 1;
      while (g1 < p1 && Mp(Mof((*cells_)[order_[g1]])) == M) ++g1;
      const int iM = (int)M, cnt = (int)(g1 - g0);
      const int64_t s0 = g0 - p0;
      const double dM = (double)M;
      if (which == 0) {
        std::vector<oila::Eigh> es;
        for (int q = 0; q < cnt; ++q)
          es.push_back(oila::Eigh{Kmm_.as<double>() + (s0 + q) * mm, eval_.as<double>() + (s0 + q) * mpmax_,
                                  EW_.as<double>() + (s0 + q) * ewd_, iM, iM,
                                  info_.as<int32_t>() + (g0 + q) * NINFO + 0});
        // algorithmic flops per phase: tridiagonalisation 4/3 M^3, tridiagonal
        // eigenpairs O(M^2), BCGS2 2 M^3, back-transform 2 M^3
        const double m3 = dM * dM * dM * cnt;
        const int kind[4] = {S_EIGH, S_EIGH_VEC, S_EIGH_ORTH, S_EIGH_BACK};
        const double fl[4] = {4.0 / 3.0 * m3, 0.0, 2.0 * m3, 2.0 * m3};
        oila::eigh(la_, st_, es, [&](int k) {
          if (k > 0) sg_.end();
          if (k < 4) sg_.begin(kind[k], fl[k], 0.0);
        });
      } else {
        // L = chol(B); half log-determinants (the lanes then form W' = C L^-T
        // by a block triangular solve with the kept diagonal-block inverses)
        sg_.begin(S_PANEL, dM * dM * dM / 3 * cnt, 0.0);
        double* B0 = B_.as<double>() + s0 * mm;
        std::vector<oila::Chol> cs;
        for (int q = 0; q < cnt; ++q)
          cs.push_back(oila::Chol{B0 + q * mm, Dinv_.as<double>() + (s0 + q) * nd64_ * 4096,
                                  info_.as<int32_t>() + (g0 + q) * NINFO + 1, iM, iM});
        oila::cholesky(la_, st_, cs);
        // the pad block is the identity: log 1 = 0 and st is 1 there (see phase3)
        hipLaunchKernelGGL(k_nys_logdet, dim3(cnt), dim3(256), 0, st_, B0, M, M, mm,
                           stl_.as<double>() + s0 * mpmax_, mpmax_,
                           res_.as<double>() + g0 * NRES, (int64_t)NRES);
        KCHK();
        // W' = C L^-T in place on each slot's C (n x M, leading dimension n): one
        // batched right-looking block solve for the whole group
        std::vector<oila::TrsmRLT> ts;
        for (int q = 0; q < cnt; ++q) {
          const CellRefs R = refs(g0 + q, s0 + q);
          ts.push_back(oila::TrsmRLT{R.C, R.B, R.dinv, R.in, R.iM, R.in, R.iMp});
        }
        oila::trsm_right_lt(la_, st_, ts);
        sg_.end();
      }
      g0 = g1;
    }
  }

  struct CellRefs {
    int64_t c, k, n, M, Mp;
    int in, iM, iMp;
    double dn, dM;
    const double* x;
    const double* r;
    const int64_t* sl;
    const double* hp;
    double *sc, *sq, *Kmm, *s, *stl, *C, *B, *rs, *dinv;
  };
  CellRefs refs(int64_t p, int64_t slot) {
    CellRefs R;
    R.k = order_[p];
    R.c = (*cells_)[R.k];
    R.n = (*tab_)[R.c].n;
    R.M = Mof(R.c);
    R.Mp = Mp(R.M);
    R.in = (int)R.n;
    R.iM = (int)R.M;
    R.iMp = (int)R.Mp;
    R.dn = (double)R.n;
    R.dM = (double)R.M;
    R.x = (*tab_)[R.c].x;
    R.r = (*tab_)[R.c].y;
    R.sl = (*tab_)[R.c].sel;
    R.hp = hyp_ + R.k * 5;
    const int64_t nmax = nmax_, mmax = mpmax_;
    R.sc = sc_.as<double>() + slot * nmax * 3;
    R.sq = sq_.as<double>() + slot * nmax * 3;
    R.Kmm = Kmm_.as<double>() + slot * mmax * mmax;
    R.s = eval_.as<double>() + slot * mmax;
    R.stl = stl_.as<double>() + slot * mmax;
    R.C = C_.as<double>() + slot * nmax * mmax;
    R.B = B_.as<double>() + slot * mmax * mmax;
    R.rs = res_.as<double>() + p * NRES;
    R.dinv = Dinv_.as<double>() + slot * nd64_ * 4096;
    return R;
  }

  // phase 3 for a whole chunk on the main stream: the per-cell elementwise
  // kernels, and each of the two n x M products as ONE batched oila::gemm over
  // the chunk's cells (per-cell launches of ~1 000 64 x 64 tiles left the
  // chip under-filled in the last wave of tiles)
  void batched3(int64_t p0, int64_t p1) {
    hipStream_t st = st_;
    const int64_t nM = nmax_ * mpmax_;
    double fl = 0.0, by = 0.0;
    for (int64_t p = p0; p < p1; ++p) {
      const CellRefs R = refs(p, p - p0);
      fl += 4 * R.dn * R.dM * R.dM;
      by += 8.0 * R.dn * R.dM;
    }
    sg_.begin(S_PANEL, fl, by);
    std::vector<oila::Gemm> g1, g2;
    for (int64_t p = p0; p < p1; ++p) {
      const CellRefs R = refs(p, p - p0);
      double* Knm = Knm_.as<double>() + (p - p0) * nM;
      double* U1 = U1_.as<double>() + (p - p0) * nM;
      hipLaunchKernelGGL(k_nys_eigpost, dim3(blocks(R.Mp, 256)), dim3(256), 0, st, R.s, R.M, R.Mp,
                         R.n, R.stl);
      KCHK();
      hipLaunchKernelGGL(k_nys_cross, dim3(blocks(R.n, 256), (unsigned)R.M), dim3(256), 0, st, R.sc,
                         nullptr, R.n, R.sc, R.sl, R.hp[3], Knm, R.n);
      KCHK();
      g1.push_back(oila::Gemm{Knm, R.Kmm, U1, R.in, R.iM, R.iM, R.in, R.iMp, R.in, 1.0, 0.0, 0});  // U1 = Knm u
      g2.push_back(oila::Gemm{U1, R.C, R.B, R.iM, R.iM, R.in, R.in, R.in, R.iMp, 1.0, 0.0, 0});    // B = ut' C
    }
    oila::gemm(la_, st, false, false, g1);
    for (int64_t p = p0; p < p1; ++p) {  // ut (in place of U1) and C
      const CellRefs R = refs(p, p - p0);
      double* U1 = U1_.as<double>() + (p - p0) * nM;
      hipLaunchKernelGGL(k_nys_ut, dim3(blocks(R.n * R.M, 256)), dim3(256), 0, st, U1, R.n, R.M, R.s,
                         std::sqrt(R.dM / R.dn), 1.0 / R.hp[4], U1, R.C);
      KCHK();
    }
    oila::gemm(la_, st, true, false, g2);
    for (int64_t p = p0; p < p1; ++p) {  // B += diag(1/st), pad block
      const CellRefs R = refs(p, p - p0);
      hipLaunchKernelGGL(k_nys_diag, dim3(blocks(R.M, 256)), dim3(256), 0, st, R.B, R.M, R.Mp, R.stl, 1,
                         0.0);
      KCHK();
      if (R.Mp > R.M) {
        hipLaunchKernelGGL(k_nys_pad, dim3(blocks(R.Mp, 256), (unsigned)R.Mp), dim3(256), 0, st, R.B,
                           R.M, R.Mp, 1.0);
        KCHK();
      }
    }
    sg_.end();
  }

  // scaled inputs, Kmm (NB1 Nystroem: SGPkernel(x[sel]))
  void phase1(Lane& L, int64_t p, int64_t slot) {
    const CellRefs R = refs(p, slot);
    hipStream_t st = L.st;
    L.sg.begin(S_BUILD, 0.0, 8.0 * R.dM * R.dM);
    hipLaunchKernelGGL(k_nys_scale, dim3(blocks(R.n, 256)), dim3(256), 0, st, R.x, R.n, R.hp[0],
                       R.hp[1], R.hp[2], R.sc, obj_ ? R.sq : nullptr);
    KCHK();
    hipLaunchKernelGGL(k_nys_cross, dim3(blocks(R.M, 256), (unsigned)R.M), dim3(256), 0, st, R.sc,
                       R.sl, R.M, R.sc, R.sl, R.hp[3], R.Kmm, R.Mp);
    KCHK();
    if (R.Mp > R.M) {
      // pad eigenvalue above every eigenvalue of K_mm (<= trace = M sf2), so the
      // M real eigenpairs stay first in syevd's ascending order
      hipLaunchKernelGGL(k_nys_pad, dim3(blocks(R.Mp, 256), (unsigned)R.Mp), dim3(256), 0, st,
                         R.Kmm, R.M, R.Mp, 2.0 * R.dM * R.hp[3] + 1.0);
      KCHK();
    }
    L.sg.end();
  }

  // s clamp, st; Knm = SGPkernel(x, xs=x[sel]); U1 = Knm u; ut, C = Vi ut;
  // B = diag(1/st) + ut' C
  void phase3(Lane& L, int64_t p, int64_t slot) {
    const CellRefs R = refs(p, slot);
    hipStream_t st = L.st;
    double* Knm = L.Knm.as<double>();
    double* U1 = L.U1.as<double>();
    double* ut = L.ut.as<double>();
    L.sg.begin(S_PANEL, 4 * R.dn * R.dM * R.dM, 8.0 * R.dn * R.dM);
    hipLaunchKernelGGL(k_nys_eigpost, dim3(blocks(R.Mp, 256)), dim3(256), 0, st, R.s, R.M, R.Mp,
                       R.n, R.stl);
    KCHK();
    hipLaunchKernelGGL(k_nys_cross, dim3(blocks(R.n, 256), (unsigned)R.M), dim3(256), 0, st, R.sc,
                       nullptr, R.n, R.sc, R.sl, R.hp[3], Knm, R.n);
    KCHK();
    // U1 = Knm u
    oila::gemm(L.la, st, false, false, {oila::Gemm{Knm, R.Kmm, U1, R.in, R.iM, R.iM, R.in, R.iMp, R.in, 1.0, 0.0, 0}});
    hipLaunchKernelGGL(k_nys_ut, dim3(blocks(R.n * R.M, 256)), dim3(256), 0, st, U1, R.n, R.M, R.s,
                       std::sqrt(R.dM / R.dn), 1.0 / R.hp[4], ut, R.C);
    KCHK();
    // B = ut' C (then + diag(1/st))
    oila::gemm(L.la, st, true, false, {oila::Gemm{ut, R.C, R.B, R.iM, R.iM, R.in, R.in, R.in, R.iMp, 1.0, 0.0, 0}});
    hipLaunchKernelGGL(k_nys_diag, dim3(blocks(R.M, 256)), dim3(256), 0, st, R.B, R.M, R.Mp, R.stl, 1,
                       0.0);
    KCHK();
    if (R.Mp > R.M) {
      hipLaunchKernelGGL(k_nys_pad, dim3(blocks(R.Mp, 256), (unsigned)R.Mp), dim3(256), 0, st, R.B,
                         R.M, R.Mp, 1.0);
      KCHK();
    }
    L.sg.end();
  }

  // W' = C L^-T;  A = r/sn2 - W'(W r);  objective (Ki, fused pass);  predict
  void phase5(Lane& L, int64_t p, int64_t slot) {
    const CellRefs R = refs(p, slot);
    hipStream_t st = L.st;
    const double sf2 = R.hp[3], isn2 = 1.0 / R.hp[4];
    const double dn = R.dn, dM = R.dM;
    double* Wt = R.C;  // n x M: W' = C L^-T, formed in place by batched()
    double* Av = L.Av.as<double>();
    double* tv = L.tv.as<double>();
    Stager& sg = L.sg;
    sg.begin(S_APPLY, 2.0 * dM * dM * dn + 4.0 * dn * dM, 16.0 * dn * dM);
    hipLaunchKernelGGL(k_nys_vi, dim3(blocks(R.n, 256)), dim3(256), 0, st, R.r, R.n, isn2, Av);
    KCHK();
    oila::gemv(L.la, st, true, {oila::Gemv{Wt, R.r, tv, R.in, R.iM, R.in, 1.0, 0.0}});     // tv = W r
    oila::gemv(L.la, st, false, {oila::Gemv{Wt, tv, Av, R.in, R.iM, R.in, -1.0, 1.0}});   // A -= W' tv
    sg.end();
    if (obj_) {
      double* Ki = L.Ki.as<double>();
      sg.begin(S_LOGDET, 2.0 * dn, 16.0 * dn);
      hipLaunchKernelGGL(k_nys_dot, dim3(1), dim3(256), 0, st, R.r, Av, R.n, R.rs + 0);
      KCHK();
      sg.end();
      if (fused_objective()) {
        // (W'W) tiles on the MFMA core, reduced against K, dK in the same kernel
        const int Tn = (int)blocks(R.n, 64), Tk = (int)blocks(R.M, 64);
        const int ntri = Tn * (Tn + 1) / 2;
        sg.begin(S_KI, dn * dn * dM, 8.0 * dn * dM);
        hipLaunchKernelGGL(k_nys_pack, dim3((unsigned)(Tn * Tk)), dim3(256), 0, st, Wt, R.n, R.M,
                           Tn, L.Wp.as<double>());
        KCHK();
        sg.end();
        sg.begin(S_GRAD, dn * dn * dM, 0.0);
        hipLaunchKernelGGL(k_nys_grad_mfma, dim3((unsigned)ntri), dim3(256), 0, st,
                           L.Wp.as<double>(), Tn, Tk, Av, R.sc, R.sq, R.n, sf2, isn2,
                           L.part.as<double>());
        KCHK();
        hipLaunchKernelGGL(k_nys_partsum, dim3(1), dim3(256), 0, st, L.part.as<double>(),
                           (int64_t)ntri, R.rs + 2);
        KCHK();
        sg.end();
      } else {
        // Ki = Vi - W'W (OI_NYS_FUSED=0 only: one full oila::gemm product; the
        // sweep below reads the lower half)
        sg.begin(S_KI, 2.0 * dn * dn * dM, 8.0 * dn * dn);
        oila::gemm(L.la, st, false, true, {oila::Gemm{Wt, Wt, Ki, R.in, R.in, R.iM, R.in, R.in, R.in, -1.0, 0.0, 0}});
        hipLaunchKernelGGL(k_nys_diag, dim3(blocks(R.n, 256)), dim3(256), 0, st, Ki, R.n, R.n, nullptr,
                           0, isn2);
        KCHK();
        sg.end();
        // the lower triangle of Ki read once (~4 n^2 bytes); inputs and A cache-resident
        sg.begin(S_GRAD, 0.0, 4.0 * dn * dn);
        const unsigned nt = blocks(R.n, 64);
        hipLaunchKernelGGL(k_nys_grad, dim3(nt, nt), dim3(256), 0, st, Ki, Av, R.sc, R.sq, R.n, sf2,
                           L.part.as<double>());
        KCHK();
        hipLaunchKernelGGL(k_nys_partsum, dim3(1), dim3(256), 0, st, L.part.as<double>(),
                           (int64_t)nt * nt, R.rs + 2);
        KCHK();
        sg.end();
      }
    }
    if (pred_) {
      // k* = SGPkernel(x, xs=xs); fs = mean + k*.A; k*'Ki k* = |k*|^2/sn2 - |W k*|^2
      sg.begin(S_PRED, 2.0 * dn * dM, 8.0 * dn * dM);
      double* ks = L.ks.as<double>();
      double* kv = L.kv.as<double>();
      hipLaunchKernelGGL(k_nys_scale, dim3(1), dim3(64), 0, st, (*tab_)[R.c].xs,
                         (int64_t)1, R.hp[0], R.hp[1], R.hp[2], L.xsc.as<double>(), nullptr);
      KCHK();
      hipLaunchKernelGGL(k_nys_cross, dim3(blocks(R.n, 256), 1), dim3(256), 0, st, R.sc, nullptr,
                         R.n, L.xsc.as<double>(), nullptr, sf2, ks, R.n);
      KCHK();
      hipLaunchKernelGGL(k_nys_dot, dim3(1), dim3(256), 0, st, ks, Av, R.n, R.rs + 7);
      KCHK();
      hipLaunchKernelGGL(k_nys_dot, dim3(1), dim3(256), 0, st, ks, ks, R.n, R.rs + 8);
      KCHK();
      oila::gemv(L.la, st, true, {oila::Gemv{Wt, ks, kv, R.in, R.iM, R.in, 1.0, 0.0}});  // kv = W k*
      hipLaunchKernelGGL(k_nys_dot, dim3(1), dim3(256), 0, st, kv, kv, R.M, R.rs + 9);
      KCHK();
      sg.end();
    }
  }

  const std::vector<CellSrc>* tab_;
  int64_t nmax_ = 0, cap_ = 0;
  hipStream_t st_;
  bool obj_ = false, pred_ = false, alloc_obj_, alloc_pred_;
  Buf res_, info_;
  Buf sc_, sq_, Kmm_, eval_, stl_, C_, B_, EW_, Dinv_, Knm_, U1_;
  bool b3_ = true;
  int64_t chunk_ = 1;
  int padq_ = 32;
  int64_t mpmax_ = 0;
  size_t ewd_ = 0;
  int64_t nd64_ = 0;
  oila::Stager la_;
  Stager sg_;
  std::vector<Lane*> lanes_;
  hipEvent_t ready_ = nullptr;
  const std::vector<int64_t>* cells_ = nullptr;
  const double* hyp_ = nullptr;
  std::vector<int64_t> order_;
  std::vector<int64_t> cellv_;
  std::vector<double> hypv_;
  int64_t ncq_ = 0;
  double mean_ = 0.0;
  bool own_ = false;
  double* hr_ = nullptr;       // pinned: the result copies stay asynchronous
  int32_t* hi_ = nullptr;
};

template <class F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const HipErr& e) {
    return oi_set_last_error(OI_E_HIP, e.msg.c_str());
  } catch (const oila::LinalgErr& e) {
    return oi_set_last_error(OI_E_HIP, e.msg.c_str());
  } catch (const std::bad_alloc&) {
    return oi_set_last_error(OI_E_NOMEM, "allocation failed");
  }
}

}  // namespace

extern "C" int oi_nystrom_batch(const double* xyt, const double* y, const int64_t* offs,
                                int64_t ncell, const int64_t* sel, const int64_t* soffs,
                                const double* hyp, const double* xs, double mean, double* nlz,
                                double* grad, double* pred, int32_t* status,
                                const oi_options* opts) {
  Batch b{xyt, y, offs, ncell, sel, soffs};
  if (int rc = check_batch(b)) return rc;
  if (ncell == 0) return 0;
  if (!hyp || !status) return oi_set_last_error(OI_E_ARG, "null pointer");
  if ((nlz == nullptr) != (grad == nullptr))
    return oi_set_last_error(OI_E_ARG, "nlz and grad go together");
  const bool want_obj = nlz != nullptr, want_pred = pred != nullptr;
  if (want_pred && !xs) return oi_set_last_error(OI_E_ARG, "pred needs xs");
  for (int64_t q = 0; q < ncell * 5; ++q)
    if (!(hyp[q] > 0.0)) return oi_set_last_error(OI_E_ARG, "hypers must be > 0");
  oi_options o;
  if (int rc = setup(opts, o)) return rc;
  return guarded([&] {
    BatchDev bd(b, want_pred ? xs : nullptr, o.device_inputs != 0, (hipStream_t)o.stream);
    Runner R(&bd.rows, b.nmax, b.mmax, ncell, o, want_obj, want_pred);
    std::vector<int64_t> cells(ncell);
    for (int64_t c = 0; c < ncell; ++c) cells[c] = c;
    std::vector<CellOut> out(ncell);
    R.run(cells, hyp, mean, out.data(), want_obj, want_pred);
    for (int64_t c = 0; c < ncell; ++c) {
      status[c] = out[c].status;
      if (want_obj) {
        nlz[c] = out[c].nlz;
        for (int q = 0; q < 5; ++q) grad[c * 5 + q] = out[c].grad[q];
      }
      if (want_pred) {
        pred[c * 3 + 0] = out[c].fs;
        pred[c * 3 + 1] = out[c].sd;
        pred[c * 3 + 2] = out[c].sprior;
      }
    }
    return 0;
  });
}

extern "C" int oi_nystrom_fit_batch(const double* xyt, const double* y, const int64_t* offs,
                                    int64_t ncell, const int64_t* sel, const int64_t* soffs,
                                    const double* x0, const double* xs, double mean, double* out,
                                    int32_t* status, int32_t* info, const oi_options* opts) {
  Batch b{xyt, y, offs, ncell, sel, soffs};
  if (int rc = check_batch(b)) return rc;
  if (ncell == 0) return 0;
  if (!x0 || !xs || !out || !status) return oi_set_last_error(OI_E_ARG, "null pointer");
  oi_options o;
  if (int rc = setup(opts, o)) return rc;
  // scipy: maxiter = len(x0) * 200 for the notebook's 5 hypers
  const int32_t maxiter = o.maxiter < 0 ? 1000 : o.maxiter;
  return guarded([&] {
    // one restated scipy CG per cell (6-slot; the sixth gradient is 0, which
    // leaves scipy's iteration unchanged), every round one pass over the cells
    // still iterating
    std::vector<oi_cg*> cg(ncell, nullptr);
    struct Free {
      std::vector<oi_cg*>& v;
      ~Free() {
        for (auto* p : v)
          if (p) oi_cg_destroy(p);
      }
    } free_{cg};
    double x6[6];
    for (int q = 0; q < 5; ++q) x6[q] = x0[q];
    x6[5] = 0.0;
    std::vector<double> req(ncell * 6);
    std::vector<char> live(ncell, 0);
    for (int64_t c = 0; c < ncell; ++c) {
      cg[c] = oi_cg_create(x6, o.gtol, maxiter);
      if (!cg[c]) throw std::bad_alloc();
      const int rc = oi_cg_step(cg[c], req.data() + c * 6);
      if (rc < 0) throw HipErr{"oi_cg_step failed"};
      live[c] = rc == 1;
    }
    // cells are independent: split them into G groups (OI_NYS_GROUPS, default 2),
    // each with its own stream and lanes, so one group's latency-bound batched
    // eigh overlaps the other's panels / objective pass; each group is
    // collected and re-queued as soon as its round is done
    int G = 2;
    if (const char* e = getenv("OI_NYS_GROUPS")) G = atoi(e);
    G = std::max(1, std::min<int>(G, (int)ncell));
    std::vector<std::vector<int64_t>> gcells(G);
    for (int64_t c = 0; c < ncell; ++c) gcells[c % G].push_back(c);
    BatchDev bd(b, xs, o.device_inputs != 0, (hipStream_t)o.stream);
    std::vector<std::unique_ptr<Runner>> RG;
    for (int g = 0; g < G; ++g)
      RG.emplace_back(new Runner(&bd.rows, b.nmax, b.mmax, (int64_t)gcells[g].size(), o, true, false, G > 1));
    std::vector<std::vector<int64_t>> qcells(G);
    std::vector<CellOut> res(ncell);
    auto queue = [&](int g) {
      qcells[g].clear();
      std::vector<double> hyp;
      for (int64_t c : gcells[g])
        if (live[c]) {
          qcells[g].push_back(c);
          for (int q = 0; q < 5; ++q) hyp.push_back(std::exp(req[c * 6 + q]));  // NB1 SMLII
        }
      if (!qcells[g].empty()) RG[g]->enqueue(qcells[g], hyp.data(), mean, true, false);
    };
    for (int g = 0; g < G; ++g) queue(g);
    for (bool any = true; any;) {
      any = false;
      for (int g = 0; g < G; ++g) {
        if (qcells[g].empty()) continue;
        any = true;
        RG[g]->collect(res.data());
        for (size_t k = 0; k < qcells[g].size(); ++k) {
          const int64_t c = qcells[g][k];
          const double g6[6] = {res[k].grad[0], res[k].grad[1], res[k].grad[2], res[k].grad[3],
                                res[k].grad[4], 0.0};
          if (oi_cg_feed(cg[c], res[k].nlz, g6) != 0) throw HipErr{"oi_cg_feed failed"};
          const int rc = oi_cg_step(cg[c], req.data() + c * 6);
          if (rc < 0) throw HipErr{"oi_cg_step failed"};
          live[c] = rc == 1;
        }
        queue(g);
      }
    }
    RG.clear();
    Runner R(&bd.rows, b.nmax, b.mmax, ncell, o, false, true);
    std::vector<int64_t> cells;
    std::vector<double> hyp;
    // NB1 code cell 5: GPR(approx=True) at the fitted hypers
    cells.clear();
    hyp.clear();
    std::vector<double> xf(ncell * 6);
    for (int64_t c = 0; c < ncell; ++c) {
      double fun;
      int32_t nit, cst;
      int64_t nfev, njev, nobj;
      oi_cg_result(cg[c], xf.data() + c * 6, &fun, &nit, &cst, &nfev, &njev, &nobj);
      if (info) {
        info[c * 4 + 0] = nit;
        info[c * 4 + 1] = cst;
        info[c * 4 + 2] = (int32_t)nfev;
        info[c * 4 + 3] = (int32_t)nobj;
      }
      cells.push_back(c);
      for (int q = 0; q < 5; ++q) hyp.push_back(std::exp(xf[c * 6 + q]));
    }
    R.run(cells, hyp.data(), mean, res.data(), false, true);
    for (int64_t c = 0; c < ncell; ++c) {
      status[c] = res[c].status;
      out[c * 8 + 0] = res[c].fs;
      out[c * 8 + 1] = res[c].sd;
      out[c * 8 + 2] = res[c].sprior;
      for (int q = 0; q < 5; ++q) out[c * 8 + 3 + q] = hyp[c * 5 + q];
    }
    return 0;
  });
}

// ---- Nystrom fit session: continuous batching across calls (NB1 code cell 5
// as a stream of batches).  Every submitted batch joins one queue of cells;
// each of the G groups (own stream, Runner) keeps up to CAP cells fitting and
// refills from the queue as cells finish, so a call's slowest cells overlap
// the next calls' cells instead of idling the GPU (the one-shot fit waits for
// its slowest cell).  A ticket completes when its last cell is fitted; its
// predictions (GPR(approx=True) at the fitted hypers) run then.  Per-cell
// arithmetic never depends on the other resident cells, so results equal
// oi_nystrom_fit_batch's bit for bit.
namespace {
struct NysTicket {
  std::unique_ptr<BatchDev> dev;
  int64_t first = 0, count = 0, unfitted = 0;
  double mean = 0.0;
  double* out = nullptr;
  int32_t* status = nullptr;
  int32_t* info = nullptr;
  bool done = false;
};
}  // namespace

struct oi_nystrom_session {
  oi_options o;
  int G = 2;
  // resident fitting cells per group (OI_NYS_CAP): the batched eigensolver's
  // per-column launches cost the same for 32 or 64 matrices, so a bigger chunk
  // amortises them -- 5.46 / 6.69 / 6.63 cells/s at 32 / 64 / 128
  // (--workload nystrom, one box, profiles/r05/nystrom_cap/)
  int64_t cap = 64;
  int32_t maxiter = 1000;
  double gtol = 1e-5;
  std::vector<CellSrc> tab;          // every submitted cell, by global id
  std::vector<int64_t> owner;        // cell -> ticket
  std::vector<oi_cg*> cg;            // per cell (null before admission / after release)
  std::vector<double> req;           // per cell: the requested point (6)
  std::vector<double> x0;            // per cell: the batch's x0 (5)
  std::deque<int64_t> queue;         // submitted, not admitted
  std::vector<std::unique_ptr<NysTicket>> tickets;
  int64_t nmax = 0, mmax = 0;        // the Runners' sizes
  struct Grp {
    std::unique_ptr<Runner> R;
    std::vector<int64_t> active, inflight;
  };
  std::vector<Grp> grp;
  std::unique_ptr<Runner> pred;      // predictions of completed tickets
  // inputs of submitted batches are allocated, copied and freed on this stream
  // (stream-ordered): dropping a completed batch never drains the groups'
  // rounds in flight (a ticket's cells are in no round by then)
  hipStream_t io = nullptr;

  ~oi_nystrom_session() {
    for (auto* p : cg)
      if (p) oi_cg_destroy(p);
    grp.clear();
    pred.reset();
    tickets.clear();
    if (io) {
      (void)hipStreamSynchronize(io);
      (void)hipStreamDestroy(io);
    }
  }

  void build_runners(int64_t nm, int64_t mm) {
    nmax = std::max(nmax, nm);
    mmax = std::max(mmax, mm);
    grp.resize(G);
    for (auto& g : grp) g.R.reset(new Runner(&tab, nmax, mmax, cap, o, true, false, G > 1));
    pred.reset(new Runner(&tab, nmax, mmax, cap, o, false, true, true));
  }

  void feed(Grp& g) {  // collect a group's round, advance its cells' CG
    if (g.inflight.empty()) return;
    std::vector<CellOut> res(g.inflight.size());
    g.R->collect(res.data());
    for (size_t k = 0; k < g.inflight.size(); ++k) {
      const int64_t c = g.inflight[k];
      const double g6[6] = {res[k].grad[0], res[k].grad[1], res[k].grad[2], res[k].grad[3], res[k].grad[4], 0.0};
      if (oi_cg_feed(cg[c], res[k].nlz, g6) != 0) throw HipErr{"oi_cg_feed failed"};
      const int rc = oi_cg_step(cg[c], req.data() + c * 6);
      if (rc < 0) throw HipErr{"oi_cg_step failed"};
      if (rc == 0) finished(c);
    }
    g.inflight.clear();
    std::vector<int64_t> keep;
    for (int64_t c : g.active)
      if (cg[c] && !fitted_[c]) keep.push_back(c);
    g.active.swap(keep);
  }

  std::vector<char> fitted_;

  void finished(int64_t c) {
    fitted_[c] = 1;
    NysTicket& t = *tickets[owner[c]];
    if (--t.unfitted == 0) complete(t);
  }

  void complete(NysTicket& t) {
    // GPR(approx=True) at the fitted hypers, in chunks of the Runner capacity
    Runner& R = *pred;
    std::vector<CellOut> res(cap);
    for (int64_t a = 0; a < t.count; a += cap) {
      const int64_t b = std::min(t.count, a + cap);
      std::vector<int64_t> cells;
      std::vector<double> hyp;
      for (int64_t k = a; k < b; ++k) {
        const int64_t c = t.first + k;
        double xf[6], fun;
        int32_t nit, cst;
        int64_t nfev, njev, nobj;
        oi_cg_result(cg[c], xf, &fun, &nit, &cst, &nfev, &njev, &nobj);
        if (t.info) {
          t.info[k * 4 + 0] = nit;
          t.info[k * 4 + 1] = cst;
          t.info[k * 4 + 2] = (int32_t)nfev;
          t.info[k * 4 + 3] = (int32_t)nobj;
        }
        cells.push_back(c);
        for (int q = 0; q < 5; ++q) hyp.push_back(std::exp(xf[q]));
      }
      R.run(cells, hyp.data(), t.mean, res.data(), false, true);
      for (int64_t k = a; k < b; ++k) {
        const CellOut& r = res[k - a];
        t.status[k] = r.status;
        t.out[k * 8 + 0] = r.fs;
        t.out[k * 8 + 1] = r.sd;
        t.out[k * 8 + 2] = r.sprior;
        for (int q = 0; q < 5; ++q) t.out[k * 8 + 3 + q] = hyp[(k - a) * 5 + q];
      }
    }
    for (int64_t k = 0; k < t.count; ++k) {
      oi_cg_destroy(cg[t.first + k]);
      cg[t.first + k] = nullptr;
    }
    t.done = true;
    t.dev.reset();  // no round reads the batch any more: freed in io-stream order
  }

  void admit(Grp& g) {
    while ((int64_t)g.active.size() < cap && !queue.empty()) {
      const int64_t c = queue.front();
      queue.pop_front();
      double x6[6];
      for (int q = 0; q < 5; ++q) x6[q] = x0[c * 5 + q];
      x6[5] = 0.0;
      cg[c] = oi_cg_create(x6, gtol, maxiter);
      if (!cg[c]) throw std::bad_alloc();
      const int rc = oi_cg_step(cg[c], req.data() + c * 6);
      if (rc < 0) throw HipErr{"oi_cg_step failed"};
      if (rc == 0) {
        finished(c);
        continue;
      }
      g.active.push_back(c);
    }
  }

  void launch(Grp& g) {  // one evaluation round of the group's live cells
    g.inflight.clear();
    std::vector<double> hyp;
    for (int64_t c : g.active) {
      g.inflight.push_back(c);
      for (int q = 0; q < 5; ++q) hyp.push_back(std::exp(req[c * 6 + q]));  // NB1 SMLII
    }
    if (!g.inflight.empty()) g.R->enqueue(g.inflight, hyp.data(), tickets[owner[g.inflight[0]]]->mean, true, false);
  }

  // rounds until ticket t (all work when t < 0) is complete
  void wait(int64_t t) {
    while (true) {
      if (t >= 0 && tickets[t]->done) return;
      bool any = false;
      for (auto& g : grp) {
        feed(g);
        admit(g);
        launch(g);
        any = any || !g.inflight.empty();
      }
      if (!any) {
        if (t >= 0 && !tickets[t]->done) throw HipErr{"nystrom session: ticket cannot complete"};
        return;
      }
    }
  }

  // every group idle (their rounds collected and fed), e.g. before the Runners are rebuilt
  void drain() {
    for (auto& g : grp) feed(g);
  }
};

extern "C" oi_nystrom_session* oi_nystrom_session_create(const oi_options* opts) {
  oi_options o;
  if (setup(opts, o)) return nullptr;
  auto* s = new oi_nystrom_session();
  s->o = o;
  if (hipStreamCreateWithFlags(&s->io, hipStreamNonBlocking) != hipSuccess) {
    delete s;
    oi_set_last_error(OI_E_HIP, "hipStreamCreate failed");
    return nullptr;
  }
  s->maxiter = o.maxiter < 0 ? 1000 : o.maxiter;  // scipy: len(x0) * 200 for NB1's 5 hypers
  s->gtol = o.gtol;
  if (const char* e = getenv("OI_NYS_GROUPS")) s->G = std::max(1, atoi(e));
  if (const char* e = getenv("OI_NYS_CAP")) s->cap = std::max(1, atoi(e));
  return s;
}

extern "C" int64_t oi_nystrom_session_submit(oi_nystrom_session* s, const double* xyt, const double* y,
                                             const int64_t* offs, int64_t ncell, const int64_t* sel,
                                             const int64_t* soffs, const double* x0, const double* xs,
                                             double mean, double* out, int32_t* status, int32_t* info) {
  if (!s) return oi_set_last_error(OI_E_ARG, "null session");
  Batch b{xyt, y, offs, ncell, sel, soffs};
  if (int rc = check_batch(b)) return rc;
  if (ncell > 0 && (!x0 || !xs || !out || !status)) return oi_set_last_error(OI_E_ARG, "null pointer");
  int64_t ticket = -1;
  const int rc = guarded([&] {
    HC(hipSetDevice(s->o.device));
    auto t = std::make_unique<NysTicket>();
    t->first = (int64_t)s->tab.size();
    t->count = ncell;
    t->unfitted = ncell;
    t->mean = mean;
    t->out = out;
    t->status = status;
    t->info = info;
    ticket = (int64_t)s->tickets.size();
    if (ncell > 0) {
      t->dev.reset(new BatchDev(b, xs, s->o.device_inputs != 0, s->io));
      if (s->grp.empty() || b.nmax > s->nmax || b.mmax > s->mmax) {
        s->drain();  // no round in flight over the old Runners' workspaces
        s->build_runners(b.nmax, b.mmax);
      }
      for (int64_t c = 0; c < ncell; ++c) {
        s->tab.push_back(t->dev->rows[c]);
        s->owner.push_back(ticket);
        s->cg.push_back(nullptr);
        s->fitted_.push_back(0);
        for (int q = 0; q < 6; ++q) s->req.push_back(0.0);
        for (int q = 0; q < 5; ++q) s->x0.push_back(x0[q]);
        s->queue.push_back(t->first + c);
      }
    } else {
      t->done = true;
    }
    s->tickets.push_back(std::move(t));
    return 0;
  });
  return rc ? rc : ticket;
}

extern "C" int oi_nystrom_session_wait(oi_nystrom_session* s, int64_t ticket) {
  if (!s) return oi_set_last_error(OI_E_ARG, "null session");
  if (ticket >= (int64_t)s->tickets.size()) return oi_set_last_error(OI_E_ARG, "unknown ticket");
  return guarded([&] {
    HC(hipSetDevice(s->o.device));
    s->wait(ticket);
    return 0;
  });
}

extern "C" void oi_nystrom_session_destroy(oi_nystrom_session* s) {
  if (!s) return;
  (void)hipSetDevice(s->o.device);
  try {
    s->drain();
  } catch (...) {
  }
  delete s;
}
