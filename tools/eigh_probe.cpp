// Phase times of oila::eigh on a chunk of Matern K_mm matrices (the Nystrom
// variant's M = 925 padded to 928, 32 per chunk) (build: tools/build_eigh_probe.sh).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../optimalinterpolation_amd/csrc/oi_linalg.h"


#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      return 1;                                                           \
    }                                                                     \
  } while (0)

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 928, nb = argc > 2 ? atoi(argv[2]) : 32, reps = 3;
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> U(-3e5, 3e5), Tt(0, 8);
  const size_t MM = (size_t)M * M, ew = oila::eigh_workspace_doubles(M);
  std::vector<double> h(MM * nb);
  for (int b = 0; b < nb; ++b) {
    std::vector<double> x(3 * M);
    for (int i = 0; i < M; ++i) {
      x[3 * i] = U(rng) / 5e4;
      x[3 * i + 1] = U(rng) / 5e4;
      x[3 * i + 2] = Tt(rng) / 1.0;
    }
    for (int j = 0; j < M; ++j)
      for (int i = 0; i < M; ++i) {
        double d = 0;
        for (int q = 0; q < 3; ++q) d += (x[3 * i + q] - x[3 * j + q]) * (x[3 * i + q] - x[3 * j + q]);
        const double Q = std::sqrt(3.0 * d);
        h[MM * b + i + (size_t)M * j] = 6e-3 * (1 + Q) * std::exp(-Q) + (i == j ? 1e-4 : 0.0);
      }
  }
  double *A, *A0, *w, *work;
  CK(hipMalloc(&A, MM * nb * 8));
  CK(hipMalloc(&A0, MM * nb * 8));
  CK(hipMalloc(&w, (size_t)M * nb * 8));
  CK(hipMalloc(&work, ew * nb * 8));
  CK(hipMemcpy(A0, h.data(), MM * nb * 8, hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  oila::Stager S;
  S.bind(st);
  std::vector<oila::Eigh> es;
  for (int b = 0; b < nb; ++b) es.push_back(oila::Eigh{A + MM * b, w + (size_t)M * b, work + ew * b, M, M});
  hipEvent_t ev[5];
  for (auto& e : ev) CK(hipEventCreate(&e));
  double ph[4] = {0, 0, 0, 0};
  for (int r = 0; r <= reps; ++r) {
    CK(hipMemcpyAsync(A, A0, MM * nb * 8, hipMemcpyDeviceToDevice, st));
    oila::eigh(S, st, es, [&](int k) { (void)hipEventRecord(ev[k], st); });
    CK(hipStreamSynchronize(st));
    S.reset();
    if (r == 0) continue;  // warm-up
    for (int k = 0; k < 4; ++k) {
      float ms;
      CK(hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
      ph[k] += ms / reps;
    }
  }
  printf("eigh M=%d x %d: sytrd %.2f ms, stebz+stein %.2f ms, orth %.2f ms, back %.2f ms\n", M, nb, ph[0],
         ph[1], ph[2], ph[3]);
  std::vector<double> wh((size_t)M * nb);
  CK(hipMemcpy(wh.data(), w, wh.size() * 8, hipMemcpyDeviceToHost));
  printf("eigenvalues of matrix 0: min %.3e max %.3e\n", wh[0], wh[M - 1]);
  // matrix 0's eigenvectors: orthogonality max |U'U - I| and residual max |AU - U diag(w)| / max|A|
  std::vector<double> Uh(MM);
  CK(hipMemcpy(Uh.data(), A, MM * 8, hipMemcpyDeviceToHost));
  double orth = 0.0, res = 0.0, amax = 0.0;
  for (size_t i = 0; i < MM; ++i) amax = std::max(amax, std::fabs(h[i]));
  for (int a = 0; a < M; ++a)
    for (int b = 0; b <= a; ++b) {
      double s = 0.0;
      for (int i = 0; i < M; ++i) s += Uh[i + (size_t)M * a] * Uh[i + (size_t)M * b];
      orth = std::max(orth, std::fabs(s - (a == b ? 1.0 : 0.0)));
    }
  for (int b = 0; b < M; ++b)
    for (int i = 0; i < M; ++i) {
      double s = 0.0;
      for (int k = 0; k < M; ++k) s += h[i + (size_t)M * k] * Uh[k + (size_t)M * b];
      res = std::max(res, std::fabs(s - wh[b] * Uh[i + (size_t)M * b]));
    }
  printf("matrix 0: orthogonality %.3e, residual %.3e x max|A|\n", orth, res / amax);
  return 0;
}
