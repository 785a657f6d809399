// TF/s of oila::gemm on the Nystrom variant's phase-3 shapes, batched over a
// chunk of cells: U1 = Knm u (n x M, k = M) and B = ut' C (M x M, k = n)
// (build: hipcc -O3 -std=c++20 --offload-arch=gfx950 -ffp-contract=off
//  tools/gemm_probe.cpp optimalinterpolation_amd/csrc/oi_linalg.hip -o tools/gemm_probe)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
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
  const int n = argc > 1 ? atoi(argv[1]) : 4600, M = argc > 2 ? atoi(argv[2]) : 928,
            nb = argc > 3 ? atoi(argv[3]) : 32, reps = 5;
  const size_t nM = (size_t)n * M, MM = (size_t)M * M;
  double *A, *U, *C;
  CK(hipMalloc(&A, nM * nb * 8));
  CK(hipMalloc(&U, MM * nb * 8));
  CK(hipMalloc(&C, nM * nb * 8));
  std::vector<double> h(nM * nb);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (double)((i * 2654435761u) % 1000) * 1e-3 - 0.5;
  CK(hipMemcpy(A, h.data(), nM * nb * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(C, h.data(), nM * nb * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(U, h.data(), MM * nb * 8, hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  oila::Stager S;
  S.bind(st);
  std::vector<oila::Gemm> g1, g2;
  for (int b = 0; b < nb; ++b) {
    g1.push_back(oila::Gemm{A + nM * b, U + MM * b, C + nM * b, n, M, M, n, M, n, 1.0, 0.0, 0});
    g2.push_back(oila::Gemm{A + nM * b, C + nM * b, U + MM * b, M, M, n, n, n, M, 1.0, 0.0, 0});
  }
  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  double t1 = 0, t2 = 0;
  for (int r = 0; r <= reps; ++r) {
    CK(hipEventRecord(e0, st));
    oila::gemm(S, st, false, false, g1);
    CK(hipEventRecord(e1, st));
    oila::gemm(S, st, true, false, g2);
    CK(hipEventRecord(e2, st));
    CK(hipStreamSynchronize(st));
    S.reset();
    if (r == 0) continue;
    float a, b;
    CK(hipEventElapsedTime(&a, e0, e1));
    CK(hipEventElapsedTime(&b, e1, e2));
    t1 += a / reps;
    t2 += b / reps;
  }
  const double fl = 2.0 * n * (double)M * M * nb;
  printf("n=%d M=%d x %d: U1 = Knm u (NN) %.3f ms %.1f TF/s; B = ut' C (TN) %.3f ms %.1f TF/s\n", n, M, nb, t1,
         fl / t1 * 1e-9, t2, fl / t2 * 1e-9);
  return 0;
}
