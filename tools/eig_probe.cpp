// Probe: rocSOLVER symmetric eigensolvers on Matern K_mm matrices (M x M),
// single vs strided-batched, to pick the Nystrom path's eigh.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#define H(x) do { if ((x) != hipSuccess) { printf("hip error %s line %d\n", #x, __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 925, B = argc > 2 ? atoi(argv[2]) : 8;
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> U(-3e5, 3e5);
  std::vector<double> A((size_t)M * M * B);
  for (int b = 0; b < B; ++b) {
    std::vector<double> p(M * 3);
    for (int i = 0; i < M; ++i) { p[i * 3] = U(g) / 9e4; p[i * 3 + 1] = U(g) / 7e4; p[i * 3 + 2] = (g() % 9) / 2.3; }
    for (int j = 0; j < M; ++j)
      for (int i = 0; i < M; ++i) {
        double d = 0; for (int k = 0; k < 3; ++k) { double t = std::sqrt(3.0) * (p[i*3+k] - p[j*3+k]); d += t * t; }
        d = std::sqrt(d);
        A[(size_t)b * M * M + i + (size_t)M * j] = 8.7e-3 * (1 + d) * std::exp(-d);
      }
  }
  double *dA, *dW, *dD, *dE, *res; int *info, *sweeps;
  H(hipMalloc(&dA, A.size() * 8)); H(hipMalloc(&dW, A.size() * 8));
  H(hipMalloc(&dD, (size_t)M * B * 8)); H(hipMalloc(&dE, (size_t)M * B * 8));
  H(hipMalloc(&res, B * 8)); H(hipMalloc(&info, B * 4)); H(hipMalloc(&sweeps, B * 4));
  rocblas_handle h; rocblas_create_handle(&h);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto reset = [&] { (void)hipMemcpy(dW, A.data(), A.size() * 8, hipMemcpyHostToDevice); };
  auto timeit = [&](const char* name, auto f, int per) {
    reset(); f(); hipDeviceSynchronize();  // warm
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
      reset(); hipDeviceSynchronize();
      hipEventRecord(e0, 0); f(); hipEventRecord(e1, 0); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1); best = ms < best ? ms : best;
    }
    printf("%-34s M=%d: %9.3f ms total, %8.3f ms per matrix\n", name, M, best, best / per);
  };
  timeit("syevd x1", [&] { rocsolver_dsyevd(h, rocblas_evect_original, rocblas_fill_lower, M, dW, M, dD, dE, info); }, 1);
  timeit("syevd loop xB", [&] { for (int b = 0; b < B; ++b) rocsolver_dsyevd(h, rocblas_evect_original, rocblas_fill_lower, M, dW + (size_t)b*M*M, M, dD + b*M, dE + b*M, info + b); }, B);
  timeit("syevd strided_batched xB", [&] { rocsolver_dsyevd_strided_batched(h, rocblas_evect_original, rocblas_fill_lower, M, dW, M, (rocblas_stride)M*M, dD, M, dE, M, info, B); }, B);
  timeit("syevdj strided_batched xB", [&] { rocsolver_dsyevdj_strided_batched(h, rocblas_evect_original, rocblas_fill_lower, M, dW, M, (rocblas_stride)M*M, dD, M, info, B); }, B);
  timeit("syevj strided_batched xB", [&] { rocsolver_dsyevj_strided_batched(h, rocblas_esort_ascending, rocblas_evect_original, rocblas_fill_lower, M, dW, M, (rocblas_stride)M*M, 0.0, res, 100, sweeps, dD, M, info, B); }, B);
  timeit("potrf x1 (reference point)", [&] { rocsolver_dpotrf(h, rocblas_fill_lower, M, dW, M, info); }, 1);
  // accuracy of syevd vs syevj eigenvalues
  std::vector<double> d1(M), d2(M);
  reset(); rocsolver_dsyevd(h, rocblas_evect_original, rocblas_fill_lower, M, dW, M, dD, dE, info);
  hipMemcpy(d1.data(), dD, M * 8, hipMemcpyDeviceToHost);
  reset(); rocsolver_dsyevj_strided_batched(h, rocblas_esort_ascending, rocblas_evect_original, rocblas_fill_lower, M, dW, M, (rocblas_stride)M*M, 0.0, res, 100, sweeps, dD, M, info, 1);
  hipMemcpy(d2.data(), dD, M * 8, hipMemcpyDeviceToHost);
  double mx = 0; for (int i = 0; i < M; ++i) mx = std::fmax(mx, std::fabs(d1[i] - d2[i]));
  int sw; hipMemcpy(&sw, sweeps, 4, hipMemcpyDeviceToHost);
  printf("max |syevd - syevj| eigenvalue diff %.3e (largest %.3e), syevj sweeps %d\n", mx, d1[M-1], sw);
  return 0;
}
