// Diagnose the fp64 tile-GEMM core (csrc/oi_gemm.h): is it MFMA-, pipeline- or
// memory-bound?  Each WG computes sum_p A_p^T B_p over P 64x64 tile pairs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../optimalinterpolation_amd/csrc/oi_gemm.h"
#define CHK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

// mode 0: A, B distinct per WG (stream from HBM); 1: A shared per group of 32 WGs; 2: tiny L2-resident set
__global__ __launch_bounds__(256) void probe(const double* A, const double* B, double* C, int P, int mode) {
  __shared__ __attribute__((aligned(16))) double lds[GEMM_LDS];
  Quad acc; quad_zero(acc);
  const int wg = blockIdx.x;
  gemm_kmajor(acc, lds, P, [&](int p, const double*& a, const double*& b) {
    size_t ta, tb;
    if (mode == 0) { ta = (size_t)wg * P + p; tb = (size_t)wg * P + p; }
    else if (mode == 1) { ta = (size_t)(wg / 32) * P + p; tb = (size_t)wg * P + p; }
    else { ta = p & 3; tb = (p + 1) & 3; }
    a = A + ta * 4096; b = B + tb * 4096;
  });
  double s = 0; for (int a = 0; a < 2; ++a) for (int b = 0; b < 2; ++b) for (int r = 0; r < 4; ++r) s += acc.c[a][b][r];
  C[(size_t)wg * 256 + threadIdx.x] = s;
}

int main(int argc, char** argv) {
  const int P = 32, nwg = 4096;
  size_t tiles = (size_t)nwg * P;
  double *A, *B, *C;
  CHK(hipMalloc(&A, tiles * 4096 * 8)); CHK(hipMalloc(&B, tiles * 4096 * 8)); CHK(hipMalloc(&C, (size_t)nwg * 256 * 8));
  CHK(hipMemset(A, 0, tiles * 4096 * 8)); CHK(hipMemset(B, 0, tiles * 4096 * 8));
  std::vector<double> h(4096 * 4); for (size_t i = 0; i < h.size(); ++i) h[i] = 1.0 + 1e-3 * (i % 97);
  CHK(hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice)); CHK(hipMemcpy(B, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  const char* names[] = {"stream A,B from HBM", "A shared by 32 WGs", "L2-resident operands"};
  for (int mode = 0; mode < 3; ++mode) {
    probe<<<nwg, 256>>>(A, B, C, P, mode); CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) probe<<<nwg, 256>>>(A, B, C, P, mode);
    CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
    double fl = 2.0 * 64 * 64 * 64 * P * nwg;
    double bytes = (mode == 0 ? 2.0 : mode == 1 ? 1.0 + 1.0/32 : 0.0) * 32768.0 * P * nwg;
    printf("%-24s %8.3f ms  %6.2f TF/s  algorithmic HBM %6.2f TB/s\n", names[mode], ms, fl / ms / 1e9, bytes / ms / 1e9);
  }
  return 0;
}
