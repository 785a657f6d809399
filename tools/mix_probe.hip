// Probe: do fp64 MFMA and fp64 VALU FMA waves run concurrently on gfx950?
// One kernel, 8 waves per workgroup (two per SIMD); `mode` picks what the
// waves do: 0 = all MFMA, 1 = all VALU, 2 = even waves MFMA + odd waves VALU,
// 3 = even waves MFMA, odd waves idle, 4 = odd waves VALU, even idle.
// Each working wave does a fixed amount of work, so mode 2's time against
// modes 3 and 4 says whether the two pipes overlap (max) or share (sum).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CHK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

__device__ __forceinline__ double do_mfma(int iters) {
  const int l = threadIdx.x & 63;
  double a = 1.0 + l * 1e-3, b = 1.0 - l * 1e-3;
  d4 c[8];
  for (int i = 0; i < 8; i++) c[i] = (d4){0, 0, 0, 0};
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < 8; i++) s += c[i][0] + c[i][1] + c[i][2] + c[i][3];
  return s;
}
__device__ __forceinline__ double do_valu(int iters) {
  const int l = threadIdx.x & 63;
  double a = 1.0 + l * 1e-9, b = 1.0 - l * 1e-9;
  double c[16];
  for (int i = 0; i < 16; i++) c[i] = 0;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < 16; i++) c[i] = fma(a, b, c[i]);
  }
  double s = 0;
  for (int i = 0; i < 16; i++) s += c[i];
  return s;
}
// MFMA wave: 8 MFMA (2048 flop each per wave) per iter; VALU wave: 16 FMA x 64 lanes x 2 flop per iter
__global__ __launch_bounds__(512) void mix(double* out, int mode, int it_m, int it_v) {
  const int w = threadIdx.x >> 6;
  double s = 0;
  const bool even = (w & 1) == 0;
  if (mode == 0 || ((mode == 2 || mode == 3) && even)) s = do_mfma(it_m);
  else if (mode == 1 || ((mode == 2 || mode == 4) && !even)) s = do_valu(it_v);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main() {
  double* out;
  CHK(hipMalloc(&out, sizeof(double) * (1 << 24)));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 256 * 2, it_m = 2000, it_v = 8000;
  const double fm = 2048.0 * 8 * it_m, fv = 2.0 * 64 * 16 * it_v;  // flops per working wave
  const char* name[5] = {"all MFMA", "all VALU", "MFMA+VALU", "MFMA half", "VALU half"};
  for (int rep = 0; rep < 2; ++rep)
    for (int mode = 0; mode < 5; ++mode) {
      mix<<<blocks, 512>>>(out, mode, 10, 40);
      CHK(hipDeviceSynchronize());
      float ms;
      hipEventRecord(e0);
      mix<<<blocks, 512>>>(out, mode, it_m, it_v);
      hipEventRecord(e1);
      CHK(hipEventSynchronize(e1));
      hipEventElapsedTime(&ms, e0, e1);
      const double waves = blocks * 8.0;
      double fl = mode == 0 ? waves * fm : mode == 1 ? waves * fv : mode == 2 ? waves / 2 * (fm + fv)
                 : mode == 3 ? waves / 2 * fm : waves / 2 * fv;
      printf("%-10s %8.3f ms  %7.2f TFLOP/s fp64\n", name[mode], ms, fl / ms / 1e9);
    }
  return 0;
}
