// k_diag_factor variants: potrf + trti2 of B independent 64x64 SPD tiles, one
// 64-lane wave per tile.  Times B = 1 (tail-round latency) and B = 256.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#define CHK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)
#define NB 64

__device__ __forceinline__ double rdlane(double v, int lane) {
  const long long x = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane((int)(x & 0xffffffffLL), lane);
  const int hi = __builtin_amdgcn_readlane((int)(x >> 32), lane);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}

// V0: the round-1 kernel (row r of the tile in lane r, readlane broadcasts)
__global__ __launch_bounds__(64) void v0(const double* A, double* L, double* D) {
  const int r = threadIdx.x;
  const double* Y = A + (size_t)blockIdx.x * 4096;
  double R[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) R[q] = Y[q * NB + r];
#pragma unroll
  for (int cc = 0; cc < NB; ++cc) {
    const double d = rdlane(R[cc], cc);
    const double l = sqrt(d);
    const double lr = r > cc ? R[cc] / l : 0.0;
    R[cc] = r > cc ? lr : (r == cc ? l : R[cc]);
#pragma unroll
    for (int s2 = cc + 1; s2 < NB; ++s2) R[s2] -= lr * rdlane(R[cc], s2);
  }
#pragma unroll
  for (int q = 0; q < NB; ++q) { if (q > r) R[q] = 0.0; L[(size_t)blockIdx.x * 4096 + q * NB + r] = R[q]; }
#pragma unroll
  for (int cc = NB - 1; cc >= 0; --cc) {
    const double ajj = 1.0 / rdlane(R[cc], cc);
    double x = 0.0;
#pragma unroll
    for (int k = cc + 1; k < NB; ++k) x += R[k] * rdlane(R[cc], k);
    R[cc] = r > cc ? -ajj * x : (r == cc ? ajj : R[cc]);
  }
#pragma unroll
  for (int q = 0; q < NB; ++q) D[(size_t)blockIdx.x * 4096 + q * NB + r] = R[q];
}

// V1: one reciprocal per column (broadcast scalar), trti2 dot split in 4 chains
__global__ __launch_bounds__(64) void v1(const double* A, double* L, double* D) {
  const int r = threadIdx.x;
  const double* Y = A + (size_t)blockIdx.x * 4096;
  double R[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) R[q] = Y[q * NB + r];
#pragma unroll
  for (int cc = 0; cc < NB; ++cc) {
    const double d = rdlane(R[cc], cc);
    const double l = sqrt(d);
    const double il = 1.0 / l;
    const double lr = r > cc ? R[cc] * il : 0.0;
    R[cc] = r > cc ? lr : (r == cc ? l : R[cc]);
#pragma unroll
    for (int s2 = cc + 1; s2 < NB; ++s2) R[s2] -= lr * rdlane(R[cc], s2);
  }
#pragma unroll
  for (int q = 0; q < NB; ++q) { if (q > r) R[q] = 0.0; L[(size_t)blockIdx.x * 4096 + q * NB + r] = R[q]; }
#pragma unroll
  for (int cc = NB - 1; cc >= 0; --cc) {
    const double ajj = 1.0 / rdlane(R[cc], cc);
    double x0 = 0.0, x1 = 0.0, x2 = 0.0, x3 = 0.0;
#pragma unroll
    for (int k = cc + 1; k < NB; ++k) {
      const double p = R[k] * rdlane(R[cc], k);
      if ((k & 3) == 0) x0 += p; else if ((k & 3) == 1) x1 += p; else if ((k & 3) == 2) x2 += p; else x3 += p;
    }
    const double x = (x0 + x1) + (x2 + x3);
    R[cc] = r > cc ? -ajj * x : (r == cc ? ajj : R[cc]);
  }
#pragma unroll
  for (int q = 0; q < NB; ++q) D[(size_t)blockIdx.x * 4096 + q * NB + r] = R[q];
}

// V2: LDS broadcasts instead of readlane.  potrf: lane r writes column cc
// entry, every lane reads the column with broadcast ds_read_b128.
// trti2: row-oriented -> column cc of Inv needs Inv[r][k] (own) and L[k][cc]
// (column cc of L, broadcast from LDS, stored once after potrf).
__global__ __launch_bounds__(64) void v2(const double* A, double* L, double* D) {
  __shared__ __attribute__((aligned(16))) double col[2][NB];
  __shared__ __attribute__((aligned(16))) double Lt[NB * NB];  // Lt[cc][k] = L[k][cc]
  const int r = threadIdx.x;
  const double* Y = A + (size_t)blockIdx.x * 4096;
  double R[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) R[q] = Y[q * NB + r];
#pragma unroll
  for (int cc = 0; cc < NB; ++cc) {
    double* cb = col[cc & 1];
    cb[r] = R[cc];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    const double d = cb[cc];
    const double l = sqrt(d);
    const double il = 1.0 / l;
    const double lr = r > cc ? R[cc] * il : 0.0;
    R[cc] = r > cc ? lr : (r == cc ? l : R[cc]);
    const double v = cb[r];  (void)v;
    // column entries L[s2][cc] = cb[s2] * il  (s2 > cc)
#pragma unroll
    for (int s2 = cc + 1; s2 < NB; ++s2) R[s2] = fma(-lr, cb[s2] * il, R[s2]);
  }
#pragma unroll
  for (int q = 0; q < NB; ++q) { if (q > r) R[q] = 0.0; L[(size_t)blockIdx.x * 4096 + q * NB + r] = R[q]; Lt[q * NB + r] = R[q]; }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int cc = NB - 1; cc >= 0; --cc) {
    const double ajj = 1.0 / Lt[cc * NB + cc];
    double x0 = 0.0, x1 = 0.0, x2 = 0.0, x3 = 0.0;
#pragma unroll
    for (int k = cc + 1; k < NB; ++k) {
      const double p = R[k] * Lt[cc * NB + k];
      if ((k & 3) == 0) x0 += p; else if ((k & 3) == 1) x1 += p; else if ((k & 3) == 2) x2 += p; else x3 += p;
    }
    const double x = (x0 + x1) + (x2 + x3);
    R[cc] = r > cc ? -ajj * x : (r == cc ? ajj : R[cc]);
  }
#pragma unroll
  for (int q = 0; q < NB; ++q) D[(size_t)blockIdx.x * 4096 + q * NB + r] = R[q];
}

int main() {
  const int B = 256;
  std::vector<double> h((size_t)B * 4096);
  for (int b = 0; b < B; ++b)
    for (int i = 0; i < 64; ++i)
      for (int k = 0; k < 64; ++k) {
        double x = exp(-0.01 * (i - k) * (i - k)) + (i == k ? 0.5 + 0.001 * b : 0.0);
        h[(size_t)b * 4096 + k * 64 + i] = x;
      }
  double *A, *L, *D;
  CHK(hipMalloc(&A, h.size() * 8)); CHK(hipMalloc(&L, h.size() * 8)); CHK(hipMalloc(&D, h.size() * 8));
  CHK(hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  std::vector<double> ref((size_t)B * 4096), out((size_t)B * 4096);
  auto run = [&](const char* name, auto kern, bool setref) {
    for (int nb : {1, 256}) {
      kern<<<nb, 64>>>(A, L, D); CHK(hipDeviceSynchronize());
      CHK(hipEventRecord(e0));
      for (int q = 0; q < 20; ++q) kern<<<nb, 64>>>(A, L, D);
      CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
      printf("%-4s B=%3d %8.1f us/launch", name, nb, ms / 20 * 1000);
      if (nb == 256) {
        CHK(hipMemcpy(out.data(), D, out.size() * 8, hipMemcpyDeviceToHost));
        if (setref) ref = out;
        double mx = 0; for (size_t q = 0; q < out.size(); ++q) mx = fmax(mx, fabs(out[q] - ref[q]) / (1e-300 + fabs(ref[q]) + 1e-3));
        printf("   max rel diff vs v0 %.2e", mx);
      }
      printf("\n");
    }
  };
  run("v0", v0, true);
  run("v1", v1, false);
  run("v2", v2, false);
  return 0;
}
