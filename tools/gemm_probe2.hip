// GEMM-core variants for sum_p A_p^T B_p over 64x64 k-major tiles, 256 threads, 64x64 out.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../optimalinterpolation_amd/csrc/oi_gemm.h"
#define CHK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)
#define MFMA(a,b,c) __builtin_amdgcn_mfma_f64_16x16x4f64(a,b,c,0,0,0)

__device__ __forceinline__ void tiles(int mode, int wg, int P, int p, const double* A, const double* B, const double*& a, const double*& b) {
  size_t ta, tb;
  if (mode == 0) { ta = (size_t)wg * P + p; tb = (size_t)wg * P + p; }
  else if (mode == 1) { ta = (size_t)(wg / 32) * P + p; tb = (size_t)wg * P + p; }
  else { ta = p & 3; tb = (p + 1) & 3; }
  a = A + ta * 4096; b = B + tb * 4096;
}

// V0: current core (KC=16, 2 LDS buffers, register staging)
__global__ __launch_bounds__(256) void v0(const double* A, const double* B, double* C, int P, int mode) {
  __shared__ __attribute__((aligned(16))) double lds[GEMM_LDS];
  Quad acc; quad_zero(acc);
  const int wg = blockIdx.x;
  gemm_kmajor(acc, lds, P, [&](int p, const double*& a, const double*& b) { tiles(mode, wg, P, p, A, B, a, b); });
  double s = 0; for (int x = 0; x < 2; ++x) for (int y = 0; y < 2; ++y) for (int r = 0; r < 4; ++r) s += acc.c[x][y][r];
  C[(size_t)wg * 256 + threadIdx.x] = s;
}

// V1: no LDS: every wave loads its own fragments from global (L1/L2), prefetch PF k4-steps ahead
template <int PF>
__global__ __launch_bounds__(256) void v1(const double* A, const double* B, double* C, int P, int mode) {
  const int wg = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
  const int fr = lane & 15, fk = lane >> 4;
  Quad acc; quad_zero(acc);
  const int nst = P * 16;  // k4 steps
  double fa0[PF], fa1[PF], fb0[PF], fb1[PF];
  auto ld = [&](int s, int slot) {
    const double *a, *b; tiles(mode, wg, P, s >> 4, A, B, a, b);
    const int k = (s & 15) * 4 + fk;
    fa0[slot] = a[k * 64 + 32 * wr + fr]; fa1[slot] = a[k * 64 + 32 * wr + 16 + fr];
    fb0[slot] = b[k * 64 + 32 * wc + fr]; fb1[slot] = b[k * 64 + 32 * wc + 16 + fr];
  };
#pragma unroll
  for (int s = 0; s < PF; ++s) ld(s, s);
  for (int s0 = 0; s0 < nst; s0 += PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      double a0 = fa0[q], a1 = fa1[q], b0 = fb0[q], b1 = fb1[q];
      if (s0 + q + PF < nst) ld(s0 + q + PF, q);
      acc.c[0][0] = MFMA(a0, b0, acc.c[0][0]); acc.c[0][1] = MFMA(a0, b1, acc.c[0][1]);
      acc.c[1][0] = MFMA(a1, b0, acc.c[1][0]); acc.c[1][1] = MFMA(a1, b1, acc.c[1][1]);
    }
  }
  double s = 0; for (int x = 0; x < 2; ++x) for (int y = 0; y < 2; ++y) for (int r = 0; r < 4; ++r) s += acc.c[x][y][r];
  C[(size_t)wg * 256 + threadIdx.x] = s;
}

// V2: LDS, KC=32 chunks (4 buffers of 32x80), one barrier per 32-deep chunk
#define KC2 32
__global__ __launch_bounds__(256) void v2(const double* A, const double* B, double* C, int P, int mode) {
  __shared__ __attribute__((aligned(16))) double lds[2 * 2 * KC2 * LDSS];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  Quad acc; quad_zero(acc);
  const int nch = P * 2;
  const int sk = t >> 4, sm = (t & 15) * 4;   // rows 0..15 and 16..31
  double2 ra[4], rb[4];
  auto load = [&](int ch) {
    const double *a, *b; tiles(mode, blockIdx.x, P, ch >> 1, A, B, a, b);
    const int off = (ch & 1) * KC2 * 64 + t * 4;
    ra[0] = *(const double2*)(a + off); ra[1] = *(const double2*)(a + off + 2);
    ra[2] = *(const double2*)(a + off + 1024); ra[3] = *(const double2*)(a + off + 1026);
    rb[0] = *(const double2*)(b + off); rb[1] = *(const double2*)(b + off + 2);
    rb[2] = *(const double2*)(b + off + 1024); rb[3] = *(const double2*)(b + off + 1026);
  };
  auto store = [&](int buf) {
    double* As = lds + buf * 2 * KC2 * LDSS; double* Bs = As + KC2 * LDSS;
    *(double2*)(As + sk * LDSS + sm) = ra[0]; *(double2*)(As + sk * LDSS + sm + 2) = ra[1];
    *(double2*)(As + (sk + 16) * LDSS + sm) = ra[2]; *(double2*)(As + (sk + 16) * LDSS + sm + 2) = ra[3];
    *(double2*)(Bs + sk * LDSS + sm) = rb[0]; *(double2*)(Bs + sk * LDSS + sm + 2) = rb[1];
    *(double2*)(Bs + (sk + 16) * LDSS + sm) = rb[2]; *(double2*)(Bs + (sk + 16) * LDSS + sm + 2) = rb[3];
  };
  load(0); store(0); __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    if (ch + 1 < nch) load(ch + 1);
    const double* As = lds + (ch & 1) * 2 * KC2 * LDSS; const double* Bs = As + KC2 * LDSS;
#pragma unroll
    for (int kk = 0; kk < KC2 / 4; ++kk) {
      const int k = kk * 4 + fk;
      double a0 = As[k * LDSS + 32 * wr + fr], a1 = As[k * LDSS + 32 * wr + 16 + fr];
      double b0 = Bs[k * LDSS + 32 * wc + fr], b1 = Bs[k * LDSS + 32 * wc + 16 + fr];
      acc.c[0][0] = MFMA(a0, b0, acc.c[0][0]); acc.c[0][1] = MFMA(a0, b1, acc.c[0][1]);
      acc.c[1][0] = MFMA(a1, b0, acc.c[1][0]); acc.c[1][1] = MFMA(a1, b1, acc.c[1][1]);
    }
    if (ch + 1 < nch) store((ch + 1) & 1);
    __syncthreads();
  }
  double s = 0; for (int x = 0; x < 2; ++x) for (int y = 0; y < 2; ++y) for (int r = 0; r < 4; ++r) s += acc.c[x][y][r];
  C[(size_t)blockIdx.x * 256 + threadIdx.x] = s;
}

// V3: 64x128 output (two B tiles sharing A), 256 threads, each wave 32x64 (2x4 blocks), LDS KC=16
__global__ __launch_bounds__(256) void v3(const double* A, const double* B, double* C, int P, int mode) {
  __shared__ __attribute__((aligned(16))) double lds[2 * (KC * LDSS + KC * 144)];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  d4 acc[2][4];
  for (int x = 0; x < 2; ++x) for (int y = 0; y < 4; ++y) acc[x][y] = (d4){0, 0, 0, 0};
  const int nch = P * 4;
  const int sk = t >> 4, sm = (t & 15) * 4;
  double2 ra0, ra1, rb[4];
  const int BS = 144;  // B row stride: 128 + 16
  auto load = [&](int ch) {
    const double *a, *b, *a2, *b2;
    tiles(mode, blockIdx.x, P, ch >> 2, A, B, a, b);
    tiles(mode, blockIdx.x + 4096, P, ch >> 2, A, B, a2, b2);  // second B tile
    const int off = (ch & 3) * KC * 64 + t * 4;
    ra0 = *(const double2*)(a + off); ra1 = *(const double2*)(a + off + 2);
    rb[0] = *(const double2*)(b + off); rb[1] = *(const double2*)(b + off + 2);
    rb[2] = *(const double2*)(b2 + off); rb[3] = *(const double2*)(b2 + off + 2);
  };
  auto store = [&](int buf) {
    double* As = lds + buf * (KC * LDSS + KC * BS); double* Bs = As + KC * LDSS;
    *(double2*)(As + sk * LDSS + sm) = ra0; *(double2*)(As + sk * LDSS + sm + 2) = ra1;
    *(double2*)(Bs + sk * BS + sm) = rb[0]; *(double2*)(Bs + sk * BS + sm + 2) = rb[1];
    *(double2*)(Bs + sk * BS + 64 + sm) = rb[2]; *(double2*)(Bs + sk * BS + 64 + sm + 2) = rb[3];
  };
  load(0); store(0); __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    if (ch + 1 < nch) load(ch + 1);
    const double* As = lds + (ch & 1) * (KC * LDSS + KC * BS); const double* Bs = As + KC * LDSS;
#pragma unroll
    for (int kk = 0; kk < KC / 4; ++kk) {
      const int k = kk * 4 + fk;
      double a0 = As[k * LDSS + 32 * wr + fr], a1 = As[k * LDSS + 32 * wr + 16 + fr];
      double b[4];
      for (int y = 0; y < 4; ++y) b[y] = Bs[k * BS + 64 * wc + 16 * y + fr];
      for (int y = 0; y < 4; ++y) { acc[0][y] = MFMA(a0, b[y], acc[0][y]); acc[1][y] = MFMA(a1, b[y], acc[1][y]); }
    }
    if (ch + 1 < nch) store((ch + 1) & 1);
    __syncthreads();
  }
  double s = 0; for (int x = 0; x < 2; ++x) for (int y = 0; y < 4; ++y) for (int r = 0; r < 4; ++r) s += acc[x][y][r];
  C[(size_t)blockIdx.x * 256 + threadIdx.x] = s;
}


// V5: v0 but all 16 fragments of a chunk are read from LDS before the 16 MFMAs
__global__ __launch_bounds__(256) void v5(const double* A, const double* B, double* C, int P, int mode) {
  __shared__ __attribute__((aligned(16))) double lds[GEMM_LDS];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  Quad acc; quad_zero(acc);
  const int nch = P * 4;
  const int sk = t >> 4, sm = (t & 15) * 4;
  double2 ra0, ra1, rb0, rb1;
  auto load = [&](int ch) {
    const double *a, *b; tiles(mode, blockIdx.x, P, ch >> 2, A, B, a, b);
    const int off = (ch & 3) * KC * 64 + t * 4;
    ra0 = *(const double2*)(a + off); ra1 = *(const double2*)(a + off + 2);
    rb0 = *(const double2*)(b + off); rb1 = *(const double2*)(b + off + 2);
  };
  auto store = [&](int buf) {
    double* As = lds + buf * 2 * STAGE; double* Bs = As + STAGE;
    *(double2*)(As + sk * LDSS + sm) = ra0; *(double2*)(As + sk * LDSS + sm + 2) = ra1;
    *(double2*)(Bs + sk * LDSS + sm) = rb0; *(double2*)(Bs + sk * LDSS + sm + 2) = rb1;
  };
  load(0); store(0); __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    if (ch + 1 < nch) load(ch + 1);
    const double* As = lds + (ch & 1) * 2 * STAGE; const double* Bs = As + STAGE;
    double a0[4], a1[4], b0[4], b1[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int k = kk * 4 + fk;
      a0[kk] = As[k * LDSS + 32 * wr + fr]; a1[kk] = As[k * LDSS + 32 * wr + 16 + fr];
      b0[kk] = Bs[k * LDSS + 32 * wc + fr]; b1[kk] = Bs[k * LDSS + 32 * wc + 16 + fr];
    }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      acc.c[0][0] = MFMA(a0[kk], b0[kk], acc.c[0][0]); acc.c[0][1] = MFMA(a0[kk], b1[kk], acc.c[0][1]);
      acc.c[1][0] = MFMA(a1[kk], b0[kk], acc.c[1][0]); acc.c[1][1] = MFMA(a1[kk], b1[kk], acc.c[1][1]);
    }
    if (ch + 1 < nch) store((ch + 1) & 1);
    __syncthreads();
  }
  double s = 0; for (int x = 0; x < 2; ++x) for (int y = 0; y < 2; ++y) for (int r = 0; r < 4; ++r) s += acc.c[x][y][r];
  C[(size_t)blockIdx.x * 256 + threadIdx.x] = s;
}

// V6: 64x128 output (A shared), each wave 32x64 (8 accumulators), KC=8 chunks -> 36 KiB LDS
#define KC6 8
__global__ __launch_bounds__(256) void v6(const double* A, const double* B, double* C, int P, int mode) {
  const int BS = 144;
  __shared__ __attribute__((aligned(16))) double lds[2 * (KC6 * LDSS + KC6 * 144)];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  d4 acc[2][4];
  for (int x = 0; x < 2; ++x) for (int y = 0; y < 4; ++y) acc[x][y] = (d4){0, 0, 0, 0};
  const int nch = P * (64 / KC6);
  // staging: A chunk 8x64 = 512 doubles (2/thread), B chunk 8x128 = 1024 (4/thread)
  const int sk = t >> 5, sm = (t & 31) * 2;
  double2 ra, rb0, rb1;
  auto load = [&](int ch) {
    const double *a, *b, *a2, *b2;
    tiles(mode, blockIdx.x, P, ch >> 3, A, B, a, b);
    tiles(mode, blockIdx.x + 4096, P, ch >> 3, A, B, a2, b2);
    const int off = (ch & 7) * KC6 * 64 + t * 2;
    ra = *(const double2*)(a + off);
    rb0 = *(const double2*)(b + off); rb1 = *(const double2*)(b2 + off);
  };
  auto store = [&](int buf) {
    double* As = lds + buf * (KC6 * LDSS + KC6 * BS); double* Bs = As + KC6 * LDSS;
    *(double2*)(As + sk * LDSS + sm) = ra;
    *(double2*)(Bs + sk * BS + sm) = rb0; *(double2*)(Bs + sk * BS + 64 + sm) = rb1;
  };
  load(0); store(0); __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    if (ch + 1 < nch) load(ch + 1);
    const double* As = lds + (ch & 1) * (KC6 * LDSS + KC6 * BS); const double* Bs = As + KC6 * LDSS;
#pragma unroll
    for (int kk = 0; kk < KC6 / 4; ++kk) {
      const int k = kk * 4 + fk;
      double a0 = As[k * LDSS + 32 * wr + fr], a1 = As[k * LDSS + 32 * wr + 16 + fr];
      double b[4];
      for (int y = 0; y < 4; ++y) b[y] = Bs[k * BS + 64 * wc + 16 * y + fr];
      for (int y = 0; y < 4; ++y) { acc[0][y] = MFMA(a0, b[y], acc[0][y]); acc[1][y] = MFMA(a1, b[y], acc[1][y]); }
    }
    if (ch + 1 < nch) store((ch + 1) & 1);
    __syncthreads();
  }
  double s = 0; for (int x = 0; x < 2; ++x) for (int y = 0; y < 4; ++y) for (int r = 0; r < 4; ++r) s += acc[x][y][r];
  C[(size_t)blockIdx.x * 256 + threadIdx.x] = s;
}

// V7: 512 threads = 8 waves, 64x128 output (A shared), each wave 32x32 (4 acc), KC=16
__global__ __launch_bounds__(512) void v7(const double* A, const double* B, double* C, int P, int mode) {
  const int BS = 144;
  __shared__ __attribute__((aligned(16))) double lds[2 * (KC * LDSS + KC * 144)];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = (w >> 2) & 1, wc = w & 3, fr = lane & 15, fk = lane >> 4;
  Quad acc; quad_zero(acc);
  const int nch = P * 4;
  // A chunk 16x64 = 1024 doubles: threads 0..255 (4 each); B chunk 16x128 = 2048: 4 each for all 512
  double2 ra0, ra1, rb0, rb1;
  auto load = [&](int ch) {
    const double *a, *b, *a2, *b2;
    tiles(mode, blockIdx.x, P, ch >> 2, A, B, a, b);
    tiles(mode, blockIdx.x + 4096, P, ch >> 2, A, B, a2, b2);
    const int tt = t & 255;
    const int off = (ch & 3) * KC * 64 + tt * 4;
    const double* bb = t < 256 ? b : b2;
    if (t < 256) { ra0 = *(const double2*)(a + off); ra1 = *(const double2*)(a + off + 2); }
    rb0 = *(const double2*)(bb + off); rb1 = *(const double2*)(bb + off + 2);
  };
  auto store = [&](int buf) {
    double* As = lds + buf * (KC * LDSS + KC * BS); double* Bs = As + KC * LDSS;
    const int tt = t & 255, sk = tt >> 4, sm = (tt & 15) * 4, half = t >> 8;
    if (t < 256) { *(double2*)(As + sk * LDSS + sm) = ra0; *(double2*)(As + sk * LDSS + sm + 2) = ra1; }
    *(double2*)(Bs + sk * BS + 64 * half + sm) = rb0; *(double2*)(Bs + sk * BS + 64 * half + sm + 2) = rb1;
  };
  load(0); store(0); __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    if (ch + 1 < nch) load(ch + 1);
    const double* As = lds + (ch & 1) * (KC * LDSS + KC * BS); const double* Bs = As + KC * LDSS;
#pragma unroll
    for (int kk = 0; kk < KC / 4; ++kk) {
      const int k = kk * 4 + fk;
      double a0 = As[k * LDSS + 32 * wr + fr], a1 = As[k * LDSS + 32 * wr + 16 + fr];
      double b0 = Bs[k * BS + 32 * wc + fr], b1 = Bs[k * BS + 32 * wc + 16 + fr];
      acc.c[0][0] = MFMA(a0, b0, acc.c[0][0]); acc.c[0][1] = MFMA(a0, b1, acc.c[0][1]);
      acc.c[1][0] = MFMA(a1, b0, acc.c[1][0]); acc.c[1][1] = MFMA(a1, b1, acc.c[1][1]);
    }
    if (ch + 1 < nch) store((ch + 1) & 1);
    __syncthreads();
  }
  double s = 0; for (int x = 0; x < 2; ++x) for (int y = 0; y < 2; ++y) for (int r = 0; r < 4; ++r) s += acc.c[x][y][r];
  C[(size_t)blockIdx.x * 512 + threadIdx.x] = s;
}

int main() {
  const int P = 32, nwg = 4096;
  size_t tiles_n = (size_t)nwg * 2 * P;
  double *A, *B, *C;
  CHK(hipMalloc(&A, tiles_n * 4096 * 8)); CHK(hipMalloc(&B, tiles_n * 4096 * 8)); CHK(hipMalloc(&C, (size_t)nwg * 512 * 8));
  CHK(hipMemset(A, 0, tiles_n * 4096 * 8)); CHK(hipMemset(B, 0, tiles_n * 4096 * 8));
  std::vector<double> h(4096 * 4); for (size_t i = 0; i < h.size(); ++i) h[i] = 1.0 + 1e-3 * (i % 97);
  CHK(hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice)); CHK(hipMemcpy(B, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  const char* mn[] = {"stream", "sharedA", "L2res"};
  auto run = [&](const char* name, auto kern, double mult, int thr = 256) {
    for (int mode = 0; mode < 3; ++mode) {
      kern<<<nwg, thr>>>(A, B, C, P, mode); CHK(hipDeviceSynchronize());
      CHK(hipEventRecord(e0));
      for (int r = 0; r < 5; ++r) kern<<<nwg, thr>>>(A, B, C, P, mode);
      CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
      double fl = mult * 2.0 * 64 * 64 * 64 * P * nwg;
      printf("%-14s %-8s %8.3f ms %6.2f TF/s\n", name, mn[mode], ms, fl / ms / 1e9);
    }
  };
  run("v0_lds_kc16", v0, 1.0);
  run("v5_preload", v5, 1.0);
  run("v6_64x128_kc8", v6, 2.0);
  run("v7_512thr_64x128", v7, 2.0, 512);
  return 0;
}
