// More 64x64-output fp64 GEMM core variants (256 threads).  sum_p A_p^T B_p, P tile pairs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../optimalinterpolation_amd/csrc/oi_gemm.h"
#define CHK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

__device__ __forceinline__ void tiles(int mode, int wg, int P, int p, const double* A, const double* B, const double*& a, const double*& b) {
  size_t ta, tb;
  if (mode == 0) { ta = (size_t)wg * P + p; tb = (size_t)wg * P + p; }
  else if (mode == 1) { ta = (size_t)(wg / 32) * P + p; tb = (size_t)wg * P + p; }
  else { ta = p & 3; tb = (p + 1) & 3; }
  a = A + ta * 4096; b = B + tb * 4096;
}

__global__ __launch_bounds__(256) void base(const double* A, const double* B, double* C, int P, int mode) {
  __shared__ __attribute__((aligned(16))) double lds[GEMM1_LDS];
  Quad acc; quad_zero(acc);
  const int wg = blockIdx.x;
  gemm1_kmajor(acc, lds, P, [&](int p, const double*& a, const double*& b) { tiles(mode, wg, P, p, A, B, a, b); });
  double s = 0; for (int x = 0; x < 2; ++x) for (int y = 0; y < 2; ++y) for (int r = 0; r < 4; ++r) s += acc.c[x][y][r];
  C[(size_t)wg * 256 + threadIdx.x] = s;
}

// generic: KCV-deep chunks, NBUF LDS buffers with (NBUF-1) chunks in flight (register ring), optional setprio
template <int KCV, int NBUF, bool PRIO>
__global__ __launch_bounds__(256) void var(const double* A, const double* B, double* C, int P, int mode) {
  constexpr int STG = KCV * LDSA;
  __shared__ __attribute__((aligned(16))) double lds[NBUF * 2 * STG];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  Quad acc; quad_zero(acc);
  constexpr int CPT = 64 / KCV;           // chunks per tile
  constexpr int PER = KCV * 64 / 256;     // doubles per thread per operand per chunk
  const int nch = P * CPT;
  const int sk = (t * PER) / 64, sm = (t * PER) % 64;
  auto ldst = [&](int ch, int buf) {
    const double *a, *b; tiles(mode, blockIdx.x, P, ch / CPT, A, B, a, b);
    const int off = (ch % CPT) * KCV * 64 + t * PER;
    double* As = lds + buf * 2 * STG; double* Bs = As + STG;
#pragma unroll
    for (int u = 0; u < PER; u += 2) {
      double2 ra = *(const double2*)(a + off + u), rb = *(const double2*)(b + off + u);
      *(double2*)(As + sk * LDSA + sm + u) = ra; *(double2*)(Bs + sk * LDSA + sm + u) = rb;
    }
  };
  for (int q = 0; q < NBUF - 1 && q < nch; ++q) ldst(q, q);
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    const double* As = lds + (ch % NBUF) * 2 * STG; const double* Bs = As + STG;
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < KCV / 4; ++kk) {
      const int k = kk * 4 + fk;
      const double a0 = As[k * LDSA + 32 * wr + fr], a1 = As[k * LDSA + 32 * wr + 16 + fr];
      const double b0 = Bs[k * LDSA + 32 * wc + fr], b1 = Bs[k * LDSA + 32 * wc + 16 + fr];
      acc.c[0][0] = MFMA64(a0, b0, acc.c[0][0]); acc.c[0][1] = MFMA64(a0, b1, acc.c[0][1]);
      acc.c[1][0] = MFMA64(a1, b0, acc.c[1][0]); acc.c[1][1] = MFMA64(a1, b1, acc.c[1][1]);
    }
    if (PRIO) __builtin_amdgcn_s_setprio(0);
    if (ch + NBUF - 1 < nch) ldst(ch + NBUF - 1, (ch + NBUF - 1) % NBUF);
    __syncthreads();
  }
  double s = 0; for (int x = 0; x < 2; ++x) for (int y = 0; y < 2; ++y) for (int r = 0; r < 4; ++r) s += acc.c[x][y][r];
  C[(size_t)blockIdx.x * 256 + threadIdx.x] = s;
}

// register ring: chunks ch+1 and ch+2 in flight while computing ch (2 LDS buffers)
typedef double dv2 __attribute__((ext_vector_type(2)));
template <bool PRIO>
__global__ __launch_bounds__(256) void pf2(const double* A, const double* B, double* C, int P, int mode) {
  __shared__ __attribute__((aligned(16))) double lds[GEMM1_LDS];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  Quad acc; quad_zero(acc);
  const int nch = P * 4;
  const int sk = t >> 4, sm = (t & 15) * 4;
  struct Rg { dv2 a0, a1, b0, b1; };
  Rg r0, r1;
  auto load = [&](int ch, Rg& rg) __attribute__((always_inline)) {
    const double *a, *b; tiles(mode, blockIdx.x, P, ch >> 2, A, B, a, b);
    const int off = (ch & 3) * KC * 64 + t * 4;
    rg.a0 = *(const dv2*)(a + off); rg.a1 = *(const dv2*)(a + off + 2);
    rg.b0 = *(const dv2*)(b + off); rg.b1 = *(const dv2*)(b + off + 2);
  };
  auto store = [&](int buf, const Rg& rg) __attribute__((always_inline)) {
    double* As = lds + buf * 2 * STAGE_A; double* Bs = As + STAGE_A;
    *(dv2*)(As + sk * LDSA + sm) = rg.a0; *(dv2*)(As + sk * LDSA + sm + 2) = rg.a1;
    *(dv2*)(Bs + sk * LDSA + sm) = rg.b0; *(dv2*)(Bs + sk * LDSA + sm + 2) = rg.b1;
  };
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const double* As = lds + buf * 2 * STAGE_A; const double* Bs = As + STAGE_A;
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < KC / 4; ++kk) {
      const int k = kk * 4 + fk;
      const double a0 = As[k * LDSA + 32 * wr + fr], a1 = As[k * LDSA + 32 * wr + 16 + fr];
      const double b0 = Bs[k * LDSA + 32 * wc + fr], b1 = Bs[k * LDSA + 32 * wc + 16 + fr];
      acc.c[0][0] = MFMA64(a0, b0, acc.c[0][0]); acc.c[0][1] = MFMA64(a0, b1, acc.c[0][1]);
      acc.c[1][0] = MFMA64(a1, b0, acc.c[1][0]); acc.c[1][1] = MFMA64(a1, b1, acc.c[1][1]);
    }
    if (PRIO) __builtin_amdgcn_s_setprio(0);
  };
  load(0, r0);
  load(1, r1);
  store(0, r0);
  __syncthreads();
  // nch is a multiple of 4 here
  for (int ch = 0; ch < nch; ch += 2) {
    if (ch + 2 < nch) load(ch + 2, r0);
    compute(0);
    store(1, r1);
    __syncthreads();
    if (ch + 3 < nch) load(ch + 3, r1);
    compute(1);
    if (ch + 2 < nch) store(0, r0);
    __syncthreads();
  }
  double s = 0;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
  for (int y = 0; y < 2; ++y)
#pragma unroll
  for (int q = 0; q < 4; ++q) s += acc.c[x][y][q];
  C[(size_t)blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  const int P = 32, nwg = 4096;
  size_t tiles_n = (size_t)nwg * P;
  double *A, *B, *C;
  CHK(hipMalloc(&A, tiles_n * 4096 * 8)); CHK(hipMalloc(&B, tiles_n * 4096 * 8)); CHK(hipMalloc(&C, (size_t)nwg * 512 * 8));
  CHK(hipMemset(A, 0, tiles_n * 4096 * 8)); CHK(hipMemset(B, 0, tiles_n * 4096 * 8));
  std::vector<double> h(4096 * 4); for (size_t i = 0; i < h.size(); ++i) h[i] = 1.0 + 1e-3 * (i % 97);
  CHK(hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice)); CHK(hipMemcpy(B, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  const char* mn[] = {"stream", "sharedA", "L2res"};
  auto run = [&](const char* name, auto kern) {
    for (int mode = 0; mode < 3; ++mode) {
      kern<<<nwg, 256>>>(A, B, C, P, mode); CHK(hipDeviceSynchronize());
      CHK(hipEventRecord(e0));
      for (int r = 0; r < 5; ++r) kern<<<nwg, 256>>>(A, B, C, P, mode);
      CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
      double fl = 2.0 * 64 * 64 * 64 * P * nwg;
      printf("%-22s %-8s %8.3f ms %6.2f TF/s\n", name, mn[mode], ms, fl / ms / 1e9);
    }
  };
  run("base_kc16_2buf", base);
  run("pf2", pf2<false>);
  run("pf2_prio", pf2<true>);
  run("kc16_2buf_prio", var<16, 2, true>);
  return 0;
}
