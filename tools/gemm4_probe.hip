// 128x128-output fp64 GEMM core (512 threads, each wave a 32x64 block of 2x4
// v_mfma_f64_16x16x4f64) vs the 64x128 gemm2 core and the 64x64 gemm1 core.
// D = sum_p A_p^T B_p over P k-major 64x64 tile pairs per output tile.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../optimalinterpolation_amd/csrc/oi_gemm.h"
#define CHK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

#define NTILES (1024 * 16 * 4)  // tiles allocated per operand array
// tile address: mode 0 every WG streams its own tiles from HBM; mode 2 a few L2-resident tiles
__device__ __forceinline__ const double* tile(const double* X, int mode, int wg, int P, int p, int which) {
  size_t t = mode == 0 ? (((size_t)wg * P + p) * 4 + which) % NTILES : (size_t)((p + which) & 7);
  return X + t * 4096;
}

struct Acc8 { d4 c[2][4]; };

template <int LDSS, int SCHED = 0>
__global__ __launch_bounds__(512) void g4(const double* A, const double* B, double* C, int P, int mode) {
  constexpr int STG = KC * LDSS;  // one 16 x 128 operand chunk
  __shared__ __attribute__((aligned(16))) double lds[4 * STG];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  Acc8 acc;
  for (int a = 0; a < 2; ++a) for (int b = 0; b < 4; ++b) acc.c[a][b] = (d4){0, 0, 0, 0};
  const int nch = P * 4;
  const int sk = t >> 5, sm = (t & 31) * 2;  // 16 B piece of a 16 x 64 chunk
  struct Rg { dv2 a0, a1, b0, b1; };
  Rg r0, r1;
  auto load = [&](int ch, Rg& q) __attribute__((always_inline)) {
    const int p = ch >> 2, off = (ch & 3) * KC * 64 + t * 2;
    q.a0 = gload2(tile(A, mode, blockIdx.x, P, p, 0) + off);
    q.a1 = gload2(tile(A, mode, blockIdx.x, P, p, 1) + off);
    q.b0 = gload2(tile(B, mode, blockIdx.x, P, p, 2) + off);
    q.b1 = gload2(tile(B, mode, blockIdx.x, P, p, 3) + off);
  };
  auto store = [&](int buf, const Rg& q) __attribute__((always_inline)) {
    double* As = lds + buf * 2 * STG;
    double* Bs = As + STG;
    *(dv2*)(As + sk * LDSS + sm) = q.a0;
    *(dv2*)(As + sk * LDSS + 64 + sm) = q.a1;
    *(dv2*)(Bs + sk * LDSS + sm) = q.b0;
    *(dv2*)(Bs + sk * LDSS + 64 + sm) = q.b1;
  };
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const double* As = lds + buf * 2 * STG;
    const double* Bs = As + STG;
#pragma unroll
    for (int kk = 0; kk < KC / 4; ++kk) {
      const int k = kk * 4 + fk;
      const double a0 = As[k * LDSS + 32 * wr + fr], a1 = As[k * LDSS + 32 * wr + 16 + fr];
      double b[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) b[q] = Bs[k * LDSS + 64 * wc + 16 * q + fr];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc.c[0][q] = MFMA64(a0, b[q], acc.c[0][q]);
        acc.c[1][q] = MFMA64(a1, b[q], acc.c[1][q]);
      }
    }
    // SCHED: interleave the chunk's 24 LDS reads with its 32 MFMAs (mask 0x100
    // DS read, 0x008 MFMA) instead of the compiler's grouping
    if (SCHED == 1) {
      __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
      for (int i = 0; i < 18; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 14, 0);
    } else if (SCHED == 2) {
      __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    }
  };
  load(0, r0);
  load(1, r1);
  store(0, r0);
  __syncthreads();
  for (int ch = 0; ch < nch; ch += 2) {
    load(min(ch + 2, nch - 1), r0);
    compute(0);
    store(1, r1);
    __syncthreads();
    load(min(ch + 3, nch - 1), r1);
    compute(1);
    if (ch + 2 < nch) store(0, r0);
    __syncthreads();
  }
  double s = 0;
  for (int a = 0; a < 2; ++a) for (int b = 0; b < 4; ++b) for (int q = 0; q < 4; ++q) s += acc.c[a][b][q];
  C[(size_t)blockIdx.x * 512 + t] = s;
}


// LDS-DMA staging (global_load_lds_dwordx4): each wave instruction fills one
// 128-double LDS row (k-row of the two 64-wide tiles side by side) linearly;
// odd rows hold the two 16-double halves of every 32-double group swapped
// (source address permuted per lane, read index m ^ 16), so ds_read_b64 of
// rows k, k+1 by one half-wave falls in opposite bank halves.
// NBUF LDS buffers, NBUF-1 chunks in flight across raw barriers (counted vmcnt).
template <int KCG, int NBUF>
__global__ __launch_bounds__(512) void g4g(const double* A, const double* B, double* C, int P, int mode) {
  constexpr int ROW = 128, STG = KCG * ROW, G = 2 * KCG / 8;  // glds per wave per chunk
  constexpr int CPP = 64 / KCG;                              // chunks per operand pair
  __shared__ __attribute__((aligned(16))) double lds[NBUF * 2 * STG];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  Acc8 acc;
  for (int a = 0; a < 2; ++a) for (int b = 0; b < 4; ++b) acc.c[a][b] = (d4){0, 0, 0, 0};
  const int nch = P * CPP;
  auto issue = [&](int ch) __attribute__((always_inline)) {
    const int p = ch / CPP, k0 = (ch % CPP) * KCG;
    double* buf = lds + (ch % NBUF) * 2 * STG;
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int gi = w * G + i, isB = gi >= KCG, k = isB ? gi - KCG : gi;
      const double* tp = tile(isB ? B : A, mode, blockIdx.x, P, p, (isB ? 2 : 0) + (lane >> 5));
      const int q = (lane & 31) ^ (8 * (k & 1));
      __builtin_amdgcn_global_load_lds((const void*)(tp + (k0 + k) * 64 + 2 * q),
                                       (void*)(buf + (isB ? STG : 0) + k * ROW), 16, 0, 0);
    }
  };
  auto compute = [&](int ch) __attribute__((always_inline)) {
    const double* As = lds + (ch % NBUF) * 2 * STG;
    const double* Bs = As + STG;
#pragma unroll
    for (int kk = 0; kk < KCG / 4; ++kk) {
      const int k = kk * 4 + fk, sw = 16 * (k & 1);
      const double a0 = As[k * ROW + ((32 * wr + fr) ^ sw)], a1 = As[k * ROW + ((32 * wr + 16 + fr) ^ sw)];
      double b[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) b[q] = Bs[k * ROW + ((64 * wc + 16 * q + fr) ^ sw)];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc.c[0][q] = MFMA64(a0, b[q], acc.c[0][q]);
        acc.c[1][q] = MFMA64(a1, b[q], acc.c[1][q]);
      }
    }
  };
#pragma unroll
  for (int d = 0; d < NBUF - 1; ++d) issue(min(d, nch - 1));
  for (int ch = 0; ch < nch; ++ch) {
    // chunk ch landed (this wave's part): NBUF-2 younger chunks may stay in flight
    if constexpr (NBUF == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (NBUF == 3) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(G) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * G) : "memory");
    __builtin_amdgcn_s_barrier();
    issue(min(ch + NBUF - 1, nch - 1));
    compute(ch);
  }
  double s = 0;
  for (int a = 0; a < 2; ++a) for (int b = 0; b < 4; ++b) for (int q = 0; q < 4; ++q) s += acc.c[a][b][q];
  C[(size_t)blockIdx.x * 512 + t] = s;
}


// 256 x 128 output per 512-thread workgroup (one workgroup per CU): wave w owns
// rows 64*(w>>1) .. +64 and columns 64*(w&1) .. +64 as 4 x 4 blocks (16 MFMAs
// per 8 LDS reads); operands A = 4 tiles (rows), B = 2 tiles (columns).
struct Acc16 { d4 c[4][4]; };
template <bool GLDS, int NBUF>
__global__ __launch_bounds__(512) void g8(const double* A, const double* B, double* C, int P, int mode) {
  constexpr int ROW = 384, STG = KC * ROW;  // one k-row: A 256 | B 128
  __shared__ __attribute__((aligned(16))) double lds[NBUF * STG];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  Acc16 acc;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc.c[a][b] = (d4){0, 0, 0, 0};
  const int nch = P * 4;
  // staging unit: 16 B pieces; chunk = 16 rows x 384 doubles = 3072 pieces = 6 per thread
  // piece q of thread t: e = t + 512 q -> row k = e / 192, piece-in-row pr = e % 192 (tile pr / 32)
  auto src = [&](int ch, int e) -> const double* {
    const int p = ch >> 2, k0 = (ch & 3) * KC, k = e / 192, pr = e % 192, tl = pr >> 5;
    const int sw = 8 * (k & 1);
    const double* tp = tile(tl < 4 ? A : B, mode, blockIdx.x, P, p, tl < 4 ? tl : 2 + (tl - 4));
    return tp + (k0 + k) * 64 + 2 * ((pr & 31) ^ sw);
  };
  // LDS image: row k, piece pr at k*ROW + 2*pr (linear); read index (m ^ 16 (k&1)) within each 64-tile
  dv2 rg[2][6];
  auto gload = [&](int ch, int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 6; ++q) rg[slot][q] = gload2(src(ch, t + 512 * q));
  };
  auto sstore = [&](int buf, int slot) __attribute__((always_inline)) {
    double* S = lds + buf * STG;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const int e = t + 512 * q;
      *(dv2*)(S + (e / 192) * ROW + 2 * (e % 192)) = rg[slot][q];
    }
  };
  auto issue = [&](int ch, int buf) __attribute__((always_inline)) {
    double* S = lds + buf * STG;
    // 48 KB per chunk = 48 wave-instructions of 1 KB: 6 per wave; instruction i of wave w covers
    // pieces (w*6 + i) * 64 .. +64 of the linear image
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int e0 = (w * 6 + i) * 64, e = e0 + lane;
      __builtin_amdgcn_global_load_lds((const void*)src(ch, e), (void*)(S + 2 * e0 + 0 * lane), 16, 0, 0);
    }
  };
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const double* S = lds + buf * STG;
#pragma unroll
    for (int kk = 0; kk < KC / 4; ++kk) {
      const int k = kk * 4 + fk, sw = 16 * (k & 1);
      double a[4], b[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] = S[k * ROW + 64 * wr + ((16 * q + fr) ^ sw)];
#pragma unroll
      for (int q = 0; q < 4; ++q) b[q] = S[k * ROW + 256 + 64 * wc + ((16 * q + fr) ^ sw)];
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc.c[x][y] = MFMA64(a[x], b[y], acc.c[x][y]);
    }
  };
  if constexpr (!GLDS) {
    gload(0, 0);
    gload(min(1, nch - 1), 1);
    sstore(0, 0);
    __syncthreads();
    for (int ch = 0; ch < nch; ch += 2) {
      gload(min(ch + 2, nch - 1), 0);
      compute(0);
      sstore(1, 1);
      __syncthreads();
      gload(min(ch + 3, nch - 1), 1);
      if (ch + 1 < nch) compute(1);
      if (ch + 2 < nch) sstore(0, 0);
      __syncthreads();
    }
  } else {
#pragma unroll
    for (int d = 0; d < NBUF - 1; ++d) issue(min(d, nch - 1), d);
    for (int ch = 0; ch < nch; ++ch) {
      if constexpr (NBUF == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      issue(min(ch + NBUF - 1, nch - 1), (ch + NBUF - 1) % NBUF);
      compute(ch % NBUF);
    }
  }
  double s = 0;
  for (int a = 0; a < 4; ++a) for (int b = 0; b < 4; ++b) for (int q = 0; q < 4; ++q) s += acc.c[a][b][q];
  C[(size_t)blockIdx.x * 512 + t] = s;
}

__global__ __launch_bounds__(512) void g2(const double* A, const double* B, double* C, int P, int mode) {
  __shared__ __attribute__((aligned(16))) double lds[GEMM2_LDS];
  Quad acc; quad_zero(acc);
  const int wg = blockIdx.x;
  gemm2_kmajor(acc, lds, P, [=](int p, const double*& a, const double*& b0, const double*& b1) {
    a = tile(A, mode, wg, P, p, 0); b0 = tile(B, mode, wg, P, p, 2); b1 = tile(B, mode, wg, P, p, 3); });
  double s = 0; for (int x = 0; x < 2; ++x) for (int y = 0; y < 2; ++y) for (int r = 0; r < 4; ++r) s += acc.c[x][y][r];
  C[(size_t)wg * 512 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void g1(const double* A, const double* B, double* C, int P, int mode) {
  __shared__ __attribute__((aligned(16))) double lds[GEMM1_LDS];
  Quad acc; quad_zero(acc);
  const int wg = blockIdx.x;
  gemm1_kmajor<false>(acc, lds, 4 * P, 0u, [=](int p, const double*& a, const double*& b) {
    a = tile(A, mode, wg, P, p, 0); b = tile(B, mode, wg, P, p, 2); });
  double s = 0; for (int x = 0; x < 2; ++x) for (int y = 0; y < 2; ++y) for (int r = 0; r < 4; ++r) s += acc.c[x][y][r];
  C[(size_t)wg * 512 + threadIdx.x] = s;
}

__global__ void fill(double* X, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) X[i] = 1.0 + 1e-3 * (double)(i % 97);
}

int main() {
  const int P = 16, nwg = 1024;
  size_t tiles_n = NTILES;
  double *A, *B, *C;
  CHK(hipMalloc(&A, tiles_n * 4096 * 8)); CHK(hipMalloc(&B, tiles_n * 4096 * 8)); CHK(hipMalloc(&C, (size_t)nwg * 4 * 512 * 8));
  const size_t nel = tiles_n * 4096;
  hipLaunchKernelGGL(fill, dim3((unsigned)((nel + 255) / 256)), dim3(256), 0, 0, A, nel);
  hipLaunchKernelGGL(fill, dim3((unsigned)((nel + 255) / 256)), dim3(256), 0, 0, B, nel);
  CHK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto kern, int threads, int nwgs, double flop_per_wg) {
    for (int mode : {0, 2}) {
      hipLaunchKernelGGL(kern, dim3(nwgs), dim3(threads), 0, 0, A, B, C, P, mode); CHK(hipDeviceSynchronize());
      CHK(hipEventRecord(e0));
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(nwgs), dim3(threads), 0, 0, A, B, C, P, mode);
      CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
      printf("%-16s %-7s %8.3f ms %6.2f TF/s\n", name, mode == 0 ? "stream" : "L2res", ms, flop_per_wg * nwgs / ms / 1e9);
    }
  };
  const double tp = 2.0 * 64 * 64 * 64 * P;  // one output tile
  auto result = [&](auto kern) {
    std::vector<double> h((size_t)nwg * 512);
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(512), 0, 0, A, B, C, P, 0); CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(h.data(), C, h.size() * 8, hipMemcpyDeviceToHost));
    return h;
  };
  {
    auto ref = result(g4<144>);
    auto chk = [&](const char* name, auto kern) {
      auto h = result(kern); size_t bad = 0;
      for (size_t i = 0; i < h.size(); ++i) bad += h[i] != ref[i];
      printf("check %-16s %zu of %zu differ\n", name, bad, h.size());
    };
    chk("g4 sched1", g4<144, 1>); chk("g4 sched2", g4<144, 2>);
    chk("g4g kc16 nbuf2", g4g<16, 2>); chk("g4g kc16 nbuf3", g4g<16, 3>); chk("g4g kc8 nbuf4", g4g<8, 4>);
    chk("g4g kc8 nbuf3", g4g<8, 3>); chk("g4g kc32 nbuf2", g4g<32, 2>);
  }
  {
    auto res8 = [&](auto kern) {
      std::vector<double> h((size_t)nwg / 2 * 512);
      hipLaunchKernelGGL(kern, dim3(nwg / 2), dim3(512), 0, 0, A, B, C, P, 0); CHK(hipDeviceSynchronize());
      CHK(hipMemcpy(h.data(), C, h.size() * 8, hipMemcpyDeviceToHost));
      return h;
    };
    auto r0 = res8(g8<false, 2>), r1 = res8(g8<true, 2>), r2 = res8(g8<true, 3>);
    size_t b1 = 0, b2 = 0;
    for (size_t i = 0; i < r0.size(); ++i) { b1 += r1[i] != r0[i]; b2 += r2[i] != r0[i]; }
    printf("check g8 glds2 %zu, glds3 %zu of %zu differ from g8 regs\n", b1, b2, r0.size());
  }
  run("g1 64x64", g1, 256, 4 * nwg, tp);
  run("g2 64x128", g2, 512, 2 * nwg, 2 * tp);
  run("g4 128x128 s144", g4<144>, 512, nwg, 4 * tp);
  run("g4 s144 sched1", g4<144, 1>, 512, nwg, 4 * tp);
  run("g4 s144 sched2", g4<144, 2>, 512, nwg, 4 * tp);
  run("g4 128x128 s144", g4<144>, 512, nwg, 4 * tp);
  run("g4 128x128 s136", g4<136>, 512, nwg, 4 * tp);
  run("g4g kc16 nbuf2", g4g<16, 2>, 512, nwg, 4 * tp);
  run("g4g kc16 nbuf3", g4g<16, 3>, 512, nwg, 4 * tp);
  run("g4g kc8 nbuf4", g4g<8, 4>, 512, nwg, 4 * tp);
  run("g4g kc8 nbuf3", g4g<8, 3>, 512, nwg, 4 * tp);
  run("g4g kc32 nbuf2", g4g<32, 2>, 512, nwg, 4 * tp);
  run("g4 128x128 s144", g4<144>, 512, nwg, 4 * tp);
  run("g4 s144 sched1", g4<144, 1>, 512, nwg, 4 * tp);
  run("g4 s144 sched2", g4<144, 2>, 512, nwg, 4 * tp);
  run("g4 128x128 s144", g4<144>, 512, nwg, 4 * tp);
  run("g8 256x128 regs", (g8<false, 2>), 512, nwg / 2, 8 * tp);
  run("g8 256x128 glds2", (g8<true, 2>), 512, nwg / 2, 8 * tp);
  run("g8 256x128 glds3", (g8<true, 3>), 512, nwg / 2, 8 * tp);
  return 0;
}
