// fp64 MFMA tile-GEMM core shared by the kernels (oi_kernels.hip) and the
// micro-benchmarks (tools/gemm_probe*.hip).
//
// A 512-thread workgroup (8 waves) computes a 64 x 128 block D = [D0 | D1]:
//   D[m][n] += sum_p sum_k A_p[k*64 + m] * Bh_p[k*64 + n']     (n = 64h + n')
// i.e. two 64x64 output tiles that share the A operand.  All operands are
// "k-major" 64x64 tiles (a column-major tile X used as X[m][k], or a row-major
// tile used as X^T), so global -> LDS staging is contiguous 16 B per lane.
// Wave w owns rows 32*((w>>2)&1) .. +32 and columns 32*(w&3) .. +32 as 2x2
// blocks of v_mfma_f64_16x16x4f64; lane l of block (mb, nb) holds
//   D[32wr + 16mb + (l>>4) + 4r][32wc + 16nb + (l&15)],  r = 0..3.
// Measured on MI355X (tools/gemm_probe2.hip, v7): 63 TF/s with both operands
// streamed from HBM vs 48.5 TF/s for a 256-thread 64x64 tile.
#pragma once
#include <type_traits>
#include <hip/hip_runtime.h>

typedef double d4 __attribute__((ext_vector_type(4)));

#define GNB 64
#define KC 16                          // k-depth of one staged chunk
#define LDSA 80                        // A chunk row stride (doubles)
#define LDSB 144                       // B chunk row stride: rows k, k+1 land in
                                       // opposite bank halves for ds_read_b64
#define STAGE_A (KC * LDSA)
#define STAGE_B (KC * LDSB)
#define GEMM2_LDS (2 * (STAGE_A + STAGE_B))  // 7168 doubles = 56 KiB
#define GEMM_THREADS 512

struct Quad {
  d4 c[2][2];
};

__device__ __forceinline__ void quad_zero(Quad& q) {
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b) q.c[a][b] = (d4){0.0, 0.0, 0.0, 0.0};
}

// coordinates in the 64 x 128 block of accumulator entry (mb, nb, r) of this lane
__device__ __forceinline__ int acc_row(int mb, int r) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  return 32 * ((w >> 2) & 1) + 16 * mb + (lane >> 4) + 4 * r;
}
__device__ __forceinline__ int acc_col(int nb) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  return 32 * (w & 3) + 16 * nb + (lane & 15);
}

#define MFMA64(a, b, c) __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0)

// pair(p, a, b0, b1): the p-th operand triple (A tile, B tile of the left
// half, B tile of the right half).  Register staging is a two-deep ring
// (chunks ch+1 and ch+2 in flight while ch is multiplied out of LDS), two LDS
// buffers; every thread stages one 16 B piece of each of A, B0 and B1, so the
// loads are branch-free and s_waitcnt can count them exactly.
typedef double dv2 __attribute__((ext_vector_type(2)));
// Operand tiles are read through global-address-space pointers: the tile
// addresses come out of OiCell records, so the compiler would otherwise emit
// FLAT loads, which count against lgkmcnt too -- every s_waitcnt lgkmcnt(0)
// of the LDS reads in compute() would then also wait for the prefetch of the
// next chunks, exposing HBM latency once per chunk.
typedef __attribute__((address_space(1))) const dv2 gdv2;
__device__ __forceinline__ dv2 gload2(const double* p) { return *(gdv2*)p; }
struct StageRegs {
  dv2 a0, a1, b0, b1;
};
struct StageRegs3 {
  dv2 a, b0, b1;
};

// Per-chunk masks (MASKED only): cmask(ch) returns more blocks to drop for
// 16-deep chunk ch alone -- the structural zeros of a triangular operand
// (Dinv_jj, W_jj,jj) in the pair that carries it, where whole chunks of k
// meet only zeros for some of the wave's output blocks.  Evaluated once per
// chunk and made wave-uniform (readfirstlane), like `skip`.
struct NoChunkMask {
  __device__ __forceinline__ unsigned operator()(int) const { return 0u; }
};

// MASKED: `skip` (wave-uniform, bit 2*mb + nb) drops this wave's 16x16
// accumulator blocks that cover only padding rows / columns of a cell (their
// exact result is 0, which the accumulator already holds).
template <bool MASKED = false, class PairFn, class CMask = NoChunkMask>
__device__ __forceinline__ void gemm2_kmajor(Quad& acc, double* lds, int npairs, PairFn pair,
                                             unsigned skip = 0u, CMask cmask = CMask()) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = (w >> 2) & 1, wc = w & 3;
  const int nch = npairs * (GNB / KC);  // even
  if (nch == 0) return;
  if (MASKED) skip = __builtin_amdgcn_readfirstlane(skip);
  const int sk = t >> 5, sm = (t & 31) * 2;  // this thread's 16 B of a 16 x 64 chunk
  const int fr = lane & 15, fk = lane >> 4;
  StageRegs3 r0, r1;
  auto load = [&](int ch, StageRegs3& q) __attribute__((always_inline)) {
    const double *pa, *pb0, *pb1;
    [[clang::always_inline]] pair(ch >> 2, pa, pb0, pb1);
    const int off = (ch & 3) * KC * GNB + t * 2;
    q.a = gload2(pa + off);
    q.b0 = gload2(pb0 + off);
    q.b1 = gload2(pb1 + off);
  };
  auto store = [&](int buf, const StageRegs3& q) __attribute__((always_inline)) {
    double* As = lds + buf * (STAGE_A + STAGE_B);
    double* Bs = As + STAGE_A;
    *(dv2*)(As + sk * LDSA + sm) = q.a;
    *(dv2*)(Bs + sk * LDSB + sm) = q.b0;
    *(dv2*)(Bs + sk * LDSB + 64 + sm) = q.b1;
  };
  auto compute = [&](int buf, int chunk) __attribute__((always_inline)) {
    const double* As = lds + buf * (STAGE_A + STAGE_B);
    const double* Bs = As + STAGE_A;
    // a wave skips a chunk only when all four of its blocks are masked (one
    // uniform branch per chunk; per-MFMA tests cost more than the partial
    // blocks they save -- those compute exact zeros or unread entries)
    if (MASKED && (skip | __builtin_amdgcn_readfirstlane(cmask(chunk))) == 0xFu) return;
#pragma unroll
    for (int kk = 0; kk < KC / 4; ++kk) {
      const int k = kk * 4 + fk;
      const double a0 = As[k * LDSA + 32 * wr + fr];
      const double a1 = As[k * LDSA + 32 * wr + 16 + fr];
      const double b0 = Bs[k * LDSB + 32 * wc + fr];
      const double b1 = Bs[k * LDSB + 32 * wc + 16 + fr];
      acc.c[0][0] = MFMA64(a0, b0, acc.c[0][0]);
      acc.c[0][1] = MFMA64(a0, b1, acc.c[0][1]);
      acc.c[1][0] = MFMA64(a1, b0, acc.c[1][0]);
      acc.c[1][1] = MFMA64(a1, b1, acc.c[1][1]);
    }
  };
  load(0, r0);
  load(1, r1);
  store(0, r0);
  __syncthreads();
  // The prefetches are unconditional (the last ones re-read the final chunk,
  // unused): a conditional load makes s_waitcnt merge "issued" and "skipped"
  // paths and wait for the newest loads too, serialising the ring.
  for (int ch = 0; ch < nch; ch += 2) {
    load(min(ch + 2, nch - 1), r0);
    compute(0, ch);
    store(1, r1);
    __syncthreads();
    load(min(ch + 3, nch - 1), r1);
    compute(1, ch + 1);
    if (ch + 2 < nch) store(0, r0);
    __syncthreads();
  }
}

// ---- 256-thread variant: one 64x64 output tile, wave w owns the 32x32
// quadrant (32*(w>>1), 32*(w&1)); LDS 2 x (A, B) chunks of 16 x 80 = 40 KiB,
// so four workgroups fit a CU.
#define GEMM1_LDS (4 * STAGE_A)
__device__ __forceinline__ int acc1_row(int mb, int r) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  return 32 * (w >> 1) + 16 * mb + (lane >> 4) + 4 * r;
}
__device__ __forceinline__ int acc1_col(int nb) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  return 32 * (w & 1) + 16 * nb + (lane & 15);
}

// Staging registers are a two-deep ring (chunks ch+1 and ch+2 in flight while
// ch is multiplied out of LDS): 66 TF/s vs 57 TF/s for a one-deep prefetch
// when one operand is L2-resident (tools/gemm_probe3.hip).  Native vector
// types (not HIP's double2 struct) keep the ring in VGPRs.
//
// `nch` counts 16-deep k-chunks (4 per operand pair; a caller may cut the
// last pair short when its k rows run into a cell's padding, which holds
// exact zeros there).  Each thread stages pieces p = t and p = t + 256 of a
// 16 x 64 chunk (16 B each, row p >> 5): consecutive lanes write consecutive
// 16 B, so the ds_write_b128 lane groups hit distinct banks.
// MASKED: `skip` (wave-uniform, bit 2*mb + nb) drops this wave's 16x16
// accumulator blocks whose outputs are never used (the upper triangle of a
// diagonal tile, padding rows / columns); their accumulators stay 0.
template <bool MASKED = false, class PairFn, class CMask = NoChunkMask>
__device__ __forceinline__ void gemm1_kmajor(Quad& acc, double* lds, int nch, unsigned skip,
                                             PairFn pair, CMask cmask = CMask()) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1;
  if (nch <= 0) return;
  const int sk = t >> 5, sm = (t & 31) * 2;
  const int fr = lane & 15, fk = lane >> 4;
  if (MASKED) skip = __builtin_amdgcn_readfirstlane(skip);
  StageRegs r0, r1;
  auto load = [&](int ch, StageRegs& q) __attribute__((always_inline)) {
    const double *pa, *pb;
    [[clang::always_inline]] pair(ch >> 2, pa, pb);
    const int off = (ch & 3) * KC * GNB + t * 2;
    q.a0 = gload2(pa + off);
    q.a1 = gload2(pa + off + 512);
    q.b0 = gload2(pb + off);
    q.b1 = gload2(pb + off + 512);
  };
  auto store = [&](int buf, const StageRegs& q) __attribute__((always_inline)) {
    double* As = lds + buf * 2 * STAGE_A;
    double* Bs = As + STAGE_A;
    *(dv2*)(As + sk * LDSA + sm) = q.a0;
    *(dv2*)(As + (sk + 8) * LDSA + sm) = q.a1;
    *(dv2*)(Bs + sk * LDSA + sm) = q.b0;
    *(dv2*)(Bs + (sk + 8) * LDSA + sm) = q.b1;
  };
  auto compute = [&](int buf, int chunk) __attribute__((always_inline)) {
    const double* As = lds + buf * 2 * STAGE_A;
    const double* Bs = As + STAGE_A;
    // per-block tests (uniform branches): on this 256-thread core they cost
    // less than the partial blocks they save (k_lauum_grad1 -2 %, k_chol_panel
    // -10 %; the 512-thread gemm2 prefers whole-chunk skips)
    unsigned sk = skip;
    if (MASKED) sk |= __builtin_amdgcn_readfirstlane(cmask(chunk));
    if (MASKED && sk == 0xFu) return;
#pragma unroll
    for (int kk = 0; kk < KC / 4; ++kk) {
      const int k = kk * 4 + fk;
      const double a0 = As[k * LDSA + 32 * wr + fr];
      const double a1 = As[k * LDSA + 32 * wr + 16 + fr];
      const double b0 = Bs[k * LDSA + 32 * wc + fr];
      const double b1 = Bs[k * LDSA + 32 * wc + 16 + fr];
      if (!MASKED || !(sk & 1u)) acc.c[0][0] = MFMA64(a0, b0, acc.c[0][0]);
      if (!MASKED || !(sk & 2u)) acc.c[0][1] = MFMA64(a0, b1, acc.c[0][1]);
      if (!MASKED || !(sk & 4u)) acc.c[1][0] = MFMA64(a1, b0, acc.c[1][0]);
      if (!MASKED || !(sk & 8u)) acc.c[1][1] = MFMA64(a1, b1, acc.c[1][1]);
    }
  };
  load(0, r0);
  load(min(1, nch - 1), r1);
  store(0, r0);
  __syncthreads();
  // unconditional prefetches: see gemm2_kmajor; an odd last chunk skips the
  // second half-step (the re-loaded duplicate is staged but never used)
  for (int ch = 0; ch < nch; ch += 2) {
    load(min(ch + 2, nch - 1), r0);
    compute(0, ch);
    store(1, r1);
    __syncthreads();
    load(min(ch + 3, nch - 1), r1);
    if (ch + 1 < nch) compute(1, ch + 1);
    if (ch + 2 < nch) store(0, r0);
    __syncthreads();
  }
}

// ---- 128 x 128 variant: 512 threads, wave w owns rows 32*(w>>1) .. +32 and
// columns 64*(w&1) .. +64 as 2 x 4 blocks of v_mfma_f64_16x16x4f64 (8
// independent accumulators, 8 MFMAs per 6 LDS reads).  Each streamed tile
// feeds two outputs: a 2 x 2 block of output tiles per workgroup, half the
// operand traffic of the 64 x 128 core and a quarter of the 64 x 64 one
// (tools/gemm4_probe.hip: 61 vs 52.5 / 35 TF/s streaming, 63 vs 59 / 53
// L2-resident).  LDS: two buffers of (A, B) 16 x 128 chunks, row stride 144.
#define GEMM4_LDSS 144
#define GEMM4_STG (KC * GEMM4_LDSS)
#define GEMM4_LDS (4 * GEMM4_STG)  // 9216 doubles = 72 KiB -> two workgroups per CU
struct Quad8 {
  d4 c[2][4];
};
__device__ __forceinline__ void quad8_zero(Quad8& q) {
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 4; ++b) q.c[a][b] = (d4){0.0, 0.0, 0.0, 0.0};
}
// coordinates in the 128 x 128 block of accumulator entry (mb, nb, r) of this lane
__device__ __forceinline__ int acc4_row(int mb, int r) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  return 32 * (w >> 1) + 16 * mb + (lane >> 4) + 4 * r;
}
__device__ __forceinline__ int acc4_col(int nb) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  return 64 * (w & 1) + 16 * nb + (lane & 15);
}

// pair(p, a0, a1, b0, b1): the p-th operand tiles -- A for output rows 0..63 /
// 64..127, B for output columns 0..63 / 64..127 (all k-major).  `nch` counts
// 16-deep chunks (4 per pair; the last pair may be cut short).  MASKED: `skip`
// (wave-uniform, bit 4*mb + nb) drops accumulator blocks whose outputs are
// never used.
template <bool MASKED, class PairFn>
__device__ __forceinline__ void gemm4_kmajor(Quad8& acc, double* lds, int nch, unsigned skip, PairFn pair) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1;
  if (nch <= 0) return;
  if (MASKED) skip = __builtin_amdgcn_readfirstlane(skip);
  const int sk = t >> 5, sm = (t & 31) * 2;  // this thread's 16 B of a 16 x 64 chunk
  const int fr = lane & 15, fk = lane >> 4;
  StageRegs r0, r1;  // a0 / a1 / b0 / b1: one 16 B piece of each operand tile
  auto load = [&](int ch, StageRegs& q) __attribute__((always_inline)) {
    const double *pa0, *pa1, *pb0, *pb1;
    [[clang::always_inline]] pair(ch >> 2, pa0, pa1, pb0, pb1);
    const int off = (ch & 3) * KC * GNB + t * 2;
    q.a0 = gload2(pa0 + off);
    q.a1 = gload2(pa1 + off);
    q.b0 = gload2(pb0 + off);
    q.b1 = gload2(pb1 + off);
  };
  auto store = [&](int buf, const StageRegs& q) __attribute__((always_inline)) {
    double* As = lds + buf * 2 * GEMM4_STG;
    double* Bs = As + GEMM4_STG;
    *(dv2*)(As + sk * GEMM4_LDSS + sm) = q.a0;
    *(dv2*)(As + sk * GEMM4_LDSS + 64 + sm) = q.a1;
    *(dv2*)(Bs + sk * GEMM4_LDSS + sm) = q.b0;
    *(dv2*)(Bs + sk * GEMM4_LDSS + 64 + sm) = q.b1;
  };
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const double* As = lds + buf * 2 * GEMM4_STG;
    const double* Bs = As + GEMM4_STG;
#pragma unroll
    for (int kk = 0; kk < KC / 4; ++kk) {
      const int k = kk * 4 + fk;
      const double a0 = As[k * GEMM4_LDSS + 32 * wr + fr];
      const double a1 = As[k * GEMM4_LDSS + 32 * wr + 16 + fr];
      double b[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) b[q] = Bs[k * GEMM4_LDSS + 64 * wc + 16 * q + fr];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (!MASKED || !(skip & (1u << q))) acc.c[0][q] = MFMA64(a0, b[q], acc.c[0][q]);
        if (!MASKED || !(skip & (1u << (4 + q)))) acc.c[1][q] = MFMA64(a1, b[q], acc.c[1][q]);
      }
    }
  };
  load(0, r0);
  load(min(1, nch - 1), r1);
  store(0, r0);
  __syncthreads();
  for (int ch = 0; ch < nch; ch += 2) {
    load(min(ch + 2, nch - 1), r0);
    compute(0);
    store(1, r1);
    __syncthreads();
    load(min(ch + 3, nch - 1), r1);
    if (ch + 1 < nch) compute(1);
    if (ch + 2 < nch) store(0, r0);
    __syncthreads();
  }
}
