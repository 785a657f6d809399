// Wave masks of the GEMM cores (oi_gemm.h), shared by the kernels
// (oi_kernels.hip) and the engine's executed-flop accounting (oi_engine.cpp):
// bit 2*mb + nb of a wave's 2 x 2 blocks of 16 x 16 at output rows r0 + 16 mb,
// columns c0 + 16 nb.
#pragma once
#include <hip/hip_runtime.h>

// Padding masks: bit 2*mb + nb of a wave's 16x16 accumulator blocks whose
// rows (m0 = row offset of the wave's quadrant, 16-row blocks mb) or columns
// (n0, blocks nb) lie at or beyond `mlim` / `nlim` (64 = no padding).
__host__ __device__ inline unsigned pad_skip(int m0, int n0, int mlim, int nlim) {
  unsigned s = 0;
  for (int mb = 0; mb < 2; ++mb)
    for (int nb = 0; nb < 2; ++nb)
      if (m0 + 16 * mb >= mlim || n0 + 16 * nb >= nlim) s |= 1u << (2 * mb + nb);
  return s;
}

// Structural zeros of triangular operands, per 16-deep k-chunk c, for a
// wave's 2 x 2 blocks (bit 2*mb + nb) at output rows r0 + 16 mb and columns
// c0 + 16 nb (gemm cores: acc(m, n) += A(m, k) B(k, n)):
//   A(m, k) = 0 for k < m (W_jj,jj as the A operand): rows_below
//   A(m, k) = 0 for k > m (Dinv_jj, column-major, as A):  rows_above
//   B(k, n) = 0 for k < n (W_jj,jj as B):                  cols_below
//   B(k, n) = 0 for k > n (Dinv_jj^T as B):                cols_above
// The skipped products are exact zeros, so results do not change.
__host__ __device__ inline unsigned rows_below(int c, int r0) {
  unsigned s = 0;
  for (int mb = 0; mb < 2; ++mb)
    if (16 * c + 15 < r0 + 16 * mb) s |= 3u << (2 * mb);
  return s;
}
__host__ __device__ inline unsigned rows_above(int c, int r0) {
  unsigned s = 0;
  for (int mb = 0; mb < 2; ++mb)
    if (16 * c > r0 + 16 * mb + 15) s |= 3u << (2 * mb);
  return s;
}
__host__ __device__ inline unsigned cols_below(int c, int c0) {
  unsigned s = 0;
  for (int nb = 0; nb < 2; ++nb)
    if (16 * c + 15 < c0 + 16 * nb) s |= 5u << nb;
  return s;
}
__host__ __device__ inline unsigned cols_above(int c, int c0) {
  unsigned s = 0;
  for (int nb = 0; nb < 2; ++nb)
    if (16 * c > c0 + 16 * nb + 15) s |= 5u << nb;
  return s;
}
// accumulator blocks strictly above (m < n) / below (m > n) the diagonal of a
// symmetric (syrk) output tile
__host__ __device__ inline unsigned upper_blocks(int r0, int c0) {
  unsigned s = 0;
  for (int mb = 0; mb < 2; ++mb)
    for (int nb = 0; nb < 2; ++nb)
      if (r0 + 16 * mb + 15 < c0 + 16 * nb) s |= 1u << (2 * mb + nb);
  return s;
}
__host__ __device__ inline unsigned lower_blocks(int r0, int c0) {
  unsigned s = 0;
  for (int mb = 0; mb < 2; ++mb)
    for (int nb = 0; nb < 2; ++nb)
      if (r0 + 16 * mb > c0 + 16 * nb + 15) s |= 1u << (2 * mb + nb);
  return s;
}

