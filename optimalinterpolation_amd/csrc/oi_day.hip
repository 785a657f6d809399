// HIP kernels (gfx950) for the day-level steps either side of the per-cell GP
// (SURVEY.md §8f rows 1-2), from 2021_paper_production/GPR_CS2S3.py (GPR:):
//
//   k_smooth_conv  GPR:65-73  inf -> NaN, clip at vmax, then astropy
//                  convolve(data, Gaussian2DKernel(std)) with its defaults:
//                  boundary 'fill' 0, nan_treatment 'interpolate' (per-pixel
//                  renormalisation over the non-NaN window entries), NaN where
//                  the whole window is NaN.  Window rows outer, columns inner,
//                  kernel flipped, no FMA contraction: bit-identical to the
//                  restatement in oracle/day_oracle.py.
//   k_smooth_fix   GPR:74-75  zeros -> np.nanmean(field) (numpy's summation
//                  order: 8192-element buffers, each pairwise), mask NaN -> NaN.
//   k_chunk_bbox / k_ball_count / k_ball_fill
//                  GPR:159  X_tree.query_ball_point(X[index], r): all training
//                  points with (dx*dx + dy*dy) <= r*r (scipy cKDTree's p=2 test),
//                  returned in ascending index order.  Points are scanned in
//                  chunks of 256 consecutive indices; a chunk whose bounding
//                  box is provably out of range is skipped (the training set is
//                  grid-ordered, so chunks are spatially compact).
//   k_gather_rows  GPR:160-161  inputs = [x_train, y_train, t_train][ID],
//                  outputs = z[ID] into the ragged layout of oi_gpr_batch.
// These are HBM/L2-bound integer and byte work; none of it is a GEMM.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#define SM_TILE 16
#define BQ_CHUNK 256

// ------------------------------------------------------------- smoothing
// One thread per output pixel of one field; the (16 + 2w)^2 input window of
// the workgroup is staged in LDS with inf -> NaN and the vmax clip applied,
// padding = fill value 0 (a valid, non-NaN 0 as in astropy's 'fill').
__global__ __launch_bounds__(256) void k_smooth_conv(const double* __restrict__ in,
                                                     double* __restrict__ out, int64_t ny,
                                                     int64_t nx, const double* __restrict__ vmax,
                                                     const double* __restrict__ kern, int ks) {
#pragma clang fp contract(off)
  extern __shared__ double tile[];  // (SM_TILE + ks - 1)^2
  const int w = ks / 2, tw = SM_TILE + ks - 1;
  const int f = blockIdx.z;
  const double vm = vmax[f];
  const double* src = in + (size_t)f * ny * nx;
  const int64_t r0 = (int64_t)blockIdx.y * SM_TILE - w, c0 = (int64_t)blockIdx.x * SM_TILE - w;
  for (int e = threadIdx.x; e < tw * tw; e += blockDim.x) {
    const int64_t r = r0 + e / tw, c = c0 + e % tw;
    double v = 0.0;
    if (r >= 0 && r < ny && c >= 0 && c < nx) {
      v = src[r * nx + c];
      if (isinf(v)) v = NAN;
      if (v > vm) v = vm;
    }
    tile[e] = v;
  }
  __syncthreads();
  const int ty = threadIdx.x / SM_TILE, tx = threadIdx.x % SM_TILE;
  const int64_t r = (int64_t)blockIdx.y * SM_TILE + ty, c = (int64_t)blockIdx.x * SM_TILE + tx;
  if (r >= ny || c >= nx) return;
  double top = 0.0, bot = 0.0;
  for (int ii = 0; ii < ks; ++ii) {
    const double* row = tile + (ty + ii) * tw + tx;
    const double* krow = kern + (ks - 1 - ii) * ks + (ks - 1);
    for (int jj = 0; jj < ks; ++jj) {
      const double val = row[jj];
      const double ker = krow[-jj];
      if (!isnan(val)) {
        top = top + val * ker;
        bot = bot + ker;
      }
    }
  }
  out[(size_t)f * ny * nx + r * nx + c] = bot == 0.0 ? NAN : top / bot;
}

// numpy pairwise_sum of a[lo .. lo+n) with NaN read as 0 (np.nanmean's
// _replace_nan), n <= 8192; explicit stack instead of recursion.
__device__ double np_pairwise_nan0(const double* a, int64_t n) {
#pragma clang fp contract(off)
  int64_t lo_s[16], n_s[16];
  double left_s[16];
  int stage_s[16];
  int sp = 0;
  lo_s[0] = 0;
  n_s[0] = n;
  stage_s[0] = 0;
  double result = 0.0;
  for (;;) {
    if (stage_s[sp] == 0) {
      const int64_t lo = lo_s[sp], m = n_s[sp];
      if (m <= 128) {
        auto at = [&](int64_t i) {
          const double v = a[lo + i];
          return isnan(v) ? 0.0 : v;
        };
        if (m < 8) {
          double res = 0.0;
          for (int64_t i = 0; i < m; ++i) res += at(i);
          result = res;
        } else {
          double r[8];
          for (int k = 0; k < 8; ++k) r[k] = at(k);
          int64_t i = 8;
          for (; i < m - (m % 8); i += 8)
            for (int k = 0; k < 8; ++k) r[k] += at(i + k);
          double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
          for (; i < m; ++i) res += at(i);
          result = res;
        }
      } else {
        int64_t n2 = m / 2;
        n2 -= n2 % 8;
        stage_s[sp] = 1;
        ++sp;
        lo_s[sp] = lo;
        n_s[sp] = n2;
        stage_s[sp] = 0;
        continue;
      }
    }
    // a value for frame sp is in `result`: return it to the parent
    for (;;) {
      if (sp == 0) return result;
      --sp;
      if (stage_s[sp] == 1) {
        left_s[sp] = result;
        stage_s[sp] = 2;
        int64_t n2 = n_s[sp] / 2;
        n2 -= n2 % 8;
        ++sp;
        lo_s[sp] = lo_s[sp - 1] + n2;
        n_s[sp] = n_s[sp - 1] - n2;
        stage_s[sp] = 0;
        break;
      }
      result = left_s[sp] + result;  // stage 2: left + right
    }
  }
}

// One workgroup per field: block sums (one 8192-element buffer per thread),
// accumulated left to right onto 0.0, / count of non-NaN; then zeros -> mean
// and mask-NaN -> NaN.
__global__ __launch_bounds__(256) void k_smooth_fix(double* __restrict__ data, int64_t npix,
                                                    const double* __restrict__ mask) {
#pragma clang fp contract(off)
  __shared__ double bsum[256];
  __shared__ double s_tot;
  __shared__ unsigned long long s_cnt;
  double* a = data + (size_t)blockIdx.x * npix;
  const int64_t nblk = (npix + 8191) / 8192;
  if (threadIdx.x == 0) {
    s_tot = 0.0;
    s_cnt = 0;
  }
  __syncthreads();
  for (int64_t b0 = 0; b0 < nblk; b0 += 256) {
    const int64_t b = b0 + threadIdx.x;
    if (b < nblk) {
      const int64_t lo = b * 8192, m = npix - lo < 8192 ? npix - lo : 8192;
      bsum[threadIdx.x] = np_pairwise_nan0(a + lo, m);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double tot = s_tot;
      for (int k = 0; k < 256 && b0 + k < nblk; ++k) tot = tot + bsum[k];
      s_tot = tot;
    }
    __syncthreads();
  }
  unsigned long long c = 0;  // non-NaN count: exact integer, order-free
  for (int64_t i = threadIdx.x; i < npix; i += blockDim.x) c += isnan(a[i]) ? 0 : 1;
  atomicAdd(&s_cnt, c);
  __syncthreads();
  const double mean = s_tot / (double)s_cnt;  // NaN when every pixel is NaN
  for (int64_t i = threadIdx.x; i < npix; i += blockDim.x) {
    double v = a[i];
    if (v == 0.0) v = mean;
    if (isnan(mask[i])) v = NAN;
    a[i] = v;
  }
}

// ------------------------------------------------------------- ball query
// Bounding box of every chunk of 256 consecutive points (pts: M x 2).
__global__ __launch_bounds__(256) void k_chunk_bbox(const double* __restrict__ pts, int64_t M,
                                                    double* __restrict__ bbox) {
  __shared__ double red[4][4];
  const int64_t i = (int64_t)blockIdx.x * BQ_CHUNK + threadIdx.x;
  double x0 = INFINITY, x1 = -INFINITY, y0 = INFINITY, y1 = -INFINITY;
  if (i < M) {
    x0 = x1 = pts[2 * i];
    y0 = y1 = pts[2 * i + 1];
  }
  for (int o = 32; o >= 1; o >>= 1) {
    x0 = fmin(x0, __shfl_xor(x0, o, 64));
    x1 = fmax(x1, __shfl_xor(x1, o, 64));
    y0 = fmin(y0, __shfl_xor(y0, o, 64));
    y1 = fmax(y1, __shfl_xor(y1, o, 64));
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[w][0] = x0;
    red[w][1] = x1;
    red[w][2] = y0;
    red[w][3] = y1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double b[4] = {red[0][0], red[0][1], red[0][2], red[0][3]};
    for (int k = 1; k < 4; ++k) {
      b[0] = fmin(b[0], red[k][0]);
      b[1] = fmax(b[1], red[k][1]);
      b[2] = fmin(b[2], red[k][2]);
      b[3] = fmax(b[3], red[k][3]);
    }
    for (int k = 0; k < 4; ++k) bbox[4 * blockIdx.x + k] = b[k];
  }
}

__device__ __forceinline__ bool chunk_may_hit(const double* bb, double qx, double qy, double r2) {
  const double dx = fmax(0.0, fmax(bb[0] - qx, qx - bb[1]));
  const double dy = fmax(0.0, fmax(bb[2] - qy, qy - bb[3]));
  return dx * dx + dy * dy <= r2 * (1.0 + 1e-9) + 1e-9;  // conservative
}

__device__ __forceinline__ bool in_ball(const double* __restrict__ pts, int64_t i, double qx,
                                        double qy, double r2) {
#pragma clang fp contract(off)
  const double dx = pts[2 * i] - qx, dy = pts[2 * i + 1] - qy;
  double d = dx * dx;
  d = d + dy * dy;
  return d <= r2;
}

// The chunks a query's ball may touch, in ascending order, 256 at a time: every
// thread tests one chunk's bounding box and the hits are compacted in order
// into LDS (wave ballots + wave prefix), so a workgroup walks nchunk / 256
// batches instead of testing every chunk serially.  Returns the batch's count.
__device__ __forceinline__ int chunk_batch(const double* __restrict__ bbox, int64_t nchunk, int64_t base,
                                           double qx, double qy, double r2, int* list, int* wcnt) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t ch = base + t;
  const bool may = ch < nchunk && chunk_may_hit(bbox + 4 * ch, qx, qy, r2);
  const unsigned long long m = __ballot(may);
  if (lane == 0) wcnt[w] = __popcll(m);
  __syncthreads();
  int before = 0;
  for (int k = 0; k < w; ++k) before += wcnt[k];
  if (may) list[before + __popcll(lane ? (m & ((1ull << lane) - 1ull)) : 0ull)] = t;
  const int total = ((wcnt[0] + wcnt[1]) + wcnt[2]) + wcnt[3];
  __syncthreads();
  return total;
}

// one workgroup (256 threads = 4 waves) per query
__global__ __launch_bounds__(256) void k_ball_count(const double* __restrict__ pts, int64_t M,
                                                    const double* __restrict__ bbox,
                                                    const double* __restrict__ q, double r2,
                                                    int64_t* __restrict__ counts) {
  __shared__ int64_t red[4];
  __shared__ int list[BQ_CHUNK], wcnt[4];
  const double qx = q[2 * blockIdx.x], qy = q[2 * blockIdx.x + 1];
  const int64_t nchunk = (M + BQ_CHUNK - 1) / BQ_CHUNK;
  int64_t cnt = 0;
  for (int64_t base = 0; base < nchunk; base += BQ_CHUNK) {
    const int nc = chunk_batch(bbox, nchunk, base, qx, qy, r2, list, wcnt);
    for (int k = 0; k < nc; ++k) {
      const int64_t i = (base + list[k]) * BQ_CHUNK + threadIdx.x;
      const bool hit = i < M && in_ball(pts, i, qx, qy, r2);
      cnt += __popcll(__ballot(hit));
    }
    __syncthreads();  // list is rewritten by the next batch
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

__global__ __launch_bounds__(256) void k_ball_fill(const double* __restrict__ pts, int64_t M,
                                                   const double* __restrict__ bbox,
                                                   const double* __restrict__ q, double r2,
                                                   const int64_t* __restrict__ offs,
                                                   int64_t* __restrict__ idx) {
  __shared__ int wcnt[4];
  __shared__ int list[BQ_CHUNK], bcnt[4];
  const double qx = q[2 * blockIdx.x], qy = q[2 * blockIdx.x + 1];
  const int64_t nchunk = (M + BQ_CHUNK - 1) / BQ_CHUNK;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t pos = offs[blockIdx.x];
  for (int64_t base = 0; base < nchunk; base += BQ_CHUNK) {
    const int nc = chunk_batch(bbox, nchunk, base, qx, qy, r2, list, bcnt);
    for (int k = 0; k < nc; ++k) {
      const int64_t i = (base + list[k]) * BQ_CHUNK + threadIdx.x;
      const bool hit = i < M && in_ball(pts, i, qx, qy, r2);
      const unsigned long long m = __ballot(hit);
      if (lane == 0) wcnt[w] = __popcll(m);
      __syncthreads();
      int before = 0;
      for (int kk = 0; kk < w; ++kk) before += wcnt[kk];
      const int total = ((wcnt[0] + wcnt[1]) + wcnt[2]) + wcnt[3];
      if (hit) {
        const unsigned long long lt = lane ? (m & ((1ull << lane) - 1ull)) : 0ull;
        idx[pos + before + __popcll(lt)] = i;
      }
      pos += total;
      __syncthreads();
    }
  }
}

// rows[k] = (x, y, t)[idx[k]], zout[k] = z[idx[k]]
__global__ __launch_bounds__(256) void k_gather_rows(const double* __restrict__ xt,
                                                     const double* __restrict__ yt,
                                                     const double* __restrict__ tt,
                                                     const double* __restrict__ zt,
                                                     const int64_t* __restrict__ idx, int64_t N,
                                                     int64_t M, double* __restrict__ xyt,
                                                     double* __restrict__ zout) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= N) return;
  const int64_t i = idx[k];
  if (i < 0 || i >= M) {  // never read out of bounds: a bad index gives NaN rows
    xyt[3 * k] = xyt[3 * k + 1] = xyt[3 * k + 2] = zout[k] = NAN;
    return;
  }
  xyt[3 * k] = xt[i];
  xyt[3 * k + 1] = yt[i];
  xyt[3 * k + 2] = tt[i];
  zout[k] = zt[i];
}

// ------------------------------------------------------------ launchers
static inline int ret() { return hipGetLastError() == hipSuccess ? 0 : -1; }

extern "C" int oi_launch_smooth(const double* in, double* out, int nf, int64_t ny, int64_t nx,
                                const double* vmax, const double* kern, int ks, const double* mask,
                                void* stream) {
  if (nf <= 0 || ny <= 0 || nx <= 0) return 0;
  const int tw = SM_TILE + ks - 1;
  dim3 grid((unsigned)((nx + SM_TILE - 1) / SM_TILE), (unsigned)((ny + SM_TILE - 1) / SM_TILE),
            (unsigned)nf);
  hipLaunchKernelGGL(k_smooth_conv, grid, dim3(256), (size_t)tw * tw * 8, (hipStream_t)stream, in,
                     out, ny, nx, vmax, kern, ks);
  if (ret()) return -1;
  hipLaunchKernelGGL(k_smooth_fix, dim3((unsigned)nf), dim3(256), 0, (hipStream_t)stream, out,
                     ny * nx, mask);
  return ret();
}

extern "C" int oi_launch_ball_count(const double* pts, int64_t M, double* bbox, const double* q,
                                    int64_t Q, double r2, int64_t* counts, void* stream) {
  if (Q <= 0) return 0;
  if (M <= 0) return hipMemsetAsync(counts, 0, (size_t)Q * 8, (hipStream_t)stream) == hipSuccess ? 0 : -1;
  const int64_t nchunk = (M + BQ_CHUNK - 1) / BQ_CHUNK;
  hipLaunchKernelGGL(k_chunk_bbox, dim3((unsigned)nchunk), dim3(256), 0, (hipStream_t)stream, pts,
                     M, bbox);
  if (ret()) return -1;
  hipLaunchKernelGGL(k_ball_count, dim3((unsigned)Q), dim3(256), 0, (hipStream_t)stream, pts, M,
                     bbox, q, r2, counts);
  return ret();
}

extern "C" int oi_launch_ball_fill(const double* pts, int64_t M, const double* bbox,
                                   const double* q, int64_t Q, double r2, const int64_t* offs,
                                   int64_t* idx, void* stream) {
  if (Q <= 0 || M <= 0) return 0;
  hipLaunchKernelGGL(k_ball_fill, dim3((unsigned)Q), dim3(256), 0, (hipStream_t)stream, pts, M,
                     bbox, q, r2, offs, idx);
  return ret();
}

extern "C" int oi_launch_gather_rows(const double* xt, const double* yt, const double* tt,
                                     const double* zt, const int64_t* idx, int64_t N, int64_t M,
                                     double* xyt, double* zout, void* stream) {
  if (N <= 0) return 0;
  hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)((N + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, xt, yt, tt, zt, idx, N, M, xyt, zout);
  return ret();
}
