// The library's own diagonal-tile kernel (oi_launch_diag_factor, through the
// OiCell descriptors the engine passes) timed on one SPD tile per cell, to set
// against tools/diag_probe's descriptor-free copy: B cells, one launch per
// repetition with the tile restored in between (events around the kernel only).
//   build: hipcc -O3 -std=c++20 --offload-arch=gfx950 -I optimalinterpolation_amd/csrc \
//          tools/diag_engine_probe.hip -o tools/diag_engine_probe
#define OI_DIAG_TIMING 1
#include "../optimalinterpolation_amd/csrc/oi_kernels.hip"

#include <algorithm>
#include <cstring>
#include <chrono>
#include <cstdio>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int T = 4, n = 200;
  const int nt = T * (T + 1) / 2;
  const int BMAX = 1024;
  std::vector<double> tile(4096);
  srand(1);
  {
    std::vector<double> Bm(4096);
    for (auto& v : Bm) v = (rand() / (double)RAND_MAX) - 0.5;
    for (int i = 0; i < 64; ++i)
      for (int jj = 0; jj < 64; ++jj) {
        double s = i == jj ? 1.0 : 0.0;
        for (int k = 0; k < 64; ++k) s += Bm[i * 64 + k] * Bm[jj * 64 + k] / 64.0;
        tile[jj * 64 + i] = s;
      }
  }
  const size_t per = (size_t)(2 * nt + 2 * T) * 4096 + 4 * T * 64 + OI_PART_SIZE(nt, T) + 64;
  double* pool;
  CHK(hipMalloc(&pool, per * BMAX * 8));
  CHK(hipMemset(pool, 0, per * BMAX * 8));
  int32_t* status;
  CHK(hipMalloc(&status, BMAX * 4));
  CHK(hipMemset(status, 0, BMAX * 4));
  double* src;
  CHK(hipMalloc(&src, 4096 * 8));
  CHK(hipMemcpy(src, tile.data(), 4096 * 8, hipMemcpyHostToDevice));
  std::vector<OiCell> hc(BMAX);
  for (int b = 0; b < BMAX; ++b) {
    double* p = pool + per * b;
    OiCell& c = hc[b];
    std::memset((void*)&c, 0, sizeof(c));
    c.L = p; p += (size_t)nt * 4096;
    c.W = p; p += (size_t)nt * 4096;
    c.Dinv = p; p += (size_t)T * 4096;
    c.P = p; p += (size_t)T * 4096;
    c.vec = p; p += 4 * T * 64;
    c.part = p; p += OI_PART_SIZE(nt, T);
    c.out = p;
    c.status = status + b;
    c.n = n; c.T = T; c.mode = OI_MODE_EVAL; c.n_obs = n;
  }
  OiCell* dc;
  CHK(hipMalloc(&dc, BMAX * sizeof(OiCell)));
  CHK(hipMemcpy(dc, hc.data(), BMAX * sizeof(OiCell), hipMemcpyHostToDevice));
  std::vector<int32_t> hl(BMAX);
  for (int b = 0; b < BMAX; ++b) hl[b] = b;
  int32_t* dl;
  CHK(hipMalloc(&dl, BMAX * 4));
  CHK(hipMemcpy(dl, hl.data(), BMAX * 4, hipMemcpyHostToDevice));
  hipStream_t st;
  CHK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  auto restore = [&](int B) {
    for (int b = 0; b < B; ++b) CHK(hipMemcpyAsync(hc[b].L, src, 4096 * 8, hipMemcpyDeviceToDevice, st));
    CHK(hipMemsetAsync(status, 0, B * 4, st));
  };
  for (int B : {1, 256, 1024}) {
    std::vector<float> v;
    for (int k = 0; k < 40; ++k) {
      restore(B);
      CHK(hipEventRecord(e0, st));
      if (oi_launch_diag_factor(dc, dl, B, 0, st)) { printf("launch failed\n"); return 1; }
      CHK(hipEventRecord(e1, st));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      if (k >= 5) v.push_back(ms * 1e3f);
    }
    std::sort(v.begin(), v.end());
    long long stamps[16];
    CHK(hipMemcpyFromSymbol(stamps, HIP_SYMBOL(g_diag_stamps), sizeof(stamps)));
    printf("  stage cycles (last launch, cell 0):");
    const char* nm[8] = {"start", "load", "potrf", "stage L", "diag inv", "offdiag+D", "fwd", "W+alpha"};
    for (int q = 1; q < 8; ++q) printf(" %s %lld", nm[q], stamps[q] - stamps[q - 1]);
    printf("  total %lld\n", stamps[7] - stamps[0]);
    int32_t s0 = -1;
    CHK(hipMemcpy(&s0, status, 4, hipMemcpyDeviceToHost));
    printf("engine k_diag_factor%s B=%5d: p50 %8.2f us/launch (min %.2f) status %d\n",
           getenv("OI_DIAG") ? getenv("OI_DIAG") : "4w", B, v[v.size() / 2], v[0], s0);
  }
  return 0;
}
