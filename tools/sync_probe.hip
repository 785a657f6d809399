// Probe: host <-> GPU round-trip latency of one tiny dependent step, the
// pattern of config 1 (one cell: the host's CG step waits for every
// evaluation).  Variants:
//   a  launch + hipStreamSynchronize
//   b  launch + 128 B D2H hipMemcpyAsync (pinned) + hipStreamSynchronize
//   c  H2D 4 KB hipMemcpyAsync + launch + D2H + hipStreamSynchronize (today's round)
//   d  launch + host spin on hipStreamQuery
//   e  launch (kernel stores its result into pinned host memory) + spin on hipStreamQuery
//   f  launch + hipEventRecord + spin on hipEventQuery
//   g  launch (kernel stores its result into pinned host memory) + host spin on
//      that value itself (no runtime call; bounded at 1 s)
//   build: hipcc -O3 --offload-arch=gfx950 tools/sync_probe.hip -o tools/sync_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void k_step(const double* in, double* out, int it) {
  if (threadIdx.x < 16) out[threadIdx.x] = in[threadIdx.x] + it;
}

int main() {
  hipStream_t st;
  CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  double *d_in, *d_out, *h_in, *h_out;
  CHK(hipMalloc(&d_in, 4096));
  CHK(hipMalloc(&d_out, 4096));
  CHK(hipMemset(d_in, 0, 4096));
  CHK(hipHostMalloc(&h_in, 4096, hipHostMallocDefault));
  CHK(hipHostMalloc(&h_out, 4096, hipHostMallocDefault));
  double* h_out_dev = nullptr;
  CHK(hipHostGetDevicePointer((void**)&h_out_dev, h_out, 0));
  hipEvent_t ev;
  CHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const char* names = "abcdefg";
  for (int rep = 0; rep < 2; ++rep)
    for (int v = 0; v < 7; ++v) {
      const int N = 2000;
      std::vector<double> us;
      for (int i = 0; i < N; ++i) {
        h_in[0] = 0.0;
        const auto t0 = std::chrono::steady_clock::now();
        if (v == 2) CHK(hipMemcpyAsync(d_in, h_in, 4096, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_step, dim3(1), dim3(64), 0, st, d_in, (v == 4 || v == 6) ? h_out_dev : d_out, i);
        if (v == 1 || v == 2) CHK(hipMemcpyAsync(h_out, d_out, 128, hipMemcpyDeviceToHost, st));
        if (v <= 2) {
          CHK(hipStreamSynchronize(st));
        } else if (v == 6) {
          volatile double* f = h_out;
          const auto ts = std::chrono::steady_clock::now();
          while (f[0] != (double)i &&
                 std::chrono::steady_clock::now() - ts < std::chrono::seconds(1)) {
          }
          if (f[0] != (double)i) printf("g: flag not seen within 1 s at i=%d\n", i);
        } else if (v == 5) {
          CHK(hipEventRecord(ev, st));
          while (hipEventQuery(ev) == hipErrorNotReady) {
          }
        } else {
          while (hipStreamQuery(st) == hipErrorNotReady) {
          }
        }
        const auto t1 = std::chrono::steady_clock::now();
        us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      }
      std::sort(us.begin(), us.end());
      printf("%c: p50 %7.2f us  p10 %7.2f  p90 %7.2f\n", names[v], us[N / 2], us[N / 10], us[N * 9 / 10]);
    }
  return 0;
}
