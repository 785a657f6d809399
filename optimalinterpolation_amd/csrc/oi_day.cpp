// C ABI of the day-level device steps (include/oi.h, "day pipeline"):
//   oi_smooth_fields  <- smooth() GPR_CS2S3.py:65-76 (called 5x, GPR:303-307)
//   oi_ball_query     <- X_tree.query_ball_point(X[index], r) GPR:159, batched
//   oi_gather_rows    <- inputs / outputs gathering GPR:160-161, batched
// Kernels: oi_day.hip.  Host mode copies through the library; with
// opts->device_inputs = 1 the array arguments are device pointers (HBM
// resident) and nothing crosses PCIe except the small host-side arrays named
// in oi.h (vmax, kern, offs).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/oi.h"

extern "C" {
int oi_launch_smooth(const double* in, double* out, int nf, int64_t ny, int64_t nx,
                     const double* vmax, const double* kern, int ks, const double* mask,
                     void* stream);
int oi_launch_ball_count(const double* pts, int64_t M, double* bbox, const double* q, int64_t Q,
                         double r2, int64_t* counts, void* stream);
int oi_launch_ball_fill(const double* pts, int64_t M, const double* bbox, const double* q,
                        int64_t Q, double r2, const int64_t* offs, int64_t* idx, void* stream);
int oi_launch_gather_rows(const double* xt, const double* yt, const double* tt, const double* zt,
                          const int64_t* idx, int64_t N, int64_t M, double* xyt, double* zout,
                          void* stream);
int oi_set_last_error(int code, const char* msg);  // oi_engine.cpp
}

namespace {

struct HipErr {
  std::string msg;
};

#define HC(expr)                                                                   \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) throw HipErr{std::string(#expr) + ": " + hipGetErrorString(e_)}; \
  } while (0)

// device buffer owned for the duration of one call, allocated and freed in
// the call's stream order: hipFree would synchronise the whole device, so a
// radius query issued between a session's rounds (bench.py's timed day) would
// drain the rounds in flight on the session's streams
struct DBuf {
  void* p = nullptr;
  hipStream_t s = nullptr;
  DBuf() = default;
  DBuf(size_t bytes, hipStream_t st) : s(st) {
    if (bytes) HC(hipMallocAsync(&p, bytes, s));
  }
  ~DBuf() {
    if (p) (void)hipFreeAsync(p, s);
  }
  DBuf(const DBuf&) = delete;
  DBuf& operator=(const DBuf&) = delete;
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

struct Ctx {
  oi_options o;
  hipStream_t s;
};

int setup(const oi_options* opts, Ctx& c) {
  oi_options_default(&c.o);
  if (opts) c.o = *opts;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return oi_set_last_error(OI_E_NODEV, "no HIP device available");
  if (c.o.device < 0 || c.o.device >= ndev) return oi_set_last_error(OI_E_ARG, "bad device ordinal");
  if (hipSetDevice(c.o.device) != hipSuccess) return oi_set_last_error(OI_E_HIP, "hipSetDevice failed");
  c.s = (hipStream_t)c.o.stream;
  return 0;
}

template <class F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const HipErr& e) {
    return oi_set_last_error(OI_E_HIP, e.msg.c_str());
  } catch (const std::bad_alloc&) {
    return oi_set_last_error(OI_E_NOMEM, "allocation failed");
  }
}

// astropy Gaussian2DKernel(x_stddev=std): Gaussian2D(amplitude 1/(2 pi std^2),
// theta 0) sampled at integer offsets, size 8*std rounded up to odd, / sum.
std::vector<double> gaussian_kernel(double std_, int& ks) {
  int i = (int)std::ceil(8.0 * std_);
  ks = (i % 2 == 0) ? i + 1 : i;
  const int h = (ks - 1) / 2;
  const double a = 0.5 * (1.0 / (std_ * std_)), amp = 1.0 / (2 * M_PI * std_ * std_);
  std::vector<double> k((size_t)ks * ks);
  double s = 0.0;
  for (int y = -h; y <= h; ++y)
    for (int x = -h; x <= h; ++x) {
      const double v = amp * std::exp(-((a * (double)(x * x)) + (a * (double)(y * y))));
      k[(size_t)(y + h) * ks + (x + h)] = v;
      s += v;
    }
  for (double& v : k) v /= s;
  return k;
}

}  // namespace

extern "C" {

int oi_smooth_fields(const double* fields, int32_t nf, int64_t ny, int64_t nx, const double* vmax,
                     const double* mask, double std_, const double* kern, int32_t ks, double* out,
                     const oi_options* opts) {
  if (nf < 0 || ny < 0 || nx < 0) return oi_set_last_error(OI_E_ARG, "negative size");
  if (nf == 0 || ny == 0 || nx == 0) return 0;
  if (!fields || !vmax || !mask || !out) return oi_set_last_error(OI_E_ARG, "null pointer");
  std::vector<double> kv;
  if (kern) {
    if (ks <= 0 || ks % 2 == 0 || ks > 65) return oi_set_last_error(OI_E_ARG, "kernel size must be odd, <= 65");
    kv.assign(kern, kern + (size_t)ks * ks);
  } else {
    if (!(std_ > 0.0) || std_ > 8.0) return oi_set_last_error(OI_E_ARG, "std must be in (0, 8]");
    kv = gaussian_kernel(std_, ks);
  }
  Ctx c;
  if (int rc = setup(opts, c)) return rc;
  return guarded([&] {
    const size_t npix = (size_t)ny * nx, fb = (size_t)nf * npix * 8;
    DBuf dk(kv.size() * 8, c.s), dv((size_t)nf * 8, c.s);
    HC(hipMemcpyAsync(dk.p, kv.data(), kv.size() * 8, hipMemcpyHostToDevice, c.s));
    HC(hipMemcpyAsync(dv.p, vmax, (size_t)nf * 8, hipMemcpyHostToDevice, c.s));
    if (c.o.device_inputs) {
      if (oi_launch_smooth(fields, out, nf, ny, nx, dv.as<double>(), dk.as<double>(), ks, mask, c.s))
        throw HipErr{"smooth kernel launch failed"};
      HC(hipStreamSynchronize(c.s));
      return 0;
    }
    DBuf din(fb, c.s), dout(fb, c.s), dm(npix * 8, c.s);
    HC(hipMemcpyAsync(din.p, fields, fb, hipMemcpyHostToDevice, c.s));
    HC(hipMemcpyAsync(dm.p, mask, npix * 8, hipMemcpyHostToDevice, c.s));
    if (oi_launch_smooth(din.as<double>(), dout.as<double>(), nf, ny, nx, dv.as<double>(),
                         dk.as<double>(), ks, dm.as<double>(), c.s))
      throw HipErr{"smooth kernel launch failed"};
    HC(hipMemcpyAsync(out, dout.p, fb, hipMemcpyDeviceToHost, c.s));
    HC(hipStreamSynchronize(c.s));
    return 0;
  });
}

int oi_ball_query(const double* pts, int64_t M, const double* q, int64_t Q, double r,
                  int64_t* offs, int64_t* idx, int64_t cap, const oi_options* opts) {
  if (M < 0 || Q < 0 || cap < 0) return oi_set_last_error(OI_E_ARG, "negative size");
  if (!offs) return oi_set_last_error(OI_E_ARG, "null offs");
  offs[0] = 0;
  if (Q == 0) return 0;
  if (!q || (M > 0 && !pts)) return oi_set_last_error(OI_E_ARG, "null pointer");
  if (!(r >= 0.0)) return oi_set_last_error(OI_E_ARG, "radius must be >= 0");
  Ctx c;
  if (int rc = setup(opts, c)) return rc;
  return guarded([&] {
    const double r2 = r * r;
    const bool dev = c.o.device_inputs != 0;
    DBuf dpts(dev ? 0 : (size_t)M * 16, c.s), dq(dev ? 0 : (size_t)Q * 16, c.s);
    const double* P = dev ? pts : dpts.as<double>();
    const double* Qp = dev ? q : dq.as<double>();
    if (!dev) {
      if (M) HC(hipMemcpyAsync(dpts.p, pts, (size_t)M * 16, hipMemcpyHostToDevice, c.s));
      HC(hipMemcpyAsync(dq.p, q, (size_t)Q * 16, hipMemcpyHostToDevice, c.s));
    }
    DBuf bbox((size_t)((M + 255) / 256 + 1) * 32, c.s), cnt((size_t)Q * 8, c.s);
    if (oi_launch_ball_count(P, M, bbox.as<double>(), Qp, Q, r2, cnt.as<int64_t>(), c.s))
      throw HipErr{"ball count launch failed"};
    std::vector<int64_t> h((size_t)Q);
    HC(hipMemcpyAsync(h.data(), cnt.p, (size_t)Q * 8, hipMemcpyDeviceToHost, c.s));
    HC(hipStreamSynchronize(c.s));
    for (int64_t k = 0; k < Q; ++k) offs[k + 1] = offs[k] + h[(size_t)k];
    const int64_t total = offs[Q];
    if (!idx || total > cap || total == 0) return 0;  // caller sizes idx from offs[Q]
    DBuf doffs((size_t)(Q + 1) * 8, c.s);
    HC(hipMemcpyAsync(doffs.p, offs, (size_t)(Q + 1) * 8, hipMemcpyHostToDevice, c.s));
    DBuf didx(dev ? 0 : (size_t)total * 8, c.s);
    int64_t* I = dev ? idx : didx.as<int64_t>();
    if (oi_launch_ball_fill(P, M, bbox.as<double>(), Qp, Q, r2, doffs.as<int64_t>(), I, c.s))
      throw HipErr{"ball fill launch failed"};
    if (!dev) HC(hipMemcpyAsync(idx, didx.p, (size_t)total * 8, hipMemcpyDeviceToHost, c.s));
    HC(hipStreamSynchronize(c.s));
    return 0;
  });
}

int oi_gather_rows(const double* x_train, const double* y_train, const double* t_train,
                   const double* z, int64_t M, const int64_t* idx, int64_t N, double* xyt,
                   double* zout, const oi_options* opts) {
  if (N < 0 || M < 0) return oi_set_last_error(OI_E_ARG, "negative size");
  if (N == 0) return 0;
  if (!x_train || !y_train || !t_train || !z || !idx || !xyt || !zout)
    return oi_set_last_error(OI_E_ARG, "null pointer");
  Ctx c;
  if (int rc = setup(opts, c)) return rc;
  return guarded([&] {
    if (c.o.device_inputs) {
      if (oi_launch_gather_rows(x_train, y_train, t_train, z, idx, N, M, xyt, zout, c.s))
        throw HipErr{"gather launch failed"};
      HC(hipStreamSynchronize(c.s));
      return 0;
    }
    for (int64_t k = 0; k < N; ++k)
      if (idx[k] < 0 || idx[k] >= M) return oi_set_last_error(OI_E_ARG, "index out of range");
    DBuf dx((size_t)M * 8, c.s), dy((size_t)M * 8, c.s), dt((size_t)M * 8, c.s), dz((size_t)M * 8, c.s),
        di((size_t)N * 8, c.s), dxyt((size_t)N * 24, c.s), dzo((size_t)N * 8, c.s);
    HC(hipMemcpyAsync(dx.p, x_train, (size_t)M * 8, hipMemcpyHostToDevice, c.s));
    HC(hipMemcpyAsync(dy.p, y_train, (size_t)M * 8, hipMemcpyHostToDevice, c.s));
    HC(hipMemcpyAsync(dt.p, t_train, (size_t)M * 8, hipMemcpyHostToDevice, c.s));
    HC(hipMemcpyAsync(dz.p, z, (size_t)M * 8, hipMemcpyHostToDevice, c.s));
    HC(hipMemcpyAsync(di.p, idx, (size_t)N * 8, hipMemcpyHostToDevice, c.s));
    if (oi_launch_gather_rows(dx.as<double>(), dy.as<double>(), dt.as<double>(), dz.as<double>(),
                              di.as<int64_t>(), N, M, dxyt.as<double>(), dzo.as<double>(), c.s))
      throw HipErr{"gather launch failed"};
    HC(hipMemcpyAsync(xyt, dxyt.p, (size_t)N * 24, hipMemcpyDeviceToHost, c.s));
    HC(hipMemcpyAsync(zout, dzo.p, (size_t)N * 8, hipMemcpyDeviceToHost, c.s));
    HC(hipStreamSynchronize(c.s));
    return 0;
  });
}

}  // extern "C"
