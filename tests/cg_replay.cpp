// Host-only replay harness for the optimiser C ABI (oi_cg_*), built with
// ASan + UBSan by `make -C optimalinterpolation_amd sanitize`
// (tests/test_cg_sanitize.py).  Reads golden CG trajectories (scipy's own
// calls, tests/golden/cg.npz, dumped as text by the test) and replays them:
// every point the restated CG requests must equal scipy's bit for bit, and the
// final x / nit / nfev / status must match.  Exit 0 = all cells equal.
#include <cstdio>
#include <cstring>
#include <vector>

#include "../include/oi.h"

extern "C" int oi_set_last_error(int code, const char* msg) {
  std::fprintf(stderr, "oi error %d: %s\n", code, msg ? msg : "");
  return code;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = std::fopen(argv[1], "r");
  if (!f) return 2;
  int ncell = 0, bad = 0;
  if (std::fscanf(f, "%d", &ncell) != 1) return 2;
  for (int c = 0; c < ncell; ++c) {
    int ncall = 0;
    double x0[6], rx[6];
    int rnit, rnfev, rstatus;
    if (std::fscanf(f, "%d", &ncall) != 1) return 2;
    for (double& v : x0) std::fscanf(f, "%la", &v);
    std::vector<double> X(6 * ncall), F(ncall), G(6 * ncall);
    for (int k = 0; k < ncall; ++k) {
      for (int q = 0; q < 6; ++q) std::fscanf(f, "%la", &X[6 * k + q]);
      std::fscanf(f, "%la", &F[k]);
      for (int q = 0; q < 6; ++q) std::fscanf(f, "%la", &G[6 * k + q]);
    }
    for (double& v : rx) std::fscanf(f, "%la", &v);
    std::fscanf(f, "%d %d %d", &rnit, &rnfev, &rstatus);
    oi_cg* h = oi_cg_create(x0, 1e-5, -1);
    double req[6];
    int k = 0, rc;
    while ((rc = oi_cg_step(h, req)) == 1) {
      if (k >= ncall || std::memcmp(req, &X[6 * k], sizeof(req)) != 0) {
        std::fprintf(stderr, "cell %d: request %d differs from scipy's\n", c, k);
        ++bad;
        break;
      }
      oi_cg_feed(h, F[k], &G[6 * k]);
      ++k;
    }
    if (rc == 0) {
      double x[6], fun;
      int32_t nit, status;
      int64_t nfev, njev, nobj;
      oi_cg_result(h, x, &fun, &nit, &status, &nfev, &njev, &nobj);
      if (std::memcmp(x, rx, sizeof(x)) != 0 || nit != rnit || nfev != rnfev || status != rstatus ||
          nobj != ncall) {
        std::fprintf(stderr, "cell %d: result differs (nit %d/%d nfev %lld/%d status %d/%d)\n", c, nit,
                     rnit, (long long)nfev, rnfev, status, rstatus);
        ++bad;
      }
    } else if (rc < 0) {
      ++bad;
    }
    oi_cg_destroy(h);
  }
  std::fclose(f);
  // misuse paths: a finished / never-started handle, null arguments
  if (oi_cg_create(nullptr, 1e-5, -1) != nullptr) ++bad;
  double z6[6] = {0, 0, 0, 0, 0, 0};
  oi_cg* h = oi_cg_create(z6, 1e-5, -1);
  if (oi_cg_feed(h, 0.0, z6) >= 0) ++bad;   // no pending request before the first step
  oi_cg_destroy(h);
  std::printf("%s %d cells\n", bad ? "FAIL" : "OK", ncell);
  return bad ? 1 : 0;
}
