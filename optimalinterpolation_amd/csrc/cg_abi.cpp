// The optimiser alone through the C ABI (include/oi.h, oi_cg_*): scipy's
// minimize(method='CG', jac=True) as called at GPR_CS2S3.py:166, restated in
// cg.cpp, driven by caller-supplied objective values.  Host-only code: it is
// also built on its own with ASan/UBSan (Makefile target `sanitize`,
// tests/test_cg_sanitize.py).
#include "../../include/oi.h"
#include "cg.hpp"

extern "C" int oi_set_last_error(int code, const char* msg);

extern "C" {

// ---- optimiser handle
struct oi_cg {
  oi::EvalSlot mail;
  oi::Task<oi::CgResult> task;
  bool started = false;
};

oi_cg* oi_cg_create(const double* x0, double gtol, int32_t maxiter) {
  if (!x0) {
    oi_set_last_error(OI_E_ARG, "null x0");
    return nullptr;
  }
  auto* h = new oi_cg();
  oi::Vec v;
  for (int k = 0; k < oi::NH; ++k) v[k] = x0[k];
  oi::CgOptions o;
  o.gtol = gtol;
  o.maxiter = maxiter;
  h->task = oi::cg_minimize(&h->mail, v, o);
  return h;
}

int oi_cg_step(oi_cg* h, double* x_req) {
  if (!h) return oi_set_last_error(OI_E_ARG, "null handle");
  if (!h->started) {
    h->started = true;
    h->task.start();
  }
  if (h->task.done()) return 0;
  if (!h->mail.pending) return oi_set_last_error(OI_E_ARG, "oi_cg_step: optimiser in an invalid state");
  if (x_req)
    for (int k = 0; k < oi::NH; ++k) x_req[k] = h->mail.x[k];
  return 1;
}

int oi_cg_feed(oi_cg* h, double f, const double* g) {
  if (!h || !g) return oi_set_last_error(OI_E_ARG, "null argument");
  if (!h->mail.pending) return oi_set_last_error(OI_E_ARG, "oi_cg_feed: no pending request");
  h->mail.f = f;
  for (int k = 0; k < oi::NH; ++k) h->mail.g[k] = g[k];
  h->mail.pending = false;
  h->mail.waiter.resume();
  return 0;
}

int oi_cg_result(oi_cg* h, double* x, double* fun, int32_t* nit, int32_t* status, int64_t* nfev,
                 int64_t* njev, int64_t* nobj) {
  if (!h || !h->task.done()) return oi_set_last_error(OI_E_ARG, "optimiser not finished");
  const oi::CgResult& r = h->task.result();
  if (x)
    for (int k = 0; k < oi::NH; ++k) x[k] = r.x[k];
  if (fun) *fun = r.fun;
  if (nit) *nit = r.nit;
  if (status) *status = r.status;
  if (nfev) *nfev = r.nfev;
  if (njev) *njev = r.njev;
  if (nobj) *nobj = r.nobj;
  return 0;
}

void oi_cg_destroy(oi_cg* h) { delete h; }

}  // extern "C"
