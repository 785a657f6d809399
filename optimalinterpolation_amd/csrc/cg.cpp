// Restatement of scipy 1.15.3's CG minimiser (see cg.hpp for the file map).
// Every arithmetic expression keeps scipy's evaluation order; Python/numpy
// semantics that matter for bit-identical iterates are made explicit:
//   * np.dot of two 6-vectors  -> sequential FMA chain (OpenBLAS ddot tail
//     loop; probed on the reference's container)
//   * np.dot(2x2, 2-vector)    -> y_i = fma(a_i0, v0, a_i1*v1) (OpenBLAS dgemv)
//   * Python max()/min()       -> first-argument-wins NaN behaviour
//   * np.clip / np.sign / np.amax -> NaN-propagating numpy definitions
//   * np.errstate(raise) in _cubicmin/_quadmin -> per-op IEEE flag checks
//   * `x ** k`                 -> libm pow(), exactly what numpy/CPython call
#include "cg.hpp"

#include <cmath>
#include <optional>

namespace oi {

namespace {

inline Vec axpy(const Vec& xk, double s, const Vec& pk) {
  Vec r;
  for (int i = 0; i < NH; ++i) r[i] = xk[i] + s * pk[i];
  return r;
}

inline bool array_equal(const Vec& a, const Vec& b) {
  for (int i = 0; i < NH; ++i)
    if (!(a[i] == b[i])) return false;
  return true;
}

// np.amax(np.abs(x)) -- NaN propagates
inline double vecnorm_inf(const Vec& x) {
  double m = std::fabs(x[0]);
  for (int i = 1; i < NH; ++i) {
    double v = std::fabs(x[i]);
    if (std::isnan(m)) break;
    if (std::isnan(v) || v > m) m = v;
  }
  return m;
}

// Python builtins: the first argument is kept unless a later one compares
// strictly greater/less (so NaN handling depends on position)
inline double py_max(double a, double b) { return b > a ? b : a; }
inline double py_max(double a, double b, double c) { return py_max(py_max(a, b), c); }
inline double py_min(double a, double b) { return b < a ? b : a; }

// numpy clip for floats: _NPY_MIN(_NPY_MAX(x, lo), hi), NaN-propagating
inline double np_clip(double x, double lo, double hi) {
  double t = std::isnan(x) ? x : (x > lo ? x : lo);
  return std::isnan(t) ? t : (t < hi ? t : hi);
}

inline double np_sign(double x) {
  if (x > 0) return 1.0;
  if (x < 0) return -1.0;
  if (x == 0) return 0.0;
  return x;  // NaN
}

// IEEE-flag emulation for `with np.errstate(divide, over, invalid='raise')`
struct Checked {
  bool err = false;
  double chk(double r, double a, double b) {
    if (std::isinf(r) && std::isfinite(a) && std::isfinite(b)) err = true;            // overflow
    if (std::isnan(r) && !std::isnan(a) && !std::isnan(b)) err = true;                // invalid
    return r;
  }
  double add(double a, double b) { return chk(a + b, a, b); }
  double sub(double a, double b) { return chk(a - b, a, b); }
  double mul(double a, double b) { return chk(a * b, a, b); }
  double div(double a, double b) {
    double r = a / b;
    if (b == 0.0) {
      if (std::isfinite(a) && a != 0.0) err = true;  // divide by zero
      if (a == 0.0) err = true;                      // 0/0 invalid
      return r;
    }
    return chk(r, a, b);
  }
  double powi(double a, double k) {
    double r = std::pow(a, k);
    if (std::isinf(r) && std::isfinite(a)) err = true;
    if (std::isnan(r) && !std::isnan(a)) err = true;
    return r;
  }
  double sqrt(double a) {
    if (a < 0.0) err = true;
    return std::sqrt(a);
  }
};

// _linesearch.py _cubicmin
std::optional<double> cubicmin(double a, double fa, double fpa, double b, double fb, double c,
                               double fc) {
  Checked k;
  double C = fpa;
  double db = k.sub(b, a);
  double dc = k.sub(c, a);
  double denom = k.mul(k.powi(k.mul(db, dc), 2.0), k.sub(db, dc));
  double d00 = k.powi(dc, 2.0);
  double d01 = -k.powi(db, 2.0);
  double d10 = -k.powi(dc, 3.0);
  double d11 = k.powi(db, 3.0);
  double v0 = k.sub(k.sub(fb, fa), k.mul(C, db));
  double v1 = k.sub(k.sub(fc, fa), k.mul(C, dc));
  if (k.err) return std::nullopt;
  // np.dot(d1, v): BLAS dgemv, flags not inspected
  double A = std::fma(d00, v0, d01 * v1);
  double B = std::fma(d10, v0, d11 * v1);
  A = k.div(A, denom);
  B = k.div(B, denom);
  double radical = k.sub(k.mul(B, B), k.mul(k.mul(3.0, A), C));
  double xmin = k.add(a, k.div(k.add(-B, k.sqrt(radical)), k.mul(3.0, A)));
  if (k.err) return std::nullopt;
  if (!std::isfinite(xmin)) return std::nullopt;
  return xmin;
}

// _linesearch.py _quadmin
std::optional<double> quadmin(double a, double fa, double fpa, double b, double fb) {
  Checked k;
  double D = fa;
  double C = fpa;
  double db = k.sub(b, k.mul(a, 1.0));
  double B = k.div(k.sub(k.sub(fb, D), k.mul(C, db)), k.mul(db, db));
  double xmin = k.sub(a, k.div(C, k.mul(2.0, B)));
  if (k.err) return std::nullopt;
  if (!std::isfinite(xmin)) return std::nullopt;
  return xmin;
}

// ---------------------------------------------------------------- DCSRCH
enum class LsTask { START, FG, CONV, WARN, ERROR };

struct Dcstep {
  double stx, fx, dx, sty, fy, dy, stp;
  bool brackt;
};

// _dcsrch.py dcstep
Dcstep dcstep(double stx, double fx, double dx, double sty, double fy, double dy, double stp,
              double fp, double dp, bool brackt, double stpmin, double stpmax) {
  double sgnd = np_sign(dp) * np_sign(dx);
  double stpf;
  if (fp > fx) {
    double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
    double s = py_max(std::fabs(theta), std::fabs(dx), std::fabs(dp));
    double gamma = s * std::sqrt(std::pow(theta / s, 2.0) - (dx / s) * (dp / s));
    if (stp < stx) gamma *= -1;
    double p = (gamma - dx) + theta;
    double q = ((gamma - dx) + gamma) + dp;
    double r = p / q;
    double stpc = stx + r * (stp - stx);
    double stpq = stx + ((dx / ((fx - fp) / (stp - stx) + dx)) / 2.0) * (stp - stx);
    if (std::fabs(stpc - stx) <= std::fabs(stpq - stx))
      stpf = stpc;
    else
      stpf = stpc + (stpq - stpc) / 2.0;
    brackt = true;
  } else if (sgnd < 0.0) {
    double theta = 3 * (fx - fp) / (stp - stx) + dx + dp;
    double s = py_max(std::fabs(theta), std::fabs(dx), std::fabs(dp));
    double gamma = s * std::sqrt(std::pow(theta / s, 2.0) - (dx / s) * (dp / s));
    if (stp > stx) gamma *= -1;
    double p = (gamma - dp) + theta;
    double q = ((gamma - dp) + gamma) + dx;
    double r = p / q;
    double stpc = stp + r * (stx - stp);
    double stpq = stp + (dp / (dp - dx)) * (stx - stp);
    if (std::fabs(stpc - stp) > std::fabs(stpq - stp))
      stpf = stpc;
    else
      stpf = stpq;
    brackt = true;
  } else if (std::fabs(dp) < std::fabs(dx)) {
    double theta = 3 * (fx - fp) / (stp - stx) + dx + dp;
    double s = py_max(std::fabs(theta), std::fabs(dx), std::fabs(dp));
    double gamma = s * std::sqrt(py_max(0.0, std::pow(theta / s, 2.0) - (dx / s) * (dp / s)));
    if (stp > stx) gamma = -gamma;
    double p = (gamma - dp) + theta;
    double q = (gamma + (dx - dp)) + gamma;
    double r = p / q;
    double stpc;
    if (r < 0 && gamma != 0)
      stpc = stp + r * (stx - stp);
    else if (stp > stx)
      stpc = stpmax;
    else
      stpc = stpmin;
    double stpq = stp + (dp / (dp - dx)) * (stx - stp);
    if (brackt) {
      if (std::fabs(stpc - stp) < std::fabs(stpq - stp))
        stpf = stpc;
      else
        stpf = stpq;
      if (stp > stx)
        stpf = py_min(stp + 0.66 * (sty - stp), stpf);
      else
        stpf = py_max(stp + 0.66 * (sty - stp), stpf);
    } else {
      if (std::fabs(stpc - stp) > std::fabs(stpq - stp))
        stpf = stpc;
      else
        stpf = stpq;
      stpf = np_clip(stpf, stpmin, stpmax);
    }
  } else {
    if (brackt) {
      double theta = 3.0 * (fp - fy) / (sty - stp) + dy + dp;
      double s = py_max(std::fabs(theta), std::fabs(dy), std::fabs(dp));
      double gamma = s * std::sqrt(std::pow(theta / s, 2.0) - (dy / s) * (dp / s));
      if (stp > sty) gamma = -gamma;
      double p = (gamma - dp) + theta;
      double q = ((gamma - dp) + gamma) + dy;
      double r = p / q;
      double stpc = stp + r * (sty - stp);
      stpf = stpc;
    } else if (stp > stx) {
      stpf = stpmax;
    } else {
      stpf = stpmin;
    }
  }
  if (fp > fx) {
    sty = stp;
    fy = fp;
    dy = dp;
  } else {
    if (sgnd < 0) {
      sty = stx;
      fy = fx;
      dy = dx;
    }
    stx = stp;
    fx = fp;
    dx = dp;
  }
  return Dcstep{stx, fx, dx, sty, fy, dy, stpf, brackt};
}

// _dcsrch.py DCSRCH._iterate (state machine; one call per trial step)
class Dcsrch {
 public:
  Dcsrch(double ftol, double gtol, double xtol, double stpmin, double stpmax)
      : ftol_(ftol), gtol_(gtol), xtol_(xtol), stpmin_(stpmin), stpmax_(stpmax) {}

  LsTask iterate(double& stp, double f, double g, LsTask task) {
    const double p5 = 0.5, p66 = 0.66, xtrapl = 1.1, xtrapu = 4.0;
    if (task == LsTask::START) {
      if (stp < stpmin_) task = LsTask::ERROR;
      if (stp > stpmax_) task = LsTask::ERROR;
      if (g >= 0) task = LsTask::ERROR;
      if (ftol_ < 0) task = LsTask::ERROR;
      if (gtol_ < 0) task = LsTask::ERROR;
      if (xtol_ < 0) task = LsTask::ERROR;
      if (stpmin_ < 0) task = LsTask::ERROR;
      if (stpmax_ < stpmin_) task = LsTask::ERROR;
      if (task == LsTask::ERROR) return task;
      brackt_ = false;
      stage_ = 1;
      finit_ = f;
      ginit_ = g;
      gtest_ = ftol_ * ginit_;
      width_ = stpmax_ - stpmin_;
      width1_ = width_ / p5;
      stx_ = 0.0;
      fx_ = finit_;
      gx_ = ginit_;
      sty_ = 0.0;
      fy_ = finit_;
      gy_ = ginit_;
      stmin_ = 0;
      stmax_ = stp + xtrapu * stp;
      return LsTask::FG;
    }
    double ftest = finit_ + stp * gtest_;
    if (stage_ == 1 && f <= ftest && g >= 0) stage_ = 2;
    if (brackt_ && (stp <= stmin_ || stp >= stmax_)) task = LsTask::WARN;
    if (brackt_ && stmax_ - stmin_ <= xtol_ * stmax_) task = LsTask::WARN;
    if (stp == stpmax_ && f <= ftest && g <= gtest_) task = LsTask::WARN;
    if (stp == stpmin_ && (f > ftest || g >= gtest_)) task = LsTask::WARN;
    if (f <= ftest && std::fabs(g) <= gtol_ * -ginit_) task = LsTask::CONV;
    if (task == LsTask::WARN || task == LsTask::CONV) return task;

    if (stage_ == 1 && f <= fx_ && f > ftest) {
      double fm = f - stp * gtest_;
      double fxm = fx_ - stx_ * gtest_;
      double fym = fy_ - sty_ * gtest_;
      double gm = g - gtest_;
      double gxm = gx_ - gtest_;
      double gym = gy_ - gtest_;
      Dcstep t = dcstep(stx_, fxm, gxm, sty_, fym, gym, stp, fm, gm, brackt_, stmin_, stmax_);
      stx_ = t.stx;
      fxm = t.fx;
      gxm = t.dx;
      sty_ = t.sty;
      fym = t.fy;
      gym = t.dy;
      stp = t.stp;
      brackt_ = t.brackt;
      fx_ = fxm + stx_ * gtest_;
      fy_ = fym + sty_ * gtest_;
      gx_ = gxm + gtest_;
      gy_ = gym + gtest_;
    } else {
      Dcstep t = dcstep(stx_, fx_, gx_, sty_, fy_, gy_, stp, f, g, brackt_, stmin_, stmax_);
      stx_ = t.stx;
      fx_ = t.fx;
      gx_ = t.dx;
      sty_ = t.sty;
      fy_ = t.fy;
      gy_ = t.dy;
      stp = t.stp;
      brackt_ = t.brackt;
    }
    if (brackt_) {
      if (std::fabs(sty_ - stx_) >= p66 * width1_) stp = stx_ + p5 * (sty_ - stx_);
      width1_ = width_;
      width_ = std::fabs(sty_ - stx_);
    }
    if (brackt_) {
      stmin_ = py_min(stx_, sty_);
      stmax_ = py_max(stx_, sty_);
    } else {
      stmin_ = stp + xtrapl * (stp - stx_);
      stmax_ = stp + xtrapu * (stp - stx_);
    }
    stp = np_clip(stp, stpmin_, stpmax_);
    if ((brackt_ && (stp <= stmin_ || stp >= stmax_)) ||
        (brackt_ && stmax_ - stmin_ <= xtol_ * stmax_))
      stp = stx_;
    return LsTask::FG;
  }

 private:
  double ftol_, gtol_, xtol_, stpmin_, stpmax_;
  bool brackt_ = false;
  int stage_ = 0;
  double ginit_ = 0, gtest_ = 0, gx_ = 0, gy_ = 0, finit_ = 0, fx_ = 0, fy_ = 0;
  double stx_ = 0, sty_ = 0, stmin_ = 0, stmax_ = 0, width_ = 0, width1_ = 0;
};

// ------------------------------------------------ CG iteration context
struct PrpStep {
  double alpha;
  Vec xkp1, pkp1, gfkp1;
  double gnorm;
};

struct CgIter {
  Vec xk, pk, gfk;
  double deltak;
  double gtol;
  std::optional<PrpStep> cached;  // cached_step

  // polak_ribiere_powell_step with a known gradient
  PrpStep step(double alpha, const Vec& gfkp1) const {
    PrpStep s;
    s.alpha = alpha;
    s.xkp1 = axpy(xk, alpha, pk);
    s.gfkp1 = gfkp1;
    Vec yk;
    for (int i = 0; i < NH; ++i) yk[i] = gfkp1[i] - gfk[i];
    double beta_k = py_max(0.0, np_dot(yk, gfkp1) / deltak);
    for (int i = 0; i < NH; ++i) s.pkp1[i] = -gfkp1[i] + beta_k * pk[i];
    s.gnorm = vecnorm_inf(gfkp1);
    return s;
  }

  // descent_condition (the extra_condition of the line searches)
  bool descent(double alpha, const Vec& gfkp1) {
    cached = step(alpha, gfkp1);
    if (cached->gnorm <= gtol) return true;
    return np_dot(cached->pkp1, cached->gfkp1) <= -0.01 * np_dot(cached->gfkp1, cached->gfkp1);
  }
};

struct LsOut {
  bool ok = false;
  double alpha = 0, fval = 0, old_fval = 0;
  std::optional<Vec> gfkp1;
};

// phi / derphi closures of the line searches
struct Line {
  Objective& ob;
  const Vec& xk;
  const Vec& pk;
  Vec gval;
  std::optional<double> gval_alpha;

  Task<double> phi(double s) { co_return co_await ob.fun(axpy(xk, s, pk)); }
  Task<double> derphi(double s) {
    gval = co_await ob.grad(axpy(xk, s, pk));
    gval_alpha = s;
    co_return np_dot(gval, pk);
  }
};

// line_search_wolfe1 + scalar_search_wolfe1 + DCSRCH.__call__
Task<LsOut> wolfe1(Objective& ob, const Vec& xk, const Vec& pk, const Vec& gfk, double old_fval,
                   double old_old_fval, double c1, double c2) {
  const double amax = 1e100, amin = 1e-100, xtol = 1e-14;
  Line ln{ob, xk, pk, gfk, std::nullopt};
  double derphi0 = np_dot(gfk, pk);
  double phi0 = old_fval, old_phi0 = old_old_fval;
  double alpha1;
  if (derphi0 != 0) {
    alpha1 = py_min(1.0, 1.01 * 2 * (phi0 - old_phi0) / derphi0);
    if (alpha1 < 0) alpha1 = 1.0;
  } else {
    alpha1 = 1.0;
  }
  Dcsrch dc(c1, c2, xtol, amin, amax);
  double phi1 = phi0, derphi1 = derphi0;
  LsTask task = LsTask::START;
  std::optional<double> stp;
  bool exhausted = true;
  for (int i = 0; i < 100; ++i) {
    double s = alpha1;
    task = dc.iterate(s, phi1, derphi1, task);
    if (!std::isfinite(s)) {
      task = LsTask::WARN;
      stp.reset();
      exhausted = false;
      break;
    }
    stp = s;
    if (task == LsTask::FG) {
      alpha1 = s;
      phi1 = co_await ln.phi(s);
      derphi1 = co_await ln.derphi(s);
    } else {
      exhausted = false;
      break;
    }
  }
  if (exhausted) stp.reset();
  if (task == LsTask::ERROR || task == LsTask::WARN) stp.reset();
  LsOut out;
  if (stp) {
    out.ok = true;
    out.alpha = *stp;
    out.fval = phi1;
    out.old_fval = phi0;
    out.gfkp1 = ln.gval;
  }
  co_return out;
}

// _linesearch.py _zoom
struct ZoomOut {
  bool ok = false;
  double a = 0, val = 0, valprime = 0;
};

Task<ZoomOut> zoom(Line& ln, CgIter& it, double a_lo, double a_hi, double phi_lo, double phi_hi,
                   double derphi_lo, double phi0, double derphi0, double c1, double c2) {
  const int maxiter = 10;
  int i = 0;
  const double delta1 = 0.2, delta2 = 0.1;
  double phi_rec = phi0;
  double a_rec = 0;
  ZoomOut out;
  while (true) {
    double dalpha = a_hi - a_lo;
    double a, b;
    if (dalpha < 0) {
      a = a_hi;
      b = a_lo;
    } else {
      a = a_lo;
      b = a_hi;
    }
    std::optional<double> a_j;
    double cchk = 0;
    if (i > 0) {
      cchk = delta1 * dalpha;
      a_j = cubicmin(a_lo, phi_lo, derphi_lo, a_hi, phi_hi, a_rec, phi_rec);
    }
    if (i == 0 || !a_j || *a_j > b - cchk || *a_j < a + cchk) {
      double qchk = delta2 * dalpha;
      a_j = quadmin(a_lo, phi_lo, derphi_lo, a_hi, phi_hi);
      if (!a_j || *a_j > b - qchk || *a_j < a + qchk) a_j = a_lo + 0.5 * dalpha;
    }
    double aj = *a_j;
    double phi_aj = co_await ln.phi(aj);
    if (phi_aj > phi0 + c1 * aj * derphi0 || phi_aj >= phi_lo) {
      phi_rec = phi_hi;
      a_rec = a_hi;
      a_hi = aj;
      phi_hi = phi_aj;
    } else {
      double derphi_aj = co_await ln.derphi(aj);
      bool accept = false;
      if (std::fabs(derphi_aj) <= -c2 * derphi0) {
        // extra_condition2: derphi(alpha) again only if the stored gradient is
        // from another alpha (never the case right after derphi(aj))
        if (!ln.gval_alpha || *ln.gval_alpha != aj) co_await ln.derphi(aj);
        accept = it.descent(aj, ln.gval);
      }
      if (accept) {
        out.ok = true;
        out.a = aj;
        out.val = phi_aj;
        out.valprime = derphi_aj;
        break;
      }
      if (derphi_aj * (a_hi - a_lo) >= 0) {
        phi_rec = phi_hi;
        a_rec = a_hi;
        a_hi = a_lo;
        phi_hi = phi_lo;
      } else {
        phi_rec = phi_lo;
        a_rec = a_lo;
      }
      a_lo = aj;
      phi_lo = phi_aj;
      derphi_lo = derphi_aj;
    }
    i += 1;
    if (i > maxiter) {
      out.ok = false;
      break;
    }
  }
  co_return out;
}

// line_search_wolfe2 + scalar_search_wolfe2 (with extra_condition2)
Task<LsOut> wolfe2(Objective& ob, CgIter& it, const Vec& xk, const Vec& pk, const Vec& gfk,
                   double old_fval, double old_old_fval, double c1, double c2) {
  const double amax = 1e100;
  const int maxiter = 10;
  Line ln{ob, xk, pk, Vec{}, std::nullopt};
  bool gval_set = false;  // gval[0] is None until the first derphi
  double derphi0 = np_dot(gfk, pk);
  double phi0 = old_fval, old_phi0 = old_old_fval;

  auto extra = [&](double alpha) -> Task<bool> {
    if (!ln.gval_alpha || *ln.gval_alpha != alpha) {
      co_await ln.derphi(alpha);
      gval_set = true;
    }
    co_return it.descent(alpha, ln.gval);
  };

  double alpha0 = 0;
  double alpha1;
  if (derphi0 != 0)
    alpha1 = py_min(1.0, 1.01 * 2 * (phi0 - old_phi0) / derphi0);
  else
    alpha1 = 1.0;
  if (alpha1 < 0) alpha1 = 1.0;
  alpha1 = py_min(alpha1, amax);
  double phi_a1 = co_await ln.phi(alpha1);
  double phi_a0 = phi0;
  double derphi_a0 = derphi0;

  std::optional<double> alpha_star;
  double phi_star = 0;
  bool have_derphi_star = false;
  bool loop_exhausted = true;
  for (int i = 0; i < maxiter; ++i) {
    if (alpha1 == 0 || alpha0 > amax) {
      alpha_star.reset();
      loop_exhausted = false;
      break;
    }
    bool not_first = i > 0;
    if (phi_a1 > phi0 + c1 * alpha1 * derphi0 || (phi_a1 >= phi_a0 && not_first)) {
      ZoomOut z = co_await zoom(ln, it, alpha0, alpha1, phi_a0, phi_a1, derphi_a0, phi0, derphi0,
                                c1, c2);
      if (z.ok) {
        alpha_star = z.a;
        phi_star = z.val;
        have_derphi_star = true;
      }
      loop_exhausted = false;
      break;
    }
    double derphi_a1 = co_await ln.derphi(alpha1);
    gval_set = true;
    if (std::fabs(derphi_a1) <= -c2 * derphi0) {
      if (co_await extra(alpha1)) {
        alpha_star = alpha1;
        phi_star = phi_a1;
        have_derphi_star = true;
        loop_exhausted = false;
        break;
      }
    }
    if (derphi_a1 >= 0) {
      ZoomOut z = co_await zoom(ln, it, alpha1, alpha0, phi_a1, phi_a0, derphi_a1, phi0, derphi0,
                                c1, c2);
      if (z.ok) {
        alpha_star = z.a;
        phi_star = z.val;
        have_derphi_star = true;
      }
      loop_exhausted = false;
      break;
    }
    double alpha2 = 2 * alpha1;
    alpha2 = py_min(alpha2, amax);
    alpha0 = alpha1;
    alpha1 = alpha2;
    phi_a0 = phi_a1;
    phi_a1 = co_await ln.phi(alpha1);
    derphi_a0 = derphi_a1;
  }
  if (loop_exhausted) {
    alpha_star = alpha1;
    phi_star = phi_a1;
    have_derphi_star = false;
  }
  LsOut out;
  if (alpha_star) {
    out.ok = true;
    out.alpha = *alpha_star;
    out.fval = phi_star;
    out.old_fval = phi0;
    if (have_derphi_star && gval_set) out.gfkp1 = ln.gval;
  }
  co_return out;
}

// _optimize.py _line_search_wolfe12
Task<LsOut> wolfe12(Objective& ob, CgIter& it, const Vec& xk, const Vec& pk, const Vec& gfk,
                    double old_fval, double old_old_fval, double c1, double c2) {
  LsOut r = co_await wolfe1(ob, xk, pk, gfk, old_fval, old_old_fval, c1, c2);
  if (r.ok) {
    if (!it.descent(r.alpha, *r.gfkp1)) r.ok = false;
  }
  if (!r.ok) r = co_await wolfe2(ob, it, xk, pk, gfk, old_fval, old_old_fval, c1, c2);
  co_return r;
}

}  // namespace

double np_dot(const Vec& a, const Vec& b) {
  double s = 0.0;
  for (int i = 0; i < NH; ++i) s = std::fma(a[i], b[i], s);
  return s;
}

// ------------------------------------------------------------ Objective
Task<int> Objective::memo(const Vec& x) {
  if (!memo_has_ || !array_equal(x, memo_x_)) {
    memo_x_ = x;
    co_await EvalRequest{slot_, x};
    memo_f_ = slot_->f;
    memo_g_ = slot_->g;
    memo_has_ = true;
    ++nobj_;
  }
  co_return 0;
}

Task<int> Objective::init(const Vec& x0) {
  sf_x_ = x0;
  f_upd_ = g_upd_ = false;
  ++nfev_;
  co_await memo(sf_x_);
  sf_f_ = memo_f_;
  f_upd_ = true;
  ++ngev_;
  co_await memo(sf_x_);
  sf_g_ = memo_g_;
  g_upd_ = true;
  co_return 0;
}

Task<double> Objective::fun(const Vec& x) {
  if (!array_equal(x, sf_x_)) {
    sf_x_ = x;
    f_upd_ = g_upd_ = false;
  }
  if (!f_upd_) {
    ++nfev_;
    co_await memo(sf_x_);
    sf_f_ = memo_f_;
    f_upd_ = true;
  }
  co_return sf_f_;
}

Task<Vec> Objective::grad(const Vec& x) {
  if (!array_equal(x, sf_x_)) {
    sf_x_ = x;
    f_upd_ = g_upd_ = false;
  }
  if (!g_upd_) {
    ++ngev_;
    co_await memo(sf_x_);
    sf_g_ = memo_g_;
    g_upd_ = true;
  }
  co_return sf_g_;
}

// ------------------------------------------------------------ _minimize_cg
Task<CgResult> cg_minimize(EvalSlot* slot, Vec x0, CgOptions opt) {
  Objective ob(slot);
  const int maxiter = opt.maxiter < 0 ? NH * 200 : opt.maxiter;
  co_await ob.init(x0);
  double old_fval = co_await ob.fun(x0);
  Vec gfk = co_await ob.grad(x0);
  int k = 0;
  Vec xk = x0;
  double old_old_fval = old_fval + std::sqrt(np_dot(gfk, gfk)) / 2;
  int warnflag = 0;
  Vec pk;
  for (int i = 0; i < NH; ++i) pk[i] = -gfk[i];
  double gnorm = vecnorm_inf(gfk);

  while (gnorm > opt.gtol && k < maxiter) {
    CgIter it{xk, pk, gfk, np_dot(gfk, gfk), opt.gtol, std::nullopt};
    LsOut ls = co_await wolfe12(ob, it, xk, pk, gfk, old_fval, old_old_fval, opt.c1, opt.c2);
    if (!ls.ok) {
      warnflag = 2;
      break;
    }
    old_fval = ls.fval;
    old_old_fval = ls.old_fval;
    PrpStep st;
    if (it.cached && ls.alpha == it.cached->alpha) {
      st = *it.cached;
    } else {
      Vec g1;
      if (ls.gfkp1)
        g1 = *ls.gfkp1;
      else
        g1 = co_await ob.grad(axpy(xk, ls.alpha, pk));
      st = it.step(ls.alpha, g1);
    }
    xk = st.xkp1;
    pk = st.pkp1;
    gfk = st.gfkp1;
    gnorm = st.gnorm;
    k += 1;
  }

  CgResult res;
  res.fun = old_fval;
  if (warnflag == 2) {
    res.status = 2;
  } else if (k >= maxiter) {
    res.status = 1;
  } else {
    bool nan = std::isnan(gnorm) || std::isnan(old_fval);
    for (int i = 0; i < NH; ++i) nan = nan || std::isnan(xk[i]);
    res.status = nan ? 3 : 0;
  }
  res.x = xk;
  res.jac = gfk;
  res.nit = k;
  res.nfev = ob.nfev();
  res.njev = ob.ngev();
  res.nobj = ob.nobj();
  co_return res;
}

}  // namespace oi
