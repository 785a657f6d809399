// Polak-Ribiere+ nonlinear conjugate gradient with Wolfe line searches:
// a restatement of the optimiser the reference calls at GPR_CS2S3.py:166
//   scipy.optimize.minimize(SMLII, x0, method='CG', jac=True)
// i.e. (scipy 1.15.3, the third-party dependency; the reference pins none)
//   _optimize.py:1695-1846  _minimize_cg
//   _optimize.py:1139-1181  _line_search_wolfe12
//   _optimize.py:61-85      MemoizeJac
//   _differentiable_functions.py  ScalarFunction fun/grad memoisation
//   _linesearch.py:37-183   line_search_wolfe1 / scalar_search_wolfe1
//   _dcsrch.py              DCSRCH / dcstep (More'-Thuente, MINPACK-2)
//   _linesearch.py:186-620  line_search_wolfe2 / _zoom / _cubicmin / _quadmin
//
// Decision logic and floating-point operation order follow scipy's so that,
// fed the same objective values, the iterates, the number of objective
// evaluations and the stop status are bit-identical (tests/test_cg_restatement.py).
// Host-only code: compile with -ffp-contract=off.
#pragma once
#include <array>
#include <coroutine>
#include <cstdint>

#include "task.hpp"

namespace oi {

constexpr int NH = 6;  // hyper-parameter vector length (GPR_CS2S3.py:217)
using Vec = std::array<double, NH>;

// One cell's request/response mailbox between its optimiser coroutine and the
// batch driver.
struct EvalSlot {
  Vec x{};                       // requested point (log hypers)
  double f = 0.0;                // objective nlZ at x
  Vec g{};                       // gradient at x
  bool pending = false;          // a request is waiting for values
  std::coroutine_handle<> waiter{};
};

// co_await EvalRequest{slot, x}: publish x, suspend until the driver filled f, g.
struct EvalRequest {
  EvalSlot* slot;
  Vec x;
  bool await_ready() const noexcept { return false; }
  void await_suspend(std::coroutine_handle<> h) noexcept {
    slot->x = x;
    slot->pending = true;
    slot->waiter = h;
  }
  void await_resume() const noexcept {}
};

struct Evaluated {
  double f;
  Vec g;
};

// MemoizeJac + ScalarFunction: the two one-deep caches between scipy's CG and
// the objective.  Only a MemoizeJac miss costs an objective evaluation.
class Objective {
 public:
  explicit Objective(EvalSlot* slot) : slot_(slot) {}
  // ScalarFunction.__init__: evaluates f and g at x0
  Task<int> init(const Vec& x0);
  Task<double> fun(const Vec& x);   // ScalarFunction.fun
  Task<Vec> grad(const Vec& x);     // ScalarFunction.grad
  int64_t nfev() const { return nfev_; }
  int64_t ngev() const { return ngev_; }
  int64_t nobj() const { return nobj_; }  // objective (SMLII) evaluations

 private:
  Task<int> memo(const Vec& x);     // MemoizeJac._compute_if_needed
  EvalSlot* slot_;
  bool memo_has_ = false;
  Vec memo_x_{};
  double memo_f_ = 0.0;
  Vec memo_g_{};
  Vec sf_x_{};
  bool f_upd_ = false, g_upd_ = false;
  double sf_f_ = 0.0;
  Vec sf_g_{};
  int64_t nfev_ = 0, ngev_ = 0, nobj_ = 0;
};

struct CgOptions {
  double gtol = 1e-5;       // _minimize_cg default
  int maxiter = -1;         // default len(x0)*200
  double c1 = 1e-4;
  double c2 = 0.4;
};

struct CgResult {
  Vec x{};
  double fun = 0.0;
  Vec jac{};
  int nit = 0;
  int status = 0;           // 0 success, 1 maxiter, 2 precision loss, 3 nan
  int64_t nfev = 0, njev = 0, nobj = 0;
};

// The whole minimisation as a coroutine; evaluations go through `slot`.
Task<CgResult> cg_minimize(EvalSlot* slot, Vec x0, CgOptions opt);

// numpy-faithful reductions used by the restatement (exposed for tests)
double np_dot(const Vec& a, const Vec& b);

}  // namespace oi
