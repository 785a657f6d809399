// Minimal C++20 coroutine task used to write the per-cell optimiser as
// straight-line code that suspends whenever it needs an objective value.
//
// A cell's optimiser is a tree of nested Task<T> coroutines (CG -> line
// search -> DCSRCH -> objective).  The innermost one suspends on an
// EvalRequest; the batch driver then evaluates every pending cell on the GPU
// in one launch sequence and resumes each cell's innermost handle.  Nested
// completion uses symmetric transfer, so resuming never grows the C stack.
#pragma once
#include <coroutine>
#include <exception>
#include <utility>

namespace oi {

template <class T>
class Task {
 public:
  struct promise_type {
    T value{};
    std::coroutine_handle<> continuation{};
    Task get_return_object() { return Task{Handle::from_promise(*this)}; }
    std::suspend_always initial_suspend() noexcept { return {}; }
    struct Final {
      bool await_ready() noexcept { return false; }
      std::coroutine_handle<> await_suspend(std::coroutine_handle<promise_type> h) noexcept {
        auto c = h.promise().continuation;
        return c ? c : std::noop_coroutine();
      }
      void await_resume() noexcept {}
    };
    Final final_suspend() noexcept { return {}; }
    void return_value(T v) { value = std::move(v); }
    void unhandled_exception() { std::terminate(); }
  };
  using Handle = std::coroutine_handle<promise_type>;

  Task() = default;
  explicit Task(Handle h) : h_(h) {}
  Task(Task&& o) noexcept : h_(std::exchange(o.h_, {})) {}
  Task& operator=(Task&& o) noexcept {
    if (this != &o) {
      if (h_) h_.destroy();
      h_ = std::exchange(o.h_, {});
    }
    return *this;
  }
  Task(const Task&) = delete;
  ~Task() {
    if (h_) h_.destroy();
  }

  // awaiting a Task starts it and resumes the awaiter when it completes
  bool await_ready() const noexcept { return false; }
  std::coroutine_handle<> await_suspend(std::coroutine_handle<> awaiter) noexcept {
    h_.promise().continuation = awaiter;
    return h_;
  }
  T await_resume() { return std::move(h_.promise().value); }

  // top-level control (used by the driver on the outermost task)
  void start() { h_.resume(); }
  bool done() const { return !h_ || h_.done(); }
  T& result() { return h_.promise().value; }

 private:
  Handle h_{};
};

}  // namespace oi
