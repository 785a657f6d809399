// liboi host engine: the C ABI of include/oi.h.
//
// Continuous batching of independent grid cells on one GPU:
//   * every cell owns a region of a device arena (packed tiles, vectors,
//     partial sums) for as long as it is resident;
//   * a fitting cell runs scipy's CG (cg.hpp) as a coroutine that suspends
//     whenever it needs SMLII at a new point;
//   * one "round" = one launch sequence that evaluates SMLII for every
//     suspended cell and the GPR3D predict block for every cell whose fit
//     has finished; then results come back, coroutines resume, finished
//     cells leave and queued cells (largest n first) take their place.
// Per-cell arithmetic never depends on which other cells share a round.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/oi.h"
#include "cg.hpp"
#include "oi_device.h"
#include "oi_masks.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define HIPC(expr)                                                                            \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess)                                                                     \
      throw HipError(std::string(#expr) + ": " + hipGetErrorString(e_));                      \
  } while (0)

struct HipError {
  std::string msg;
  explicit HipError(std::string m) : msg(std::move(m)) {}
};

inline int tiles_of(int64_t n) { return (int)((n + OI_NB - 1) / OI_NB); }

// ------------------------------------------------------------- arena
// First-fit free list over one device allocation (256-byte granules).
class Arena {
 public:
  void init(size_t bytes) {
    HIPC(hipMalloc(&base_, bytes));
    size_ = bytes;
    free_.clear();
    free_[0] = bytes;
  }
  ~Arena() {
    if (base_) (void)hipFree(base_);
  }
  size_t size() const { return size_; }
  // returns offset or SIZE_MAX
  size_t alloc(size_t bytes) {
    bytes = (bytes + 255) & ~size_t(255);
    for (auto it = free_.begin(); it != free_.end(); ++it) {
      if (it->second >= bytes) {
        size_t off = it->first, len = it->second;
        free_.erase(it);
        if (len > bytes) free_[off + bytes] = len - bytes;
        return off;
      }
    }
    return SIZE_MAX;
  }
  void release(size_t off, size_t bytes) {
    bytes = (bytes + 255) & ~size_t(255);
    // a block the arena never handed out (SIZE_MAX = a failed alloc) must not
    // enter the free list: it would alias live allocations after wrap-around
    if (off >= size_ || bytes > size_ - off) return;
    auto it = free_.emplace(off, bytes).first;
    auto nx = std::next(it);
    if (nx != free_.end() && it->first + it->second == nx->first) {
      it->second += nx->second;
      free_.erase(nx);
    }
    if (it != free_.begin()) {
      auto pv = std::prev(it);
      if (pv->first + pv->second == it->first) {
        pv->second += it->second;
        free_.erase(it);
      }
    }
  }
  char* ptr(size_t off) const { return static_cast<char*>(base_) + off; }

 private:
  void* base_ = nullptr;
  size_t size_ = 0;
  std::map<size_t, size_t> free_;
};

size_t cell_bytes(int64_t n, bool eval) {
  const size_t T = (size_t)tiles_of(n), nt = T * (T + 1) / 2;
  size_t b = 0;
  auto add = [&](size_t x) { b += (x + 255) & ~size_t(255); };
  add(nt * OI_TILE * 8);                         // L
  if (eval) add(nt * OI_TILE * 8);               // W
  add(T * OI_TILE * 8);                          // Dinv
  add(4 * T * OI_NB * 8);                        // vec
  add((size_t)OI_PART_SIZE(nt, T) * 8);          // part
  return b;
}

// ------------------------------------------------------------- profiling
enum KernelId { K_BUILD, K_CHOL, K_TRSM, K_EVEN, K_LAUUM, K_FINAL, K_EVEN4, K_COUNT };
const char* kKernelName[K_COUNT] = {"k_build", "k_diag_factor", "k_chol_panel", "k_panel_even",
                                    "k_lauum_grad", "k_finalize", "k_panel4"};

// Panel scheme, read per call from OI_PANEL:
//   2 (default): even/odd block-column pairs share one stream (k_panel_even +
//                k_chol_panel(kbeg = j-1)): half the L / W traffic of the
//                one-column scheme and k_scale only every other column;
//                +2.5 % on the day workload;
//   1          : one-column left-looking panels, every column streams its
//                whole block row of L (and of W = L^-1).
bool legacy_panels() {
  const char* e = getenv("OI_PANEL");
  return e && atoi(e) == 1;
}
// Even-column panel core, read per call from OI_PANEL4: 1 (default) => k_panel4
// (two block rows per workgroup on the 128 x 128 gemm4 core; day 137.2 vs
// 135.5 cells/s back to back on one box, profiles/r03/), 0 => k_panel_even
// (64 x 128 gemm2 core).  Post-form only.
bool panel4_enabled() {
  const char* e = getenv("OI_PANEL4");
  return !(e && atoi(e) == 0);
}
// k_panel4 from even column OI_PANEL4_MINJ on (k_panel_even below it: with few
// streamed pairs per workgroup the paired-row epilogue costs more than the
// shared operand stream saves)
int panel4_minj() {
  const char* e = getenv("OI_PANEL4_MINJ");
  return e ? atoi(e) : 0;
}
// ... and only in rounds whose largest cell has at least OI_PANEL4_MINT (12)
// block columns: on small cells (config 2, n = 500, T = 8: 271 k vs 284 k
// cells/s; config 1) k_panel_even's one-tile workgroups finish sooner, on the
// day (T up to 35) k_panel4 wins (138.1 vs 136.3 cells/s with it from j = 8 on)
int panel4_mint() {
  const char* e = getenv("OI_PANEL4_MINT");
  return e ? atoi(e) : 12;
}
// ... and only when the launch has at least OI_PANEL4_MINWG (512: two
// k_panel4 workgroups per CU) workgroups -- the day's tail rounds of a few
// slow-converging cells run the one-row kernel, twice as many workgroups
int panel4_minwg() {
  const char* e = getenv("OI_PANEL4_MINWG");
  return e ? atoi(e) : 512;
}
// rounds of at least OI_FUSE_DIAG_MIN cells factor diagonal tile j+1 inside
// column j's panel launch (k_diag_factor4w then runs for column 0 only)
int fuse_diag_min() {
  const char* e = getenv("OI_FUSE_DIAG_MIN");
  return e ? atoi(e) : 1;
}
// Executed MFMA flops per cell and launch (profile mode), mirroring the
// kernels' wave masks (oi_masks.h): a 16x16 accumulator block over one
// 16-deep k-chunk is 8192 flops.  gemm2 (k_panel_even: 8 waves, wr 0..1,
// wc 0..3) skips whole chunks only; gemm1 (k_chol_panel, k_lauum_grad1: 4
// waves) skips per block.  Every count is closed-form in the cell's tile
// geometry (O(T) per round at most).
namespace acct {
constexpr double BLK = 2.0 * 16 * 16 * 16;
inline int live(unsigned m) { return __builtin_popcount(~m & 0xFu); }

// post_right / post_left (post-form): the triangular product S Dinv^T /
// Dinv S of one tile, 160 MFMAs of 16x16x4 over the workgroup's waves (no
// masks), in BLK units
constexpr double POST_BLOCKS = 160.0 / 4.0;

double panel_even(int T, int n, int j, bool eval, bool post) {
  const int rT = n - OI_NB * (T - 1), nf = T - 1 - j;
  auto factor_wg = [&](int x) {
    const int i = j + 1 + x, mlim = i == T - 1 ? rT : OI_NB;
    double b = 0;
    for (int w = 0; w < 8; ++w) {
      const int wr = (w >> 2) & 1, wc = w & 3;
      const int nlim = (wc >= 2 && j + 1 == T - 1) ? rT : OI_NB;
      const unsigned s = pad_skip(32 * wr, 32 * (wc & 1), mlim, nlim) |
                         (x == 0 && wc >= 2 ? upper_blocks(32 * wr, 32 * (wc - 2)) : 0u);
      if (s == 0xFu) continue;
      b += 16.0 * j;  // pairs p < j: 4 chunks x 4 blocks each
      if (!post)
        for (int c = 0; c < 4; ++c)
          if ((s | (wc >= 2 ? 0xFu : cols_above(c, 32 * wc))) != 0xFu) b += 4;
    }
    if (x == 0) b += 64;  // the fresh L_j+1,j L_j+1,j^T product of the look-ahead
    if (post) b += POST_BLOCKS;  // (A_ij - acc) Dinv_jj^T
    return b;
  };
  double blocks = 0;
  if (nf > 0) blocks += factor_wg(0);
  if (nf > 1) blocks += factor_wg(nf - 1);
  if (nf > 2) blocks += (nf - 2) * factor_wg(1);
  if (eval && j > 0) {
    const bool has_next = j + 1 < T;
    if (post) blocks += j * POST_BLOCKS;  // -acc Dinv_jj^T, one per W tile
    for (int w = 0; w < 8; ++w) {
      const int wr = (w >> 2) & 1, wc = w & 3;
      const int nlim = ((wc < 2 && j == T - 1) || (wc >= 2 && j + 1 == T - 1)) ? rT : OI_NB;
      const unsigned s = pad_skip(0, 32 * (wc & 1), OI_NB, nlim) | (!has_next && wc >= 2 ? 0xFu : 0u);
      if (s == 0xFu) continue;
      double first = 0;  // the pair k = jj (W_jj,jj): its 4 chunks
      for (int c = 0; c < 4; ++c)
        if ((s | rows_below(c, 32 * wr)) != 0xFu) first += 4;
      blocks += 16.0 * (j * (j - 1) / 2.0) + j * first;
    }
  }
  return blocks * BLK;
}

// k_panel4 (gemm4: 8 waves of 2 x 4 blocks; per-MFMA masks when `masked`)
inline int live8(unsigned m) { return __builtin_popcount(~m & 0xFFu); }
double panel4(int T, int n, int j, bool eval) {
  const int rT = n - OI_NB * (T - 1), nfp = (T - j) >> 1;
  double blocks = 0;
  for (int x = 0; x < nfp; ++x) {
    const int i1 = j + 1 + 2 * x, i2 = i1 + 1;
    const bool masked = x == 0 || i2 >= T - 1 || j + 1 == T - 1;
    for (int w = 0; w < 8; ++w) {
      const int wr = w >> 1, wc = w & 1, ti = wr >= 2 ? i2 : i1, tj = wc ? j + 1 : j;
      unsigned skip = 0;
      for (int mb = 0; mb < 2; ++mb)
        for (int nb = 0; nb < 4; ++nb) {
          const int m0 = 32 * (wr & 1) + 16 * mb, n0 = 16 * nb;
          if (ti >= T || (ti == T - 1 && m0 >= rT) || (tj == T - 1 && n0 >= rT) ||
              (x == 0 && wr < 2 && wc == 1 && m0 + 15 < n0))
            skip |= 1u << (4 * mb + nb);
        }
      blocks += 4.0 * j * (masked ? live8(skip) : 8);
    }
    blocks += POST_BLOCKS * (i2 < T ? 2 : 1);
    if (x == 0) blocks += 40;  // the look-ahead's 10 lower blocks x 16 MFMAs
  }
  if (eval)
    for (int y = 0; 2 * y < j; ++y) {
      const bool masked = j >= T - 2;
      for (int w = 0; w < 8; ++w) {
        const int wc = w & 1, tj = wc ? j + 1 : j;
        unsigned skip = 0;
        for (int nb = 0; nb < 4; ++nb)
          if ((wc == 1 && j + 1 >= T) || (tj == T - 1 && 16 * nb >= rT)) skip |= 0x11u << nb;
        blocks += 4.0 * (j - 2 * y) * (masked ? live8(skip) : 8);
      }
      blocks += 2 * POST_BLOCKS;
    }
  return blocks * BLK;
}

double chol_panel(int T, int n, int j, int kbeg, bool eval, bool post) {
  const int rT = n - OI_NB * (T - 1), nf = T - 1 - j;
  auto factor_wg = [&](int x) {
    const int i = j + 1 + x;
    double b = 0;
    for (int w = 0; w < 4; ++w) {
      const int wr = w >> 1, wc = w & 1;
      const unsigned s = i == T - 1 ? pad_skip(32 * wr, 32 * wc, OI_NB, rT) : 0u;
      b += 4.0 * (j - kbeg) * live(s);
      if (!post)
        for (int c = 0; c < 4; ++c) b += live(s | rows_above(c, 32 * wr));  // the Dinv_jj pair
      if (x == 0) b += 4.0 * j * live(lower_blocks(32 * wr, 32 * wc));  // look-ahead syrk
    }
    if (x == 0) b += 64;  // its fresh L_ij L_ij^T product
    if (post) b += POST_BLOCKS;  // Dinv_jj (A_ij^T - acc)
    return b;
  };
  double blocks = 0;
  if (nf > 0) blocks += factor_wg(0);
  if (nf > 1) blocks += factor_wg(nf - 1);
  if (nf > 2) blocks += (nf - 2) * factor_wg(1);
  if (eval && j > 0) {
    for (int w = 0; w < 4; ++w) {
      const int wr = w >> 1, wc = w & 1;
      const unsigned s = j == T - 1 ? pad_skip(32 * wr, 32 * wc, rT, OI_NB) : 0u;
      // pair k = jj (B = W_jj,jj) when the tile starts there, pair k = j (A = Dinv_jj)
      double tri_first = 0, dinv_last = 0;
      for (int c = 0; c < 4; ++c) {
        tri_first += live(s | cols_below(c, 32 * wc));
        dinv_last += live(s | rows_above(c, 32 * wr));
      }
      if (post) dinv_last = POST_BLOCKS / 4;  // Dinv_jj (Vneg - acc), every W tile (per wave: 4 waves)
      for (int jj = 0; jj < j && jj < kbeg; ++jj)  // extra pair: k = kbeg .. j
        blocks += 4.0 * (j - kbeg) * live(s) + dinv_last;
      // kfirst = jj (jj >= kbeg): pairs k = jj .. j-1, the first against W_jj,jj
      const int lo = kbeg < j ? kbeg : j;
      for (int jj = lo; jj < j; ++jj)
        blocks += 4.0 * (j - jj - 1) * live(s) + tri_first + (post ? dinv_last : 0.0);
    }
  }
  return blocks * BLK;
}

double lauum(int T, int n) {
  const int rT = n - OI_NB * (T - 1);
  double blocks = 0;
  for (int i = 0; i < T; ++i) {
    const int nch = 4 * (T - i - 1) + (rT + 15) / 16;
    for (int diag = 0; diag < 2; ++diag) {  // tile (i, i), then one of the i tiles (i, j < i)
      if (!diag && i == 0) continue;
      const int jt = diag ? i : 0;
      double b = 0;
      for (int w = 0; w < 4; ++w) {
        const int wr = w >> 1, wc = w & 1;
        unsigned s = 0;
        for (int mb = 0; mb < 2; ++mb)
          for (int nb = 0; nb < 2; ++nb) {
            const int m0 = 32 * wr + 16 * mb, n0 = 32 * wc + 16 * nb;
            if ((diag && m0 + 15 < n0) || (i == T - 1 && m0 >= rT) || (jt == T - 1 && n0 >= rT))
              s |= 1u << (2 * mb + nb);
          }
        for (int c = 0; c < nch && c < 4; ++c)
          b += live(s | rows_below(c, 32 * wr) | (diag ? cols_below(c, 32 * wc) : 0u));
        if (nch > 4) b += (nch - 4.0) * live(s);
      }
      blocks += diag ? b : i * b;
    }
  }
  return blocks * BLK;
}
}  // namespace acct

struct KStat {
  int64_t launches = 0;
  double ms = 0.0;
  double flops = 0.0;  // executed tile-GEMM flops (2*64^3 per tile product)
};
std::mutex g_prof_mu;
KStat g_prof[K_COUNT];
struct RunStat {
  int64_t rounds = 0, evals = 0, predicts = 0;
  double wall_s = 0.0;
  double setup_s = 0.0;  // run() entry -> first round (uploads, residuals)
  double sync_s = 0.0;   // host blocked on round completion
  double consume_s = 0.0;  // consume(): sync + results + coroutine steps
  double prep_s = 0.0;     // launch_round() before its first kernel (lists, sort, copy)
  double launch_s = 0.0;   // launch_round() in total (incl. every launch call)
} g_run;
struct LaunchRec {
  int kind, j, cells;
  double ms;
};
std::vector<LaunchRec> g_last_round;  // per-launch times of the latest profiled round
// per (kernel, block column j) totals over every profiled round: launches,
// resident cells, HIP-event ms, executed MFMA flops (the launch-shape analysis
// of DESIGN §6: how much time goes to launches with few cells left at large j)
struct ByJ {
  int64_t launches = 0, cells = 0;
  double ms = 0.0, flops = 0.0;
};
std::map<std::pair<int, int>, ByJ> g_byj;
struct RoundRec {
  int n_eval, n_pred, maxT;
  double work;  // sum over evaluated cells of T^3
  double ms;    // GPU time of the round's launches
};
std::vector<RoundRec> g_rounds;  // every profiled round since the last reset
// stages timed by the other translation units (oi_nystrom.hip), by name
struct ExtStat {
  int64_t launches = 0;
  double ms = 0.0, flops = 0.0, bytes = 0.0;
};
std::vector<std::pair<std::string, ExtStat>> g_ext;

// ------------------------------------------------------------- context
struct Context {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t sub_stream = nullptr;  // submissions (residuals, sites): never behind a round in flight
  std::vector<hipStream_t> aux;  // extra streams for concurrent cell groups
  hipStream_t aux_stream(int g) {
    while ((int)aux.size() < g) {
      hipStream_t s;
      HIPC(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      aux.push_back(s);
    }
    return aux[g - 1];
  }
  Arena arena;
  size_t arena_bytes = 0;
  int live_sessions = 0;  // the arena is never re-sized under a live session
  std::mutex mu;
};

std::mutex g_ctx_mu;
std::map<int, std::unique_ptr<Context>> g_ctx;

Context& context(int device, int64_t pool_bytes) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  auto& p = g_ctx[device];
  if (!p) {
    p = std::make_unique<Context>();
    p->device = device;
    HIPC(hipSetDevice(device));
    HIPC(hipStreamCreateWithFlags(&p->own_stream, hipStreamNonBlocking));
    HIPC(hipStreamCreateWithFlags(&p->sub_stream, hipStreamNonBlocking));
  }
  HIPC(hipSetDevice(device));
  size_t want = (size_t)pool_bytes;
  if (want == 0) {
    if (p->arena_bytes == SIZE_MAX - 1) return *p;  // keep the automatic arena between calls
    size_t fr = 0, tot = 0;
    HIPC(hipMemGetInfo(&fr, &tot));
    // OI_ARENA_FRAC: the share of free HBM the automatic arena takes (0.6);
    // bench.py lowers it when several rank processes share one GPU
    static const double frac = [] {
      const char* e = getenv("OI_ARENA_FRAC");
      const double f = e ? atof(e) : 0.6;
      return f > 0.0 && f <= 0.95 ? f : 0.6;
    }();
    want = (size_t)(fr * frac);
  }
  if (want != p->arena_bytes && p->live_sessions == 0) {
    p->arena.~Arena();
    new (&p->arena) Arena();
    p->arena_bytes = 0;
    // several processes sharing a device size their arenas from the same
    // hipMemGetInfo snapshot: on failure, halve the automatic size and retry
    const bool automatic = pool_bytes == 0;
    while (true) {
      try {
        p->arena.init(want);
        break;
      } catch (const HipError&) {
        (void)hipGetLastError();
        if (!automatic || want < (size_t(1) << 30)) throw;
        want /= 2;
      }
    }
    p->arena_bytes = automatic ? SIZE_MAX - 1 : want;  // automatic: keep between calls
  }
  return *p;
}

// device buffer RAII
struct DBuf {
  void* p = nullptr;
  size_t n = 0;
  void reserve(size_t bytes) {
    if (bytes <= n) return;
    if (p) HIPC(hipFree(p));
    p = nullptr;
    HIPC(hipMalloc(&p, bytes));
    n = bytes;
  }
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
};
struct HBuf {  // pinned host
  void* p = nullptr;
  size_t n = 0;
  void reserve(size_t bytes, unsigned flags = hipHostMallocDefault) {
    if (bytes <= n) return;
    if (p) HIPC(hipHostFree(p));
    p = nullptr;
    HIPC(hipHostMalloc(&p, bytes, flags));
    n = bytes;
  }
  ~HBuf() {
    if (p) (void)hipHostFree(p);
  }
};

// ------------------------------------------------------------- the batch
// One submitted ragged batch of cells ("ticket").  Host metadata is copied at
// submission; host inputs are copied to the device at submission; outputs go
// to the caller's arrays as each cell finishes.
struct Job {
  // inputs (device after submission)
  const double* xyt = nullptr;  // device rows of the batch (caller's or own copy)
  const double* r = nullptr;    // device residuals y - mX
  std::vector<int64_t> offs;    // ncell + 1
  int64_t ncell = 0;
  std::vector<double> xs;       // ncell x 3 (predict)
  double mean = 0.0;
  // per-cell work description
  enum Kind { FIT_PREDICT, PREDICT_ONLY, EVAL_ONLY } kind = FIT_PREDICT;
  std::vector<double> x0;       // FIT_PREDICT: 6
  std::vector<double> hyp;      // PREDICT_ONLY: ncell x 5
  std::vector<double> h;        // EVAL_ONLY: ncell x 6
  oi::CgOptions cg;
  // outputs (caller-owned)
  double* out = nullptr;        // FIT/PRED: ncell x 8
  int32_t* status = nullptr;
  int32_t* info = nullptr;
  double* nlz = nullptr;        // EVAL_ONLY
  double* grad = nullptr;
  // distinct sites per cell (k_dedup; oi_device.h "Duplicate sites")
  const double* sites = nullptr;  // device, 3 per site at the cell's observation offset
  const double* v = nullptr;      // device, site residuals
  const double* dw = nullptr;     // device, site weights
  std::vector<int32_t> m;         // sites per cell
  std::vector<double> ssw;        // within-site residual sum of squares per cell
  // bookkeeping
  int64_t id = 0;
  int64_t remaining = 0;
  size_t in_off = SIZE_MAX, in_bytes = 0;  // arena block holding the inputs' device copies
  DBuf own;                                // fallback when the arena is full
  std::vector<double> r_host;              // staging for host inputs
};

bool dedup_enabled() {
  const char* e = getenv("OI_DEDUP");
  return !(e && atoi(e) == 0);
}

struct Slot {
  Job* job = nullptr;
  int64_t cell = -1;
  size_t off = 0, bytes = 0;
  int phase = 0;  // 0 fit (eval), 1 predict, 2 eval-only
  oi::EvalSlot mail;
  oi::Task<oi::CgResult> task;
  double hyp[5] = {0, 0, 0, 0, 0};
  oi::CgResult res;
};

// Continuous-batching engine over one device context.  Cells of every
// submitted batch wait in one FIFO queue (largest n first inside a batch) and
// are admitted while the arena has room; rounds evaluate every resident cell.
// wait(id) drives rounds until batch `id` is complete and returns with the
// next round already in flight, so the GPU keeps working while the caller
// submits more batches (oi_session_*); a one-shot oi_gpr_batch is
// submit + drain on a private engine.
class Engine {
 public:
  Engine(Context& ctx, const oi_options& o, int64_t cap_hint)
      : ctx_(ctx), o_(o), legacy_(legacy_panels()), panel4_(panel4_enabled()),
        panel4_minj_(panel4_minj()), panel4_mint_(panel4_mint()), panel4_minwg_(panel4_minwg()),
        fuse_diag_min_(fuse_diag_min()) {
    HIPC(hipSetDevice(ctx.device));
    st_ = o.stream ? (hipStream_t)o.stream : ctx.own_stream;
    ss_ = ctx.sub_stream;
    static const bool debug_set = [] {
      const char* e = getenv("OI_DEBUG");
      if (e && atoi(e) == 1) oi_set_debug(1);
      return true;
    }();
    (void)debug_set;
    const char* ep = getenv("OI_POISON");
    poison_ = ep && atoi(ep) == 1;
    cap_ = (int)std::max<int64_t>(1, std::min<int64_t>(cap_hint, o.max_pool > 0 ? o.max_pool : 2048));
    slots_ = std::vector<Slot>(cap_);
    // Resident cells are split into G groups with their own stream: while one
    // group's round runs, the host consumes the other group's results and its
    // kernels fill the GPU around the first group's latency-bound launches.
    G_ = 1;  // OI_GROUPS=2..8: measured no gain on the day workload (round 1)
    if (const char* eg = getenv("OI_GROUPS")) G_ = std::max(1, std::min(8, atoi(eg)));
    if (cap_ < 2 * G_) G_ = 1;
    capG_ = (cap_ + G_ - 1) / G_;
    // one block per group, mirrored on the host, so a round uploads its cell
    // records, lists and cleared status words in ONE copy (and the status comes
    // back inside the result rows, OI_OUT_STATUS): two copies per round, not five
    blk_ = ((size_t)capG_ * (sizeof(OiCell) + 4 * 3 + 4) + 255) & ~size_t(255);
    d_blk_.reserve(G_ * blk_);
    h_blk_.reserve(G_ * blk_);
    // result rows and the per-group completion flags: fine-grained pinned host
    // memory the kernels write directly (k_finalize), no D2H copy per round
    h_res_.reserve(cap_ * OI_OUT_N * 8, hipHostMallocCoherent | hipHostMallocMapped);
    hres_ = (double*)h_res_.p;
    HIPC(hipHostGetDevicePointer((void**)&dres_, hres_, 0));
    h_flag_.reserve(G_ * 64, hipHostMallocCoherent | hipHostMallocMapped);
    std::memset(h_flag_.p, 0, G_ * 64);
    HIPC(hipHostGetDevicePointer((void**)&dflag_, h_flag_.p, 0));
    d_done_.reserve(G_ * 64);
    HIPC(hipMemset(d_done_.p, 0, G_ * 64));
    groups_.resize(G_);
    for (int g = 0; g < G_; ++g) {
      Group& gr = groups_[g];
      gr.s0 = g * capG_;
      gr.cap = std::max(0, std::min(capG_, cap_ - g * capG_));
      gr.st = g == 0 ? st_ : ctx.aux_stream(g);
      for (int s = gr.s0 + gr.cap - 1; s >= gr.s0; --s) gr.free_slots.push_back(s);
      char* hb = (char*)h_blk_.p + g * blk_;
      char* db = (char*)d_blk_.p + g * blk_;
      gr.hc = (OiCell*)hb;
      gr.dc = (OiCell*)db;
      gr.hl = (int32_t*)(hb + capG_ * sizeof(OiCell));
      gr.dl = (int32_t*)(db + capG_ * sizeof(OiCell));
      gr.hstat = gr.hl + 3 * capG_;
      gr.dstat = gr.dl + 3 * capG_;
      if (o.profile) {
        gr.ev.resize(2 * (3 * 1024 + 16));
        for (auto& ee : gr.ev) HIPC(hipEventCreate(&ee));
      }
    }
    HIPC(hipEventCreateWithFlags(&ready_, hipEventDisableTiming));
    t_start_ = std::chrono::steady_clock::now();
  }

  ~Engine() {
    // never leave a round running over memory the engine is about to free
    for (Group& gr : groups_)
      if (gr.inflight) (void)hipStreamSynchronize(gr.st);
    for (Group& gr : groups_)
      for (auto& ee : gr.ev) (void)hipEventDestroy(ee);
    if (ready_) (void)hipEventDestroy(ready_);
    for (auto& sl : slots_)
      if (sl.cell >= 0) ctx_.arena.release(sl.off, sl.bytes);
    for (auto& kv : jobs_)
      if (kv.second->in_off != SIZE_MAX) ctx_.arena.release(kv.second->in_off, kv.second->in_bytes);
    flush_stats();
  }

  // Takes ownership of `job` (metadata filled by the caller; `y`, `mX`, `xyt_in`
  // are the caller's input pointers, host or device per o.device_inputs).
  int64_t submit(std::unique_ptr<Job> job, const double* xyt_in, const double* y, const double* mX) {
    Job& jb = *job;
    jb.id = next_id_++;
    const int64_t N = jb.offs[jb.ncell], nc = jb.ncell;
    // device inputs: order after the caller's stream (or the legacy null
    // stream, torch's default) so producers of xyt / y / mX have finished
    if (o_.device_inputs && N > 0) {
      HIPC(hipEventRecord(ready_, o_.stream ? (hipStream_t)o_.stream : (hipStream_t)0));
      for (Group& gr : groups_) HIPC(hipStreamWaitEvent(gr.st, ready_, 0));
      HIPC(hipStreamWaitEvent(ss_, ready_, 0));
    }
    // The submission's own work (residuals, copies, k_dedup, the m / SSW
    // read-back) runs on the submit stream: the host waits for it alone, not
    // for the round in flight on the group streams (a session's submit used to
    // drain the GPU once per batch).  Arena blocks are released only after the
    // rounds that used them completed, so the new block never overlaps them.
    // one block: residuals | sites | v | d | offs | m | SSW (| host inputs' copy)
    auto rnd = [](size_t b) { return (b + 255) & ~size_t(255); };
    const size_t N1 = (size_t)std::max<int64_t>(N, 1), C1 = (size_t)std::max<int64_t>(nc, 1);
    const size_t sz[8] = {rnd(N1 * 8), rnd(N1 * 24), rnd(N1 * 8), rnd(N1 * 8), rnd((C1 + 1) * 8),
                          rnd(C1 * 4), rnd(C1 * 8), o_.device_inputs ? 0 : rnd(N1 * 24)};
    jb.in_bytes = 0;
    for (size_t b : sz) jb.in_bytes += b;
    jb.in_off = ctx_.arena.alloc(jb.in_bytes);
    char* base;
    if (jb.in_off != SIZE_MAX) {
      base = ctx_.arena.ptr(jb.in_off);
    } else {
      jb.own.reserve(jb.in_bytes);
      base = (char*)jb.own.p;
    }
    char* q = base;
    auto take = [&](size_t b) {
      char* p = q;
      q += b;
      return p;
    };
    double* d_r = (double*)take(sz[0]);
    double* d_sites = (double*)take(sz[1]);
    double* d_v = (double*)take(sz[2]);
    double* d_dw = (double*)take(sz[3]);
    int64_t* d_offs = (int64_t*)take(sz[4]);
    int32_t* d_m = (int32_t*)take(sz[5]);
    double* d_ssw = (double*)take(sz[6]);
    const double* d_x = xyt_in;
    if (o_.device_inputs) {
      if (N > 0 && oi_launch_residual(y, mX, jb.mean, d_r, N, ss_))
        throw HipError("residual kernel launch failed");
    } else {
      double* dx = (double*)take(sz[7]);
      d_x = dx;
      if (N > 0) {
        jb.r_host.resize(N);
        for (int64_t a = 0; a < N; ++a) jb.r_host[a] = y[a] - (mX ? mX[a] : 1.0 * jb.mean);
        HIPC(hipMemcpyAsync(dx, xyt_in, N * 3 * 8, hipMemcpyHostToDevice, ss_));
        HIPC(hipMemcpyAsync(d_r, jb.r_host.data(), N * 8, hipMemcpyHostToDevice, ss_));
      }
    }
    // distinct sites of every cell; the host needs m to size and order cells
    jb.m.assign(nc, 0);
    jb.ssw.assign(nc, 0.0);
    if (nc > 0) {
      int64_t maxn = 0;
      for (int64_t c = 0; c < nc; ++c) maxn = std::max(maxn, jb.offs[c + 1] - jb.offs[c]);
      HIPC(hipMemcpyAsync(d_offs, jb.offs.data(), (nc + 1) * 8, hipMemcpyHostToDevice, ss_));
      if (oi_launch_dedup(d_x, d_r, d_offs, (int)nc, (int)std::min<int64_t>(maxn, INT32_MAX),
                          dedup_enabled() ? 0 : 1, d_sites, d_v, d_dw, d_m, d_ssw, ss_))
        throw HipError(std::string("dedup kernel launch failed: ") + hipGetErrorString(hipGetLastError()));
      HIPC(hipMemcpyAsync(jb.m.data(), d_m, nc * 4, hipMemcpyDeviceToHost, ss_));
      HIPC(hipMemcpyAsync(jb.ssw.data(), d_ssw, nc * 8, hipMemcpyDeviceToHost, ss_));
    }
    HIPC(hipStreamSynchronize(ss_));  // m known; host inputs may be released on return
    jb.xyt = d_x;
    jb.r = d_r;
    jb.sites = d_sites;
    jb.v = d_v;
    jb.dw = d_dw;
    size_t max_cell = 0;
    for (int64_t c = 0; c < nc; ++c)
      max_cell = std::max(max_cell, cell_bytes(jb.m[c], jb.kind != Job::PREDICT_ONLY));
    if (max_cell > ctx_.arena.size()) {
      // in_off == SIZE_MAX: the inputs went to the job's own buffer, nothing
      // of the arena to return
      if (jb.in_off != SIZE_MAX) ctx_.arena.release(jb.in_off, jb.in_bytes);
      jb.in_off = SIZE_MAX;
      throw NoMem("a cell needs " + std::to_string(max_cell) + " bytes of workspace, pool is " +
                  std::to_string(ctx_.arena.size()));
    }
    // (the submission completed on the host's clock: every group stream's later
    // launches see its outputs)
    // admission order inside the batch: largest cells first (cost ~ m^3), ties by index
    std::vector<int64_t> order(nc);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return jb.m[a] > jb.m[b]; });
    jb.remaining = nc;
    Job* jp = job.get();
    const int64_t id = jb.id;
    for (int64_t c : order) queue_.push_back({jp, c});
    if (nc == 0)
      release_job(jp);
    else
      jobs_[id] = std::move(job);
    return id;
  }

  bool done(int64_t id) const { return id < next_id_ && !jobs_.count(id); }


  // k_panel4 (two block rows per 512-thread workgroup) when the launch still
  // fills the chip, else k_panel_even (one block row: twice the workgroups);
  // the two are bitwise equal (round 5), so the choice never changes a result
  bool use_panel4(int j, int maxT, int cnt, bool trtri) const {
    if (!(panel4_ && j >= panel4_minj_ && maxT >= panel4_mint_)) return false;
    const int64_t wg = (int64_t)cnt * (((maxT - j) >> 1) + (trtri ? j / 2 : 0));
    return wg >= panel4_minwg_;
  }

  // The stream later submissions' device inputs are ordered after (the rounds
  // keep the stream chosen at construction).
  void set_input_stream(void* stream) { o_.stream = stream; }

  // Drive rounds until batch `id` (or every batch, id < 0) is complete.
  void wait(int64_t id) {
    const auto tw = std::chrono::steady_clock::now();
    while (true) {
      bool any = false;
      for (Group& gr : groups_) {
        if (gr.inflight) consume(gr);
        admit(gr);
        if (!gr.active.empty()) {
          launch_round(gr);
          any = true;
        }
      }
      if (id >= 0 ? done(id) : (jobs_.empty() && !any)) break;
      if (!any) {
        if (!queue_.empty()) throw NoMem("workspace exhausted with no resident cell");
        break;
      }
    }
    if (id < 0)
      for (Group& gr : groups_)
        if (gr.inflight) consume(gr);
    wall_s_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - tw).count();
    flush_stats();
  }

  struct NoMem {
    std::string msg;
    explicit NoMem(std::string m) : msg(std::move(m)) {}
  };

 private:
  struct Group {
    int s0 = 0, cap = 0;
    hipStream_t st = nullptr;
    std::vector<int> free_slots, active, ev_slots, pr_slots;
    OiCell* hc = nullptr;   // cell records of the group's slots (host mirror / device)
    OiCell* dc = nullptr;
    int32_t* hl = nullptr;  // lists all | eval | predict (capG each), group-local slot indices
    int32_t* dl = nullptr;
    int32_t* hstat = nullptr;  // status words (cleared on the host every round)
    int32_t* dstat = nullptr;
    bool inflight = false;
    bool flagged = false;         // completion by host flag (else stream synchronise)
    unsigned long long seq = 0;   // rounds launched: the flag value of the latest
    int maxT = 0;
    std::vector<hipEvent_t> ev;
    std::vector<int> ev_kind;
    std::vector<std::pair<int, int>> ev_meta;
  };

  OiCell& hcell(int s) {
    Group& gr = groups_[s / capG_];
    return gr.hc[s - gr.s0];
  }

  void release_job(Job* jp) {
    if (jp->in_off != SIZE_MAX) ctx_.arena.release(jp->in_off, jp->in_bytes);
    jp->in_off = SIZE_MAX;
    auto it = jobs_.find(jp->id);
    if (it != jobs_.end()) jobs_.erase(it);  // frees the job (its own DBuf, if any)
  }

  void admit(Group& gr) {
    while (!queue_.empty() && !gr.free_slots.empty()) {
      Job* jp = queue_.front().first;
      const int64_t c = queue_.front().second;
      const Job& job = *jp;
      const int64_t n = job.m[c];  // the cell's problem size: its distinct sites
      const bool eval_mem = job.kind != Job::PREDICT_ONLY;
      const size_t bytes = cell_bytes(n, eval_mem);
      const size_t off = ctx_.arena.alloc(bytes);
      if (off == SIZE_MAX) break;
      queue_.pop_front();
      const int s = gr.free_slots.back();
      gr.free_slots.pop_back();
      Slot& sl = slots_[s];
      sl = Slot();
      sl.job = jp;
      sl.cell = c;
      sl.off = off;
      sl.bytes = bytes;
      if (poison_)  // debug: NaN-fill the cell's workspace so any read-before-write shows
        HIPC(hipMemsetAsync(ctx_.arena.ptr(off), 0xFF, bytes, gr.st));
      OiCell& cd = hcell(s);
      std::memset(&cd, 0, sizeof(cd));
      const int T = tiles_of(n);
      const size_t nt = (size_t)T * (T + 1) / 2;
      char* p = ctx_.arena.ptr(off);
      auto take = [&](size_t x) {
        char* q = p;
        p += (x + 255) & ~size_t(255);
        return (double*)q;
      };
      cd.L = take(nt * OI_TILE * 8);
      cd.W = eval_mem ? take(nt * OI_TILE * 8) : nullptr;
      cd.Dinv = take((size_t)T * OI_TILE * 8);
      cd.vec = take(4 * (size_t)T * OI_NB * 8);
      cd.part = take((size_t)OI_PART_SIZE(nt, T) * 8);
      cd.xyt = job.sites + 3 * job.offs[c];
      cd.r = job.v + job.offs[c];
      cd.dw = job.dw + job.offs[c];
      cd.out = dres_ + (size_t)s * OI_OUT_N;
      cd.status = gr.dstat + (s - gr.s0);
      cd.n = (int32_t)n;
      cd.n_obs = (int32_t)(job.offs[c + 1] - job.offs[c]);
      cd.ssw = job.ssw[c];
      cd.T = T;
      if (!job.xs.empty())
        for (int d = 0; d < 3; ++d) cd.xs[d] = job.xs[3 * c + d];
      cd.mean = job.mean;
      if (job.kind == Job::FIT_PREDICT) {
        sl.phase = 0;
        oi::Vec x0;
        for (int k = 0; k < oi::NH; ++k) x0[k] = job.x0[k];
        sl.task = oi::cg_minimize(&sl.mail, x0, job.cg);
        sl.task.start();  // runs to the first objective request
      } else if (job.kind == Job::PREDICT_ONLY) {
        sl.phase = 1;
        for (int k = 0; k < 5; ++k) sl.hyp[k] = job.hyp[5 * c + k];
      } else {
        sl.phase = 2;
        for (int k = 0; k < 5; ++k) sl.hyp[k] = std::exp(job.h[6 * c + k]);
      }
      gr.active.push_back(s);
    }
  }

  void launch_round(Group& gr) {
    const auto tl0 = std::chrono::steady_clock::now();
    hipStream_t gst = gr.st;
    auto hc = [&](int s) -> OiCell& { return gr.hc[s - gr.s0]; };
    gr.ev_slots.clear();
    gr.pr_slots.clear();
    for (int s : gr.active) {
      Slot& sl = slots_[s];
      OiCell& cd = hc(s);
      if (sl.phase == 0) {
        for (int k = 0; k < 5; ++k) cd.hyp[k] = std::exp(sl.mail.x[k]);  // GPR:120-122
        cd.mode = OI_MODE_EVAL;
        gr.ev_slots.push_back(s);
      } else if (sl.phase == 2) {
        for (int k = 0; k < 5; ++k) cd.hyp[k] = sl.hyp[k];
        cd.mode = OI_MODE_EVAL;
        gr.ev_slots.push_back(s);
      } else {
        for (int k = 0; k < 5; ++k) cd.hyp[k] = sl.hyp[k];
        cd.mode = OI_MODE_PREDICT;
        gr.pr_slots.push_back(s);
      }
    }
    auto byT = [&](std::vector<int>& v) {
      std::stable_sort(v.begin(), v.end(), [&](int a, int b) { return hc(a).T > hc(b).T; });
    };
    byT(gr.ev_slots);
    byT(gr.pr_slots);
    std::vector<int> all_slots;
    all_slots.reserve(gr.active.size());
    std::merge(gr.ev_slots.begin(), gr.ev_slots.end(), gr.pr_slots.begin(), gr.pr_slots.end(),
               std::back_inserter(all_slots), [&](int a, int b) { return hc(a).T > hc(b).T; });
    const int na = (int)all_slots.size(), ne = (int)gr.ev_slots.size(),
              np_ = (int)gr.pr_slots.size();
    int32_t* l_all = gr.hl;
    int32_t* l_ev = gr.hl + capG_;
    int32_t* l_pr = gr.hl + 2 * capG_;
    for (int k = 0; k < na; ++k) l_all[k] = all_slots[k] - gr.s0;
    for (int k = 0; k < ne; ++k) l_ev[k] = gr.ev_slots[k] - gr.s0;
    for (int k = 0; k < np_; ++k) l_pr[k] = gr.pr_slots[k] - gr.s0;
    const int maxT = na ? hc(all_slots[0]).T : 0;
    const int maxTe = ne ? hc(gr.ev_slots[0]).T : 0;
    gr.maxT = maxT;

    std::memset(gr.hstat, 0, (size_t)capG_ * 4);
    HIPC(hipMemcpyAsync(gr.dc, gr.hc, blk_, hipMemcpyHostToDevice, gst));
    const int32_t* dl_all = gr.dl;
    const int32_t* dl_ev = gr.dl + capG_;
    const OiCell* dc = gr.dc;

    gr.ev_kind.clear();
    gr.ev_meta.clear();
    int cur_j = -1, cur_cells = 0;
    auto mark = [&](int k, bool end) {
      if (!o_.profile) return;
      if (!end) {
        gr.ev_kind.push_back(k);
        gr.ev_meta.emplace_back(cur_j, cur_cells);
      }
      const size_t idx = 2 * (gr.ev_kind.size() - 1) + (end ? 1 : 0);
      if (idx < gr.ev.size()) HIPC(hipEventRecord(gr.ev[idx], gst));
    };
    int rc = 0;
    cur_cells = na;
    prep_s_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - tl0).count();
    // (no k_build since round 5: the factor kernels generate K + sn2 I where they read it)
    for (int j = 0; j < maxT; ++j) {
      int cnt = 0;
      while (cnt < na && hc(all_slots[cnt]).T > j) ++cnt;
      cur_j = j;
      cur_cells = cnt;
      // diagonal tile 0 has its own launch; tile j+1 is factored by the
      // look-ahead workgroup of column j's panel launch (round 5) -- unless the
      // round holds fewer than OI_FUSE_DIAG_MIN cells (the lone cell of config
      // 1: there a launch of its own is cheaper than the long look-ahead
      // workgroup); bitwise the same either way
      const bool fuse = na >= fuse_diag_min_;
      if (j == 0 || !fuse) {
        mark(K_CHOL, false);
        rc |= oi_launch_diag_factor(dc, dl_all, cnt, j, gst);
        mark(K_CHOL, true);
      }
      const bool even = !legacy_ && (j % 2 == 0);
      const int kbeg = (legacy_ || even) ? 0 : j - 1;
      // the last column of a round with no fitting cell has neither factor
      // tiles below the diagonal nor a W row: its panel launch would be empty
      const bool empty_panel = j == maxT - 1 && ne == 0;
      if (empty_panel) {
      } else if (even) {
        const int ke = use_panel4(j, maxT, cnt, ne > 0) ? K_EVEN4 : K_EVEN;
        mark(ke, false);
        if (ke == K_EVEN4)
          rc |= oi_launch_panel4(dc, dl_all, cnt, maxT, j, ne > 0 ? 1 : 0, fuse, gst);
        else
          rc |= oi_launch_panel_even(dc, dl_all, cnt, maxT, j, ne > 0 ? 1 : 0, fuse, gst);
        mark(ke, true);
      } else {
        mark(K_TRSM, false);
        rc |= oi_launch_chol_panel(dc, dl_all, cnt, maxT, j, kbeg, ne > 0 ? 1 : 0, fuse, gst);
        mark(K_TRSM, true);
      }
      if (o_.profile) {  // executed MFMA flops, mirroring the kernels' masks (acct::)
        for (int k = 0; k < cnt; ++k) {
          const OiCell& cd = hc(all_slots[k]);
          const bool ev = cd.mode == OI_MODE_EVAL;
          if (empty_panel) continue;
          const int kk = even ? (use_panel4(j, maxT, cnt, ne > 0) ? K_EVEN4 : K_EVEN) : K_TRSM;
          const double f = kk == K_EVEN4 ? acct::panel4(cd.T, cd.n, j, ev)
                           : kk == K_EVEN ? acct::panel_even(cd.T, cd.n, j, ev, true)
                                          : acct::chol_panel(cd.T, cd.n, j, kbeg, ev, true);
          kfl_[kk] += f;
          std::lock_guard<std::mutex> pl(g_prof_mu);
          g_byj[{kk, j}].flops += f;
        }
      }
    }
    cur_j = -1;
    cur_cells = ne;
    // z = L^-1 r and alpha = W^T z were built during the factorisation
    // (k_diag_factor and the panels), quad = z^T z
    if (ne > 0) {  // (an empty launch would still be profiled)
      mark(K_LAUUM, false);
      rc |= oi_launch_lauum_grad(dc, dl_ev, ne, maxTe, gst);
      mark(K_LAUUM, true);
    }
    // nlZ / dnlZ of the fitting cells and fs / sd / lZ of the predicting ones
    cur_cells = na;
    // the host spins on the group's flag (profiling rounds synchronise the
    // stream: their events are read back)
    const int g = (int)(&gr - groups_.data());
    gr.flagged = !o_.profile && na > 0;
    mark(K_FINAL, false);
    rc |= oi_launch_finalize(dc, dl_all, na, (unsigned*)d_done_.p + 16 * g,
                             gr.flagged ? (unsigned long long*)(dflag_ + 64 * g) : nullptr, ++gr.seq, gst);
    mark(K_FINAL, true);
    if (rc) throw HipError(std::string("kernel launch failed: ") + hipGetErrorString(hipGetLastError()));
    if (o_.profile) {
      for (int k = 0; k < ne; ++k) {
        const OiCell& cd = hc(gr.ev_slots[k]);
        kfl_[K_LAUUM] += acct::lauum(cd.T, cd.n);
      }
    }
    gr.inflight = true;
    launch_s_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - tl0).count();
  }

  // Wait for the group's round: spin on its host flag (k_finalize stores the
  // round's sequence number after the last result row), checking the stream
  // every ~1 ms so a failed launch surfaces as an error instead of a hang.
  void wait_round(Group& gr) {
    if (!gr.flagged) {
      HIPC(hipStreamSynchronize(gr.st));
      return;
    }
    const int g = (int)(&gr - groups_.data());
    const volatile unsigned long long* f = (const volatile unsigned long long*)((char*)h_flag_.p + 64 * g);
    auto last = std::chrono::steady_clock::now();
    for (unsigned spin = 0; *f != gr.seq; ++spin) {
      if ((spin & 1023u) != 0) continue;
      const auto now = std::chrono::steady_clock::now();
      if (now - last < std::chrono::milliseconds(1)) continue;
      last = now;
      const hipError_t e = hipStreamQuery(gr.st);
      if (e == hipErrorNotReady) continue;
      if (e != hipSuccess) throw HipError(std::string("round failed: ") + hipGetErrorString(e));
      if (*f != gr.seq) throw HipError("round completed without its completion flag");
    }
    std::atomic_thread_fence(std::memory_order_acquire);
  }

  void consume(Group& gr) {
    const auto ts0 = std::chrono::steady_clock::now();
    wait_round(gr);
    sync_s_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - ts0).count();
    gr.inflight = false;
    ++rounds_;
    if (o_.profile) {
      std::vector<LaunchRec> recs;
      for (size_t q = 0; q < gr.ev_kind.size() && 2 * q + 1 < gr.ev.size(); ++q) {
        float a = 0;
        HIPC(hipEventElapsedTime(&a, gr.ev[2 * q], gr.ev[2 * q + 1]));
        kms_[gr.ev_kind[q]] += a;
        kln_[gr.ev_kind[q]]++;
        recs.push_back({gr.ev_kind[q], gr.ev_meta[q].first, gr.ev_meta[q].second, (double)a});
      }
      {
        std::lock_guard<std::mutex> pl(g_prof_mu);
        for (const auto& rr : recs) {
          ByJ& b = g_byj[{rr.kind, rr.j}];
          b.launches++;
          b.cells += rr.cells;
          b.ms += rr.ms;
        }
      }
      double rms = 0.0, work = 0.0;
      for (const auto& rr : recs) rms += rr.ms;
      for (int s : gr.ev_slots) work += std::pow((double)hcell(s).T, 3.0);
      std::lock_guard<std::mutex> pl(g_prof_mu);
      g_last_round.swap(recs);
      g_rounds.push_back({(int)gr.ev_slots.size(), (int)gr.pr_slots.size(), gr.maxT, work, rms});
    }
    std::vector<int> still;
    still.reserve(gr.active.size());
    for (int s : gr.active) {
      Slot& sl = slots_[s];
      Job& job = *sl.job;
      const double* rr = hres_ + (size_t)s * OI_OUT_N;
      const int32_t st = (int32_t)rr[OI_OUT_STATUS];
      const int64_t c = sl.cell;
      bool done = false;
      if (sl.phase == 0) {
        ++evals_;
        sl.mail.f = rr[0];
        for (int k = 0; k < oi::NH; ++k) sl.mail.g[k] = rr[1 + k];
        sl.mail.pending = false;
        sl.mail.waiter.resume();
        if (sl.task.done()) {
          sl.res = sl.task.result();
          sl.phase = 1;
          for (int k = 0; k < 5; ++k) sl.hyp[k] = std::exp(sl.res.x[k]);  // GPR:166-168
        }
      } else if (sl.phase == 2) {
        ++evals_;
        job.nlz[c] = rr[0];
        for (int k = 0; k < oi::NH; ++k) job.grad[6 * c + k] = rr[1 + k];
        if (job.status) job.status[c] = st;
        done = true;
      } else {
        ++predicts_;
        double* dst = job.out + 8 * c;
        dst[0] = rr[0];
        dst[1] = rr[1];
        dst[2] = rr[2];
        for (int k = 0; k < 5; ++k) dst[3 + k] = sl.hyp[k];
        if (st != OI_OK) {
          for (int k = 0; k < 8; ++k) dst[k] = NAN;  // GPR:187-189
        }
        if (job.status) job.status[c] = st;
        if (job.info) {
          int32_t* inf = job.info + 4 * c;
          inf[0] = sl.res.nit;
          inf[1] = sl.res.status;
          inf[2] = (int32_t)sl.res.nfev;
          inf[3] = (int32_t)sl.res.nobj;
        }
        done = true;
      }
      if (done) {
        ctx_.arena.release(sl.off, sl.bytes);
        sl.task = oi::Task<oi::CgResult>();
        sl.cell = -1;
        sl.job = nullptr;
        gr.free_slots.push_back(s);
        if (--job.remaining == 0) release_job(&job);
      } else {
        still.push_back(s);
      }
    }
    gr.active.swap(still);
    consume_s_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - ts0).count();
  }

  void flush_stats() {
    std::lock_guard<std::mutex> pl(g_prof_mu);
    if (o_.profile) {
      for (int k = 0; k < K_COUNT; ++k) {
        g_prof[k].launches += kln_[k];
        g_prof[k].ms += kms_[k];
        g_prof[k].flops += kfl_[k];
        kln_[k] = 0;
        kms_[k] = kfl_[k] = 0.0;
      }
    }
    g_run.rounds += rounds_;
    g_run.evals += evals_;
    g_run.predicts += predicts_;
    g_run.sync_s += sync_s_;
    g_run.wall_s += wall_s_;
    g_run.consume_s += consume_s_;
    g_run.prep_s += prep_s_;
    g_run.launch_s += launch_s_;
    rounds_ = evals_ = predicts_ = 0;
    sync_s_ = wall_s_ = consume_s_ = prep_s_ = launch_s_ = 0.0;
  }

  Context& ctx_;
  oi_options o_;
  bool legacy_ = false, poison_ = false, panel4_ = false;
  int panel4_minj_ = 0, panel4_mint_ = 12, panel4_minwg_ = 512, fuse_diag_min_ = 1;
  hipStream_t st_ = nullptr, ss_ = nullptr;
  hipEvent_t ready_ = nullptr;
  int cap_ = 1, G_ = 1, capG_ = 1;
  std::vector<Slot> slots_;
  std::vector<Group> groups_;
  DBuf d_blk_, d_done_;
  HBuf h_blk_, h_res_, h_flag_;
  size_t blk_ = 0;  // bytes of one group's round block
  double* hres_ = nullptr;  // result rows (host view)
  double* dres_ = nullptr;  // the same rows, device view
  char* dflag_ = nullptr;   // device view of h_flag_ (64 B per group)
  std::deque<std::pair<Job*, int64_t>> queue_;
  std::map<int64_t, std::unique_ptr<Job>> jobs_;
  int64_t next_id_ = 0;
  double kms_[K_COUNT] = {0}, kfl_[K_COUNT] = {0};
  int64_t kln_[K_COUNT] = {0};
  int64_t rounds_ = 0, evals_ = 0, predicts_ = 0;
  double sync_s_ = 0.0, wall_s_ = 0.0;
  double consume_s_ = 0.0, prep_s_ = 0.0, launch_s_ = 0.0;  // host time per phase
  std::chrono::steady_clock::time_point t_start_;
};

bool check_offs(const int64_t* offs, int64_t ncell) {
  if (!offs || offs[0] != 0) return false;
  for (int64_t c = 0; c < ncell; ++c)
    if (offs[c + 1] < offs[c]) return false;
  return true;
}

oi_options resolve(const oi_options* opts) {
  oi_options o;
  oi_options_default(&o);
  if (opts) o = *opts;
  return o;
}

int check_device(const oi_options& o) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(OI_E_NODEV, "no HIP device available");
  if (o.device < 0 || o.device >= ndev) return fail(OI_E_ARG, "bad device ordinal");
  return 0;
}

// Validates the oi_gpr_batch arguments and fills a Job (host metadata copied).
int make_gpr_job(const double* xyt, const double* z, const int64_t* offs, int64_t ncell,
                 const double* xs, double mean, const double* x0, int32_t opt, const double* hyp,
                 double* out, int32_t* status, int32_t* info, const oi_options& o,
                 std::unique_ptr<Job>& job) {
  if (ncell < 0 || !check_offs(offs, ncell)) return fail(OI_E_ARG, "bad offs / ncell");
  const int64_t N = ncell ? offs[ncell] : 0;
  if (ncell > 0 && ((N > 0 && (!xyt || !z)) || !xs || !out)) return fail(OI_E_ARG, "null input/output pointer");
  if (opt && !x0) return fail(OI_E_ARG, "opt=1 needs x0");
  if (!opt && !hyp) return fail(OI_E_ARG, "opt=0 needs hyp");
  job = std::make_unique<Job>();
  Job& jb = *job;
  jb.offs.assign(offs, offs + ncell + 1);
  jb.ncell = ncell;
  if (ncell > 0) jb.xs.assign(xs, xs + 3 * ncell);
  jb.mean = mean;  // outputs - mX with mX = ones(n)*mean  (GPR:163, GPR:178)
  jb.kind = opt ? Job::FIT_PREDICT : Job::PREDICT_ONLY;
  if (opt) jb.x0.assign(x0, x0 + 6);
  else jb.hyp.assign(hyp, hyp + 5 * ncell);
  jb.cg.gtol = o.gtol;
  jb.cg.maxiter = o.maxiter;
  jb.out = out;
  jb.status = status;
  jb.info = info;
  return 0;
}

// One-shot batch: a private engine, submit + drain.
int run_once(std::unique_ptr<Job> job, const double* xyt, const double* y, const double* mX,
             const oi_options& o) {
  try {
    if (int rc = check_device(o)) return rc;
    if (job->ncell == 0) return 0;
    Context& ctx = context(o.device, o.pool_bytes);
    std::lock_guard<std::mutex> lk(ctx.mu);
    const auto t0 = std::chrono::steady_clock::now();
    Engine eng(ctx, o, job->ncell);
    eng.submit(std::move(job), xyt, y, mX);
    const double setup = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    {
      std::lock_guard<std::mutex> pl(g_prof_mu);
      g_run.setup_s += setup;
    }
    eng.wait(-1);
    return 0;
  } catch (const HipError& e) {
    return fail(OI_E_HIP, e.msg);
  } catch (const Engine::NoMem& e) {
    return fail(OI_E_NOMEM, e.msg);
  } catch (const std::bad_alloc&) {
    return fail(OI_E_NOMEM, "host allocation failed");
  }
}

}  // namespace

// =================================================================== C ABI
extern "C" {

void oi_options_default(oi_options* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->device = 0;
  o->maxiter = -1;
  o->gtol = 1e-5;
  o->stream = nullptr;
  o->pool_bytes = 0;
  o->max_pool = 0;
  o->profile = 0;
  o->device_inputs = 0;
}

int oi_gpr_batch(const double* xyt, const double* z, const int64_t* offs, int64_t ncell,
                 const double* xs, double mean, const double* x0, int32_t opt, const double* hyp,
                 double* out, int32_t* status, int32_t* info, const oi_options* opts) {
  if (ncell < 0 || !check_offs(offs, ncell)) return fail(OI_E_ARG, "bad offs / ncell");
  if (ncell == 0) return 0;
  const oi_options o = resolve(opts);
  std::unique_ptr<Job> job;
  if (int rc = make_gpr_job(xyt, z, offs, ncell, xs, mean, x0, opt, hyp, out, status, info, o, job))
    return rc;
  return run_once(std::move(job), xyt, z, nullptr, o);
}

int oi_nlml_grad_batch(const double* xyt, const double* y, const double* mX, const int64_t* offs,
                       int64_t ncell, const double* h, double* nlz, double* grad, int32_t* status,
                       const oi_options* opts) {
  if (ncell < 0 || !check_offs(offs, ncell)) return fail(OI_E_ARG, "bad offs / ncell");
  if (ncell == 0) return 0;
  const int64_t N = offs[ncell];
  if ((N > 0 && (!xyt || !y || !mX)) || !h || !nlz || !grad)
    return fail(OI_E_ARG, "null input/output pointer");
  auto job = std::make_unique<Job>();
  job->offs.assign(offs, offs + ncell + 1);
  job->ncell = ncell;
  job->kind = Job::EVAL_ONLY;  // y - mX, GPR:127
  job->h.assign(h, h + 6 * ncell);
  job->nlz = nlz;
  job->grad = grad;
  job->status = status;
  return run_once(std::move(job), xyt, y, mX, resolve(opts));
}

// ---- session: continuous batching across calls
struct oi_session {
  oi_options o;
  Context* ctx = nullptr;
  std::unique_ptr<Engine> eng;
};

oi_session* oi_session_create(const oi_options* opts) {
  const oi_options o = resolve(opts);
  try {
    if (check_device(o)) return nullptr;
    auto* s = new oi_session();
    s->o = o;
    s->ctx = &context(o.device, o.pool_bytes);
    std::lock_guard<std::mutex> lk(s->ctx->mu);
    s->eng = std::make_unique<Engine>(*s->ctx, o, INT64_MAX);
    s->ctx->live_sessions++;
    return s;
  } catch (const HipError& e) {
    fail(OI_E_HIP, e.msg);
  } catch (const std::bad_alloc&) {
    fail(OI_E_NOMEM, "host allocation failed");
  }
  return nullptr;
}

int64_t oi_session_submit(oi_session* s, const double* xyt, const double* z, const int64_t* offs,
                          int64_t ncell, const double* xs, double mean, const double* x0, int32_t opt,
                          const double* hyp, double* out, int32_t* status, int32_t* info) {
  if (!s) return fail(OI_E_ARG, "null session");
  std::unique_ptr<Job> job;
  if (int rc = make_gpr_job(xyt, z, offs, ncell, xs, mean, x0, opt, hyp, out, status, info, s->o, job))
    return rc;
  try {
    std::lock_guard<std::mutex> lk(s->ctx->mu);
    HIPC(hipSetDevice(s->o.device));
    return s->eng->submit(std::move(job), xyt, z, nullptr);
  } catch (const HipError& e) {
    return fail(OI_E_HIP, e.msg);
  } catch (const Engine::NoMem& e) {
    return fail(OI_E_NOMEM, e.msg);
  } catch (const std::bad_alloc&) {
    return fail(OI_E_NOMEM, "host allocation failed");
  }
}

int oi_session_set_stream(oi_session* s, void* stream) {
  if (!s) return fail(OI_E_ARG, "null session");
  std::lock_guard<std::mutex> lk(s->ctx->mu);
  s->eng->set_input_stream(stream);
  return 0;
}

int oi_session_wait(oi_session* s, int64_t ticket) {
  if (!s) return fail(OI_E_ARG, "null session");
  try {
    std::lock_guard<std::mutex> lk(s->ctx->mu);
    HIPC(hipSetDevice(s->o.device));
    s->eng->wait(ticket < 0 ? -1 : ticket);
    return 0;
  } catch (const HipError& e) {
    return fail(OI_E_HIP, e.msg);
  } catch (const Engine::NoMem& e) {
    return fail(OI_E_NOMEM, e.msg);
  } catch (const std::bad_alloc&) {
    return fail(OI_E_NOMEM, "host allocation failed");
  }
}

int oi_session_done(oi_session* s, int64_t ticket) {
  if (!s) return fail(OI_E_ARG, "null session");
  std::lock_guard<std::mutex> lk(s->ctx->mu);
  return s->eng->done(ticket) ? 1 : 0;
}

void oi_session_destroy(oi_session* s) {
  if (!s) return;
  {
    std::lock_guard<std::mutex> lk(s->ctx->mu);
    (void)hipSetDevice(s->o.device);
    s->eng.reset();
    s->ctx->live_sessions--;
  }
  delete s;
}


const char* oi_last_error(void) { return g_last_error.c_str(); }
// internal: lets the other translation units (oi_day.cpp) report errors
int oi_set_last_error(int code, const char* msg) { return fail(code, msg ? msg : ""); }
int32_t oi_version(void) { return OI_VERSION; }
// internal: per-stage HIP-event timings from the other translation units
void oi_profile_add(const char* name, int64_t launches, double ms, double flops, double bytes) {
  std::lock_guard<std::mutex> pl(g_prof_mu);
  for (auto& e : g_ext)
    if (e.first == name) {
      e.second.launches += launches;
      e.second.ms += ms;
      e.second.flops += flops;
      e.second.bytes += bytes;
      return;
    }
  g_ext.push_back({name, ExtStat{launches, ms, flops, bytes}});
}

int64_t oi_profile_json(char* buf, int64_t len) {
  std::lock_guard<std::mutex> pl(g_prof_mu);
  std::string s = "{\"kernels\":{";
  for (int k = 0; k < K_COUNT; ++k) {
    char tmp[256];
    std::snprintf(tmp, sizeof(tmp), "%s\"%s\":{\"launches\":%lld,\"total_ms\":%.6f,\"flops\":%.6e}",
                  k ? "," : "", kKernelName[k], (long long)g_prof[k].launches, g_prof[k].ms,
                  g_prof[k].flops);
    s += tmp;
  }
  for (const auto& e : g_ext) {
    char tmp[320];
    std::snprintf(tmp, sizeof(tmp),
                  ",\"%s\":{\"launches\":%lld,\"total_ms\":%.6f,\"flops\":%.6e,\"bytes\":%.6e}",
                  e.first.c_str(), (long long)e.second.launches, e.second.ms, e.second.flops,
                  e.second.bytes);
    s += tmp;
  }
  char tmp[512];
  std::snprintf(tmp, sizeof(tmp),
                "},\"rounds\":%lld,\"evals\":%lld,\"predicts\":%lld,\"wall_s\":%.6f,\"sync_s\":%.6f,"
                "\"setup_s\":%.6f,\"consume_s\":%.6f,\"prep_s\":%.6f,\"launch_s\":%.6f",
                (long long)g_run.rounds, (long long)g_run.evals, (long long)g_run.predicts,
                g_run.wall_s, g_run.sync_s, g_run.setup_s, g_run.consume_s, g_run.prep_s, g_run.launch_s);
  s += tmp;
  s += ",\"last_round\":[";
  for (size_t q = 0; q < g_last_round.size(); ++q) {
    const LaunchRec& r = g_last_round[q];
    std::snprintf(tmp, sizeof(tmp), "%s[\"%s\",%d,%d,%.4f]", q ? "," : "", kKernelName[r.kind], r.j,
                  r.cells, r.ms);
    s += tmp;
  }
  s += "],\"by_j\":[";
  {
    bool first = true;
    for (const auto& kv : g_byj) {
      std::snprintf(tmp, sizeof(tmp), "%s[\"%s\",%d,%lld,%lld,%.4f,%.6e]", first ? "" : ",",
                    kKernelName[kv.first.first], kv.first.second, (long long)kv.second.launches,
                    (long long)kv.second.cells, kv.second.ms, kv.second.flops);
      s += tmp;
      first = false;
    }
  }
  s += "],\"rounds_log\":[";
  for (size_t q = 0; q < g_rounds.size(); ++q) {
    const RoundRec& r = g_rounds[q];
    std::snprintf(tmp, sizeof(tmp), "%s[%d,%d,%d,%.0f,%.4f]", q ? "," : "", r.n_eval, r.n_pred, r.maxT,
                  r.work, r.ms);
    s += tmp;
  }
  s += "]}";
  if (buf && len > 0) {
    std::strncpy(buf, s.c_str(), (size_t)len);
    buf[len - 1] = 0;
  }
  return (int64_t)s.size() + 1;
}

void oi_profile_reset(void) {
  std::lock_guard<std::mutex> pl(g_prof_mu);
  for (auto& k : g_prof) k = KStat();
  g_run = RunStat();
  g_rounds.clear();
  g_byj.clear();
  g_ext.clear();
}

}  // extern "C"
