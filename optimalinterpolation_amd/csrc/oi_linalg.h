// Hand-written dense fp64 kernels for the Nystrom variant (oi_nystrom.hip):
// what GP_example.ipynb does with LAPACK / BLAS -- np.linalg.eigh(Kmm)
// (NB1 Nystroem), np.linalg.cholesky and the n x M products -- as batched
// HIP kernels for gfx950, one matrix per cell of a chunk (oi_linalg.hip).
//
// Every routine takes a host vector of per-matrix descriptors, stages them
// into a Stager (pinned host ring -> device copy, stream ordered) and
// launches over the whole batch; matrices of different sizes share a launch.
// All matrices are column-major.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

namespace oila {

struct LinalgErr {  // thrown by the host routines on a HIP error or an operand too large
  std::string msg;
};

// C = alpha op(A) op(B) + beta C  (m x n, inner dimension k); tri:
//   0  all output tiles;
//   1  lower output tiles only (64-tile row >= 64-tile column; syrk-like);
//   2  op(B) upper triangular: output column tile jt only sums k < 64 (jt + 1)
struct Gemm {
  const double* A;
  const double* B;
  double* C;
  int m, n, k, lda, ldb, ldc;
  double alpha, beta;
  int tri;
};

// y = alpha op(A) x + beta y (A m x n; op = A' when trans)
struct Gemv {
  const double* A;
  const double* x;
  double* y;
  int m, n, lda;
  double alpha, beta;
};

// One symmetric matrix for the eigensolver: A (M x M, lower triangle read;
// destroyed, then overwritten with the eigenvectors), w (M eigenvalues,
// ascending), its workspace (workspace_doubles(M) doubles), and info (device,
// may be null): set to 1 -- LAPACK syevd's info > 0, numpy's LinAlgError --
// when the orthogonalisation cannot produce a finite column in its four
// attempts; left untouched otherwise (NaN input propagates as NaN).
struct Eigh {
  double* A;
  double* w;
  double* work;
  int M, lda;
  int* info;
};
size_t eigh_workspace_doubles(int M);

// One SPD matrix for the blocked Cholesky: A (M x M, lower triangle; the
// factor L overwrites it), dinv (ceil(M/64) x 4096 doubles: the inverses of
// L's 64 x 64 diagonal blocks, kept for trsm_right_lt), info (0, or 1 when
// a pivot is <= 0, as LAPACK dpotrf's info > 0; a NaN pivot propagates, as
// numpy + OpenBLAS's dpotrf let it).
struct Chol {
  double* A;
  double* dinv;
  int* info;
  int M, lda;
};

// X (m x M) <- X L^-T for a factored Chol (right-looking block triangular solve)
struct TrsmRLT {
  double* X;
  const double* L;
  const double* dinv;
  int m, M, ldx, ldl;
};

// Pinned-host -> device staging of descriptor arrays, one ring per stream.
// reset() may be called once the stream has drained every launch that used it.
class Stager {
 public:
  Stager() = default;
  ~Stager();
  Stager(const Stager&) = delete;
  Stager& operator=(const Stager&) = delete;
  void bind(hipStream_t st) { st_ = st; }
  template <class T>
  const T* put(const std::vector<T>& v) {
    return static_cast<const T*>(put_bytes(v.data(), v.size() * sizeof(T)));
  }
  void reset() { off_ = 0; }

 private:
  const void* put_bytes(const void* p, size_t bytes);
  hipStream_t st_ = nullptr;
  char* host_ = nullptr;
  char* dev_ = nullptr;
  size_t cap_ = 0, off_ = 0;
  std::vector<std::pair<char*, char*>> retired_;  // grown-out buffers, freed at destruction
};

void gemm(Stager& S, hipStream_t st, bool ta, bool tb, const std::vector<Gemm>& g);
void gemv(Stager& S, hipStream_t st, bool trans, const std::vector<Gemv>& g);
void cholesky(Stager& S, hipStream_t st, const std::vector<Chol>& c);
void trsm_right_lt(Stager& S, hipStream_t st, const std::vector<TrsmRLT>& t);
// mark(k), k = 0..4, is called between the phases (tridiagonalisation,
// eigenpairs of the tridiagonal, orthogonalisation, back-transform, end)
void eigh(Stager& S, hipStream_t st, const std::vector<Eigh>& e,
          const std::function<void(int)>& mark = nullptr);

}  // namespace oila
