// Geometry of the fictitious-domain method (components C2, C3, C4 of SURVEY §2.1).
//
// Reference behaviour (all stages carry a copy):
//   * domain predicate  x^2 + 4y^2 < 1            stage0/Withoutopenmp1.cpp:14-16
//   * face ∩ ellipse length (vertical/horizontal)  stage0/Withoutopenmp1.cpp:19-39,
//                                                  stage4-mpi+cuda/poisson_mpi_cuda_f.cu:46-76
//   * coefficient a_ij / b_ij from the face length stage0/Withoutopenmp1.cpp:53-54
//
// MI355X design: the 2D coefficient arrays a, b (and D) are never materialised
// on the device.  a_ij depends only on (x_i, y_j) through a *column-constant*
// clip root (the ellipse half-height at the face's x) and *row-constant* face
// ends, so we tabulate six 1D arrays (O(M+N) bytes) on the host and the HIP
// kernels rebuild a, b, D per point with a handful of min/max/compare ops
// (see csrc/hip/pcg_kernels.hip).  That removes 24 B/pt/iter of coefficient
// traffic relative to the reference's stored a/b arrays.
//
// Every function below reproduces the reference arithmetic order exactly and is
// compiled with FP contraction disabled, so host and device coefficients are
// bit-identical to the reference CPU code.
#pragma once

#include <cmath>
#include <limits>
#include <vector>

#include "pmx/spec.hpp"

#if defined(__HIPCC__)
#define PMX_HD __host__ __device__
#else
#define PMX_HD
#endif

#if defined(__clang__)
#define PMX_NO_CONTRACT _Pragma("clang fp contract(off)")
#else
#define PMX_NO_CONTRACT
#endif

namespace pmx {
namespace geo {

// std::min / std::max semantics (first argument wins ties) written out so the
// device code matches libstdc++ bit for bit, signed zeros included.
PMX_HD inline double smin(double a, double b) { return (b < a) ? b : a; }
PMX_HD inline double smax(double a, double b) { return (a < b) ? b : a; }

// Length of [lo, hi] ∩ [-root, root]; root = -inf encodes "the face's line misses
// the ellipse" (the reference's `lij = 0` branch).  Equals
// max(0, min(hi, root) - max(lo, -root))  (stage0/Withoutopenmp1.cpp:28,36).
PMX_HD inline double clip_len(double lo, double hi, double root) {
  PMX_NO_CONTRACT
  const double d = smin(hi, root) - smax(lo, -root);
  return smax(0.0, d);
}

// a_ij / b_ij from the face length l and the face size h
// (stage0/Withoutopenmp1.cpp:53-54; note the reference evaluates 1.0/eps inline).
PMX_HD inline double face_coef(double l, double h, double eps, double inv_eps) {
  PMX_NO_CONTRACT
  if (std::fabs(l - h) < 1e-9) return 1.0;
  if (l < 1e-9) return inv_eps;
  return (l / h) + (1.0 - l / h) / eps;
}

// Half-height of the ellipse on the vertical line x = x0, or -inf when the line
// misses it (stage0/Withoutopenmp1.cpp:22-27).
inline double vertical_root(double x0, double ax, double by, bool reference) {
  PMX_NO_CONTRACT
  if (reference) {
    if (std::fabs(x0) >= 1.0) return -std::numeric_limits<double>::infinity();
    return std::sqrt(std::max(0.0, (1.0 - x0 * x0) / 4.0));
  }
  if (std::fabs(x0) >= ax) return -std::numeric_limits<double>::infinity();
  const double t = x0 / ax;
  return by * std::sqrt(std::max(0.0, 1.0 - t * t));
}

// Half-width of the ellipse on the horizontal line y = y0 (stage0/Withoutopenmp1.cpp:30-35).
inline double horizontal_root(double y0, double ax, double by, bool reference) {
  PMX_NO_CONTRACT
  if (reference) {
    if (std::fabs(2.0 * y0) >= 1.0) return -std::numeric_limits<double>::infinity();
    return std::sqrt(std::max(0.0, 1.0 - 4.0 * y0 * y0));
  }
  if (std::fabs(y0) >= by) return -std::numeric_limits<double>::infinity();
  const double t = y0 / by;
  return ax * std::sqrt(std::max(0.0, 1.0 - t * t));
}

// Domain predicate (stage0/Withoutopenmp1.cpp:14-16), generalised to any axes.
PMX_HD inline bool inside(double x, double y, double ax, double by, bool reference) {
  PMX_NO_CONTRACT
  if (reference) return x * x + 4.0 * y * y < 1.0;
  const double u = x / ax, v = y / by;
  return u * u + v * v < 1.0;
}

// Analytic solution of -Δu = F in the ellipse, u = 0 on its boundary: used for
// accuracy reports (the reference states (1-x^2-4y^2)/10 in its report but never
// computes the error: итоговый отчёт/Этап_4_1213.pdf p.1).
inline double exact_solution(double x, double y, const ProblemSpec& s) {
  const double u = x / s.ax, v = y / s.by;
  const double q = 1.0 - u * u - v * v;
  return q > 0.0 ? s.F * q / (2.0 / (s.ax * s.ax) + 2.0 / (s.by * s.by)) : 0.0;
}

// Six 1D tables indexed by GLOBAL node index, covering ghost nodes 0..M+1 / 0..N+1.
//   a(i,j) = face_coef(clip_len(ylo[j], yhi[j], rv[i]), h2)   vertical face at x_i - h1/2
//   b(i,j) = face_coef(clip_len(xlo[i], xhi[i], rh[j]), h1)   horizontal face at y_j - h2/2
//   x[i], y[j] node coordinates (RHS predicate, ASCII dump)
struct FaceTables {
  std::vector<double> rv, xlo, xhi, x;  // size M+2
  std::vector<double> rh, ylo, yhi, y;  // size N+2

  FaceTables(const ProblemSpec& s, const GridInfo& g) {
    PMX_NO_CONTRACT
    const bool ref = s.reference_ellipse();
    rv.resize(s.M + 2); xlo.resize(s.M + 2); xhi.resize(s.M + 2); x.resize(s.M + 2);
    rh.resize(s.N + 2); ylo.resize(s.N + 2); yhi.resize(s.N + 2); y.resize(s.N + 2);
    for (int i = 0; i <= s.M + 1; ++i) {
      const double xi = s.A1 + i * g.h1;  // stage0/Withoutopenmp1.cpp:49
      x[i] = xi;
      xlo[i] = xi - 0.5 * g.h1;
      xhi[i] = xi + 0.5 * g.h1;
      rv[i] = vertical_root(xi - 0.5 * g.h1, s.ax, s.by, ref);
    }
    for (int j = 0; j <= s.N + 1; ++j) {
      const double yj = s.A2 + j * g.h2;  // stage0/Withoutopenmp1.cpp:50
      y[j] = yj;
      ylo[j] = yj - 0.5 * g.h2;
      yhi[j] = yj + 0.5 * g.h2;
      rh[j] = horizontal_root(yj - 0.5 * g.h2, s.ax, s.by, ref);
    }
  }
};

// Host versions of a_ij, b_ij, B_ij (the reference's fic_reg, stage0/Withoutopenmp1.cpp:42-61).
inline double coef_a(const FaceTables& t, const GridInfo& g, int i, int j) {
  return face_coef(clip_len(t.ylo[j], t.yhi[j], t.rv[i]), g.h2, g.eps, g.inv_eps);
}
inline double coef_b(const FaceTables& t, const GridInfo& g, int i, int j) {
  return face_coef(clip_len(t.xlo[i], t.xhi[i], t.rh[j]), g.h1, g.eps, g.inv_eps);
}
inline double rhs(const FaceTables& t, const ProblemSpec& s, int i, int j) {
  return inside(t.x[i], t.y[j], s.ax, s.by, s.reference_ellipse()) ? s.F : 0.0;
}

}  // namespace geo
}  // namespace pmx
