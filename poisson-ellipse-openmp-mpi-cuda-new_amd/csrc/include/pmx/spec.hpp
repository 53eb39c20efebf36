// Problem definition (component C1 + C11 of SURVEY.md §2.1).
//
// The reference hard-codes the box, the ellipse x^2+4y^2<1, F=1, delta=1e-6 and
// max_iter=(M-1)(N-1) in every stage (stage0/Withoutopenmp1.cpp:9-11,178,182;
// stage4-mpi+cuda/poisson_mpi_cuda_f.cu:11-13,1006-1007).  Here they are one
// CLI-overridable struct; the defaults reproduce the reference exactly.
#pragma once

#include <algorithm>
#include <cstdint>
#include <string>

#include "pmx/common.hpp"

namespace pmx {

// Stop-rule / breakdown-guard semantics of the reference stages.
//  kWeighted  : sqrt(h1*h2*sum dw^2) < delta, |denom| < breakdown_tol (1e-15)  (stages 1-4)
//  kUnweighted: sqrt(sum dw^2) < delta,        denom  < breakdown_tol (1e-15)  (stage 0)
enum class Norm : int { kWeighted = 0, kUnweighted = 1 };

enum class Status : int { kRunning = 0, kConverged = 1, kBreakdown = 2, kMaxIter = 3 };

inline const char* status_name(Status s) {
  switch (s) {
    case Status::kRunning: return "running";
    case Status::kConverged: return "converged";
    case Status::kBreakdown: return "breakdown";
    case Status::kMaxIter: return "max_iter";
  }
  return "?";
}

struct ProblemSpec {
  int M = 40, N = 40;                 // grid cells along x / y
  double A1 = -1.0, B1 = 1.0;         // box x-range  (stage0/Withoutopenmp1.cpp:9)
  double A2 = -0.6, B2 = 0.6;         // box y-range  (stage0/Withoutopenmp1.cpp:10)
  double ax = 1.0, by = 0.5;          // ellipse semi-axes: x^2/ax^2 + y^2/by^2 < 1
  double F = 1.0;                     // RHS value in D (stage0/Withoutopenmp1.cpp:11)
  double delta = 1e-6;                // stop tolerance (stage0/Withoutopenmp1.cpp:178)
  int64_t max_iter = -1;              // <0 -> (M-1)(N-1) (stage0/Withoutopenmp1.cpp:182)
  Norm norm = Norm::kWeighted;
  // CG breakdown guard on (A p, p): |denom| < tol (weighted) / denom < tol (unweighted), 1e-15 in
  // every reference stage (stage0/Withoutopenmp1.cpp:130, stage4-mpi+cuda/...:876).  The value is
  // absolute and (A p, p) shrinks like h^3 for this problem, so grids beyond ~100000^2 trip it at
  // the first iteration; lower it (e.g. 0) there.
  double breakdown_tol = 1e-15;

  int64_t effective_max_iter() const {
    return max_iter >= 0 ? max_iter : int64_t(M - 1) * int64_t(N - 1);
  }
  // The reference ellipse uses a specific arithmetic order (x*x + 4*y*y < 1,
  // sqrt((1-x0*x0)/4), sqrt(1-4*y0*y0)).  When the axes are the reference ones we
  // keep that order so coefficients are bit-identical to the reference.
  bool reference_ellipse() const { return ax == 1.0 && by == 0.5; }

  void validate() const {
    PMX_CHECK(M >= 2 && N >= 2, "grid must be at least 2x2 cells, got " << M << "x" << N);
    PMX_CHECK(B1 > A1 && B2 > A2, "empty box");
    PMX_CHECK(ax > 0 && by > 0, "ellipse semi-axes must be positive");
    PMX_CHECK(delta > 0, "delta must be positive");
    PMX_CHECK(breakdown_tol >= 0, "breakdown tolerance must be >= 0");
  }
};

// Derived grid quantities (stage0/Withoutopenmp1.cpp:107-108).
struct GridInfo {
  double h1, h2, eps, inv_eps, h1h2;
  explicit GridInfo(const ProblemSpec& s) {
    h1 = (s.B1 - s.A1) / s.M;
    h2 = (s.B2 - s.A2) / s.N;
    eps = std::max(h1, h2) * std::max(h1, h2);
    inv_eps = 1.0 / eps;
    h1h2 = h1 * h2;
  }
};

}  // namespace pmx
