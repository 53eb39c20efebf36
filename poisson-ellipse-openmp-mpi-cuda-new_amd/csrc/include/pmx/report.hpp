// Output: reference-compatible stdout lines, ASCII solution/error dumps, accuracy norms,
// one-line JSON summaries (components X3, X7 of SURVEY §2.6 and §5.5/§5.6).
//
// Reference formats kept byte-compatible:
//   stage 0/1: "Converged after k iterations (||w(k+1)-w(k)|| < δ)."     stage0/Withoutopenmp1.cpp:157-158
//             "M=40, N=40 | Iter=61 | Time=0.0034 s"                     stage0/Withoutopenmp1.cpp:189-192
//   stage 1 : banner + "Threads =  4 | Time = 0.123 s"                  stage1-openmp/Withopenmp1.cpp:208-224
//   stage 2 : "Pure MPI 2D run with P processes; M=.., N=.."            stage2-mpi/poisson_mpi_decomp.cpp:476-477
//   stage 3 : "MPI/OpenMP run with P MPI processes; M=.., N=.."         stage3-openmp+mpi/hybrid.cpp:486-487
//   stage 2-4: "Converged after k iterations (||w(k+1)-w(k)|| < 1e-06)." stage2-mpi/poisson_mpi_decomp.cpp:444-445
//   stage 2/3: "M=.., N=.. | Iter=.. | Time=%.6f s"                     stage2-mpi/poisson_mpi_decomp.cpp:494-497
//   stage 4 : "MPI + CUDA 2D run with P processes; M=.., N=.." + 5 bucket lines + "Total Time" block
//                                                                       stage4-mpi+cuda/poisson_mpi_cuda_f.cu:970-979,1002-1003,1028-1034
// The reference never writes the solution; the ASCII dump is new: gnuplot-friendly
// "x y w u_exact err" rows with a blank line between x-rows, then an error footer.
#pragma once

#include <cmath>
#include <cstdio>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "pmx/geometry.hpp"
#include "pmx/spec.hpp"

namespace pmx {

struct ErrorNorms {
  double l2 = 0, max_err = 0, max_w = 0;
};

// Error of a global (M+1) x (N+1) solution against the analytic one inside D (h-weighted L2).
inline ErrorNorms error_norms(const ProblemSpec& s, const std::vector<double>& w) {
  const GridInfo g(s);
  const geo::FaceTables t(s, g);
  ErrorNorms e;
  double sum = 0.0;
  for (int i = 0; i <= s.M; ++i)
    for (int j = 0; j <= s.N; ++j) {
      const double wij = w[size_t(i) * (s.N + 1) + j];
      e.max_w = std::max(e.max_w, wij);
      if (!geo::inside(t.x[i], t.y[j], s.ax, s.by, s.reference_ellipse())) continue;
      const double d = wij - geo::exact_solution(t.x[i], t.y[j], s);
      sum += d * d;
      e.max_err = std::max(e.max_err, std::fabs(d));
    }
  e.l2 = std::sqrt(sum * g.h1 * g.h2);
  return e;
}

inline void write_ascii(const std::string& path, const ProblemSpec& s, const std::vector<double>& w,
                        int stride, int64_t iters) {
  std::ofstream f(path);
  if (!f) throw Error("cannot open dump file " + path);
  const GridInfo g(s);
  const geo::FaceTables t(s, g);
  const ErrorNorms e = error_norms(s, w);
  stride = std::max(1, stride);
  f << "# pmx solution: M=" << s.M << " N=" << s.N << " ellipse ax=" << s.ax << " by=" << s.by
    << " F=" << s.F << " iters=" << iters << "\n# columns: x y w u_exact err\n";
  f << std::setprecision(12);
  for (int i = 0; i <= s.M; i += stride) {
    for (int j = 0; j <= s.N; j += stride) {
      const double wij = w[size_t(i) * (s.N + 1) + j];
      const double u = geo::exact_solution(t.x[i], t.y[j], s);
      f << t.x[i] << ' ' << t.y[j] << ' ' << wij << ' ' << u << ' ' << (wij - u) << '\n';
    }
    f << '\n';
  }
  f << "# L2_error_in_D=" << e.l2 << " max_error_in_D=" << e.max_err << " max_w=" << e.max_w << '\n';
}

// symbolic: stages 0/1 print the literal "δ" (stage0/Withoutopenmp1.cpp:157-158,
// stage1-openmp/Withopenmp1.cpp:192); stages 2-4 print the value with default stream formatting
inline void print_converged(int64_t k, double delta, bool symbolic) {
  if (symbolic) {
    std::cout << "Converged after " << k << " iterations (||w(k+1)-w(k)|| < δ)." << std::endl;
  } else {
    std::ostringstream d;  // independent of any std::fixed left on std::cout
    d << delta;
    std::cout << "Converged after " << k << " iterations (||w(k+1)-w(k)|| < " << d.str() << ").\n";
  }
}

struct JsonLine {
  std::ostringstream os;
  bool first = true;
  JsonLine() { os << std::setprecision(10) << '{'; }
  template <typename V>
  JsonLine& kv(const std::string& k, const V& v) {
    os << (first ? "" : ", ") << '"' << k << "\": " << v;
    first = false;
    return *this;
  }
  JsonLine& ks(const std::string& k, const std::string& v) {
    os << (first ? "" : ", ") << '"' << k << "\": \"" << v << '"';
    first = false;
    return *this;
  }
  std::string str() { return os.str() + "}"; }
};

}  // namespace pmx
