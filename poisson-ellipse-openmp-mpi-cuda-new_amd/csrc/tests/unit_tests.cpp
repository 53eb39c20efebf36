// Native unit tests of the host core (SURVEY §4.2 "unit (CPU)"): geometry, decomposition, CPU
// PCG goldens, report formats.  No framework: each CHECK prints file:line on failure and the
// binary exits non-zero.  Built as bin/pmx_unit_tests by utils/build.py and as a CTest target by
// CMakeLists.txt; tests/test_native_unit.py runs it under pytest.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <sstream>
#include <string>
#include <vector>

#include "pmx/cpu_pcg.hpp"
#include "pmx/decomp.hpp"
#include "pmx/geometry.hpp"
#include "pmx/report.hpp"
#include "pmx/spec.hpp"

namespace {

int g_failed = 0, g_checks = 0;

#define CHECK(cond)                                                         \
  do {                                                                      \
    ++g_checks;                                                             \
    if (!(cond)) {                                                          \
      ++g_failed;                                                           \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
    }                                                                       \
  } while (0)

using namespace pmx;

// stage2-mpi/poisson_mpi_decomp.cpp:60-64: Px = floor(sqrt(P)), decremented until it divides P
void test_process_grid() {
  const int expect[][3] = {{1, 1, 1}, {2, 1, 2}, {3, 1, 3}, {4, 2, 2}, {6, 2, 3},
                           {7, 1, 7}, {8, 2, 4}, {12, 3, 4}, {16, 4, 4}, {20, 4, 5}};
  for (const auto& e : expect) {
    const ProcGrid g = choose_process_grid(e[0]);
    CHECK(g.Px == e[1] && g.Py == e[2]);
  }
  CHECK(make_process_grid(8, 16384, 16384, Split::kRows).Px == 8);
  CHECK(make_process_grid(8, 16384, 16384, Split::kCols).Py == 8);
}

// every interior node owned exactly once; sizes differ by <= 1; neighbours are symmetric
void test_decomposition_cover() {
  for (int P : {1, 2, 3, 4, 6, 7, 8, 12}) {
    const int M = 97, N = 131;
    const ProcGrid g = choose_process_grid(P);
    std::vector<int> owner(size_t(M + 1) * (N + 1), -1);
    int nx_min = 1 << 30, nx_max = 0, ny_min = 1 << 30, ny_max = 0;
    for (int r = 0; r < P; ++r) {
      const Subdomain d = decompose_2d(M, N, g, r);
      nx_min = std::min(nx_min, d.nx); nx_max = std::max(nx_max, d.nx);
      ny_min = std::min(ny_min, d.ny); ny_max = std::max(ny_max, d.ny);
      for (int i = d.i_start; i <= d.i_end; ++i)
        for (int j = d.j_start; j <= d.j_end; ++j) {
          int& o = owner[size_t(i) * (N + 1) + j];
          CHECK(o == -1);
          o = r;
        }
      const int nbs[4] = {d.nb_xlo, d.nb_xhi, d.nb_ylo, d.nb_yhi};
      for (int s = 0; s < 4; ++s) {
        if (nbs[s] < 0) continue;
        const Subdomain n = decompose_2d(M, N, g, nbs[s]);
        const int back[4] = {n.nb_xlo, n.nb_xhi, n.nb_ylo, n.nb_yhi};
        CHECK(back[s ^ 1] == r);
      }
    }
    for (int i = 1; i < M; ++i)
      for (int j = 1; j < N; ++j) CHECK(owner[size_t(i) * (N + 1) + j] >= 0);
    CHECK(nx_max - nx_min <= 1 && ny_max - ny_min <= 1);
  }
}

// coefficient invariants: 1 deep inside D, 1/eps far outside, symmetric about both axes
void test_geometry() {
  ProblemSpec s;
  s.M = 80; s.N = 60;
  const GridInfo g(s);
  const geo::FaceTables t(s, g);
  CHECK(geo::inside(0.0, 0.0, s.ax, s.by, true));
  CHECK(!geo::inside(0.99, 0.45, s.ax, s.by, true));
  CHECK(geo::coef_a(t, g, s.M / 2, s.N / 2) == 1.0);
  CHECK(geo::coef_b(t, g, s.M / 2, s.N / 2) == 1.0);
  CHECK(geo::coef_a(t, g, 1, 1) == g.inv_eps);
  for (int i = 1; i <= s.M; ++i)
    for (int j = 1; j <= s.N; ++j) {
      // a(i, j) uses the face at x_i - h1/2: mirror i -> M + 1 - i, j -> N - j
      const double a = geo::coef_a(t, g, i, j), am = geo::coef_a(t, g, s.M + 1 - i, s.N - j);
      CHECK(std::fabs(a - am) <= 1e-9 * std::fabs(a));
    }
  // analytic solution vanishes on the ellipse, F / (2/ax^2 + 2/by^2) at the centre
  CHECK(std::fabs(geo::exact_solution(0.0, 0.0, s) - 0.1) < 1e-15);
  CHECK(geo::exact_solution(1.0, 0.0, s) == 0.0);
}

// SURVEY §4.1 goldens (reproduced from the reference code)
void test_cpu_goldens() {
  const int weighted[][3] = {{10, 10, 15}, {20, 20, 26}, {40, 40, 50}};
  for (const auto& e : weighted) {
    ProblemSpec s;
    s.M = e[0]; s.N = e[1];
    const SolveResult r = cpu_solve(s, 1, true);
    CHECK(r.status == Status::kConverged && r.iters == e[2]);
  }
  const int unweighted[][3] = {{10, 10, 17}, {20, 20, 31}, {40, 40, 61}};
  for (const auto& e : unweighted) {
    ProblemSpec s;
    s.M = e[0]; s.N = e[1]; s.norm = Norm::kUnweighted;
    CHECK(cpu_solve(s, 1, false).iters == e[2]);
  }
  ProblemSpec s;  // 40x40: max w and error vs analytic
  const SolveResult r = cpu_solve(s, 1, true);
  const ErrorNorms e = error_norms(s, r.w);
  CHECK(std::fabs(e.max_w - 0.09797040155) < 1e-9);
  CHECK(std::fabs(e.l2 - 3.6773e-3) < 1e-7);
  // threaded decomposition reproduces the serial solve
  const SolveResult d = cpu_solve_decomposed(s, 4, Split::kReference, 1, true);
  CHECK(d.iters == r.iters);
  double dmax = 0.0;
  for (size_t k = 0; k < r.w.size(); ++k) dmax = std::max(dmax, std::fabs(d.w[k] - r.w[k]));
  CHECK(dmax < 1e-12);
}

void test_report_formats() {
  JsonLine j;
  j.ks("backend", "cpu").kv("M", 40).kv("x", 0.125);
  CHECK(j.str() == "{\"backend\": \"cpu\", \"M\": 40, \"x\": 0.125}");
  CHECK(std::string(status_name(Status::kConverged)) == "converged");
  CHECK(std::string(status_name(Status::kBreakdown)) == "breakdown");
}

void test_spec_validation() {
  ProblemSpec s;
  s.M = 1;
  bool threw = false;
  try { s.validate(); } catch (const Error&) { threw = true; }
  CHECK(threw);
  ProblemSpec t;
  CHECK(t.effective_max_iter() == 39 * 39);
  t.max_iter = 7;
  CHECK(t.effective_max_iter() == 7);
}

}  // namespace

int main() {
  test_process_grid();
  test_decomposition_cover();
  test_geometry();
  test_cpu_goldens();
  test_report_formats();
  test_spec_validation();
  std::printf("pmx_unit_tests: %d checks, %d failed\n", g_checks, g_failed);
  return g_failed ? 1 : 0;
}
