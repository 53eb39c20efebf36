// CPU PCG oracle (serial / OpenMP / decomposed).  See pmx/cpu_pcg.hpp.
//
// The arithmetic of every operator reproduces the reference exactly:
//   mat_A  stage0/Withoutopenmp1.cpp:83-85  (-1/h1 * (a(w+-w)/h1 - ...))
//   mat_D  stage0/Withoutopenmp1.cpp:98-99  (D = (a+a)/(h1*h1) + (b+b)/(h2*h2), z = r/D)
//   dot    stage0/Withoutopenmp1.cpp:64-72  (sum * h1 * h2)
// so serial runs are bit-identical to the reference and reproduce its iteration
// counts (15/26/50/546/989 weighted, 17/31/61/801 unweighted).
#include "pmx/cpu_pcg.hpp"

#include <chrono>
#include <cmath>
#include <cstring>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace pmx {
namespace {

struct Timer {
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  double seconds() const {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
};

inline double norm_of(double sum_sq, const ProblemSpec& s, const GridInfo& g) {
  // stage0/Withoutopenmp1.cpp:154 (unweighted) vs stage2-mpi/poisson_mpi_decomp.cpp:440 (weighted)
  return s.norm == Norm::kWeighted ? std::sqrt(sum_sq * g.h1 * g.h2) : std::sqrt(sum_sq);
}

inline bool breakdown(double denom, const ProblemSpec& s) {
  // stage0/Withoutopenmp1.cpp:128 vs stage2-mpi/poisson_mpi_decomp.cpp:413
  return s.norm == Norm::kWeighted ? std::fabs(denom) < s.breakdown_tol : denom < s.breakdown_tol;
}

}  // namespace

void cpu_assemble(const ProblemSpec& spec, std::vector<double>& a, std::vector<double>& b,
                  std::vector<double>& B) {
  spec.validate();
  const GridInfo g(spec);
  const geo::FaceTables t(spec, g);
  const int M = spec.M, N = spec.N, pa = N + 2, pB = N + 1;
  a.assign(size_t(M + 2) * pa, 0.0);
  b.assign(size_t(M + 2) * pa, 0.0);
  B.assign(size_t(M + 1) * pB, 0.0);
  for (int i = 0; i <= M + 1; ++i)
    for (int j = 0; j <= N + 1; ++j) {
      a[size_t(i) * pa + j] = geo::coef_a(t, g, i, j);
      b[size_t(i) * pa + j] = geo::coef_b(t, g, i, j);
    }
  for (int i = 1; i <= M - 1; ++i)
    for (int j = 1; j <= N - 1; ++j) B[size_t(i) * pB + j] = geo::rhs(t, spec, i, j);
}

SolveResult cpu_solve(const ProblemSpec& spec, int threads, bool keep_solution) {
  spec.validate();
  const GridInfo g(spec);
  const geo::FaceTables t(spec, g);
  const int M = spec.M, N = spec.N;
  const int P = N + 2;  // pitch; arrays (M+2) x (N+2), index i*P + j
  const size_t n = size_t(M + 2) * P;
  const double h1 = g.h1, h2 = g.h2;
  const int nt = threads < 1 ? 1 : threads;
  (void)nt;

  std::vector<double> a(n), b(n), w(n, 0.0), r(n, 0.0), z(n, 0.0), p(n, 0.0), Ap(n, 0.0),
      wprev(n, 0.0);
  for (int i = 0; i <= M + 1; ++i)
    for (int j = 0; j <= N + 1; ++j) {
      a[size_t(i) * P + j] = geo::coef_a(t, g, i, j);
      b[size_t(i) * P + j] = geo::coef_b(t, g, i, j);
    }
  for (int i = 1; i <= M - 1; ++i)
    for (int j = 1; j <= N - 1; ++j) r[size_t(i) * P + j] = geo::rhs(t, spec, i, j);

  Timer timer;
  auto dot = [&](const std::vector<double>& u, const std::vector<double>& v) {
    double sum = 0.0;
#pragma omp parallel for collapse(2) reduction(+ : sum) num_threads(nt) if (nt > 1)
    for (int i = 1; i <= M - 1; ++i)
      for (int j = 1; j <= N - 1; ++j) sum += u[size_t(i) * P + j] * v[size_t(i) * P + j];
    return sum * h1 * h2;
  };
  auto mat_D = [&]() {
#pragma omp parallel for collapse(2) num_threads(nt) if (nt > 1)
    for (int i = 1; i <= M - 1; ++i)
      for (int j = 1; j <= N - 1; ++j) {
        const size_t c = size_t(i) * P + j;
        const double D = (a[c + P] + a[c]) / (h1 * h1) + (b[c + 1] + b[c]) / (h2 * h2);
        z[c] = (D != 0.0) ? r[c] / D : 0.0;
      }
  };
  auto mat_A = [&]() {
#pragma omp parallel for collapse(2) num_threads(nt) if (nt > 1)
    for (int i = 1; i <= M - 1; ++i)
      for (int j = 1; j <= N - 1; ++j) {
        const size_t c = size_t(i) * P + j;
        const double Ax = -1.0 / h1 * (a[c + P] * (p[c + P] - p[c]) / h1 - a[c] * (p[c] - p[c - P]) / h1);
        const double Ay = -1.0 / h2 * (b[c + 1] * (p[c + 1] - p[c]) / h2 - b[c] * (p[c] - p[c - 1]) / h2);
        Ap[c] = Ax + Ay;
      }
  };

  mat_D();
  p = z;
  double zr_old = dot(z, r);
  SolveResult res;
  const int64_t max_iter = spec.effective_max_iter();
  for (int64_t k = 1; k <= max_iter; ++k) {
    res.iters = k;
    mat_A();
    const double denom = dot(Ap, p);
    if (breakdown(denom, spec)) { res.status = Status::kBreakdown; break; }
    const double alpha = zr_old / denom;
    double dsum = 0.0;
#pragma omp parallel for collapse(2) reduction(+ : dsum) num_threads(nt) if (nt > 1)
    for (int i = 1; i <= M - 1; ++i)
      for (int j = 1; j <= N - 1; ++j) {
        const size_t c = size_t(i) * P + j;
        const double w_old = w[c];
        w[c] = w_old + alpha * p[c];
        r[c] -= alpha * Ap[c];
        const double d = w[c] - w_old;
        dsum += d * d;
      }
    mat_D();
    const double zr_new = dot(z, r);
    res.last_diff = norm_of(dsum, spec, g);
    if (res.last_diff < spec.delta) { res.status = Status::kConverged; break; }
    const double beta = zr_new / zr_old;
    zr_old = zr_new;
#pragma omp parallel for collapse(2) num_threads(nt) if (nt > 1)
    for (int i = 1; i <= M - 1; ++i)
      for (int j = 1; j <= N - 1; ++j) {
        const size_t c = size_t(i) * P + j;
        p[c] = z[c] + beta * p[c];
      }
  }
  if (res.status == Status::kRunning) res.status = Status::kMaxIter;
  res.seconds = timer.seconds();
  if (keep_solution) {
    res.w.assign(size_t(M + 1) * (N + 1), 0.0);
    for (int i = 0; i <= M; ++i)
      for (int j = 0; j <= N; ++j) res.w[size_t(i) * (N + 1) + j] = w[size_t(i) * P + j];
  }
  return res;
}

// ---------------------------------------------------------------------------
// CpuSubdomain (stage2-mpi/poisson_mpi_decomp.cpp:124-232 semantics)
// ---------------------------------------------------------------------------

CpuSubdomain::CpuSubdomain(const ProblemSpec& spec, const Subdomain& sd, int threads)
    : spec_(spec), g_(spec), sd_(sd), threads_(threads < 1 ? 1 : threads) {
  const geo::FaceTables t(spec, g_);
  const int nx = sd.nx, ny = sd.ny, P = ny + 2;
  const size_t n = size_t(nx + 2) * P;
  a_.assign(n, 0.0); b_.assign(n, 0.0); B_.assign(n, 0.0);
  w_.assign(n, 0.0); r_.assign(n, 0.0); z_.assign(n, 0.0); p_.assign(n, 0.0); Ap_.assign(n, 0.0);
  // coefficients include the 1-cell halo, computed analytically (never communicated),
  // exactly like fic_reg_local (stage2-mpi/poisson_mpi_decomp.cpp:132-133)
  for (int li = 0; li <= nx + 1; ++li)
    for (int lj = 0; lj <= ny + 1; ++lj) {
      const int gi = sd.gi0() + li, gj = sd.gj0() + lj;
      a_[size_t(li) * P + lj] = geo::coef_a(t, g_, gi, gj);
      b_[size_t(li) * P + lj] = geo::coef_b(t, g_, gi, gj);
    }
  for (int li = 1; li <= nx; ++li)
    for (int lj = 1; lj <= ny; ++lj)
      B_[size_t(li) * P + lj] = geo::rhs(t, spec, sd.gi0() + li, sd.gj0() + lj);
}

double CpuSubdomain::init() {
  r_ = B_;
  std::fill(w_.begin(), w_.end(), 0.0);
  const double zr = precond_dot();
  p_ = z_;
  return zr;
}

double CpuSubdomain::matvec_dot() {
  const int nx = sd_.nx, ny = sd_.ny, P = ny + 2, nt = threads_;
  const double h1 = g_.h1, h2 = g_.h2;
  const double* a = a_.data(); const double* b = b_.data(); const double* p = p_.data();
  double* Ap = Ap_.data();
  double sum = 0.0;
#pragma omp parallel for collapse(2) reduction(+ : sum) num_threads(nt) if (nt > 1)
  for (int li = 1; li <= nx; ++li)
    for (int lj = 1; lj <= ny; ++lj) {
      const size_t c = size_t(li) * P + lj;
      const double Ax = -1.0 / h1 * (a[c + P] * (p[c + P] - p[c]) / h1 - a[c] * (p[c] - p[c - P]) / h1);
      const double Ay = -1.0 / h2 * (b[c + 1] * (p[c + 1] - p[c]) / h2 - b[c] * (p[c] - p[c - 1]) / h2);
      Ap[c] = Ax + Ay;
      sum += Ap[c] * p[c];
    }
  return sum * h1 * h2;
}

void CpuSubdomain::update_wr(double alpha, double* diff_local) {
  const int nx = sd_.nx, ny = sd_.ny, P = ny + 2, nt = threads_;
  double* w = w_.data(); double* r = r_.data();
  const double* p = p_.data(); const double* Ap = Ap_.data();
  double dsum = 0.0;
#pragma omp parallel for collapse(2) reduction(+ : dsum) num_threads(nt) if (nt > 1)
  for (int li = 1; li <= nx; ++li)
    for (int lj = 1; lj <= ny; ++lj) {
      const size_t c = size_t(li) * P + lj;
      const double w_old = w[c];
      w[c] = w_old + alpha * p[c];
      r[c] -= alpha * Ap[c];
      const double d = w[c] - w_old;
      dsum += d * d;
    }
  *diff_local = dsum;
}

double CpuSubdomain::precond_dot() {
  const int nx = sd_.nx, ny = sd_.ny, P = ny + 2, nt = threads_;
  const double h1 = g_.h1, h2 = g_.h2;
  const double* a = a_.data(); const double* b = b_.data(); const double* r = r_.data();
  double* z = z_.data();
  double sum = 0.0;
#pragma omp parallel for collapse(2) reduction(+ : sum) num_threads(nt) if (nt > 1)
  for (int li = 1; li <= nx; ++li)
    for (int lj = 1; lj <= ny; ++lj) {
      const size_t c = size_t(li) * P + lj;
      const double D = (a[c + P] + a[c]) / (h1 * h1) + (b[c + 1] + b[c]) / (h2 * h2);
      z[c] = (D != 0.0) ? r[c] / D : 0.0;
      sum += z[c] * r[c];
    }
  return sum * h1 * h2;
}

void CpuSubdomain::update_p(double beta) {
  const int nx = sd_.nx, ny = sd_.ny, P = ny + 2, nt = threads_;
  double* p = p_.data(); const double* z = z_.data();
#pragma omp parallel for collapse(2) num_threads(nt) if (nt > 1)
  for (int li = 1; li <= nx; ++li)
    for (int lj = 1; lj <= ny; ++lj) {
      const size_t c = size_t(li) * P + lj;
      p[c] = z[c] + beta * p[c];
    }
}

void CpuSubdomain::get_edge(int side, double* out) const {
  const int nx = sd_.nx, ny = sd_.ny, P = ny + 2;
  switch (side) {
    case 0: std::memcpy(out, &p_[size_t(1) * P + 1], sizeof(double) * ny); break;
    case 1: std::memcpy(out, &p_[size_t(nx) * P + 1], sizeof(double) * ny); break;
    case 2: for (int li = 1; li <= nx; ++li) out[li - 1] = p_[size_t(li) * P + 1]; break;
    case 3: for (int li = 1; li <= nx; ++li) out[li - 1] = p_[size_t(li) * P + ny]; break;
    default: PMX_CHECK(false, "bad side " << side);
  }
}

void CpuSubdomain::set_ghost(int side, const double* in) {
  const int nx = sd_.nx, ny = sd_.ny, P = ny + 2;
  switch (side) {
    case 0: std::memcpy(&p_[1], in, sizeof(double) * ny); break;
    case 1: std::memcpy(&p_[size_t(nx + 1) * P + 1], in, sizeof(double) * ny); break;
    case 2: for (int li = 1; li <= nx; ++li) p_[size_t(li) * P] = in[li - 1]; break;
    case 3: for (int li = 1; li <= nx; ++li) p_[size_t(li) * P + ny + 1] = in[li - 1]; break;
    default: PMX_CHECK(false, "bad side " << side);
  }
}

void CpuSubdomain::zero_ghost(int side) {
  std::vector<double> zeros(size_t(edge_len(side)), 0.0);
  set_ghost(side, zeros.data());
}

void CpuSubdomain::scatter_w_into(std::vector<double>& global) const {
  const int P = sd_.ny + 2, GP = sd_.N + 1;
  for (int li = 1; li <= sd_.nx; ++li)
    for (int lj = 1; lj <= sd_.ny; ++lj)
      global[size_t(sd_.gi0() + li) * GP + sd_.gj0() + lj] = w_[size_t(li) * P + lj];
}

// ---------------------------------------------------------------------------
// Lock-step PCG over subdomains (stage2-mpi/poisson_mpi_decomp.cpp:391-457)
// ---------------------------------------------------------------------------

SolveResult cpu_pcg_loop(const ProblemSpec& spec, std::vector<CpuSubdomain*>& local,
                         HostCollectives& coll) {
  const GridInfo g(spec);
  auto local_sum = [&](auto&& f) {
    double s = 0.0;
    for (auto* d : local) s += f(*d);  // fixed rank order -> deterministic
    return coll.allreduce_sum(s);
  };
  Timer timer;
  double zr_old = local_sum([](CpuSubdomain& d) { return d.init(); });
  SolveResult res;
  const int64_t max_iter = spec.effective_max_iter();
  for (int64_t k = 1; k <= max_iter; ++k) {
    res.iters = k;
    for (auto* d : local) coll.exchange_p_halos(*d);
    const double denom = local_sum([](CpuSubdomain& d) { return d.matvec_dot(); });
    if (breakdown(denom, spec)) { res.status = Status::kBreakdown; break; }
    const double alpha = zr_old / denom;
    double dl = 0.0;
    for (auto* d : local) { double x; d->update_wr(alpha, &x); dl += x; }
    const double zr_new = local_sum([](CpuSubdomain& d) { return d.precond_dot(); });
    res.last_diff = norm_of(coll.allreduce_sum(dl), spec, g);
    if (res.last_diff < spec.delta) { res.status = Status::kConverged; break; }
    const double beta = zr_new / zr_old;
    zr_old = zr_new;
    for (auto* d : local) d->update_p(beta);
  }
  if (res.status == Status::kRunning) res.status = Status::kMaxIter;
  res.seconds = timer.seconds();
  return res;
}

SolveResult cpu_solve_decomposed(const ProblemSpec& spec, int nranks, Split split,
                                 int threads_per_rank, bool keep_solution) {
  spec.validate();
  const ProcGrid pg = make_process_grid(nranks, spec.M, spec.N, split);
  std::vector<CpuSubdomain> subs;
  subs.reserve(nranks);
  for (int r = 0; r < nranks; ++r)
    subs.emplace_back(spec, decompose_2d(spec.M, spec.N, pg, r), threads_per_rank);
  std::vector<CpuSubdomain*> local;
  for (auto& s : subs) local.push_back(&s);

  HostCollectives coll;
  coll.allreduce_sum = [](double x) { return x; };  // all ranks are local
  coll.exchange_p_halos = [&](CpuSubdomain& d) {
    // opposite sides: 0<->1 (x), 2<->3 (y); tags as in stage2-mpi/poisson_mpi_decomp.cpp:249-252
    const Subdomain& s = d.sd();
    const int nb[4] = {s.nb_xlo, s.nb_xhi, s.nb_ylo, s.nb_yhi};
    for (int side = 0; side < 4; ++side) {
      if (nb[side] < 0) { d.zero_ghost(side); continue; }
      CpuSubdomain& o = subs[nb[side]];
      std::vector<double> buf(size_t(o.edge_len(side ^ 1)));
      o.get_edge(side ^ 1, buf.data());
      d.set_ghost(side, buf.data());
    }
  };
  SolveResult res = cpu_pcg_loop(spec, local, coll);
  if (keep_solution) {
    res.w.assign(size_t(spec.M + 1) * (spec.N + 1), 0.0);
    for (auto& s : subs) s.scatter_w_into(res.w);
  }
  return res;
}

}  // namespace pmx
