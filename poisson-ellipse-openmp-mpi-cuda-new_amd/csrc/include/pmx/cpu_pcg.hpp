// CPU PCG — the validation oracle and the "no-GPU" configuration
// (components C4-C10 and P1 of SURVEY §2; stages 0/1/2/3 of the reference).
//
//  * cpu_solve()            : global grid, serial or OpenMP (stage 0 / stage 1 semantics,
//                             stage0/Withoutopenmp1.cpp:106-172, stage1-openmp/Withopenmp1.cpp:133-199)
//  * CpuSubdomain           : one rank's block with a 1-cell halo, phase-structured so the same
//                             code runs under an in-process multi-subdomain driver
//                             (cpu_solve_decomposed) and under MPI (apps/pmx_mpi.cpp)
//                             (stage2-mpi/poisson_mpi_decomp.cpp:356-460, stage3-openmp+mpi/hybrid.cpp:364-470)
#pragma once

#include <cstdint>
#include <functional>
#include <vector>

#include "pmx/decomp.hpp"
#include "pmx/geometry.hpp"
#include "pmx/spec.hpp"

namespace pmx {

struct SolveResult {
  int64_t iters = 0;
  Status status = Status::kRunning;
  double last_diff = 0.0;  // final ||w^{k+1}-w^k|| (norm per spec.norm)
  double seconds = 0.0;    // solver wall time
  // solution on the global grid, (M+1) x (N+1) row-major, boundary = 0
  std::vector<double> w;
};

// Serial (threads<=1) or OpenMP PCG over the whole grid.
SolveResult cpu_solve(const ProblemSpec& spec, int threads = 1, bool keep_solution = true);

// Assemble the reference's 2D arrays on the host (tests: kernel bit-equality).
// a, b are (M+2) x (N+2) including ghost nodes; B is (M+1) x (N+1).
void cpu_assemble(const ProblemSpec& spec, std::vector<double>& a, std::vector<double>& b,
                  std::vector<double>& B);

// One rank's block (local arrays (nx+2) x (ny+2), row-major, pitch ny+2).
class CpuSubdomain {
 public:
  CpuSubdomain(const ProblemSpec& spec, const Subdomain& sd, int threads);

  const Subdomain& sd() const { return sd_; }
  int pitch() const { return sd_.ny + 2; }

  double init();                         // r=B, z=D^-1 r, p=z, w=0 -> local (z,r)
  double matvec_dot();                   // Ap = A p (needs p halos) -> local (Ap,p)
  void update_wr(double alpha, double* diff_local);   // w+=ap, r-=aAp, local sum dw^2
  double precond_dot();                  // z = D^-1 r -> local (z,r)
  void update_p(double beta);            // p = z + beta p

  // halo access for p (the only field with halos, stage2-mpi/poisson_mpi_decomp.cpp:241-347)
  // side: 0 = x-lo (row 1), 1 = x-hi (row nx), 2 = y-lo (col 1), 3 = y-hi (col ny)
  int edge_len(int side) const { return side < 2 ? sd_.ny : sd_.nx; }
  void get_edge(int side, double* out) const;
  void set_ghost(int side, const double* in);
  void zero_ghost(int side);

  // gather local interior of w into a global (M+1)x(N+1) array
  void scatter_w_into(std::vector<double>& global) const;

 private:
  ProblemSpec spec_;
  GridInfo g_;
  Subdomain sd_;
  int threads_;
  std::vector<double> a_, b_, B_, w_, r_, z_, p_, Ap_;
};

// In-process multi-subdomain driver: P subdomains stepped in lock-step with a
// deterministic rank-ordered reduction.  This is the "fake cluster" used to test
// decomposition + halo logic without MPI (SURVEY §4.2 'distributed (fake)').
SolveResult cpu_solve_decomposed(const ProblemSpec& spec, int nranks, Split split,
                                 int threads_per_rank = 1, bool keep_solution = true);

// Generic lock-step PCG over CpuSubdomains with pluggable collectives.  The MPI
// app supplies MPI-backed callbacks; the in-process driver supplies local ones.
struct HostCollectives {
  std::function<double(double)> allreduce_sum;          // global sum of one double
  std::function<void(CpuSubdomain&)> exchange_p_halos;  // fill p ghosts (Dirichlet zero at boundary)
};
SolveResult cpu_pcg_loop(const ProblemSpec& spec, std::vector<CpuSubdomain*>& local,
                         HostCollectives& coll);

}  // namespace pmx
