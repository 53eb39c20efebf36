// pmx_mpi — CPU MPI / MPI+OpenMP backend (stages 2 and 3 of the reference).
//
// Same CpuSubdomain phases as the in-process driver (csrc/cpu/cpu_pcg.cpp), with real MPI
// collectives: MPI_Allreduce for the scalars (stage2-mpi/poisson_mpi_decomp.cpp:396,412,435,439)
// and non-blocking 4-neighbour ghost exchange of p (stage2-mpi/poisson_mpi_decomp.cpp:241-347,
// same tag scheme :249-252).  Output lines match the reference banners.
//
//   mpirun -np 4 pmx_mpi 800 1200 [--threads T] [--split reference|auto|rows|cols]
//          [--norm weighted|unweighted] [--json] [--dump FILE] [--dump-stride S] [--phases]
//
// --phases: per-rank time split into compute / halo exchange / all-reduce (the all-reduce bucket
// includes waiting for the slowest rank), reduced with MPI_MAX over ranks and printed by rank 0 in
// the reference's "(max over ranks)" style (stage4-mpi+cuda/poisson_mpi_cuda_f.cu:956-980).
#include <mpi.h>

#include <cstdlib>
#include <cstring>
#include <iomanip>
#include <iostream>
#include <string>
#include <vector>

#include "pmx/cpu_pcg.hpp"
#include "pmx/report.hpp"

using namespace pmx;

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rank = 0, size = 1;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  ProblemSpec spec;
  int threads = 1, stride = 1;
  bool json = false, phases = false;
  std::string dump;
  Split split = Split::kReference;
  std::vector<std::string> pos;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto val = [&]() { return std::string(i + 1 < argc ? argv[++i] : ""); };
    if (a == "--threads") threads = std::atoi(val().c_str());
    else if (a == "--json") json = true;
    else if (a == "--phases") phases = true;
    else if (a == "--dump") dump = val();
    else if (a == "--dump-stride") stride = std::atoi(val().c_str());
    else if (a == "--norm") spec.norm = val() == "unweighted" ? Norm::kUnweighted : Norm::kWeighted;
    else if (a == "--split") {
      const std::string v = val();
      split = v == "auto" ? Split::kAuto : v == "rows" ? Split::kRows : v == "cols" ? Split::kCols : Split::kReference;
    } else if (a == "--delta") spec.delta = std::atof(val().c_str());
    else if (a == "--max-iter") spec.max_iter = std::atoll(val().c_str());
    else if (a == "--breakdown-tol") spec.breakdown_tol = std::atof(val().c_str());
    else pos.push_back(a);
  }
  if (pos.size() >= 2) {
    spec.M = std::atoi(pos[0].c_str());
    spec.N = std::atoi(pos[1].c_str());
  }
  try {
    spec.validate();
    if (rank == 0) {
      if (threads > 1)
        std::cout << "MPI/OpenMP run with " << size << " MPI processes; M=" << spec.M << ", N=" << spec.N << std::endl;
      else
        std::cout << "Pure MPI 2D run with " << size << " processes; M=" << spec.M << ", N=" << spec.N << std::endl;
    }
    const ProcGrid pg = make_process_grid(size, spec.M, spec.N, split);
    CpuSubdomain sub(spec, decompose_2d(spec.M, spec.N, pg, rank), threads);
    std::vector<CpuSubdomain*> local{&sub};
    HostCollectives coll;
    double t_allreduce = 0.0, t_halo = 0.0;
    coll.allreduce_sum = [&](double x) {
      double y = 0.0;
      const double t = MPI_Wtime();
      MPI_Allreduce(&x, &y, 1, MPI_DOUBLE, MPI_SUM, MPI_COMM_WORLD);
      t_allreduce += MPI_Wtime() - t;
      return y;
    };
    std::vector<std::vector<double>> sbuf(4), rbuf(4);
    coll.exchange_p_halos = [&](CpuSubdomain& d) {
      const double t = MPI_Wtime();
      const Subdomain& s = d.sd();
      const int nb[4] = {s.nb_xlo, s.nb_xhi, s.nb_ylo, s.nb_yhi};
      MPI_Request req[8];
      int nreq = 0;
      for (int side = 0; side < 4; ++side) {
        if (nb[side] < 0) { d.zero_ghost(side); continue; }
        const int len = d.edge_len(side);
        sbuf[side].resize(len);
        rbuf[side].resize(len);
        d.get_edge(side, sbuf[side].data());
        // tag = sender's side (0 left, 1 right, 2 down, 3 up): stage2-mpi/poisson_mpi_decomp.cpp:249-252
        MPI_Irecv(rbuf[side].data(), len, MPI_DOUBLE, nb[side], side ^ 1, MPI_COMM_WORLD, &req[nreq++]);
        MPI_Isend(sbuf[side].data(), len, MPI_DOUBLE, nb[side], side, MPI_COMM_WORLD, &req[nreq++]);
      }
      MPI_Waitall(nreq, req, MPI_STATUSES_IGNORE);
      for (int side = 0; side < 4; ++side)
        if (nb[side] >= 0) d.set_ghost(side, rbuf[side].data());
      t_halo += MPI_Wtime() - t;
    };
    MPI_Barrier(MPI_COMM_WORLD);
    const double t0 = MPI_Wtime();
    SolveResult r = cpu_pcg_loop(spec, local, coll);
    MPI_Barrier(MPI_COMM_WORLD);
    const double elapsed = MPI_Wtime() - t0;
    // per-rank buckets, MAX over ranks (each bucket's slowest rank, as the reference reports them)
    const double mine[3] = {elapsed - t_halo - t_allreduce, t_halo, t_allreduce};
    double tmax[3] = {0.0, 0.0, 0.0};
    MPI_Reduce(mine, tmax, 3, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
    // gather the solution on rank 0 (sum of disjoint scattered pieces)
    std::vector<double> w(size_t(spec.M + 1) * (spec.N + 1), 0.0), g;
    if (json || !dump.empty()) {
      sub.scatter_w_into(w);
      if (rank == 0) g.assign(w.size(), 0.0);
      MPI_Reduce(w.data(), rank == 0 ? g.data() : nullptr, int(w.size()), MPI_DOUBLE, MPI_SUM, 0, MPI_COMM_WORLD);
    }
    if (rank == 0) {
      if (r.status == Status::kConverged) print_converged(r.iters, spec.delta, false);
      std::cout << "M=" << spec.M << ", N=" << spec.N << " | Iter=" << r.iters << " | Time=" << std::fixed
                << std::setprecision(6) << elapsed << " s\n";
      if (phases)
        std::cout << "   Compute time (stencil + updates, max over ranks) ~ " << tmax[0] << " s\n"
                  << "   MPI halo exchange time (max over ranks)         ~ " << tmax[1] << " s\n"
                  << "   MPI_Allreduce time (dots, max over ranks)       ~ " << tmax[2] << " s\n";
      if (!dump.empty()) write_ascii(dump, spec, g, stride, r.iters);
      if (json) {
        const ErrorNorms e = error_norms(spec, g);
        JsonLine j;
        j.ks("backend", "mpi").kv("M", spec.M).kv("N", spec.N).kv("ranks", size).kv("threads", threads)
            .kv("iters", r.iters).ks("status", status_name(r.status)).kv("seconds", elapsed)
            .kv("mlups", double(spec.M - 1) * (spec.N - 1) * r.iters / elapsed / 1e6)
            .kv("l2_error", e.l2).kv("max_error", e.max_err).kv("max_w", e.max_w)
            .kv("t_compute_max", tmax[0]).kv("t_halo_max", tmax[1]).kv("t_allreduce_max", tmax[2]);
        std::cout << j.str() << std::endl;
      }
    }
  } catch (const std::exception& e) {
    std::cerr << "rank " << rank << ": " << e.what() << std::endl;
    MPI_Abort(MPI_COMM_WORLD, 1);
  }
  MPI_Finalize();
  return 0;
}
