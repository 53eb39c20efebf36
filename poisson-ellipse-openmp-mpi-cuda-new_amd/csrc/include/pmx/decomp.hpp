// 2D block domain decomposition (component P2 of SURVEY §2.2).
//
// Reference: choose_process_grid  stage2-mpi/poisson_mpi_decomp.cpp:60-64
//            decompose_2d         stage2-mpi/poisson_mpi_decomp.cpp:75-111
//            neighbour map        stage2-mpi/poisson_mpi_decomp.cpp:246-252
// The default process grid is identical to the reference (P=2 -> 1x2, 4 -> 2x2,
// 8 -> 2x4).  `Split::kAuto` instead cuts only the slow (row) axis while the strips stay
// >= kMinStripRows tall, else minimises the halo perimeter.
#pragma once

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "pmx/common.hpp"

namespace pmx {

enum class Split : int { kReference = 0, kAuto = 1, kRows = 2, kCols = 3 };

struct ProcGrid {
  int Px = 1, Py = 1;
  int size() const { return Px * Py; }
};

// stage2-mpi/poisson_mpi_decomp.cpp:60-64
inline ProcGrid choose_process_grid(int size) {
  PMX_CHECK(size >= 1, "process count must be >= 1");
  ProcGrid g;
  g.Px = static_cast<int>(std::sqrt(static_cast<double>(size)));
  while (g.Px > 1 && size % g.Px != 0) --g.Px;
  g.Py = size / g.Px;
  return g;
}

// Split::kAuto uses row strips while they are at least this many rows tall (see make_process_grid)
constexpr int kMinStripRows = 128;

inline ProcGrid make_process_grid(int size, int M, int N, Split split) {
  if (split == Split::kReference) return choose_process_grid(size);
  if (split == Split::kRows) return ProcGrid{size, 1};
  if (split == Split::kCols) return ProcGrid{1, size};
  // kAuto: row strips (py = 1, the longest contiguous rows) when every strip keeps at least
  // kMinStripRows rows.  The sweep streams whole rows, so at equal points per rank long rows are
  // faster: 2048x16384 strips 337.6 us/iter vs 4096x8192 blocks 356.9 and 8192x4096 378.9
  // (profiles/r2/small_shapes/README.md); the ghost exchange (~32 B per column per side in fp64)
  // runs under the interior sweep and stays well below it while strips are >= 128 rows tall.
  // Otherwise: the least halo perimeter (nx + ny), ties -> more x cuts (x halos are contiguous
  // rows in our row-major [i][j] layout).
  if ((M - 1) / size >= kMinStripRows) return ProcGrid{size, 1};
  ProcGrid best{size, 1};
  double best_cost = 1e300;
  for (int px = 1; px <= size; ++px) {
    if (size % px) continue;
    const int py = size / px;
    const double nx = double(M - 1) / px, ny = double(N - 1) / py;
    const double cost = (px > 1 ? 2.0 * ny : 0.0) + (py > 1 ? 2.0 * nx * 1.0001 : 0.0);
    if (cost < best_cost) { best_cost = cost; best = ProcGrid{px, py}; }
  }
  return best;
}

struct Subdomain {
  int M = 0, N = 0;
  ProcGrid grid;
  int rank = 0, px = 0, py = 0;
  int i_start = 1, i_end = 0, j_start = 1, j_end = 0;  // global interior ranges (inclusive)
  int nx = 0, ny = 0;                                   // local interior sizes
  // neighbour ranks (-1 = global Dirichlet boundary); x = slow/row axis, y = contiguous axis
  int nb_xlo = -1, nb_xhi = -1, nb_ylo = -1, nb_yhi = -1;

  // global index of local (li, lj): gi = i_start - 1 + li  (li = 0 .. nx+1)
  int gi0() const { return i_start - 1; }
  int gj0() const { return j_start - 1; }
  // rank across halo slot s (pmx/device_types.hpp kHaloSlots: 4 sides, then 4 corners), or -1
  int peer(int s) const {
    static constexpr int dx[8] = {-1, 1, 0, 0, -1, -1, 1, 1};
    static constexpr int dy[8] = {0, 0, -1, 1, -1, 1, -1, 1};
    const int qx = px + dx[s], qy = py + dy[s];
    return (qx >= 0 && qx < grid.Px && qy >= 0 && qy < grid.Py) ? qy * grid.Px + qx : -1;
  }
  double aspect() const {
    return nx > 0 && ny > 0 ? double(std::max(nx, ny)) / double(std::min(nx, ny)) : 0.0;
  }
};

// stage2-mpi/poisson_mpi_decomp.cpp:75-111 (block sizes differ by at most 1,
// rank -> (px = rank % Px, py = rank / Px)).
inline Subdomain decompose_2d(int M, int N, ProcGrid g, int rank) {
  PMX_CHECK(rank >= 0 && rank < g.size(), "rank " << rank << " outside process grid");
  PMX_CHECK(M - 1 >= g.Px && N - 1 >= g.Py,
            "grid " << M << "x" << N << " too small for " << g.Px << "x" << g.Py << " ranks");
  Subdomain d;
  d.M = M; d.N = N; d.grid = g; d.rank = rank;
  d.px = rank % g.Px;
  d.py = rank / g.Px;
  auto split = [](int total, int parts, int idx, int& start, int& end) {
    const int base = total / parts, rem = total % parts;
    int off = 1;
    for (int k = 0; k < idx; ++k) off += base + (k < rem ? 1 : 0);
    const int n = base + (idx < rem ? 1 : 0);
    start = off;
    end = off + n - 1;
  };
  split(M - 1, g.Px, d.px, d.i_start, d.i_end);
  split(N - 1, g.Py, d.py, d.j_start, d.j_end);
  d.nx = d.i_end - d.i_start + 1;
  d.ny = d.j_end - d.j_start + 1;
  d.nb_xlo = d.px > 0 ? rank - 1 : -1;
  d.nb_xhi = d.px < g.Px - 1 ? rank + 1 : -1;
  d.nb_ylo = d.py > 0 ? rank - g.Px : -1;
  d.nb_yhi = d.py < g.Py - 1 ? rank + g.Px : -1;
  return d;
}

}  // namespace pmx
