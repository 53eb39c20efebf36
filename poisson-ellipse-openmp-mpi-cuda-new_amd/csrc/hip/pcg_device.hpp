// Device helpers shared by the HIP kernels: on-the-fly coefficients, Dirichlet
// masks, wave64/block reductions.
#pragma once

#include <hip/hip_runtime.h>

#include "pmx/device_types.hpp"
#include "pmx/geometry.hpp"

namespace pmx {
namespace dev {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

// a(gi, gj) / b(gi, gj) rebuilt from the 1D tables; bit-identical to the reference's
// fic_reg (stage0/Withoutopenmp1.cpp:51-54) because geo:: disables FP contraction.
__device__ __forceinline__ double coef_a(const DevTables& T, const DevGeom& G, int gi, int gj) {
  return geo::face_coef(geo::clip_len(T.ylo[gj], T.yhi[gj], T.rv[gi]), G.h2, G.eps, G.inv_eps);
}
__device__ __forceinline__ double coef_b(const DevTables& T, const DevGeom& G, int gi, int gj) {
  return geo::face_coef(geo::clip_len(T.xlo[gi], T.xhi[gi], T.rh[gj]), G.h1, G.eps, G.inv_eps);
}

// Row/column-split evaluation used in the marching kernels: the column terms
// (ylo, yhi, rh) live in registers for the whole tile, the row terms are uniform.
struct ColConst {
  double ylo, yhi, rh0, rh1;  // rh0 = rh[gj], rh1 = rh[gj+1]
};
struct RowConst {
  double rv0, rv1, xlo, xhi;  // rv0 = rv[gi], rv1 = rv[gi+1]
};
__device__ __forceinline__ ColConst load_col(const DevTables& T, int gj) {
  return ColConst{T.ylo[gj], T.yhi[gj], T.rh[gj], T.rh[gj + 1]};
}
__device__ __forceinline__ RowConst load_row(const DevTables& T, int gi) {
  return RowConst{T.rv[gi], T.rv[gi + 1], T.xlo[gi], T.xhi[gi]};
}
__device__ __forceinline__ double face_a(const ColConst& c, double rv, const DevGeom& G) {
  return geo::face_coef(geo::clip_len(c.ylo, c.yhi, rv), G.h2, G.eps, G.inv_eps);
}
__device__ __forceinline__ double face_b(const RowConst& r, double rh, const DevGeom& G) {
  return geo::face_coef(geo::clip_len(r.xlo, r.xhi, rh), G.h1, G.eps, G.inv_eps);
}

// Diagonal D_ij (stage0/Withoutopenmp1.cpp:98).  EXACT reproduces the reference's
// division order; the fast form multiplies by precomputed 1/h^2.
template <bool EXACT>
__device__ __forceinline__ double diag(double a0, double a1, double b0, double b1, const DevGeom& G) {
  if constexpr (EXACT) {
    PMX_NO_CONTRACT
    return (a1 + a0) / (G.h1 * G.h1) + (b1 + b0) / (G.h2 * G.h2);
  } else {
    return (a1 + a0) * G.cx + (b1 + b0) * G.cy;
  }
}

// (A p)_ij from the 5-point values (stage0/Withoutopenmp1.cpp:83-85).
template <bool EXACT>
__device__ __forceinline__ double apply_a(double pc, double pim, double pip, double pjm, double pjp,
                                          double a0, double a1, double b0, double b1,
                                          const DevGeom& G) {
  if constexpr (EXACT) {
    PMX_NO_CONTRACT
    const double Ax = -1.0 / G.h1 * (a1 * (pip - pc) / G.h1 - a0 * (pc - pim) / G.h1);
    const double Ay = -1.0 / G.h2 * (b1 * (pjp - pc) / G.h2 - b0 * (pc - pjm) / G.h2);
    return Ax + Ay;
  } else {
    return G.cx * (a1 * (pc - pip) + a0 * (pc - pim)) + G.cy * (b1 * (pc - pjp) + b0 * (pc - pjm));
  }
}

__device__ __forceinline__ bool dirichlet(const DevGeom& G, int gi, int gj) {
  return gi <= 0 || gi >= G.M || gj <= 0 || gj >= G.N;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// Deterministic block sum of up to two values; result valid in thread 0.
template <int BLOCK>
__device__ __forceinline__ void block_sum2(double& v0, double& v1, double* lds /*2*BLOCK/64*/) {
  constexpr int NW = BLOCK / kWave;
  v0 = wave_sum(v0);
  v1 = wave_sum(v1);
  const int wid = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  if (lane == 0) { lds[wid] = v0; lds[NW + wid] = v1; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) { s0 += lds[w]; s1 += lds[NW + w]; }
    v0 = s0; v1 = s1;
  }
}

// Linear tile id -> (ti, tj).  Tiles are TI rows x BLOCK columns.
struct Tile {
  int i0, iend, j0, jend, id;
};
__device__ __forceinline__ Tile tile_of(int id, int tiles_j, int TI, int BLOCK, const DevGeom& G) {
  Tile t;
  t.id = id;
  const int ti = id / tiles_j, tj = id - ti * tiles_j;
  t.i0 = 1 + ti * TI;
  t.iend = min(t.i0 + TI - 1, G.nx);
  t.j0 = 1 + tj * BLOCK;
  t.jend = min(t.j0 + BLOCK - 1, G.ny);
  return t;
}

}  // namespace dev
}  // namespace pmx
