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
// (ylo, yhi, rh) live in registers for the whole tile, the row terms (clip roots, face ends and
// the per-row coefficient classes of DevTables::acls/bcls) are wave-uniform scalar loads.
struct ColConst {
  double ylo, yhi, rh0, rh1;  // rh0 = rh[gj], rh1 = rh[gj+1]
  int gj;
};
struct RowConst {
  double rv0, rv1, xlo, xhi;  // rv0 = rv[gi], rv1 = rv[gi+1]
  int ca0[4], ca1[4], cb[4];  // classes of a(gi, .), a(gi+1, .), b(gi, .)
};
__device__ __forceinline__ ColConst load_col(const DevTables& T, int gj) {
  return ColConst{T.ylo[gj], T.yhi[gj], T.rh[gj], T.rh[gj + 1], gj};
}
// Wave-uniform loads from the read-only tables through the scalar cache: the tables are
// never written by a kernel that reads them, but the compiler cannot prove that (they may alias
// the fields), so without the constant address space it issues VECTOR loads -- and waiting for
// those (vmcnt is in-order) also drains every row prefetch issued before them.
template <typename T>
__device__ __forceinline__ T ld_uniform(const T* p, int i) {
  typedef const __attribute__((address_space(4))) T CT;
  return ((CT*)p)[i];
}
// Hand-off between the blocks of one launch (the ticketed last-block reductions): each block
// publishes its chunk sums write-through (relaxed agent-scope atomic stores, sc1), drains them
// (vmcnt 0) before its relaxed ticket add, and the last arriver reads every chunk with agent-scope
// atomic loads (sc1, past its CU's L1).  No __threadfence(): that is an L2 writeback plus an L2
// invalidate (~3.5 us each side) in a kernel of a few microseconds.
// Memory-model status: relaxed atomics give no happens-before edge in the HIP/C++ model; this is
// the hardware-level form MI355X_MICROARCH.md lists as measured valid on gfx950 / ROCm 7.2 ('Valid
// forms', first row of its hand-off table: one lane per storing workgroup, sc1 stores, vmcnt(0)
// before one agent-scope add to an unsharded counter, the last adder loads sc1 after its add
// returned, the other lanes after a workgroup barrier; <= 1 workgroup per CU -- the reductions run
// <= 64 blocks).  Not an architectural guarantee: tests/test_gpu_ops.py::
// test_reduction_handoff_stress checks every result of 200 back-to-back launches on one workspace
// under uneven load against the exactly rounded host sum.
typedef __attribute__((address_space(1))) double gdouble;
typedef __attribute__((address_space(1))) unsigned gunsigned;
__device__ __forceinline__ void st_publish(double* p, double v) {
  __hip_atomic_store((gdouble*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // NOLINT
}
__device__ __forceinline__ double ld_published(const double* p) {
  return __hip_atomic_load((gdouble*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // NOLINT
}
// true for the block whose arrival completes the count (n arrivals in all)
__device__ __forceinline__ bool ticket_arrive_last(unsigned* ticket, int n) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the published chunk is in L2 first
  return __hip_atomic_fetch_add((gunsigned*)ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==  // NOLINT
         unsigned(n - 1);
}
__device__ __forceinline__ RowConst load_row(const DevTables& T, int gi) {
  RowConst r;
  gi = __builtin_amdgcn_readfirstlane(gi);
  r.rv0 = ld_uniform(T.rv, gi);
  r.rv1 = ld_uniform(T.rv, gi + 1);
  r.xlo = ld_uniform(T.xlo, gi);
  r.xhi = ld_uniform(T.xhi, gi);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    r.ca0[q] = ld_uniform(T.acls, 4 * gi + q);
    r.ca1[q] = ld_uniform(T.acls, 4 * (gi + 1) + q);
    r.cb[q] = ld_uniform(T.bcls, 4 * gi + q);
  }
  return r;
}
// exact evaluation (bit-identical to the reference formula)
__device__ __forceinline__ double face_a(const ColConst& c, double rv, const DevGeom& G) {
  return geo::face_coef(geo::clip_len(c.ylo, c.yhi, rv), G.h2, G.eps, G.inv_eps);
}
__device__ __forceinline__ double face_b(const RowConst& r, double rh, const DevGeom& G) {
  return geo::face_coef(geo::clip_len(r.xlo, r.xhi, rh), G.h1, G.eps, G.inv_eps);
}
// class -> 1/eps, 1 or "cut" (exact formula).  The classes were produced by k_classify from the
// exact formula, so the fast values are bit-identical; the cut branch is rare (faces crossed by
// the ellipse) and skipped by whole waves away from the boundary.
__device__ __forceinline__ bool cls_fast(int j, const int* c, double inv_eps, double& v) {
  if (j < c[0] || j > c[3]) { v = inv_eps; return true; }
  if (j >= c[1] && j <= c[2]) { v = 1.0; return true; }
  return false;
}
__device__ __forceinline__ double face_a0c(const ColConst& cc, const RowConst& rc, const DevGeom& G) {
  double v;
  if (!cls_fast(cc.gj, rc.ca0, G.inv_eps, v)) v = face_a(cc, rc.rv0, G);
  return v;
}
__device__ __forceinline__ double face_a1c(const ColConst& cc, const RowConst& rc, const DevGeom& G) {
  double v;
  if (!cls_fast(cc.gj, rc.ca1, G.inv_eps, v)) v = face_a(cc, rc.rv1, G);
  return v;
}
__device__ __forceinline__ double face_b0c(const ColConst& cc, const RowConst& rc, const DevGeom& G) {
  double v;
  if (!cls_fast(cc.gj, rc.cb, G.inv_eps, v)) v = face_b(rc, cc.rh0, G);
  return v;
}
__device__ __forceinline__ double face_b1c(const ColConst& cc, const RowConst& rc, const DevGeom& G) {
  double v;
  if (!cls_fast(cc.gj + 1, rc.cb, G.inv_eps, v)) v = face_b(rc, cc.rh1, G);
  return v;
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

// z = r / D for a row of known uniform class (1 inside / 2 outside), else the general path.
template <bool EXACT>
__device__ __forceinline__ double zdiv_u(int ucls, double r, double a0, double a1, double b0,
                                         double b1, const DevGeom& G);

// z = r / D.  Fast mode: the two common stencils (all faces inside / all outside D) use a
// precomputed 1/D; only cut stencils divide.
template <bool EXACT>
__device__ __forceinline__ double zdiv(double r, double a0, double a1, double b0, double b1,
                                       const DevGeom& G) {
  if constexpr (EXACT) {
    return r / diag<true>(a0, a1, b0, b1, G);
  } else {
    const bool in = (a0 == 1.0) & (a1 == 1.0) & (b0 == 1.0) & (b1 == 1.0);
    const bool out = (a0 == G.inv_eps) & (a1 == G.inv_eps) & (b0 == G.inv_eps) & (b1 == G.inv_eps);
    if (in) return r * G.dinv_in;
    if (out) return r * G.dinv_out;
    return r / diag<false>(a0, a1, b0, b1, G);
  }
}

template <bool EXACT>
__device__ __forceinline__ double zdiv_u(int ucls, double r, double a0, double a1, double b0,
                                         double b1, const DevGeom& G) {
  if constexpr (!EXACT) {
    if (ucls == 1) return r * G.dinv_in;
    if (ucls == 2) return r * G.dinv_out;
  }
  return zdiv<EXACT>(r, a0, a1, b0, b1, G);
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
    // explicit FMAs: every kernel that evaluates A p (pcg_a, pcg_b, edge_r) gets bit-identical
    // values whatever the compiler's contraction choices in the surrounding code
    const double x = __builtin_fma(a1, pc - pip, a0 * (pc - pim));
    const double y = __builtin_fma(b1, pc - pjp, b0 * (pc - pjm));
    return __builtin_fma(G.cx, x, G.cy * y);
  }
}

// w + alpha p and r - alpha A p.  EXACT: the reference's separate multiply and add
// (stage0/Withoutopenmp1.cpp:135-143); fast: one explicit FMA each, so the r values packed for the
// halo by k_edge_r equal those k_pcg_b stores.
template <bool EXACT>
__device__ __forceinline__ double upd_w(double wo, double alpha, double p) {
  if constexpr (EXACT) {
    PMX_NO_CONTRACT
    return wo + alpha * p;
  } else {
    return __builtin_fma(alpha, p, wo);
  }
}
template <bool EXACT>
__device__ __forceinline__ double upd_r(double ro, double alpha, double Ap) {
  if constexpr (EXACT) {
    PMX_NO_CONTRACT
    return ro - alpha * Ap;
  } else {
    return __builtin_fma(-alpha, Ap, ro);
  }
}

__device__ __forceinline__ bool dirichlet(const DevGeom& G, int gi, int gj) {
  return gi <= 0 || gi >= G.M || gj <= 0 || gj >= G.N;
}

// ---- wave64 reductions on the matrix cores --------------------------------------------------
// v_mfma_*_16x16x4 with B = ones computes D[i][j] = sum_k A[i][k], where lane l supplies
// A[l % 16][l / 16]: one MFMA folds the 64 lanes into 16 row sums (lanes i, i+16, i+32, i+48).
// Lane l receives 4 of those rows (a set fixed by l / 16 that partitions the 16 rows; f64 and f32
// interleave them differently, see wave_sum2_mfma), so after
// adding its 4 outputs every lane of group g = l / 16 holds the same group sum S_g, and a second
// MFMA with A[.][g] = S_g sums the 4 groups.  No LDS and no cross-lane permutes; deterministic.
// Requires a full EXEC mask (all callers reduce after their wave-uniform control flow).
typedef double v4f64 __attribute__((ext_vector_type(4)));
typedef float v4f32 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4f64 mfma_rowsum(double a) {
  const v4f64 z = {0.0, 0.0, 0.0, 0.0};
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, 1.0, z, 0, 0, 0);
}
__device__ __forceinline__ v4f32 mfma_rowsum(float a) {
  const v4f32 z = {0.f, 0.f, 0.f, 0.f};
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, 1.0f, z, 0, 0, 0);
}

__device__ __forceinline__ double readlane_t(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane(int(b), lane);
  const int hi = __builtin_amdgcn_readlane(int(b >> 32), lane);
  return __longlong_as_double((long long)(unsigned)lo | ((long long)hi << 32));
}
__device__ __forceinline__ float readlane_t(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// sum over the wave, returned in every lane
template <typename T>
__device__ __forceinline__ T wave_sum_mfma(T v) {
  auto d = mfma_rowsum(v);
  const T g = (d[0] + d[1]) + (d[2] + d[3]);
  d = mfma_rowsum(g);
  return d[0];
}

// Packed pair: two first-stage MFMAs, then ONE second-stage MFMA whose rows 0-7 carry the group
// sums of v0 and rows 8-15 those of v1.  Lanes 0-31 end with sum(v0), lanes 32-63 with sum(v1);
// both are returned wave-uniform.
template <typename T>
__device__ __forceinline__ void wave_sum2_mfma(T& v0, T& v1) {
  const auto d0 = mfma_rowsum(v0);
  const auto d1 = mfma_rowsum(v1);
  const T g0 = (d0[0] + d0[1]) + (d0[2] + d0[3]);
  const T g1 = (d1[0] + d1[1]) + (d1[2] + d1[3]);
  const int lane = __lane_id();
  const auto e = mfma_rowsum((lane & 15) < 8 ? g0 : g1);
  // D[i][j] = sum_k A[i][k]: rows 0-7 hold sum(v0), rows 8-15 sum(v1).  Output rows of lane l,
  // register r (measured on gfx950, bench/probe/mfma_layout.hip): f64 row l/16 + 4r, f32 row
  // 4(l/16) + r.  So f64 reads lane 0 registers 0 / 2 and f32 lanes 0 / 32 of register 0.
  if constexpr (sizeof(T) == 8) {
    v0 = readlane_t(e[0], 0);
    v1 = readlane_t(e[2], 0);
  } else {
    v0 = readlane_t(e[0], 0);
    v1 = readlane_t(e[0], 32);
  }
}

__device__ __forceinline__ double wave_sum(double v) { return wave_sum_mfma(v); }

// Deterministic block sum of up to two values; result valid in thread 0.
template <int BLOCK>
__device__ __forceinline__ void block_sum2(double& v0, double& v1, double* lds /*2*BLOCK/64*/) {
  constexpr int NW = BLOCK / kWave;
  wave_sum2_mfma(v0, v1);
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

// Bijective XCD-aware remap (cdna_hip_programming.md §5.5 T1): hardware dispatch deals workgroup b
// to XCD b % 8, so hand each XCD a contiguous range of logical tiles.  Neighbouring tiles share
// halo cache lines and rows; keeping them on one XCD turns those re-reads into L2 hits.  Speed
// only: any placement gives the same result.
__device__ __forceinline__ int xcd_remap(int b, int nb) {
  const int q = nb / 8, r = nb % 8;
  const int xcd = b % 8, idx = b / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// Wave-uniform row class of a tile: 1 = every face of every column in [jlo, jhi] lies inside D
// (all coefficients exactly 1), 2 = all outside (all exactly 1/eps), 0 = cut faces present.
__device__ __forceinline__ int row_class(const RowConst& rc, int jlo, int jhi) {
  const bool in = jlo >= rc.ca0[1] && jhi <= rc.ca0[2] && jlo >= rc.ca1[1] && jhi <= rc.ca1[2] &&
                  jlo >= rc.cb[1] && jhi + 1 <= rc.cb[2];
  if (in) return 1;
  auto out = [&](const int* c, int hi) { return jlo > c[3] || hi < c[0]; };
  if (out(rc.ca0, jhi) && out(rc.ca1, jhi) && (jlo > rc.cb[3] || jhi + 1 < rc.cb[0])) return 2;
  return 0;
}

// Linear tile id -> (ti, tj).  Tiles are TI rows x BLOCK columns.
struct Tile {
  int i0, iend, j0, jend, id;
};
__device__ __forceinline__ Tile tile_of(int id, int tiles_j, int TI, int BLOCK, const DevGeom& G) {
  id = xcd_remap(id, int(gridDim.x));
  Tile t;
  t.id = id;
  const int ti = id / tiles_j, tj = id - ti * tiles_j;
  t.i0 = 1 + ti * TI;
  t.iend = min(t.i0 + TI - 1, G.nx);
  t.j0 = 1 + tj * BLOCK;
  t.jend = min(t.j0 + BLOCK - 1, G.ny);
  return t;
}

// ---- wave-tile helpers (pcg_kernels_dpp.hip, pcg1_kernels.hip) -------------------------------
// DPP wave shifts on a double: lane l receives lane l-1's (SHR) / l+1's (SHL) value; the edge lane
// that has no source keeps `edge`.
constexpr int kWaveShl1 = 0x130;
constexpr int kWaveShr1 = 0x138;
template <int CTRL>
__device__ __forceinline__ float dpp_shift(float v, float edge) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(edge), __float_as_int(v), CTRL, 0xf,
                                                    0xf, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp_shift_f64(double v, double edge);
template <int CTRL>
__device__ __forceinline__ double dpp_shift(double v, double edge) { return dpp_shift_f64<CTRL>(v, edge); }
template <int CTRL>
__device__ __forceinline__ double dpp_shift_f64(double v, double edge) {
  const long long b = __double_as_longlong(v);
  const long long e = __double_as_longlong(edge);
  const int lo = __builtin_amdgcn_update_dpp(int(e), int(b), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(int(e >> 32), int(b >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double((long long)(unsigned)lo | ((long long)hi << 32));
}

template <typename T, int VEC> struct VecT;
template <> struct VecT<double, 1> { using type = double; };
template <> struct VecT<double, 2> { using type = double2; };
template <> struct VecT<double, 4> { using type = double4; };
template <> struct VecT<float, 1> { using type = float; };
template <> struct VecT<float, 2> { using type = float2; };
template <> struct VecT<float, 4> { using type = float4; };

// Loads keep the storage type: prefetch rings hold raw T (half the VGPRs in fp32 storage mode)
// and values are widened to fp64 where they are used.
template <typename T, int VEC>
__device__ __forceinline__ void vload_raw(const T* p, T (&out)[VEC]) {
  using V = typename VecT<T, VEC>::type;
  const V v = *reinterpret_cast<const V*>(p);
  const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
  for (int u = 0; u < VEC; ++u) out[u] = e[u];
}

template <typename T, int VEC>
__device__ __forceinline__ void vload(const T* p, double (&out)[VEC]) {
  using V = typename VecT<T, VEC>::type;
  const V v = *reinterpret_cast<const V*>(p);
  const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
  for (int u = 0; u < VEC; ++u) out[u] = double(e[u]);
}

template <typename T, int VEC>
__device__ __forceinline__ void vstore(T* p, const T (&in)[VEC]) {
  using V = typename VecT<T, VEC>::type;
  V v;
  T* e = reinterpret_cast<T*>(&v);
#pragma unroll
  for (int u = 0; u < VEC; ++u) e[u] = in[u];
  *reinterpret_cast<V*>(p) = v;
}

}  // namespace dev
}  // namespace pmx
