// Unfused device ops: assembly, operator A, preconditioner, dot partials.
//
// They mirror the reference's one-op-per-kernel structure (stage4-mpi+cuda/poisson_mpi_cuda_f.cu:
// apply_A_kernel :507-536, apply_Dinv_kernel :541-562, dot_kernel :574-598) but with the
// CDNA-friendly mapping: threadIdx.x runs along the contiguous axis lj (the reference maps it to
// the strided li axis, :514-515), and coefficients come from the 1D face tables.  Used by the
// unit tests (each op vs a PyTorch fp64 reference) and by the solver's `naive` kernel mode.
#include <algorithm>
#include <climits>
#include <cmath>

#include "pcg_device.hpp"
#include "pmx/common.hpp"
#include "pmx/kernels.hpp"

namespace pmx {

using namespace dev;

__global__ void __launch_bounds__(256)
k_assemble(DevGeom G, DevTables Tb, double* a, double* b, double* B, int64_t pab) {
  const int lj = blockIdx.x * 64 + (threadIdx.x & 63);
  const int li = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (li > G.nx + 1 || lj > G.ny + 1) return;
  const int gi = G.gi0 + li, gj = G.gj0 + lj;
  a[li * pab + lj] = coef_a(Tb, G, gi, gj);
  b[li * pab + lj] = coef_b(Tb, G, gi, gj);
  const bool interior = li >= 1 && li <= G.nx && lj >= 1 && lj <= G.ny;
  B[li * pab + lj] =
      interior && geo::inside(Tb.x[gi], Tb.y[gj], G.ax, G.by, G.ref_ellipse != 0) ? G.F : 0.0;
}

template <typename T, bool EXACT>
__global__ void __launch_bounds__(256)
k_apply_a(DevGeom G, DevTables Tb, const T* __restrict__ p, T* __restrict__ Ap) {
  const int lj = 1 + blockIdx.x * 64 + (threadIdx.x & 63);
  const int li = 1 + blockIdx.y * 4 + (threadIdx.x >> 6);
  if (li > G.nx || lj > G.ny) return;
  const int gi = G.gi0 + li, gj = G.gj0 + lj;
  const int64_t c = li * G.pitch + lj;
  const double a0 = coef_a(Tb, G, gi, gj), a1 = coef_a(Tb, G, gi + 1, gj);
  const double b0 = coef_b(Tb, G, gi, gj), b1 = coef_b(Tb, G, gi, gj + 1);
  Ap[c] = static_cast<T>(apply_a<EXACT>(double(p[c]), double(p[c - G.pitch]),
                                        double(p[c + G.pitch]), double(p[c - 1]),
                                        double(p[c + 1]), a0, a1, b0, b1, G));
}

template <typename T, bool EXACT>
__global__ void __launch_bounds__(256)
k_precond(DevGeom G, DevTables Tb, const T* __restrict__ r, T* __restrict__ z) {
  const int lj = 1 + blockIdx.x * 64 + (threadIdx.x & 63);
  const int li = 1 + blockIdx.y * 4 + (threadIdx.x >> 6);
  if (li > G.nx || lj > G.ny) return;
  const int gi = G.gi0 + li, gj = G.gj0 + lj;
  const int64_t c = li * G.pitch + lj;
  const double a0 = coef_a(Tb, G, gi, gj), a1 = coef_a(Tb, G, gi + 1, gj);
  const double b0 = coef_b(Tb, G, gi, gj), b1 = coef_b(Tb, G, gi, gj + 1);
  const double D = diag<EXACT>(a0, a1, b0, b1, G);
  z[c] = static_cast<T>((D != 0.0) ? double(r[c]) / D : 0.0);
}

template <typename T>
__global__ void __launch_bounds__(256)
k_dot_partials(DevGeom G, const T* __restrict__ x, const T* __restrict__ y, double* partials) {
  __shared__ double lds[2 * 256 / kWave];
  double s = 0.0, unused = 0.0;
  const int64_t n = int64_t(G.nx) * G.ny;
  for (int64_t k = int64_t(blockIdx.x) * 256 + threadIdx.x; k < n; k += int64_t(gridDim.x) * 256) {
    const int li = int(k / G.ny) + 1, lj = int(k % G.ny) + 1;
    const int64_t c = li * G.pitch + lj;
    s += double(x[c]) * double(y[c]);
  }
  block_sum2<256>(s, unused, lds);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

// Error of the solution against the analytic u = F (1 - x^2/ax^2 - y^2/by^2) / (2/ax^2 + 2/by^2)
// inside D (итоговый отчёт/Этап_4_1213.pdf p.1: (1 - x^2 - 4y^2)/10; the reference never computes
// it).  w_eff = w + sum_q c_q p_q applies the single-pass solver's pending w steps (see
// GpuSubdomainSolver::download_w) without moving w to the host.  Per block: sum of e^2 over the
// owned nodes in D, max |e| in D, max w_eff; the caller finishes on the host (and over ranks).
template <typename T>
__global__ void __launch_bounds__(256)
k_error_norms(DevGeom G, DevTables Tb, const T* __restrict__ w, const T* __restrict__ pa, double ca,
              const T* __restrict__ pb, double cb, int npend, double* out) {
  __shared__ double lds[3][256 / kWave];
  const double den = 2.0 / (G.ax * G.ax) + 2.0 / (G.by * G.by);  // as geo::exact_solution
  double se = 0.0, me = 0.0, mw = -HUGE_VAL;
  const int64_t n = int64_t(G.nx) * G.ny;
  for (int64_t k = int64_t(blockIdx.x) * 256 + threadIdx.x; k < n; k += int64_t(gridDim.x) * 256) {
    const int li = int(k / G.ny) + 1, lj = int(k % G.ny) + 1;
    const int64_t c = li * G.pitch + lj;
    double v = double(w[c]);
    if (npend > 0) v = __builtin_fma(ca, double(pa[c]), v);
    if (npend > 1) v = __builtin_fma(cb, double(pb[c]), v);
    if (npend > 0 && sizeof(T) == 4) v = double(static_cast<float>(v));
    mw = fmax(mw, v);
    const double x = Tb.x[G.gi0 + li], y = Tb.y[G.gj0 + lj];
    if (geo::inside(x, y, G.ax, G.by, G.ref_ellipse != 0)) {
      const double u = x / G.ax, t = y / G.by;
      const double q = 1.0 - u * u - t * t;
      const double e = v - (q > 0.0 ? G.F * q / den : 0.0);
      se = __builtin_fma(e, e, se);
      me = fmax(me, fabs(e));
    }
  }
  se = wave_sum_mfma(se);
  for (int o = 32; o >= 1; o >>= 1) {
    me = fmax(me, __shfl_xor(me, o));
    mw = fmax(mw, __shfl_xor(mw, o));
  }
  const int wid = threadIdx.x / kWave;
  if ((threadIdx.x % kWave) == 0) {
    lds[0][wid] = se;
    lds[1][wid] = me;
    lds[2][wid] = mw;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0, m = -HUGE_VAL;
    for (int q = 0; q < 256 / kWave; ++q) {
      a += lds[0][q];
      b = fmax(b, lds[1][q]);
      m = fmax(m, lds[2][q]);
    }
    out[3 * blockIdx.x] = a;
    out[3 * blockIdx.x + 1] = b;
    out[3 * blockIdx.x + 2] = m;
  }
}

template <typename T>
int launch_error_norms(const DevGeom& G, const DevTables& Tb, const T* w, const T* pa, double ca,
                       const T* pb, double cb, int npend, double* out, int max_blocks, hipStream_t s) {
  const int64_t n = int64_t(G.nx) * G.ny;
  const int nb = int(std::max<int64_t>(1, std::min<int64_t>(max_blocks, (n + 255) / 256)));
  hipLaunchKernelGGL((k_error_norms<T>), dim3(nb), dim3(256), 0, s, G, Tb, w, pa, ca, pb, cb, npend, out);
  HIP_CHECK(hipGetLastError());
  return nb;
}
template int launch_error_norms<double>(const DevGeom&, const DevTables&, const double*, const double*,
                                        double, const double*, double, int, double*, int, hipStream_t);
template int launch_error_norms<float>(const DevGeom&, const DevTables&, const float*, const float*, double,
                                       const float*, double, int, double*, int, hipStream_t);

// MFMA wave reductions (pcg_device.hpp) on arbitrary data, for the unit tests: per wave64 of x,
// out[3w] = sum x, out[3w+1] = sum x (packed pair), out[3w+2] = sum x^2 (packed pair)
template <typename T>
__global__ void __launch_bounds__(256) k_wave_sums(const T* __restrict__ x, T* __restrict__ out, int nw) {
  const int w = blockIdx.x * 4 + int(threadIdx.x >> 6);
  if (w >= nw) return;  // wave-uniform: EXEC stays full for the MFMAs
  const T v = x[int64_t(w) * 64 + (threadIdx.x & 63)];
  const T s = wave_sum_mfma(v);
  T a = v, b = v * v;
  wave_sum2_mfma(a, b);
  if ((threadIdx.x & 63) == 0) {
    out[3 * w] = s;
    out[3 * w + 1] = a;
    out[3 * w + 2] = b;
  }
}

template <typename T>
void launch_wave_sums(const T* x, T* out, int nw, hipStream_t s) {
  hipLaunchKernelGGL((k_wave_sums<T>), dim3((nw + 3) / 4), dim3(256), 0, s, x, out, nw);
  HIP_CHECK(hipGetLastError());
}
template void launch_wave_sums<double>(const double*, double*, int, hipStream_t);
template void launch_wave_sums<float>(const float*, float*, int, hipStream_t);

// one workgroup per global row gi: out range (first/last j whose coefficient is not 1/eps) and
// in range (first/last j equal to 1, kept only if every j between is exactly 1)
__global__ void __launch_bounds__(256)
k_classify(DevGeom G, DevTables Tb, int* acls, int* bcls) {
  // acc: a out lo/hi, a in lo/hi, b out lo/hi, b in lo/hi, #a==1, #b==1
  __shared__ int acc[10];
  const int gi = blockIdx.x;
  int ao_lo = INT_MAX, ao_hi = INT_MIN, ai_lo = INT_MAX, ai_hi = INT_MIN;
  int bo_lo = INT_MAX, bo_hi = INT_MIN, bi_lo = INT_MAX, bi_hi = INT_MIN;
  int na1 = 0, nb1 = 0;
  if (threadIdx.x < 10)
    acc[threadIdx.x] = threadIdx.x >= 8 ? 0 : (threadIdx.x % 2 == 0 ? INT_MAX : INT_MIN);
  __syncthreads();
  for (int j = threadIdx.x; j <= G.N + 1; j += 256) {
    const double a = coef_a(Tb, G, gi, j);
    const double b = coef_b(Tb, G, gi, j);
    if (a != G.inv_eps) { ao_lo = min(ao_lo, j); ao_hi = max(ao_hi, j); }
    if (a == 1.0) { ai_lo = min(ai_lo, j); ai_hi = max(ai_hi, j); ++na1; }
    if (b != G.inv_eps) { bo_lo = min(bo_lo, j); bo_hi = max(bo_hi, j); }
    if (b == 1.0) { bi_lo = min(bi_lo, j); bi_hi = max(bi_hi, j); ++nb1; }
  }
  atomicMin(&acc[0], ao_lo); atomicMax(&acc[1], ao_hi);
  atomicMin(&acc[2], ai_lo); atomicMax(&acc[3], ai_hi);
  atomicMin(&acc[4], bo_lo); atomicMax(&acc[5], bo_hi);
  atomicMin(&acc[6], bi_lo); atomicMax(&acc[7], bi_hi);
  atomicAdd(&acc[8], na1); atomicAdd(&acc[9], nb1);
  __syncthreads();
  if (threadIdx.x == 0) {
    int* A = acls + 4 * gi;
    int* B = bcls + 4 * gi;
    const bool a_contig = acc[8] > 0 && acc[8] == acc[3] - acc[2] + 1;
    const bool b_contig = acc[9] > 0 && acc[9] == acc[7] - acc[6] + 1;
    A[0] = acc[0]; A[1] = a_contig ? acc[2] : 1; A[2] = a_contig ? acc[3] : 0; A[3] = acc[1];
    B[0] = acc[4]; B[1] = b_contig ? acc[6] : 1; B[2] = b_contig ? acc[7] : 0; B[3] = acc[5];
  }
}

void launch_classify(const DevGeom& G, const DevTables& Tb, int* acls, int* bcls, hipStream_t s) {
  hipLaunchKernelGGL(k_classify, dim3(G.M + 2), dim3(256), 0, s, G, Tb, acls, bcls);
  HIP_CHECK(hipGetLastError());
}

void launch_assemble(const DevGeom& G, const DevTables& Tb, double* a, double* b, double* B,
                     int64_t pab, hipStream_t s) {
  dim3 grid((G.ny + 2 + 63) / 64, (G.nx + 2 + 3) / 4);
  hipLaunchKernelGGL(k_assemble, grid, dim3(256), 0, s, G, Tb, a, b, B, pab);
  HIP_CHECK(hipGetLastError());
}

template <typename T>
void launch_apply_a(const DevGeom& G, const DevTables& Tb, const T* p, T* Ap, bool exact,
                    hipStream_t s) {
  dim3 grid((G.ny + 63) / 64, (G.nx + 3) / 4);
  if (exact) hipLaunchKernelGGL((k_apply_a<T, true>), grid, dim3(256), 0, s, G, Tb, p, Ap);
  else hipLaunchKernelGGL((k_apply_a<T, false>), grid, dim3(256), 0, s, G, Tb, p, Ap);
  HIP_CHECK(hipGetLastError());
}

template <typename T>
void launch_precond(const DevGeom& G, const DevTables& Tb, const T* r, T* z, bool exact,
                    hipStream_t s) {
  dim3 grid((G.ny + 63) / 64, (G.nx + 3) / 4);
  if (exact) hipLaunchKernelGGL((k_precond<T, true>), grid, dim3(256), 0, s, G, Tb, r, z);
  else hipLaunchKernelGGL((k_precond<T, false>), grid, dim3(256), 0, s, G, Tb, r, z);
  HIP_CHECK(hipGetLastError());
}

template <typename T>
int launch_dot_partials(const DevGeom& G, const T* x, const T* y, double* partials, int max_blocks,
                        hipStream_t s) {
  const int64_t n = int64_t(G.nx) * G.ny;
  int blocks = int(std::min<int64_t>(max_blocks, (n + 255) / 256));
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL((k_dot_partials<T>), dim3(blocks), dim3(256), 0, s, G, x, y, partials);
  HIP_CHECK(hipGetLastError());
  return blocks;
}

#define PMX_INST(T)                                                                          \
  template void launch_apply_a<T>(const DevGeom&, const DevTables&, const T*, T*, bool,     \
                                  hipStream_t);                                              \
  template void launch_precond<T>(const DevGeom&, const DevTables&, const T*, T*, bool,     \
                                  hipStream_t);                                              \
  template int launch_dot_partials<T>(const DevGeom&, const T*, const T*, double*, int,     \
                                      hipStream_t);
PMX_INST(double)
PMX_INST(float)
#undef PMX_INST

}  // namespace pmx
