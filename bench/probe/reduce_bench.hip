// Wave64 fp64 reduction micro-benchmark ("measure the MFMA reduction against a
// DPP/shuffle reduction and keep whichever is faster").  Each wave runs a dependent chain of
// `reps` reductions of one (single) or two (pair) values; reported as ns per reduction per wave
// and as chip throughput.  Variants: MFMA (pcg_device.hpp's scheme), __shfl_xor butterfly
// (ds_bpermute), DPP row/bank shuffles + readlane.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double v4d __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double sum_mfma(double v) {
  const v4d z = {0, 0, 0, 0};
  v4d d = __builtin_amdgcn_mfma_f64_16x16x4f64(v, 1.0, z, 0, 0, 0);
  const double g = (d[0] + d[1]) + (d[2] + d[3]);
  d = __builtin_amdgcn_mfma_f64_16x16x4f64(g, 1.0, z, 0, 0, 0);
  return d[0];
}
__device__ __forceinline__ void sum2_mfma(double& a, double& b) {
  const v4d z = {0, 0, 0, 0};
  const v4d d0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, 1.0, z, 0, 0, 0);
  const v4d d1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, 1.0, z, 0, 0, 0);
  const double g0 = (d0[0] + d0[1]) + (d0[2] + d0[3]), g1 = (d1[0] + d1[1]) + (d1[2] + d1[3]);
  const v4d e = __builtin_amdgcn_mfma_f64_16x16x4f64((__lane_id() & 15) < 8 ? g0 : g1, 1.0, z, 0, 0, 0);
  a = e[0];
  b = e[2];
}
__device__ __forceinline__ double sum_shfl(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, int(b), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, int(b >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double((long long)(unsigned)lo | ((long long)hi << 32));
}
__device__ __forceinline__ double rl(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane(int(b), lane), hi = __builtin_amdgcn_readlane(int(b >> 32), lane);
  return __longlong_as_double((long long)(unsigned)lo | ((long long)hi << 32));
}
// DPP: quad_perm swaps, row_shr 4/8 (row = 16 lanes), then combine the 4 rows with readlanes
__device__ __forceinline__ double sum_dpp(double v) {
  v += dpp<0xb1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4e>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x114>(v);  // row_shr:4
  v += dpp<0x118>(v);  // row_shr:8
  return (rl(v, 15) + rl(v, 31)) + (rl(v, 47) + rl(v, 63));
}

template <int MODE>
__global__ void __launch_bounds__(256) k(const double* x, double* out, int reps) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  double a = x[i], b = x[i] * 0.5;
  for (int r = 0; r < reps; ++r) {
    if (MODE == 0) a = sum_mfma(a) * 1e-3 + x[i];
    if (MODE == 1) a = sum_shfl(a) * 1e-3 + x[i];
    if (MODE == 2) a = sum_dpp(a) * 1e-3 + x[i];
    if (MODE == 3) { sum2_mfma(a, b); a = a * 1e-3 + x[i]; b = b * 1e-3 + x[i]; }
    if (MODE == 4) { a = sum_shfl(a) * 1e-3 + x[i]; b = sum_shfl(b) * 1e-3 + x[i]; }
    if (MODE == 5) { a = sum_dpp(a) * 1e-3 + x[i]; b = sum_dpp(b) * 1e-3 + x[i]; }
  }
  out[i] = a + b;
}

int main() {
  const int blocks = 4096, reps = 2000, n = blocks * 256;
  double *x, *o;
  hipMalloc(&x, n * 8);
  hipMalloc(&o, n * 8);
  hipMemset(x, 0, n * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[6] = {"mfma", "shfl_xor", "dpp", "mfma_pair", "shfl_xor_pair", "dpp_pair"};
  for (int m = 0; m < 6; ++m) {
    auto launch = [&] {
      switch (m) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, x, o, reps); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, x, o, reps); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, x, o, reps); break;
        case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, x, o, reps); break;
        case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, x, o, reps); break;
        case 5: hipLaunchKernelGGL(k<5>, dim3(blocks), dim3(256), 0, 0, x, o, reps); break;
      }
    };
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double waves = blocks * 4.0;
    printf("{\"reduction\": \"%s\", \"ms\": %.3f, \"wave_reductions_per_s\": %.3e}\n", names[m], ms,
           waves * reps / (ms * 1e-3));
  }
  return 0;
}
