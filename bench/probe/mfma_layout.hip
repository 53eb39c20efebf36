// Probe: output-row layout of v_mfma_{f64,f32}_16x16x4 (lane l supplies A[l%16][l/16] = l%16,
// B = ones, so D[i][j] = 4i and each output register reveals its row).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
__global__ void k(double* od, float* of) {
  const int l = threadIdx.x;
  const v4d zd = {0, 0, 0, 0};
  const v4f zf = {0, 0, 0, 0};
  v4d d = __builtin_amdgcn_mfma_f64_16x16x4f64(double(l % 16), 1.0, zd, 0, 0, 0);
  v4f f = __builtin_amdgcn_mfma_f32_16x16x4f32(float(l % 16), 1.0f, zf, 0, 0, 0);
  for (int r = 0; r < 4; ++r) { od[l * 4 + r] = d[r] / 4; of[l * 4 + r] = f[r] / 4; }
}
int main() {
  double* od; float* of;
  hipMalloc(&od, 256 * 8); hipMalloc(&of, 256 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, od, of);
  double hd[256]; float hf[256];
  hipMemcpy(hd, od, sizeof hd, hipMemcpyDeviceToHost);
  hipMemcpy(hf, of, sizeof hf, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; l += 8)
    printf("lane %2d f64 rows %g %g %g %g | f32 rows %g %g %g %g\n", l, hd[4*l], hd[4*l+1], hd[4*l+2], hd[4*l+3], hf[4*l], hf[4*l+1], hf[4*l+2], hf[4*l+3]);
  return 0;
}
