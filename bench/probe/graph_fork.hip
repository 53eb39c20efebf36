// Standalone reproducer for the round-3 host segfault in hipGraphLaunch (verdict r3 item 7): a
// captured graph whose iterations fork onto side streams and join back -- the shape of
// PcgDriver::enqueue_split_iteration (csrc/hip/gpu_solver.hip) -- launched in a process with
// GPU_MAX_HW_QUEUES=1.  No pmx code: three streams, events reused every iteration (as the
// driver does), trivial kernels and device-to-device copies standing in for the sweep parts, the
// pack/unpack kernels, the reduction and the LocalComm ghost copies.
//
//   hipcc --offload-arch=gfx950 -O2 bench/probe/graph_fork.hip -o bench/probe/graph_fork
//   GPU_MAX_HW_QUEUES=1 bench/probe/graph_fork [iters_per_graph=3] [launches=20] [copies=4]
//
// Prints one line per step; exit 0 = no crash and every kernel ran the expected number of times.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(2);                                                                  \
    }                                                                                \
  } while (0)

__global__ void k_tick(unsigned long long* counter, int slot) {
  if (threadIdx.x == 0 && blockIdx.x == 0) atomicAdd(counter + slot, 1ull);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 3;
  const int launches = argc > 2 ? std::atoi(argv[2]) : 20;
  const int copies = argc > 3 ? std::atoi(argv[3]) : 4;
  const char* hwq = std::getenv("GPU_MAX_HW_QUEUES");
  std::printf("graph_fork: iters/graph %d, launches %d, copies/iter %d, GPU_MAX_HW_QUEUES=%s\n", iters, launches,
              copies, hwq ? hwq : "(default)");
  int rt = 0, drv = 0;
  CK(hipRuntimeGetVersion(&rt));
  CK(hipDriverGetVersion(&drv));
  std::printf("HIP runtime %d, driver %d\n", rt, drv);
  std::fflush(stdout);
  unsigned long long* counter = nullptr;
  CK(hipMalloc(&counter, 8 * sizeof(unsigned long long)));
  CK(hipMemset(counter, 0, 8 * sizeof(unsigned long long)));
  const size_t nbytes = 64 * 1024;
  std::vector<char*> buf(2 * copies);
  for (auto& b : buf) CK(hipMalloc(&b, nbytes));
  hipStream_t C, F, H;  // compute, frame, comm
  CK(hipStreamCreateWithFlags(&C, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&F, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&H, hipStreamNonBlocking));
  hipEvent_t ev_ar, ev_fdone, ev_swept, ev_pk, ev_halo;
  for (hipEvent_t* e : {&ev_ar, &ev_fdone, &ev_swept, &ev_pk, &ev_halo})
    CK(hipEventCreateWithFlags(e, hipEventDisableTiming));

  CK(hipStreamBeginCapture(C, hipStreamCaptureModeThreadLocal));
  bool halo_pending = false;
  for (int k = 0; k < iters; ++k) {
    CK(hipEventRecord(ev_ar, C));
    CK(hipStreamWaitEvent(F, ev_ar, 0));
    if (halo_pending) CK(hipStreamWaitEvent(F, ev_halo, 0));
    hipLaunchKernelGGL(k_tick, dim3(64), dim3(64), 0, C, counter, 0);  // interior tiles
    hipLaunchKernelGGL(k_tick, dim3(8), dim3(64), 0, F, counter, 1);   // frame tiles
    CK(hipEventRecord(ev_fdone, F));
    CK(hipStreamWaitEvent(C, ev_fdone, 0));
    CK(hipEventRecord(ev_swept, C));
    CK(hipStreamWaitEvent(H, ev_swept, 0));
    hipLaunchKernelGGL(k_tick, dim3(8), dim3(64), 0, H, counter, 2);  // pack
    CK(hipEventRecord(ev_pk, H));
    for (int c = 0; c < copies; ++c)  // LocalComm ghost copies
      CK(hipMemcpyAsync(buf[2 * c + 1], buf[2 * c], nbytes, hipMemcpyDeviceToDevice, H));
    hipLaunchKernelGGL(k_tick, dim3(8), dim3(64), 0, H, counter, 3);  // unpack
    CK(hipEventRecord(ev_halo, H));
    halo_pending = true;
    hipLaunchKernelGGL(k_tick, dim3(1), dim3(64), 0, C, counter, 4);  // reduction
    CK(hipStreamWaitEvent(C, ev_pk, 0));
  }
  CK(hipStreamWaitEvent(C, ev_halo, 0));  // join
  hipGraph_t g = nullptr;
  CK(hipStreamEndCapture(C, &g));
  size_t nn = 0;
  CK(hipGraphGetNodes(g, nullptr, &nn));
  std::printf("captured %zu nodes\n", nn);
  std::fflush(stdout);
  hipGraphExec_t ex = nullptr;
  CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  std::printf("instantiated\n");
  std::fflush(stdout);
  for (int l = 0; l < launches; ++l) {
    CK(hipGraphLaunch(ex, C));
    if (l == 0) {
      std::printf("first launch enqueued\n");
      std::fflush(stdout);
    }
  }
  CK(hipStreamSynchronize(C));
  unsigned long long h[8];
  CK(hipMemcpy(h, counter, sizeof(h), hipMemcpyDeviceToHost));
  const unsigned long long want = (unsigned long long)iters * launches;
  bool ok = true;
  for (int s = 0; s < 5; ++s) ok &= h[s] == want * (s == 0 ? 1 : 1);
  std::printf("counts %llu %llu %llu %llu %llu (want %llu each): %s\n", h[0], h[1], h[2], h[3], h[4], want,
              ok ? "ok" : "MISMATCH");
  CK(hipGraphExecDestroy(ex));
  CK(hipGraphDestroy(g));
  return ok ? 0 : 1;
}
