// pmx — MI355X-native Poisson/fictitious-domain PCG solver.
// Common error handling.  Replaces the reference's `checkCuda(err,msg)` helper
// (stage4-mpi+cuda/poisson_mpi_cuda_f.cu:20-27), which printed and exit()ed.
// Here every failure carries file:line and is raised as pmx::Error so the
// Python bindings surface it as a RuntimeError instead of killing the process.
#pragma once

#include <cstdio>
#include <cstdlib>
#include <sstream>
#include <stdexcept>
#include <string>

namespace pmx {

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

[[noreturn]] inline void fail(const char* file, int line, const std::string& what) {
  std::ostringstream os;
  os << "pmx error at " << file << ":" << line << ": " << what;
  throw Error(os.str());
}

}  // namespace pmx

#define PMX_CHECK(cond, msg)                                                   \
  do {                                                                         \
    if (!(cond)) {                                                             \
      std::ostringstream pmx_os_;                                              \
      pmx_os_ << "check failed: " #cond " — " << msg;                          \
      ::pmx::fail(__FILE__, __LINE__, pmx_os_.str());                          \
    }                                                                          \
  } while (0)

#if defined(__HIPCC__) || defined(PMX_WITH_HIP)
#include <hip/hip_runtime.h>
#define HIP_CHECK(expr)                                                        \
  do {                                                                         \
    hipError_t pmx_e_ = (expr);                                                \
    if (pmx_e_ != hipSuccess)                                                  \
      ::pmx::fail(__FILE__, __LINE__,                                          \
                  std::string(#expr " -> ") + hipGetErrorString(pmx_e_));      \
  } while (0)
#endif
