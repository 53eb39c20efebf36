// roctx ranges/marks for rocprofv3 --marker-trace.  Host-side ranges: they bracket
// the enqueue/poll work of the driver (init, graph batches, state polls, checkpoints) and, with
// --kernel-trace, line up with the kernels those calls launch.  Streams are named so traces
// show "pmx:compute" / "pmx:comm".  Compiled in only where the HIP runtime is used.
#pragma once

#include <rocprofiler-sdk-roctx/roctx.h>

namespace pmx {

class TraceRange {
 public:
  explicit TraceRange(const char* name) { roctxRangePushA(name); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

inline void trace_mark(const char* msg) { roctxMarkA(msg); }

}  // namespace pmx
