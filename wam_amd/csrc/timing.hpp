// Optional live per-launch timing: when enabled (wam_timing_enable), every kernel launch of the
// library is bracketed by hipEventRecord on the launch stream and logged with its kernel name and
// ALGORITHMIC bytes (each input element read once, each output written once). bench.py drains the
// records to report achieved GB/s per kernel measured on the stream the kernels run on.
#pragma once
#include <hip/hip_runtime.h>

struct WamTimer {
  hipStream_t st;
  const char* name;
  double bytes;
  hipEvent_t s = nullptr, e = nullptr;
  WamTimer(hipStream_t st_, const char* name_, double bytes_);
  ~WamTimer();
};
