// hip_check.h — error propagation for HIP runtime calls.  The reference throws
// std::runtime_error from PHANTOM_CHECK_CUDA (include/cuda_wrapper.cuh:19-47); this engine
// does the same on the C++ side and converts to status codes at the C-ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdexcept>
#include <string>

namespace phantom {

class hip_error : public std::runtime_error {
 public:
  hip_error(hipError_t e, const char* what_call)
      : std::runtime_error(std::string(what_call) + ": " + hipGetErrorString(e)), code(e) {}
  hipError_t code;
};

// Status of a kernel launch (or any HIP call) -> exception.  PHX_DEBUG_SYNC=1 also synchronises
// the device after every checked call, so an asynchronous failure is reported by the launch that
// caused it (debugging aid; off by default).
bool debug_sync_enabled();
inline void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw hip_error(e, what);
  if (debug_sync_enabled()) {
    const hipError_t s = hipDeviceSynchronize();
    if (s != hipSuccess) throw hip_error(s, what);
  }
}

}  // namespace phantom

#define PHX_CHECK(call)                                         \
  do {                                                          \
    hipError_t phx_err_ = (call);                               \
    if (phx_err_ != hipSuccess) throw ::phantom::hip_error(phx_err_, #call); \
  } while (0)
