// capi_internal.h — helpers shared by the C-ABI translation units.
#pragma once

#include <new>
#include <stdexcept>

#include "phantom_amd.h"
#include "hip_check.h"

namespace phantom::capi {
int fail(int code, const char* msg);
int from_hip(hipError_t e);
}  // namespace phantom::capi

// Run `body` (which returns an int status) and map C++ exceptions to status codes, the way
// the reference's exception classes map (std::invalid_argument, std::logic_error,
// std::runtime_error from CUDA checks).
#define PHX_CAPI_GUARD(...)                                                                   \
  try {                                                                                       \
    __VA_ARGS__                                                                                   \
  } catch (const ::phantom::hip_error& e) {                                                   \
    return ::phantom::capi::fail(PHANTOM_ERR_HIP, e.what());                                  \
  } catch (const std::invalid_argument& e) {                                                  \
    return ::phantom::capi::fail(PHANTOM_ERR_INVALID_ARGUMENT, e.what());                     \
  } catch (const std::logic_error& e) {                                                       \
    return ::phantom::capi::fail(PHANTOM_ERR_LOGIC, e.what());                                \
  } catch (const std::bad_alloc&) {                                                           \
    return ::phantom::capi::fail(PHANTOM_ERR_INTERNAL, "out of host memory");                 \
  } catch (const std::exception& e) {                                                         \
    return ::phantom::capi::fail(PHANTOM_ERR_INTERNAL, e.what());                             \
  }
