// Host-side error checking shared by .hip and .cpp sources.
#pragma once

#include <hip/hip_runtime_api.h>
#include <c10/util/Exception.h>

#define DMP_HIP_CHECK(expr)                                                   \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    if (_e != hipSuccess) {                                                   \
      TORCH_CHECK(false, "HIP error ", hipGetErrorString(_e), " at ", __FILE__, \
                  ":", __LINE__);                                             \
    }                                                                         \
  } while (0)
