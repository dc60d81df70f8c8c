// Shared device/host helpers for the torchmetrics_forked_amd native library (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include <cstdint>

#include "device_common.h"

namespace tmx {

inline hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define TMX_CHECK_HIP(expr)                                                              \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    TORCH_CHECK(_e == hipSuccess, "HIP error: ", hipGetErrorString(_e), " at ", #expr); \
  } while (0)

#define TMX_LAUNCH_CHECK() TMX_CHECK_HIP(hipGetLastError())

}  // namespace tmx



// Dispatch over the float dtypes the framework accepts for score tensors.
#define TMX_DISPATCH_FLOAT(dtype, NAME, ...)                                       \
  [&] {                                                                            \
    switch (dtype) {                                                               \
      case at::kFloat: { using scalar_t = float; return __VA_ARGS__(); }           \
      case at::kDouble: { using scalar_t = double; return __VA_ARGS__(); }         \
      case at::kBFloat16: { using scalar_t = __hip_bfloat16; return __VA_ARGS__(); } \
      case at::kHalf: { using scalar_t = __half; return __VA_ARGS__(); }           \
      default: TORCH_CHECK(false, NAME, ": unsupported dtype ", dtype);            \
    }                                                                              \
  }()

#define TMX_DISPATCH_HALF(dtype, NAME, ...)                                        \
  [&] {                                                                            \
    switch (dtype) {                                                               \
      case at::kBFloat16: { using scalar_t = __hip_bfloat16; return __VA_ARGS__(); } \
      case at::kHalf: { using scalar_t = __half; return __VA_ARGS__(); }           \
      default: TORCH_CHECK(false, NAME, ": expected a 16-bit float tensor, got ", dtype); \
    }                                                                              \
  }()
