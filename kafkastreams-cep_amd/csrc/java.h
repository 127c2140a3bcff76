// java.h — Java primitive semantics on the device (JLS 5.1.3 casts, 15.17 division).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cep_layout.h"
#include "kernel_args.h"

namespace cep {

__device__ __forceinline__ double as_f64(int64_t x) { return __longlong_as_double(x); }
__device__ __forceinline__ int64_t from_f64(double x) { return __double_as_longlong(x); }

__device__ __forceinline__ int64_t java_d2i(double d) {
  if (d != d) return 0;
  if (d >= 2147483647.0) return 2147483647;
  if (d <= -2147483648.0) return -2147483648LL;
  return (int64_t)(int32_t)d;
}
__device__ __forceinline__ int64_t java_d2l(double d) {
  if (d != d) return 0;
  if (d >= 9223372036854775807.0) return INT64_MAX;
  if (d <= -9223372036854775808.0) return INT64_MIN;
  return (int64_t)d;
}
__device__ __forceinline__ int64_t wrap32(int64_t x) { return (int64_t)(int32_t)(uint32_t)(uint64_t)x; }

}  // namespace cep
