// watermark.hip — the batch's largest event time (cep_watermark; multi-GPU runs reduce the
// ranks' values with min over RCCL).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cep {

// The batch's largest timestamp (the watermark).  A streaming read of 8 bytes per event:
// 16-byte loads, four in flight per thread, one wave reduction and one atomic per wave.
__global__ void __launch_bounds__(256) max_kernel(const int64_t* __restrict__ ts, uint64_t n,
                                                  unsigned long long* out) {
  int64_t m = INT64_MIN;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (((uintptr_t)ts & 15) == 0) {
    const longlong2* t2 = reinterpret_cast<const longlong2*>(ts);
    const uint64_t n2 = n / 2;
    for (; i + 3 * stride < n2; i += 4 * stride) {
      const longlong2 a = t2[i], b = t2[i + stride], c = t2[i + 2 * stride], d = t2[i + 3 * stride];
      const int64_t x = a.x > a.y ? a.x : a.y, y = b.x > b.y ? b.x : b.y;
      const int64_t z = c.x > c.y ? c.x : c.y, w = d.x > d.y ? d.x : d.y;
      const int64_t xy = x > y ? x : y, zw = z > w ? z : w;
      const int64_t v = xy > zw ? xy : zw;
      m = v > m ? v : m;
    }
    for (; i < n2; i += stride) {
      const longlong2 a = t2[i];
      const int64_t v = a.x > a.y ? a.x : a.y;
      m = v > m ? v : m;
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) m = ts[n - 1] > m ? ts[n - 1] : m;
  } else {
    for (; i < n; i += stride) m = ts[i] > m ? ts[i] : m;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t y = __shfl_down(m, o, 64);
    m = y > m ? y : m;
  }
  // order-preserving map of signed to unsigned for atomicMax
  if ((threadIdx.x & 63) == 0) atomicMax(out, (unsigned long long)m ^ 0x8000000000000000ull);
}

hipError_t launch_max(const int64_t* ts, uint64_t n, unsigned long long* out, hipStream_t st) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = (n / 2 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL(max_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, ts, n, out);
  return hipGetLastError();
}

}  // namespace cep
