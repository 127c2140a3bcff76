// synth.hip — on-device synthetic streams (kafkastreams-cep_amd/workloads.py, bit for bit)
// plus small utility kernels (watermark).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cep {

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// workloads._h: splitmix64(splitmix64(seed ^ key*C1 ^ j*C2))
__host__ __device__ __forceinline__ uint64_t synth_hash(uint64_t seed, uint64_t key, uint64_t j) {
  return splitmix64(splitmix64(seed ^ (key * 0xD1B54A32D192ED03ull) ^ (j * 0x9E3779B97F4A7C15ull)));
}

__global__ void __launch_bounds__(256) synth_kernel(int kind, uint64_t seed, uint64_t n_keys, uint64_t key_base,
                                                    const uint64_t* __restrict__ key_off, int32_t* __restrict__ c0,
                                                    int32_t* __restrict__ c1) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_keys) return;
  const uint64_t gk = k + key_base;
  const uint64_t a = key_off[k], b = key_off[k + 1];
  if (kind == 0) {  // "abc": v = h % 16
    for (uint64_t p = a; p < b; p++) c0[p] = (int32_t)(synth_hash(seed, gk, p - a) % 16);
    return;
  }
  // "stock": price random walk clamped at 1, volume mixture
  int64_t price = 100 + (int64_t)(gk % 100);
  for (uint64_t p = a; p < b; p++) {
    const uint64_t h = synth_hash(seed, gk, p - a);
    price += (int64_t)(h % 5) - 2;
    if (price < 1) price = 1;
    const uint64_t u = (h >> 8) % 500, r = h >> 20;
    int64_t vol;
    if (u == 0) vol = 1001 + (int64_t)(r % 100);
    else if (u == 1) vol = (int64_t)(r % 700);
    else vol = 900 + (int64_t)(r % 101);
    c0[p] = (int32_t)price;
    c1[p] = (int32_t)vol;
  }
}

hipError_t launch_synth(int kind, uint64_t seed, uint64_t n_keys, uint64_t key_base, const uint64_t* key_off,
                        int32_t* c0, int32_t* c1, hipStream_t st) {
  if (n_keys == 0) return hipSuccess;
  hipLaunchKernelGGL(synth_kernel, dim3((uint32_t)((n_keys + 255) / 256)), dim3(256), 0, st, kind, seed, n_keys,
                     key_base, key_off, c0, c1);
  return hipGetLastError();
}

// event timestamps of a synthetic CSR stream: base + CSR position (each key's events in time
// order, as the reference's stream time advances per record)
__global__ void __launch_bounds__(256) ts_kernel(int64_t* ts, uint64_t n, int64_t base) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    ts[i] = base + (int64_t)i;
}

hipError_t launch_synth_ts(int64_t* ts, uint64_t n, int64_t base, hipStream_t st) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(ts_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, ts, n, base);
  return hipGetLastError();
}

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

namespace cep {
uint64_t synth_hash_host(uint64_t seed, uint64_t key, uint64_t j) { return synth_hash(seed, key, j); }
}  // namespace cep
