// synth_gen.hip — the synthetic streams of the bench and the tests, generated on the device
// (kafkastreams-cep_amd/workloads.py bit for bit), in CSR or arrival order, plus StockEvent
// JSON record values.  A separate library (libcep_synth.so, include/cep_synth.h): test and
// bench infrastructure, not part of the matcher (libcep.so), which links nothing of it.  The
// arrival-order permutation and the JSON offsets use hipCUB here; the product path's sorts
// and scans are hand-written (partition.hip, symbol.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <functional>
#include <hipcub/hipcub.hpp>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/cep_synth.h"

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

__global__ void __launch_bounds__(256) iota_u32(uint32_t* v, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) v[i] = (uint32_t)i;
}

// ---- synthetic arrival order: CSR position p of key k, index j -> sort key j * n_keys + k
__global__ void __launch_bounds__(256) arrival_keys(const uint64_t* __restrict__ key_off, uint64_t n_keys,
                                                    uint64_t* skey, uint32_t* kid) {
  const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n_keys) return;
  for (uint64_t p = key_off[k]; p < key_off[k + 1]; p++) {
    skey[p] = (p - key_off[k]) * n_keys + k;
    kid[p] = (uint32_t)k;
  }
}

__global__ void __launch_bounds__(256) arrival_gather(const uint32_t* __restrict__ order, uint64_t n, const uint32_t* kid,
                                                      const int32_t* c0, const int32_t* c1, uint32_t* key_out,
                                                      int32_t* o0, int32_t* o1) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = order[i];
  key_out[i] = kid[p];
  o0[i] = c0[p];
  if (c1) o1[i] = c1[p];
}

// CSR stream (key_off, c0, c1) -> arrival order (key_out, o0, o1), on the device
hipError_t csr_to_arrival(const uint64_t* key_off, uint64_t n_keys, uint64_t n, uint64_t max_nk, const int32_t* c0,
                          const int32_t* c1, uint32_t* key_out, int32_t* o0, int32_t* o1, hipStream_t st) {
  if (n == 0 || n_keys == 0) return hipSuccess;
  uint64_t *skey = nullptr, *skey2 = nullptr;
  uint32_t *kid = nullptr, *idx = nullptr, *order = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  hipError_t e = hipSuccess;
  auto ok = [&](hipError_t x) { if (e == hipSuccess) e = x; return e == hipSuccess; };
  int bits = 1;  // sort keys < max_nk * n_keys
  while (bits < 64 && (max_nk * n_keys) >> bits) bits++;
  if (ok(hipMalloc(&skey, 8 * n)) && ok(hipMalloc(&skey2, 8 * n)) && ok(hipMalloc(&kid, 4 * n)) &&
      ok(hipMalloc(&idx, 4 * n)) && ok(hipMalloc(&order, 4 * n))) {
    hipLaunchKernelGGL(arrival_keys, dim3((uint32_t)((n_keys + 255) / 256)), dim3(256), 0, st, key_off, n_keys, skey, kid);
    hipLaunchKernelGGL(iota_u32, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, idx, n);
    ok(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, skey, skey2, idx, order, (int)n, 0, bits, st));
    if (ok(hipMalloc(&tmp, tmp_bytes + 256)) &&
        ok(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, skey, skey2, idx, order, (int)n, 0, bits, st))) {
      hipLaunchKernelGGL(arrival_gather, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, order, n, kid, c0, c1,
                         key_out, o0, o1);
      ok(hipGetLastError());
      ok(hipStreamSynchronize(st));
    }
  }
  for (void* p : {(void*)skey, (void*)skey2, (void*)kid, (void*)idx, (void*)order, tmp})
    if (p) (void)hipFree(p);
  return e;
}

// ---- synthetic records: json-simple's toJSONString of the demo's StockEvent
// (StockEventSerDe.java:75-82), {"name":"e<i+1>","price":P,"volume":V}, the README's format
// (README.md:73-80) ----

__device__ __forceinline__ uint32_t ndigits(int64_t v) {
  uint64_t m = v < 0 ? 0ull - (uint64_t)v : (uint64_t)v;
  uint32_t d = 1;
  while (m >= 10) { m /= 10; d++; }
  return d + (v < 0);
}

__global__ void __launch_bounds__(256) json_len_kernel(const int32_t* price, const int32_t* volume, uint64_t n,
                                                       uint64_t* len) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) len[i] = 31 + ndigits((int64_t)i + 1) + ndigits(price[i]) + ndigits(volume[i]);
}

__device__ __forceinline__ uint64_t put_str(uint8_t* o, uint64_t p, const char* s) {
  while (*s) o[p++] = (uint8_t)*s++;
  return p;
}
__device__ __forceinline__ uint64_t put_int(uint8_t* o, uint64_t p, int64_t v) {
  const uint32_t d = ndigits(v);
  uint64_t m = v < 0 ? 0ull - (uint64_t)v : (uint64_t)v;
  if (v < 0) o[p] = '-';
  for (uint32_t k = 0; k < d - (v < 0); k++) {
    o[p + d - 1 - k] = (uint8_t)('0' + m % 10);
    m /= 10;
  }
  return p + d;
}

__global__ void __launch_bounds__(256) json_write_kernel(const int32_t* price, const int32_t* volume, uint64_t n,
                                                         const uint64_t* off, uint8_t* out) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint64_t p = off[i];
  // json-simple's JSONObject (a HashMap) iterates volume, price, name (StockEventSerDe.java:75-82)
  p = put_str(out, p, "{\"volume\":");
  p = put_int(out, p, volume[i]);
  p = put_str(out, p, ",\"price\":");
  p = put_int(out, p, price[i]);
  p = put_str(out, p, ",\"name\":\"e");
  p = put_int(out, p, (int64_t)i + 1);
  p = put_str(out, p, "\"}");
}

// lengths -> rec_off (inclusive scan into rec_off+1) ; total bytes returned through *total
hipError_t synth_stock_json(const int32_t* price, const int32_t* volume, uint64_t n, uint8_t* out, uint64_t cap,
                            uint64_t* rec_off, uint64_t* total) {
  hipError_t e;
  if ((e = hipMemset(rec_off, 0, 8)) != hipSuccess) return e;
  if (n == 0) { *total = 0; return hipSuccess; }
  const dim3 g((uint32_t)((n + 255) / 256));
  hipLaunchKernelGGL(json_len_kernel, g, dim3(256), 0, 0, price, volume, n, rec_off + 1);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  size_t tmp = 0;
  if ((e = hipcub::DeviceScan::InclusiveSum(nullptr, tmp, rec_off + 1, rec_off + 1, (int)n)) != hipSuccess) return e;
  void* scratch = nullptr;
  if ((e = hipMalloc(&scratch, tmp + 16)) != hipSuccess) return e;
  e = hipcub::DeviceScan::InclusiveSum(scratch, tmp, rec_off + 1, rec_off + 1, (int)n);
  if (e == hipSuccess) e = hipMemcpy(total, rec_off + n, 8, hipMemcpyDeviceToHost);
  (void)hipFree(scratch);
  if (e != hipSuccess) return e;
  if (*total > cap) return hipSuccess;  // caller sees total > cap and retries with more room
  hipLaunchKernelGGL(json_write_kernel, g, dim3(256), 0, 0, price, volume, n, rec_off, out);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  return hipDeviceSynchronize();
}

}  // namespace cep

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define HIPCHECK(x)                                                                          \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess)                                                                    \
      throw HipError(std::string(#x) + ": " + hipGetErrorString(e_));                        \
  } while (0)

struct DeviceGuard {
  int prev = 0;
  explicit DeviceGuard(int d) {
    (void)hipGetDevice(&prev);
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DeviceGuard() { (void)hipSetDevice(prev); }
};

struct DevMem {  // scratch device buffer for one call
  void* p = nullptr;
  explicit DevMem(size_t n) {
    if (n && hipMalloc(&p, n) != hipSuccess) throw std::bad_alloc();
  }
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
  ~DevMem() {
    if (p) (void)hipFree(p);
  }
};

int guarded(const std::function<void()>& f) {
  try {
    f();
    return CEP_SYNTH_OK;
  } catch (HipError& e) {
    return fail(CEP_SYNTH_E_HIP, e.what());
  } catch (std::bad_alloc&) {
    return fail(CEP_SYNTH_E_NOMEM, "device allocation failed");
  } catch (std::exception& e) {
    return fail(CEP_SYNTH_E_INVALID, e.what());
  }
}

}  // namespace

using namespace cep;

extern "C" {

const char* cep_synth_last_error(void) { return g_err.c_str(); }

static std::vector<uint64_t> synth_offsets(int kind, uint64_t seed, uint64_t n_keys, uint64_t key_base,
                                           uint32_t mean) {
  (void)kind;
  std::vector<uint64_t> off(n_keys + 1, 0);
  const uint64_t sp = (uint64_t)std::floor(std::sqrt((double)mean));
  for (uint64_t k = 0; k < n_keys; k++) {
    const uint64_t h = cep::synth_hash(seed, k + key_base, 0xFFFFFFFFull);
    off[k + 1] = off[k] + (mean - sp + h % (2 * sp + 1));
  }
  return off;
}

int cep_synth_count(int device, int kind, uint64_t seed, uint64_t n_keys, uint64_t key_base, uint32_t mean_events,
                    uint64_t* n_events) {
  (void)device;
  if (!n_events || mean_events == 0) return fail(CEP_SYNTH_E_INVALID, "bad argument");
  *n_events = synth_offsets(kind, seed, n_keys, key_base, mean_events)[n_keys];
  return CEP_SYNTH_OK;
}

int cep_synth_generate(int device, int kind, uint64_t seed, uint64_t n_keys, uint64_t key_base, uint32_t mean_events,
                       uint64_t* key_off_dev, int32_t* const* cols_dev) {
  if (!key_off_dev || !cols_dev || mean_events == 0) return fail(CEP_SYNTH_E_INVALID, "bad argument");
  if (kind != 0 && kind != 1) return fail(CEP_SYNTH_E_INVALID, "kind must be 0 (abc) or 1 (stock)");
  return guarded([&] {
    DeviceGuard g(device);
    HIPCHECK(hipSetDevice(device));
    auto off = synth_offsets(kind, seed, n_keys, key_base, mean_events);
    HIPCHECK(hipMemcpy(key_off_dev, off.data(), sizeof(uint64_t) * (n_keys + 1), hipMemcpyHostToDevice));
    HIPCHECK(launch_synth(kind, seed, n_keys, key_base, key_off_dev, cols_dev[0], kind == 1 ? cols_dev[1] : nullptr,
                          nullptr));
    HIPCHECK(hipDeviceSynchronize());
  });
}

int cep_synth_ts(int device, uint64_t n_events, int64_t base, int64_t* ts_dev) {
  if (!ts_dev && n_events) return fail(CEP_SYNTH_E_INVALID, "null argument");
  return guarded([&] {
    DeviceGuard g(device);
    HIPCHECK(hipSetDevice(device));
    HIPCHECK(launch_synth_ts(ts_dev, n_events, base, nullptr));
    HIPCHECK(hipDeviceSynchronize());
  });
}

int cep_synth_generate_arrival(int device, int kind, uint64_t seed, uint64_t n_keys, uint64_t key_base,
                               uint32_t mean_events, uint32_t* keys_dev, int32_t* const* cols_dev) {
  if (!keys_dev || !cols_dev || mean_events == 0) return fail(CEP_SYNTH_E_INVALID, "bad argument");
  if (kind != 0 && kind != 1) return fail(CEP_SYNTH_E_INVALID, "kind must be 0 (abc) or 1 (stock)");
  return guarded([&] {
    DeviceGuard g(device);
    HIPCHECK(hipSetDevice(device));
    auto off = synth_offsets(kind, seed, n_keys, key_base, mean_events);
    const uint64_t n = off[n_keys];
    uint64_t max_nk = 1;
    for (uint64_t k = 0; k < n_keys; k++) max_nk = std::max<uint64_t>(max_nk, off[k + 1] - off[k]);
    DevMem d_off(8 * (n_keys + 1)), c0(4 * std::max<uint64_t>(n, 1)), c1(kind == 1 ? 4 * std::max<uint64_t>(n, 1) : 0);
    HIPCHECK(hipMemcpy(d_off.p, off.data(), 8 * (n_keys + 1), hipMemcpyHostToDevice));
    HIPCHECK(launch_synth(kind, seed, n_keys, key_base, d_off.as<uint64_t>(), c0.as<int32_t>(),
                          kind == 1 ? c1.as<int32_t>() : nullptr, nullptr));
    HIPCHECK(csr_to_arrival(d_off.as<uint64_t>(), n_keys, n, max_nk, c0.as<int32_t>(),
                            kind == 1 ? c1.as<int32_t>() : nullptr, keys_dev, cols_dev[0],
                            kind == 1 ? cols_dev[1] : nullptr, nullptr));
    HIPCHECK(hipDeviceSynchronize());
  });
}

int cep_synth_stock_json(int device, const int32_t* price_dev, const int32_t* volume_dev, uint64_t n,
                         uint8_t* out_dev, uint64_t cap, uint64_t* rec_off_dev, uint64_t* total) {
  if (!rec_off_dev || !total || (n && (!price_dev || !volume_dev))) return fail(CEP_SYNTH_E_INVALID, "null argument");
  if (n >= (1ull << 31)) return fail(CEP_SYNTH_E_INVALID, "at most 2^31 - 1 records");
  return guarded([&] {
    DeviceGuard g(device);
    HIPCHECK(hipSetDevice(device));
    HIPCHECK(synth_stock_json(price_dev, volume_dev, n, out_dev, out_dev ? cap : 0, rec_off_dev, total));
  });
}

}  // extern "C"
