// partition.hip — arrival-order batches -> the key-partitioned (CSR) layout the matchers read.
//
// The reference's processor receives records one at a time in arrival order
// (CEPProcessor.process, CEPProcessor.java:155-163) and each key's NFA sees that key's records
// in that order.  A batch handed over in arrival order (one key id per event) is
// partitioned on the device: a stable LSD radix sort of (key, arrival index) pairs by key
// (rocPRIM through hipCUB), key_off by a binary search per key over the sorted keys, then one
// gather per column.
// Stability is what keeps every key's events in arrival order.  All passes are HBM-bound.
//
// Also the synthetic arrival-order stream of the bench/tests: the CSR stream of
// workloads.generate interleaved round-robin, arrival order = (index within key, key).
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "kernel_args.h"

namespace cep {

__global__ void __launch_bounds__(256) iota_u32(uint32_t* v, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) v[i] = (uint32_t)i;
}

// range check of the key ids (the sort only looks at the bits of n_keys - 1)
__global__ void __launch_bounds__(256) check_keys(const uint32_t* __restrict__ key, uint64_t n, uint64_t n_keys,
                                                  unsigned* bad) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n && key[i] >= n_keys) atomicOr(bad, 1u);
}

// key_off[k] = first position of a key >= k in the sorted keys (binary search per key)
__global__ void __launch_bounds__(256) key_offsets(const uint32_t* __restrict__ sorted, uint64_t n, uint64_t n_keys,
                                                   uint64_t* key_off) {
  const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (k > n_keys) return;
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) / 2;
    if (sorted[mid] < k) lo = mid + 1;
    else hi = mid;
  }
  key_off[k] = lo;
}

// CSR position p <- arrival index perm[p], for every column (4- or 8-byte values) and ts
__global__ void __launch_bounds__(256) gather_cols(const uint32_t* __restrict__ perm, uint64_t n, int nf, Cols in,
                                                   Cols out, uint32_t wide_mask, const int64_t* ts_in,
                                                   int64_t* ts_out) {
  const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= n) return;
  const uint32_t src = perm[p];
  for (int f = 0; f < nf; f++) {
    if ((wide_mask >> f) & 1u)
      ((int64_t*)out.p[f])[p] = ((const int64_t*)in.p[f])[src];
    else
      ((int32_t*)out.p[f])[p] = ((const int32_t*)in.p[f])[src];
  }
  if (ts_in) ts_out[p] = ts_in[src];
}

static int key_bits(uint64_t n_keys) {
  int b = 1;
  while (b < 32 && (1ull << b) < n_keys) b++;
  return b;
}

// Device scratch of partition(): bytes needed for n events over n_keys keys.
size_t partition_scratch_bytes(uint64_t n, uint64_t n_keys) {
  (void)n_keys;
  size_t tmp = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                     (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)std::max<uint64_t>(n, 1));
  return tmp + 256;
}

// arrival-order batch -> key_off[n_keys + 1], perm[n] (arrival index of each CSR position),
// columns in CSR order.  scratch: partition_scratch_bytes; sorted_keys, idx: n u32 each.
hipError_t partition(const uint32_t* key, uint64_t n, uint64_t n_keys, int nf, Cols in, Cols out, uint32_t wide_mask,
                     const int64_t* ts_in, int64_t* ts_out, uint64_t* key_off, uint64_t* cnt, uint32_t* perm,
                     uint32_t* sorted_keys, uint32_t* idx, void* scratch, size_t scratch_bytes, unsigned* bad,
                     hipStream_t st) {
  (void)cnt;
  const uint32_t blocks = (uint32_t)((n + 255) / 256);
  hipError_t e = hipSuccess;
  if (n) {
    hipLaunchKernelGGL(check_keys, dim3(blocks), dim3(256), 0, st, key, n, n_keys, bad);
    hipLaunchKernelGGL(iota_u32, dim3(blocks), dim3(256), 0, st, idx, n);
    size_t tmp = scratch_bytes;
    e = hipcub::DeviceRadixSort::SortPairs(scratch, tmp, key, sorted_keys, idx, perm, (int)n, 0, key_bits(n_keys), st);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(key_offsets, dim3((uint32_t)((n_keys + 256) / 256)), dim3(256), 0, st, sorted_keys, n, n_keys,
                     key_off);
  if (n) hipLaunchKernelGGL(gather_cols, dim3(blocks), dim3(256), 0, st, perm, n, nf, in, out, wide_mask, ts_in, ts_out);
  return hipGetLastError();
}

// keys by estimated work, longest first (the NFA's lane order, session.cpp)
hipError_t sort_keys_by_work(const uint32_t* est, uint32_t* est_sorted, uint32_t* iota_tmp, uint32_t* order,
                             uint64_t n, void*& tmp, size_t& tmp_bytes, hipStream_t st) {
  hipLaunchKernelGGL(iota_u32, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, iota_tmp, n);
  size_t need = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairsDescending(nullptr, need, est, est_sorted, iota_tmp, order, (int)n,
                                                              0, 32, st);
  if (e != hipSuccess) return e;
  if (need > tmp_bytes) {
    if (tmp) (void)hipFree(tmp);
    tmp = nullptr;
    tmp_bytes = 0;
    if ((e = hipMalloc(&tmp, need)) != hipSuccess) return e;
    tmp_bytes = need;
  }
  return hipcub::DeviceRadixSort::SortPairsDescending(tmp, need, est, est_sorted, iota_tmp, order, (int)n, 0, 32, st);
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

}  // namespace cep
