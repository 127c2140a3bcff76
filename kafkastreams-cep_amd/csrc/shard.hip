// shard.hip — a rank's shard of a key-partitioned stream (multi-GPU key sharding).
//
// The keys a rank owns are chosen on the host (kafkastreams-cep_amd/shard.py: Kafka's
// DefaultPartitioner over the key ids); this kernel gathers their events into the shard's own
// CSR batch: one wave per owned key, each column copied with coalesced 256-B wave accesses.
// HBM-bound (reads and writes the shard's bytes once).
#include <hip/hip_runtime.h>

#include "kernel_args.h"

namespace cep {

__global__ void __launch_bounds__(256) gather_keys_kernel(uint64_t n_sel, const uint32_t* __restrict__ sel,
                                                          const uint64_t* __restrict__ src_off,
                                                          const uint64_t* __restrict__ dst_off, Cols src, Cols dst,
                                                          uint32_t wide, int nf, const int64_t* __restrict__ src_ts,
                                                          int64_t* __restrict__ dst_ts) {
  const uint64_t k = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  if (k >= n_sel) return;
  const uint64_t s0 = src_off[sel[k]], n = src_off[sel[k] + 1] - s0, d0 = dst_off[k];
  for (int f = 0; f < nf; f++) {
    if ((wide >> f) & 1u) {
      const uint64_t* a = static_cast<const uint64_t*>(src.p[f]) + s0;
      uint64_t* b = static_cast<uint64_t*>(const_cast<void*>(dst.p[f])) + d0;
      for (uint64_t j = lane; j < n; j += 64) b[j] = a[j];
    } else {
      const uint32_t* a = static_cast<const uint32_t*>(src.p[f]) + s0;
      uint32_t* b = static_cast<uint32_t*>(const_cast<void*>(dst.p[f])) + d0;
      for (uint64_t j = lane; j < n; j += 64) b[j] = a[j];
    }
  }
  if (src_ts && dst_ts)
    for (uint64_t j = lane; j < n; j += 64) dst_ts[d0 + j] = src_ts[s0 + j];
}

hipError_t gather_keys(uint64_t n_sel, const uint32_t* sel, const uint64_t* src_off, const uint64_t* dst_off,
                       int nf, const uint32_t* col_bytes, const void* const* src_cols, void* const* dst_cols,
                       const int64_t* src_ts, int64_t* dst_ts, hipStream_t st) {
  if (n_sel == 0) return hipSuccess;
  if (nf < 0 || nf > kMaxFields) return hipErrorInvalidValue;
  Cols s{}, d{};
  uint32_t wide = 0;
  for (int f = 0; f < nf; f++) {
    if (col_bytes[f] != 4 && col_bytes[f] != 8) return hipErrorInvalidValue;
    wide |= (col_bytes[f] == 8 ? 1u : 0u) << f;
    s.p[f] = src_cols[f];
    d.p[f] = dst_cols[f];
  }
  hipLaunchKernelGGL(gather_keys_kernel, dim3((uint32_t)((n_sel + 3) / 4)), dim3(256), 0, st, n_sel, sel, src_off,
                     dst_off, s, d, wide, nf, src_ts, dst_ts);
  return hipGetLastError();
}

}  // namespace cep
