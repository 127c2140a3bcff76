// floor.hip — per key, the oldest event a streaming session's shared buffer still holds
// (cep_live_floor).  The reference's buffer keeps an event for as long as a node of it is in
// the store (KVSharedVersionedBuffer.java:143-171 deletes a node when its last reference is
// walked); only those events can appear in a later Sequence, so a host that keeps the
// records it forwards (processor.py) may drop every older one.  One pass over the node
// pool: a live node lowers its key's floor to its event (atomicMin), HBM-bound.
#include <hip/hip_runtime.h>

#include "kernel_args.h"

namespace cep {

__global__ void __launch_bounds__(256) live_floor_kernel(const Node* __restrict__ nodes, uint64_t n, uint64_t n_keys,
                                                         uint32_t* __restrict__ floor) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint4 q = reinterpret_cast<const uint4*>(nodes + i)[0];   // {event, refs, head, tail}
  const uint4 q1 = reinterpret_cast<const uint4*>(nodes + i)[1];  // {same_next, meta, lk, key}
  if ((q1.y & 0x100u) && q1.w < n_keys) atomicMin(floor + q1.w, q.x);
}

hipError_t launch_live_floor(const Node* nodes, uint64_t n_nodes, uint64_t n_keys, uint32_t* floor, hipStream_t st) {
  hipError_t e = hipMemsetAsync(floor, 0xFF, 4 * n_keys, st);
  if (e != hipSuccess || n_nodes == 0) return e;
  hipLaunchKernelGGL(live_floor_kernel, dim3((uint32_t)((n_nodes + 255) / 256)), dim3(256), 0, st, nodes, n_nodes,
                     n_keys, floor);
  return hipGetLastError();
}

}  // namespace cep
