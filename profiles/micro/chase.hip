// chase.hip — per-hop latency of one lane's dependent pointer chase on MI355X, shaped like a
// buffer walk step (nfa_lane.h walk_node): per hop four independent 16-B loads (a 32-B node and
// the first 32 B of its 64-B predecessor slot), a refcount store, then the next index from the
// loaded data.  Working sets from L2-resident (256 KiB) to HBM-sized.  Prints ns per hop.
//   hipcc --offload-arch=gfx950 -O3 -o chase chase.hip && ./chase
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ void chase(const v4u* nodes, const v4u* preds, uint32_t* refs_out, uint32_t start, int hops, int store,
                      uint32_t* sink) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t s = start, acc = 0;
  for (int h = 0; h < hops; h++) {
    const v4u n0 = nodes[2 * s], n1 = nodes[2 * s + 1];
    const v4u f0 = preds[4 * s], f1 = preds[4 * s + 1];
    if (store) refs_out[s] = n0.y + 1;
    acc += n1.y + f1.x;
    s = f0.x ^ (n0.z & 0);  // the next node: the first predecessor's key
  }
  sink[0] = acc + s;
}

int main() {
  const int hops = 200000;
  for (uint32_t n : {4096u, 65536u, 1u << 20, 1u << 24}) {
    std::vector<uint32_t> perm(n);
    for (uint32_t i = 0; i < n; i++) perm[i] = i;
    srand(1);
    for (uint32_t i = n - 1; i > 0; i--) std::swap(perm[i], perm[rand() % (i + 1)]);
    std::vector<v4u> nodes(2 * (size_t)n), preds(4 * (size_t)n);
    for (uint32_t i = 0; i < n; i++) {
      nodes[2 * i] = v4u{i, 1, 0, 0};
      nodes[2 * i + 1] = v4u{0, 7, 0, 0};
      preds[4 * i] = v4u{perm[i], 0, 0, 0};  // a single cycle through all nodes (random order)
    }
    // make it one cycle: follow perm as a successor table built from a shuffled order
    for (uint32_t k = 0; k < n; k++) preds[4 * perm[k]].x = perm[(k + 1) % n];
    v4u *dn, *dp;
    uint32_t *dr, *sink;
    hipMalloc(&dn, nodes.size() * 16);
    hipMalloc(&dp, preds.size() * 16);
    hipMalloc(&dr, 4 * (size_t)n);
    hipMalloc(&sink, 4);
    hipMemcpy(dn, nodes.data(), nodes.size() * 16, hipMemcpyHostToDevice);
    hipMemcpy(dp, preds.data(), preds.size() * 16, hipMemcpyHostToDevice);
    for (int store = 0; store < 2; store++) {
      hipEvent_t a, b;
      hipEventCreate(&a);
      hipEventCreate(&b);
      chase<<<1, 64>>>(dn, dp, dr, perm[0], hops / 10, store, sink);  // warm
      hipEventRecord(a);
      chase<<<1, 64>>>(dn, dp, dr, perm[0], hops, store, sink);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      printf("{\"nodes\": %u, \"bytes\": %zu, \"store\": %d, \"ns_per_hop\": %.1f}\n", n, (size_t)n * 96, store,
             ms * 1e6 / hops);
    }
    hipFree(dn);
    hipFree(dp);
    hipFree(dr);
    hipFree(sink);
  }
  return 0;
}
