// walk_bench.hip — the NFA's real buffer-walk code (csrc/nfa_lane.h Lane::walk_now / flush) on
// a synthetic chain, one lane, outside the matcher kernel: ns per walk node, to compare with
// profiles/micro/chase.hip (the bare dependent-load chase) and with a heavy key's per-node
// cost inside cep_nfa_jit.  A chain of N nodes, node i's only predecessor is node i-1 with
// version [1, 0] (the stock query's Kleene path); an emit walk from the last node visits all
// N (extraction: refs 1 -> 0, nodes deleted, pointers removed), a branch walk first raises the
// refs (refs++ along the path).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../kafkastreams-cep_amd/csrc -o walk_bench walk_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "cep_layout.h"
#include "kernel_args.h"
#include "dewey.h"
#include "nfa_lane.h"

using namespace cep;

struct BenchQ {
  struct EvT {
    int64_t ts;
  };
  static constexpr bool kBeginReg = true, kFold32 = true, quiet = true;
  static constexpr uint32_t kRingLds = 0, begin_stage = 0;
  __device__ uint32_t stage_sk(uint32_t) const { return 1; }
  __device__ uint16_t sk_name(uint32_t sk) const { return (uint16_t)sk; }
};

// mode 0: one emit walk over the chain (walk_now); 1: a branch walk then an emit walk, both
// queued and drained by flush() (the deferred path)
__global__ void walk_kernel(NfaArgs A, uint32_t last, int mode, uint32_t* out_stats) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  BenchQ q;
  Lane<2, BenchQ> L(A, q);
  L.wb = reinterpret_cast<v4u*>(A.walks);
  L.j = last + 1;
  Dewey v;
  dw_init(v, 1);
  v.n = 2;
  v.len = 2;
  v.v[1] = 0;
  v.c[1] = 1;
  if (mode == 0) {
    L.walk_now(kWalkEmit, 1, last, last, v, last + 1);
  } else {
    L.walk(kWalkBranch, 1, last, last, v);
    L.walk(kWalkEmit, 1, last, last, v);
    L.flush();
  }
  out_stats[0] = L.n_pairs;
  out_stats[1] = (uint32_t)L.err;
}

int main() {
  for (uint32_t n : {4096u, 65536u}) {
    std::vector<Node> nodes(n);
    std::vector<Pred> preds0(n);
    for (uint32_t i = 0; i < n; i++) {
      nodes[i] = Node{i, 1, kPred0 | i, kPred0 | i, CEP_NONE, 1u | 0x100u | (1u << 16), 0, 0};
      Pred p{};
      p.prev = i ? i - 1 : CEP_NONE;
      p.next = CEP_NONE;
      p.flags = 2u << 8;
      p.len = 2;
      p.pair[0] = 1;
      p.pair[1] = 1;
      p.pair[2] = 0;
      p.pair[3] = 1;
      preds0[i] = p;
    }
    Node* dn;
    Pred *dp0, *dp;
    uint32_t *out, *top, *stats;
    void* walks;
    hipMalloc(&dn, n * sizeof(Node));
    hipMalloc(&dp0, n * sizeof(Pred));
    hipMalloc(&dp, 1024 * sizeof(Pred));
    hipMalloc(&out, (size_t)(2 * n / 255 + 64) * kOutChunkWords * 4 * 2);
    hipMalloc(&top, 16);
    hipMalloc(&stats, 16);
    hipMalloc(&walks, walkq_bytes(64, 64));
    for (int mode = 0; mode < 2; mode++) {
      float best = 1e30f;
      for (int rep = 0; rep < 3; rep++) {
        hipMemcpy(dn, nodes.data(), n * sizeof(Node), hipMemcpyHostToDevice);
        hipMemcpy(dp0, preds0.data(), n * sizeof(Pred), hipMemcpyHostToDevice);
        hipMemset(top, 0, 16);
        NfaArgs a{};
        a.nodes = dn;
        a.preds0 = dp0;
        a.preds = dp;
        a.out = out;
        a.out_pool = Pool{top, (uint32_t)(4 * n / 255 + 64), 1};
        a.walks = walks;
        a.wcap = 64;
        a.defer = mode == 1;
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        walk_kernel<<<1, 64>>>(a, n - 1, mode, stats);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      uint32_t st[2];
      hipMemcpy(st, stats, 8, hipMemcpyDeviceToHost);
      const double nodes_visited = mode == 0 ? n : 2.0 * n;
      printf("{\"nodes\": %u, \"mode\": \"%s\", \"pairs\": %u, \"err\": %u, \"ns_per_node\": %.1f}\n", n,
             mode == 0 ? "walk_now emit" : "flush: branch + emit", st[0], st[1], best * 1e6 / nodes_visited);
    }
    hipFree(dn);
    hipFree(dp0);
    hipFree(dp);
    hipFree(out);
    hipFree(top);
    hipFree(stats);
    hipFree(walks);
  }
  return 0;
}
