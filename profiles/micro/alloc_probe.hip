// alloc_probe.hip — tests the two allocator hazards behind the round-5 arrival-order flake
//  on the GPU box, without the matcher:
//  1. does hipFree wait for a kernel still using the buffer on a hipStreamNonBlocking stream?
//     (DBuf::ensure frees a buffer before re-allocating it; the stencil path returns without a
//     host sync, so a kernel of the previous push may still run)
//  2. does the stream-ordered pool (hipMallocAsync / hipFreeAsync, the pre-fix scan_u32 and
//     today's symbol_keys) ever hand out memory that overlaps a live hipMalloc buffer, and does
//     a victim buffer filled with a pattern stay intact while small pool blocks are written,
//     freed, trimmed at synchronisation and re-allocated around hipMalloc / hipFree churn on
//     several streams?
// Build: hipcc --offload-arch=gfx950 -O2 -o alloc_probe alloc_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                         \
    }                                                                                       \
  } while (0)

__global__ void spin_write(uint32_t* p, uint64_t n, long long cycles, uint32_t v) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(10);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

__global__ void fill(uint32_t* p, uint64_t n, uint32_t v) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

__global__ void count_not(const uint32_t* p, uint64_t n, uint32_t v, unsigned* bad) {
  unsigned c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    c += p[i] != v;
  if (c) atomicAdd(bad, c);
}

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

struct Range {
  uintptr_t a, b;
};
static bool overlaps(const std::vector<Range>& v, uintptr_t a, uintptr_t b) {
  for (const Range& r : v)
    if (a < r.b && r.a < b) return true;
  return false;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 4000;
  // ---- 1. hipFree vs a running kernel on a non-blocking stream
  {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t done;
    CK(hipEventCreate(&done));
    for (int trial = 0; trial < 3; trial++) {
      uint32_t* x = nullptr;
      const uint64_t n = 16u << 20;
      CK(hipMalloc(&x, 4 * n));
      hipLaunchKernelGGL(spin_write, dim3(1024), dim3(256), 0, s, x, n, 400000000ll, 7u);  // ~0.2 s
      CK(hipEventRecord(done, s));
      auto t = std::chrono::steady_clock::now();
      CK(hipFree(x));
      const double free_ms = ms_since(t);
      const hipError_t q = hipEventQuery(done);
      std::printf("hipFree_vs_running_kernel trial=%d free_ms=%.2f kernel_done_at_return=%d\n", trial, free_ms,
                  q == hipSuccess ? 1 : 0);
      CK(hipStreamSynchronize(s));
    }
    CK(hipEventDestroy(done));
    CK(hipStreamDestroy(s));
  }
  // ---- 2. stream-ordered pool blocks vs live hipMalloc buffers
  {
    std::mt19937_64 rng(12345);
    std::vector<hipStream_t> streams(4);
    for (auto& s : streams) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const uint64_t vn = 8u << 20;  // victim: 32 MB of 0x5A5A5A5A
    uint32_t* victim = nullptr;
    CK(hipMalloc(&victim, 4 * vn));
    hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, streams[0], victim, vn, 0x5A5A5A5Au);
    CK(hipStreamSynchronize(streams[0]));
    unsigned* bad = nullptr;
    CK(hipMalloc(&bad, 4));
    std::vector<Range> live;  // hipMalloc buffers
    std::vector<void*> livep;
    live.push_back({(uintptr_t)victim, (uintptr_t)victim + 4 * vn});
    livep.push_back(victim);
    uint64_t n_async = 0, n_overlap_async = 0, n_overlap_malloc = 0, n_checks = 0, n_corrupt = 0;
    std::vector<Range> async_live;
    for (int it = 0; it < iters; it++) {
      const int act = (int)(rng() % 10);
      hipStream_t s = streams[rng() % streams.size()];
      if (act < 5) {  // a scan_u32-like use of the pool: small blocks, a kernel, stream-ordered frees
        const size_t b1 = 4 * (1 + rng() % 4096), b2 = 4 * (1 + rng() % 4096);
        uint32_t *p1 = nullptr, *p2 = nullptr;
        CK(hipMallocAsync((void**)&p1, b1, s));
        CK(hipMallocAsync((void**)&p2, b2, s));
        n_async += 2;
        for (auto [p, b] : {std::pair<uint32_t*, size_t>{p1, b1}, {p2, b2}}) {
          if (overlaps(live, (uintptr_t)p, (uintptr_t)p + b)) n_overlap_async++;
          async_live.push_back({(uintptr_t)p, (uintptr_t)p + b});
        }
        hipLaunchKernelGGL(fill, dim3(16), dim3(256), 0, s, p1, b1 / 4, 0xDEADBEEFu);
        hipLaunchKernelGGL(fill, dim3(16), dim3(256), 0, s, p2, b2 / 4, 0xFEEDFACEu);
        CK(hipFreeAsync(p1, s));
        CK(hipFreeAsync(p2, s));
        if (rng() % 2) {
          CK(hipStreamSynchronize(s));
          async_live.clear();  // (freed and complete)
        }
      } else if (act < 7) {  // DBuf::ensure-like churn
        const size_t b = 256 + (rng() % (8u << 20));
        void* p = nullptr;
        CK(hipMalloc(&p, b));
        if (overlaps(async_live, (uintptr_t)p, (uintptr_t)p + b)) n_overlap_malloc++;
        live.push_back({(uintptr_t)p, (uintptr_t)p + b});
        livep.push_back(p);
      } else if (act < 9 && livep.size() > 1) {
        const size_t k = 1 + rng() % (livep.size() - 1);  // never the victim
        CK(hipFree(livep[k]));
        livep.erase(livep.begin() + (long)k);
        live.erase(live.begin() + (long)k);
      } else {
        for (auto& t : streams) CK(hipStreamSynchronize(t));
        async_live.clear();
        CK(hipMemsetAsync(bad, 0, 4, streams[0]));
        hipLaunchKernelGGL(count_not, dim3(1024), dim3(256), 0, streams[0], victim, vn, 0x5A5A5A5Au, bad);
        unsigned h = 0;
        CK(hipMemcpyAsync(&h, bad, 4, hipMemcpyDeviceToHost, streams[0]));
        CK(hipStreamSynchronize(streams[0]));
        n_checks++;
        if (h) {
          n_corrupt++;
          std::printf("victim corrupted at iteration %d: %u words\n", it, h);
          hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, streams[0], victim, vn, 0x5A5A5A5Au);
        }
      }
    }
    for (auto& t : streams) CK(hipStreamSynchronize(t));
    std::printf("pool_probe iters=%d async_allocs=%llu async_overlapping_live_malloc=%llu "
                "malloc_overlapping_inflight_async=%llu victim_checks=%llu victim_corrupted=%llu\n",
                iters, (unsigned long long)n_async, (unsigned long long)n_overlap_async,
                (unsigned long long)n_overlap_malloc, (unsigned long long)n_checks, (unsigned long long)n_corrupt);
    for (void* p : livep) CK(hipFree(p));
    CK(hipFree(bad));
    for (auto& s : streams) CK(hipStreamDestroy(s));
  }
  return 0;
}
