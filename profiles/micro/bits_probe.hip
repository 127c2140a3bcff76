// bits_probe.hip — the begin-hit bitmap pass of the headline step (cep_nfa_bits as compile.cpp
// generates it for the README query: volume > 1000 from one int32 column, the block's largest
// timestamp from the int64 ts column) over 1e9 events, in variants of its shape, to see how close
// the 12 bytes per event can come to the HBM read rate.
//   S        strips of 1024 positions a 256-thread block covers (the product: 4)
//   NT       non-temporal (streaming) loads of both columns
// Build: hipcc --offload-arch=gfx950 -O3 -o bits_probe bits_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                         \
    }                                                                                       \
  } while (0)

__global__ void fill(int32_t* v, int64_t* ts, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 31)) * 0xBF58476D1CE4E5B9ull;
    v[i] = (int32_t)((z >> 40) % 2000);
    ts[i] = 1600000000000ll + (int64_t)i;
  }
}

__device__ __forceinline__ uint64_t spread4(uint32_t x16) {
  uint64_t x = x16;
  x = (x | (x << 24)) & 0x000000FF000000FFull;
  x = (x | (x << 12)) & 0x000F000F000F000Full;
  x = (x | (x << 6)) & 0x0303030303030303ull;
  x = (x | (x << 3)) & 0x1111111111111111ull;
  return x;
}

template <int S, bool NT>
__global__ void __launch_bounds__(256) bits(const int32_t* __restrict__ vol, const int64_t* __restrict__ tsc, uint64_t n,
                                            uint64_t* bh, int64_t* wmb) {
  const uint64_t b0 = (uint64_t)blockIdx.x * (1024 * S);
  const uint32_t lane = threadIdx.x & 63;
  int64_t t[S][4];
  int4 v[S];
#pragma unroll
  for (int k = 0; k < S; k++) {
    const uint64_t p = b0 + (uint64_t)k * 1024 + (uint64_t)threadIdx.x * 4;
    if (p + 4 <= n) {
      const longlong2* q = reinterpret_cast<const longlong2*>(tsc + p);
      longlong2 a, c;
      if (NT) {
        typedef long long ll2v __attribute__((ext_vector_type(2)));
        typedef int i4v __attribute__((ext_vector_type(4)));
        const ll2v x = __builtin_nontemporal_load(reinterpret_cast<const ll2v*>(q));
        const ll2v y = __builtin_nontemporal_load(reinterpret_cast<const ll2v*>(q) + 1);
        const i4v z = __builtin_nontemporal_load(reinterpret_cast<const i4v*>(vol + p));
        a.x = x.x;
        a.y = x.y;
        c.x = y.x;
        c.y = y.y;
        v[k] = int4{z.x, z.y, z.z, z.w};
      } else {
        a = q[0];
        c = q[1];
        v[k] = *reinterpret_cast<const int4*>(vol + p);
      }
      t[k][0] = a.x;
      t[k][1] = a.y;
      t[k][2] = c.x;
      t[k][3] = c.y;
    } else {
#pragma unroll
      for (int j = 0; j < 4; j++) t[k][j] = p + j < n ? tsc[p + j] : INT64_MIN;
      v[k] = int4{p < n ? vol[p] : 0, p + 1 < n ? vol[p + 1] : 0, p + 2 < n ? vol[p + 2] : 0, p + 3 < n ? vol[p + 3] : 0};
    }
  }
  int64_t m = INT64_MIN;
#pragma unroll
  for (int k = 0; k < S; k++)
#pragma unroll
    for (int j = 0; j < 4; j++) m = t[k][j] > m ? t[k][j] : m;
#pragma unroll
  for (int k = 0; k < S; k++) {
    const uint64_t p = b0 + (uint64_t)k * 1024 + (uint64_t)threadIdx.x * 4;
    uint64_t B[4];
    B[0] = __ballot(p < n && v[k].x > 1000);
    B[1] = __ballot(p + 1 < n && v[k].y > 1000);
    B[2] = __ballot(p + 2 < n && v[k].z > 1000);
    B[3] = __ballot(p + 3 < n && v[k].w > 1000);
    uint64_t w = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      uint64_t x = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) x |= spread4((uint32_t)(B[j] >> (16 * q)) & 0xFFFFu) << j;
      if (lane == (uint32_t)q) w = x;
    }
    const uint64_t ws = b0 + (uint64_t)k * 1024 + (uint64_t)(threadIdx.x >> 6) * 256 + (uint64_t)lane * 64;
    if (lane < 4 && ws < n) bh[ws >> 6] = w;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t y = __shfl_down(m, o, 64);
    m = y > m ? y : m;
  }
  __shared__ int64_t wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t x = wm[0];
    for (int i = 1; i < 4; i++) x = wm[i] > x ? wm[i] : x;
    wmb[blockIdx.x] = x;
  }
}

template <int S, bool NT>
static void run(const char* name, const int32_t* vol, const int64_t* ts, uint64_t n, uint64_t* bh, int64_t* wmb,
                hipStream_t st, int reps) {
  const uint64_t blocks = (n + 1024 * S - 1) / (1024 * S);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((bits<S, NT>), dim3((uint32_t)blocks), dim3(256), 0, st, vol, ts, n, bh, wmb);
  CK(hipStreamSynchronize(st));
  float best = 1e30f, sum = 0;
  for (int r = 0; r < reps; r++) {
    CK(hipEventRecord(a, st));
    hipLaunchKernelGGL((bits<S, NT>), dim3((uint32_t)blocks), dim3(256), 0, st, vol, ts, n, bh, wmb);
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
    sum += ms;
  }
  const double bytes = 12.0 * (double)n;
  std::printf("%-10s best %.3f ms mean %.3f ms  %.2f TB/s (best)\n", name, best, sum / reps, bytes / (best * 1e-3) / 1e12);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : 1000000000ull;
  const int reps = 20;
  int32_t* vol;
  int64_t* ts;
  uint64_t* bh;
  int64_t* wmb;
  CK(hipMalloc(&vol, 4 * n));
  CK(hipMalloc(&ts, 8 * n));
  CK(hipMalloc(&bh, 8 * ((n + 63) / 64)));
  CK(hipMalloc(&wmb, 8 * ((n + 1023) / 1024)));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, st, vol, ts, n);
  CK(hipStreamSynchronize(st));
  run<4, false>("S4", vol, ts, n, bh, wmb, st, reps);
  run<2, false>("S2", vol, ts, n, bh, wmb, st, reps);
  run<8, false>("S8", vol, ts, n, bh, wmb, st, reps);
  run<4, true>("S4nt", vol, ts, n, bh, wmb, st, reps);
  run<8, true>("S8nt", vol, ts, n, bh, wmb, st, reps);
  run<4, false>("S4again", vol, ts, n, bh, wmb, st, reps);
  CK(hipFree(vol));
  CK(hipFree(ts));
  CK(hipFree(bh));
  CK(hipFree(wmb));
  return 0;
}
