// Achievable HBM read rate on this box for the stencil's access shape: each wave streams
// 16 KiB with 16-B loads (one 1-KiB wave instruction per step), 256-thread blocks.
// Build: hipcc --offload-arch=gfx950 -O3 hbm_read.hip -o hbm_read ; run: ./hbm_read [MB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <unistd.h>

typedef int v4i __attribute__((ext_vector_type(4)));

template <int D>
__global__ void __launch_bounds__(256) rd(const v4i* __restrict__ p, size_t n_quads, int* out) {
  const size_t base = ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 1024 + (threadIdx.x & 63);
  v4i acc = {0, 0, 0, 0};
  v4i x[D];
#pragma unroll
  for (int c = 0; c < 16 / D; c++) {
#pragma unroll
    for (int d = 0; d < D; d++) {
      const size_t i = base + (size_t)(c * D + d) * 64;
      x[d] = i < n_quads ? __builtin_nontemporal_load(p + i) : v4i{0, 0, 0, 0};
    }
#pragma unroll
    for (int d = 0; d < D; d++) acc ^= x[d];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678) out[0] = 1;
}

int main(int argc, char** argv) {
  const size_t mb = argc > 1 ? atol(argv[1]) : 400;
  const size_t bytes = mb << 20, nq = bytes / 16;
  v4i* p;
  int* o;
  hipMalloc(&p, bytes);
  hipMalloc(&o, 4);
  hipMemset(p, 1, bytes);
  const unsigned blocks = (unsigned)((nq + 4095) / 4096);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  // the same kernel with the host idle between launches (like a push() per batch)
  for (int gap : {0, 50, 500}) {
    float best = 1e9, sum = 0;
    for (int it = 0; it < 20; it++) {
      hipDeviceSynchronize();
      if (gap) usleep(gap);
      hipEventRecord(a);
      hipLaunchKernelGGL(rd<16>, dim3(blocks), dim3(256), 0, 0, p, nq, o);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
      sum += ms;
    }
    printf("read %zu MB after %d us idle: best %.1f us, mean %.1f us\n", mb, gap, best * 1e3, sum / 20 * 1e3);
  }
  for (int D : {1, 4, 16}) {
    float best = 1e9;
    for (int it = 0; it < 20; it++) {
      hipEventRecord(a);
      if (D == 1) hipLaunchKernelGGL(rd<1>, dim3(blocks), dim3(256), 0, 0, p, nq, o);
      if (D == 4) hipLaunchKernelGGL(rd<4>, dim3(blocks), dim3(256), 0, 0, p, nq, o);
      if (D == 16) hipLaunchKernelGGL(rd<16>, dim3(blocks), dim3(256), 0, 0, p, nq, o);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    printf("read %zu MB, %d loads in flight per wave: %.1f us, %.2f TB/s\n", mb, D, best * 1e3, bytes / (best * 1e-3) / 1e12);
  }
  return 0;
}
