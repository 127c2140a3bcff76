// CPU stand-in for the HIP device runtime: lets tests/lane_cpu build a query's generated NFA
// kernel (compile.cpp generate_jit + csrc/nfa_lane.h) as ordinary host code, one lane at a
// time, to debug and fuzz the lane logic without a GPU.  Test infrastructure only.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>

#define __device__
#define __host__
#define __global__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define __shared__ static  // one lane at a time: the block's LDS is one static array
#define CEP_LDS_AS           // (no address spaces on the host)
#define asm(...) ((void)0)

struct LaneDim3 {
  unsigned x = 0, y = 0, z = 0;
};
extern thread_local LaneDim3 blockIdx, threadIdx, blockDim, gridDim;

inline unsigned atomicAdd(unsigned* p, unsigned v) {
  const unsigned o = *p;
  *p += v;
  return o;
}
inline unsigned long long atomicMax(unsigned long long* p, unsigned long long v) {
  const unsigned long long o = *p;
  if (v > o) *p = v;
  return o;
}
inline unsigned atomicOr(unsigned* p, unsigned v) {
  const unsigned o = *p;
  *p = o | v;
  return o;
}
inline void __syncthreads() {}  // one lane at a time
inline bool __any(int x) { return x != 0; }  // a wave of one lane
// a wave of one lane: the calling lane's own bit (its lane id is threadIdx.x & 63)
inline unsigned long long __ballot(int x) { return x ? 1ull << (threadIdx.x & 63) : 0ull; }
inline int __ffsll(unsigned long long x) { return __builtin_ffsll((long long)x); }
inline int __popcll(unsigned long long x) { return __builtin_popcountll(x); }
template <class T>
inline T __shfl(T v, int, int = 64) {  // a wave of one lane: its own value
  return v;
}
inline double __longlong_as_double(long long x) {
  double d;
  std::memcpy(&d, &x, 8);
  return d;
}
inline long long __double_as_longlong(double d) {
  long long x;
  std::memcpy(&x, &d, 8);
  return x;
}
inline double __dadd_rn(double a, double b) { return a + b; }
inline double __dsub_rn(double a, double b) { return a - b; }
inline double __dmul_rn(double a, double b) { return a * b; }
inline double __ddiv_rn(double a, double b) { return a / b; }
// a wave of one lane: there is no lane below/above to read from
template <class T>
inline T __shfl_down(T, int, int = 64) {
  return T(0);
}
