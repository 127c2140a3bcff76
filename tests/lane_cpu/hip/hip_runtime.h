// CPU stand-in for the HIP device runtime: lets tests/lane_cpu build a query's generated NFA
// kernel (compile.cpp generate_jit + csrc/nfa_lane.h) as ordinary host code, to debug and
// fuzz the lane logic without a GPU.  Test infrastructure only.
//
// Two modes.  Without a wave (emu::g_wave null) a lane runs alone: a wave of one lane, whose
// cross-lane operations see only itself.  With a wave (tests/lane_cpu/wave_emu.h) the 64
// lanes of a wavefront run as fibers and every cross-lane operation (__ballot, __any,
// __shfl*) is a rendezvous of the wave's live lanes: each lane runs until it reaches one, and
// once every live lane is parked the results are computed from all their values, as the
// hardware computes them for a wavefront whose live lanes are all active.  The kernel code
// calls them convergently (every live lane of the wave, the same call); a lane that reaches a
// different one than the others is a bug of the kernel and aborts the run.  A lane that has
// returned from the kernel is inactive, as on the GPU.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>

#define __device__
#define __host__
#define __global__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define __shared__ static  // the block's LDS: one static array (its waves run one after another)
#define CEP_LDS_AS           // (no address spaces on the host)
#define asm(...) ((void)0)
// (lanes run one at a time: a wave-uniform value is the lane's own)
#define CEP_UNIFORM(x) ((uint32_t)(x))

// (the vector types the generated bitmap kernel's 16-B loads use)
struct int4 {
  int x, y, z, w;
};
struct longlong2 {
  long long x, y;
};
struct double2 {
  double x, y;
};

struct LaneDim3 {
  unsigned x = 0, y = 0, z = 0;
};
extern thread_local LaneDim3 blockIdx, threadIdx, blockDim, gridDim;

namespace emu {
// cross-lane operations of the wave emulator (wave_emu.h; absent: a wave of one lane)
enum Op : int { kBallot = 1, kShfl = 2, kShflXor = 3, kShflUp = 4, kShflDown = 5 };
struct Wave;
extern Wave* g_wave;
uint64_t collective(int op, uint64_t val, int arg, const char* site);
}  // namespace emu

inline unsigned atomicAdd(unsigned* p, unsigned v) {
  const unsigned o = *p;
  *p += v;
  return o;
}
inline unsigned long long atomicAdd(unsigned long long* p, unsigned long long v) {
  const unsigned long long o = *p;
  *p += v;
  return o;
}
inline unsigned long long atomicMax(unsigned long long* p, unsigned long long v) {
  const unsigned long long o = *p;
  if (v > o) *p = v;
  return o;
}
inline unsigned atomicMax(unsigned* p, unsigned v) {
  const unsigned o = *p;
  if (v > o) *p = v;
  return o;
}
inline unsigned atomicOr(unsigned* p, unsigned v) {
  const unsigned o = *p;
  *p = o | v;
  return o;
}
inline void __syncthreads() {}  // (the NFA kernels do not synchronise their waves)
#define CEP_HOST_LANES 1
inline bool cep_host_single_lane() { return emu::g_wave == nullptr; }  // (a wave of one lane)

#define CEP_EMU_SITE __FILE__ ":" CEP_EMU_STR(__LINE__)
#define CEP_EMU_STR(x) CEP_EMU_STR2(x)
#define CEP_EMU_STR2(x) #x

inline unsigned long long cep_emu_ballot(int x, const char* site) {
  if (!emu::g_wave) return x ? 1ull << (threadIdx.x & 63) : 0ull;  // a wave of one lane
  return emu::collective(emu::kBallot, x ? 1u : 0u, 0, site);
}
#define __ballot(x) cep_emu_ballot((x) ? 1 : 0, CEP_EMU_SITE)
#define __any(x) (cep_emu_ballot((x) ? 1 : 0, CEP_EMU_SITE) != 0ull)
#define __all(x) (cep_emu_ballot((x) ? 0 : 1, CEP_EMU_SITE) == 0ull)
inline int __ffsll(unsigned long long x) { return __builtin_ffsll((long long)x); }
inline int __popcll(unsigned long long x) { return __builtin_popcountll(x); }
inline int __popc(unsigned x) { return __builtin_popcount(x); }

template <class T>
inline uint64_t cep_emu_bits(T v) {
  static_assert(sizeof(T) <= 8, "cross-lane values of at most 8 bytes");
  uint64_t b = 0;
  std::memcpy(&b, &v, sizeof(T));
  return b;
}
template <class T>
inline T cep_emu_from(uint64_t b) {
  T v;
  std::memcpy(&v, &b, sizeof(T));
  return v;
}
template <class T>
inline T cep_emu_shfl(int op, T v, int arg, const char* site) {
  if (!emu::g_wave) {  // a wave of one lane: its own value, or nothing below/above it
    if (op == emu::kShflUp || op == emu::kShflDown) return arg == 0 ? v : T(0);
    return v;
  }
  return cep_emu_from<T>(emu::collective(op, cep_emu_bits(v), arg, site));
}
#define __shfl(v, src, ...) cep_emu_shfl(emu::kShfl, (v), (int)(src), CEP_EMU_SITE)
#define __shfl_xor(v, m, ...) cep_emu_shfl(emu::kShflXor, (v), (int)(m), CEP_EMU_SITE)
#define __shfl_up(v, d, ...) cep_emu_shfl(emu::kShflUp, (v), (int)(d), CEP_EMU_SITE)
#define __shfl_down(v, d, ...) cep_emu_shfl(emu::kShflDown, (v), (int)(d), CEP_EMU_SITE)

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
