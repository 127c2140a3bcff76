// wave_emu.h — runs the 64 lanes of a wavefront as fibers (ucontext) so that the kernel's
// cross-lane operations (hip/hip_runtime.h: __ballot, __any, __shfl*) see every live lane of
// the wave, as on the GPU.  Test infrastructure only (tests/lane_cpu/driver.cpp).
//
// Each lane runs until it reaches a cross-lane operation (or returns from the kernel), then
// the next lane runs; once every live lane is parked, all must be at the same operation (the
// same call site: the kernel calls them convergently) - the results are computed from their
// values and the lanes resume in lane order.  Lanes that returned are inactive: they take no
// part and read as 0 through a shuffle.
#pragma once
#include <sys/mman.h>
#include <ucontext.h>

#include <cstdio>
#include <cstdlib>

namespace emu {

struct Wave {
  static constexpr size_t kStack = 1u << 20;
  ucontext_t sched;
  ucontext_t ctx[64];
  void* stack[64] = {};
  bool live[64] = {};
  bool parked[64] = {};
  int op[64] = {};
  uint64_t val[64] = {};
  int arg[64] = {};
  const char* site[64] = {};
  uint64_t res[64] = {};
  int cur = 0;
  unsigned block = 0, tid0 = 0, bdim = 256;
  void (*body)(void*) = nullptr;
  void* user = nullptr;
  uint64_t rendezvous = 0;
};

Wave* g_wave = nullptr;

static void lane_entry(unsigned lo, unsigned hi) {
  Wave* w = reinterpret_cast<Wave*>(((uint64_t)hi << 32) | lo);
  w->body(w->user);
  w->live[w->cur] = false;  // returned: inactive from now on (back to the scheduler: uc_link)
}

uint64_t collective(int op, uint64_t val, int arg, const char* site) {
  Wave& w = *g_wave;
  const int l = w.cur;
  w.op[l] = op;
  w.val[l] = val;
  w.arg[l] = arg;
  w.site[l] = site;
  w.parked[l] = true;
  swapcontext(&w.ctx[l], &w.sched);
  return w.res[l];
}

static void set_lane(Wave& w, int l) {
  w.cur = l;
  threadIdx.x = w.tid0 + (unsigned)l;
  blockIdx.x = w.block;
  blockDim.x = w.bdim;
}

// Runs body(user) on the 64 lanes of the wave whose first thread is (block, tid0).
inline void run_wave(unsigned block, unsigned tid0, void (*body)(void*), void* user) {
  static Wave W;
  Wave& w = W;
  w.block = block;
  w.tid0 = tid0;
  w.body = body;
  w.user = user;
  const uint64_t wp = (uint64_t)&w;
  for (int l = 0; l < 64; l++) {
    if (!w.stack[l]) {
      w.stack[l] = mmap(nullptr, Wave::kStack, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (w.stack[l] == MAP_FAILED) std::abort();
    }
    getcontext(&w.ctx[l]);
    w.ctx[l].uc_stack.ss_sp = w.stack[l];
    w.ctx[l].uc_stack.ss_size = Wave::kStack;
    w.ctx[l].uc_link = &w.sched;
    makecontext(&w.ctx[l], (void (*)())lane_entry, 2, (unsigned)(wp & 0xFFFFFFFFu), (unsigned)(wp >> 32));
    w.live[l] = true;
    w.parked[l] = false;
  }
  g_wave = &w;
  for (;;) {
    // run every live lane up to its next cross-lane operation (or its return)
    for (int l = 0; l < 64; l++) {
      if (!w.live[l]) continue;
      set_lane(w, l);
      w.parked[l] = false;
      swapcontext(&w.sched, &w.ctx[l]);
    }
    int first = -1, n = 0;
    for (int l = 0; l < 64; l++)
      if (w.live[l]) {
        n++;
        if (first < 0) first = l;
        if (!w.parked[l]) {
          std::fprintf(stderr, "wave_emu: lane %d neither returned nor parked\n", l);
          std::abort();
        }
      }
    if (n == 0) break;
    w.rendezvous++;
    for (int l = 0; l < 64; l++)
      if (w.live[l] && (w.op[l] != w.op[first] || w.site[l] != w.site[first])) {
        std::fprintf(stderr, "wave_emu: divergent cross-lane operation (rendezvous %llu): lane %d at %s, lane %d at %s\n",
                     (unsigned long long)w.rendezvous, first, w.site[first], l, w.site[l]);
        std::abort();
      }
    const int op = w.op[first];
    uint64_t ballot = 0;
    if (op == kBallot)
      for (int l = 0; l < 64; l++)
        if (w.live[l] && w.val[l]) ballot |= 1ull << l;
    auto lane_val = [&](int s) -> uint64_t { return (s >= 0 && s < 64 && w.live[s]) ? w.val[s] : 0ull; };
    for (int l = 0; l < 64; l++) {
      if (!w.live[l]) continue;
      switch (op) {
        case kBallot: w.res[l] = ballot; break;
        case kShfl: w.res[l] = lane_val(w.arg[l] & 63); break;
        case kShflXor: w.res[l] = lane_val((l ^ w.arg[l]) & 63); break;
        // (__shfl_up / __shfl_down: a lane with no source lane keeps its own value)
        case kShflUp: w.res[l] = l - w.arg[l] >= 0 ? lane_val(l - w.arg[l]) : w.val[l]; break;
        case kShflDown: w.res[l] = l + w.arg[l] < 64 ? lane_val(l + w.arg[l]) : w.val[l]; break;
        default: std::abort();
      }
    }
  }
  g_wave = nullptr;
}

}  // namespace emu
