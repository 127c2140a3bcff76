// Stencil mask-phase probe (round 5): where config 2's mask pass spends its time.
//   rd        : a pure read of the column in the mask pass's shape (the memory floor)
//   stencil_mask, stencil_emit: the product's passes (stencil.hip)
//   v2<SPW,PF,KEY>: the same stage ballots and window ANDs with a double-buffered load ring
//                 (PF steps in flight while the other PF compute), SPW 256-event steps per wave,
//                 KEY = 0 skips the key-start preamble (measurement only: wrong at key starts)
// Synthetic cfg-2 stream: n events, v = mix(i) % 16, keys of n / n_keys events.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../../kafkastreams-cep_amd/csrc stencil_probe.hip -o stencil_probe
#include "stencil.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace cep;

__global__ void gen(int32_t* v, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) v[i] = (int32_t)(mix64s(i * 0x9E3779B97F4A7C15ull + 12345) % 16);
}

__global__ void gen_off(uint64_t* off, uint64_t n_keys, uint64_t n) {
  const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (k <= n_keys) off[k] = k == n_keys ? n : (n / n_keys) * k + (mix64s(k) % 977);
}

__global__ void __launch_bounds__(256) rd(const v4i* __restrict__ p, size_t nq, uint64_t* out) {
  const size_t base = ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 1024 + (threadIdx.x & 63);
  v4i acc = {0, 0, 0, 0};
#pragma unroll
  for (int c = 0; c < 16; c++) {
    const size_t i = base + (size_t)c * 64;
    acc ^= i < nq ? __builtin_nontemporal_load(p + i) : v4i{0, 0, 0, 0};
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678) out[0] = 1;
}

// v2: ballots + windows as in wave_mask's fast path, keys optional, double-buffered loads
template <int M, int SPW, int PF, bool KEY>
__global__ void __launch_bounds__(256) v2(StencilArgs A, uint64_t* out) {
  constexpr int H = M - 1;
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t wbase = ((uint64_t)blockIdx.x * 4 + wv) * (uint64_t)SPW * 256;
  const StEval<M, true, 1> ev(A);
  if (wbase + (uint64_t)SPW * 256 > A.n_events) return;  // (probe: whole waves only)
  const v4i* c0 = reinterpret_cast<const v4i*>(A.col[0] + wbase) + lane;
  v4i xa[PF], xb[PF];
#pragma unroll
  for (int d = 0; d < PF; d++) xa[d] = __builtin_nontemporal_load(c0 + d * 64);
  uint64_t bw = 0;
  uint32_t wkey = 0;
  if (KEY) {  // the product's preamble (first chunk only): wave_key, then key_off around it
    const uint32_t k0 = A.wave_key[wbase / kStWave];
    const uint64_t wend = wbase + (uint64_t)SPW * 256;
    const uint64_t lo = wbase >= 8 ? wbase - 8 : 0;
    for (int64_t i0 = (int64_t)k0 - 8;; i0 += 64) {
      const int64_t i = i0 + lane;
      const bool valid = i >= 0 && (uint64_t)i < A.n_keys;
      const uint64_t sj = valid ? A.key_off[i] : 0;
      uint64_t inr = __ballot(valid && sj >= lo && sj < wend);
      while (inr) {
        const int j = __builtin_ctzll(inr);
        inr &= inr - 1;
        const uint64_t sjj = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(sj >> 32), j) << 32) |
                             (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)sj, j);
        if (sjj >= wbase && ((sjj - wbase) >> 6) % 64 == (uint64_t)lane) bw |= 1ull << (sjj & 63);
        wkey = (uint32_t)(i0 + j);
      }
      const uint64_t s63 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(sj >> 32), 63) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)sj, 63);
      if (!(i0 + 64 < (int64_t)A.n_keys && s63 < wend)) break;
    }
  }
  const uint64_t kstep = H > 0 ? __ballot(bw != 0) : 0;
  uint64_t pW[M][4];
#pragma unroll
  for (int s = 0; s < M; s++)
#pragma unroll
    for (int k = 0; k < 4; k++) pW[s][k] = 0;
  uint64_t myword = 0;
  auto step = [&](const int q, const v4i x) {
    uint64_t W[M][4];
#pragma unroll
    for (int s = 0; s < M; s++) ev.ballot4(s, x, x, W[s]);
    uint64_t m[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      m[k] = ~0ull;
#pragma unroll
      for (int s = 0; s < M; s++) {
        const int t = k - (M - 1 - s);
        const int cr = t >= 0 ? 0 : (3 - t) / 4;
        const int kk = t + 4 * cr;
        m[k] &= cr == 0 ? W[s][kk] : ((W[s][kk] << cr) | (pW[s][kk] >> (64 - cr)));
      }
    }
    if (KEY && ((kstep >> (4 * (q & 15))) & 0xF)) {  // (probe: the key-start masking's branch only)
#pragma unroll
      for (int k = 0; k < 4; k++) m[k] &= ~(uint64_t)__shfl(bw, 4 * (q & 15) + k, 64);
    }
    const int lrel = lane - 4 * (q & 15);
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (lrel == k) myword ^= m[k];
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int s = 0; s < M; s++) pW[s][k] = W[s][k];
  };
  // two buffers of PF steps: while one chunk computes, the other's loads are in flight
#pragma unroll 1
  for (int c = 0; c < SPW; c += 2 * PF) {
    const int nb = c + PF < SPW ? c + PF : c;
#pragma unroll
    for (int d = 0; d < PF; d++) xb[d] = __builtin_nontemporal_load(c0 + (nb + d) * 64);
#pragma unroll
    for (int d = 0; d < PF; d++) step(c + d, xa[d]);
    const int na = c + 2 * PF < SPW ? c + 2 * PF : c;
#pragma unroll
    for (int d = 0; d < PF; d++) xa[d] = __builtin_nontemporal_load(c0 + (na + d) * 64);
#pragma unroll
    for (int d = 0; d < PF; d++) step(c + PF + d, xb[d]);
  }
  out[(wbase / 64) % (1u << 20) + lane] = myword ^ wkey;
}

// emit ablation (probe): ABL 0 loads + scans only, 1 + LDS staging, 2 = stencil_emit
template <int M, int ABL>
__global__ void __launch_bounds__(kStThreads) emit_abl(StencilArgs A) {
  __shared__ uint32_t s_wsum[kStThreads / 64];
  __shared__ uint64_t s_toff[kStThreads / 64];
  __shared__ uint2 s_stage[kEmStage];  // (key, sequence number of the final event)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint64_t t0 = (uint64_t)blockIdx.x * kEmW;  // the block's first mask tile
  const uint64_t n_words = (A.n_events + 63) / 64;
  const uint64_t w0 = t0 * (kStTile / 64) + (uint64_t)tid * kEmW;  // this thread's first word
  // Every independent load is issued before the first use: the thread's words (a 16-B record
  // each: match bits, first key, sequence number) and the counts of the blocks before this one.
  uint64_t wm[kEmW];
  uint32_t wk[kEmW], ws[kEmW];
#pragma unroll
  for (int i = 0; i < kEmW; i++) {
    const uint4 x = w0 + i < n_words ? A.words[w0 + i] : uint4{0, 0, 0, 0};
    wm[i] = ((uint64_t)x.y << 32) | x.x;
    wk[i] = x.z;
    ws[i] = x.w;
  }
  uint64_t part = 0;  // the matches of the blocks before this one: their group counts
  // (the first 8 per thread issued together: a late block of 1e8 events has ~1500 before it)
#pragma unroll
  for (int r = 0; r < 8; r++) {
    const uint32_t i = (uint32_t)tid + (uint32_t)r * kStThreads;
    part += i < blockIdx.x ? A.group_cnt[i] : 0u;
  }
  for (uint64_t i = (uint64_t)tid + 8 * kStThreads; i < blockIdx.x; i += kStThreads) part += A.group_cnt[i];
  uint32_t cnt = 0;
#pragma unroll
  for (int i = 0; i < kEmW; i++) cnt += (uint32_t)__popcll(wm[i]);
  // block exclusive scan of the threads' match counts
  uint32_t incl = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) part += __shfl_down(part, off, 64);
  if (lane == 63) s_wsum[wv] = incl;
  if (lane == 0) s_toff[wv] = part;
  __syncthreads();
  uint32_t woff = 0;
#pragma unroll
  for (int w = 0; w < kStThreads / 64; w++)
    if (w < wv) woff += s_wsum[w];
  const uint32_t excl = woff + incl - cnt;
  const uint64_t toff = s_toff[0] + s_toff[1] + s_toff[2] + s_toff[3];
  if (blockIdx.x + 1 == gridDim.x && tid == kStThreads - 1) {  // all matches
    *A.total = toff + woff + incl;
    if (A.total_host) *A.total_host = toff + woff + incl;  // pinned host memory, read after the batch's event
  }
  const uint32_t block_total = s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
  if (ABL == 0) return;
  const bool staged = block_total <= kEmStage;  // block-uniform
  uint64_t o = toff + excl;
  uint32_t so = excl;  // slot within the block
#pragma unroll
  for (int i = 0; i < kEmW; i++) {
    uint64_t match = wm[i];
    if (!match) continue;
    const uint64_t p0 = (w0 + i) * 64;
    uint32_t key = wk[i] & 0x7FFFFFFFu;
    const bool cross = (wk[i] >> 31) != 0;  // a key starts inside this word
    uint64_t kstart = 0, knext = 0;
    if (cross) {
      kstart = A.key_off[key];
      knext = A.key_off[key + 1];
    }
    while (match) {
      const int b = __builtin_ctzll(match);
      match &= match - 1;
      const uint64_t p = p0 + b;
      uint32_t seq = ws[i] + (uint32_t)b;
      if (cross) {
        while (p >= knext) {  // the next key (empty keys share their offset: skipped too)
          key++;
          kstart = knext;
          knext = A.key_off[key + 1];
        }
        seq = (uint32_t)(p - kstart);
      }
      if (staged) {
        s_stage[so++] = uint2{key, seq};
      } else if (o < A.out_cap) {
        A.m_key[o] = key;
#pragma unroll
        for (int x = 0; x < M; x++) A.p_seq[o * M + x] = seq - x;
      } else {
        atomicOr(A.overflow, 1u);
      }
      o++;
    }
  }
  if (!staged) return;
  __syncthreads();
  if (ABL == 1) return;
  // thread i writes matches i, i + 256, ...: adjacent threads, adjacent slots
  for (uint32_t i = tid; i < block_total; i += kStThreads) {
    const uint64_t slot = toff + i;
    const uint2 e = s_stage[i];
    if (slot < A.out_cap) {
      A.m_key[slot] = e.x;
      if (M == 3) {  // one 12-B store per match
        *reinterpret_cast<uint3*>(A.p_seq + slot * 3) = uint3{e.y, e.y - 1, e.y - 2};
      } else {
#pragma unroll
        for (int x = 0; x < M; x++) A.p_seq[slot * M + x] = e.y - x;
      }
    } else {
      atomicOr(A.overflow, 1u);
    }
  }
}


template <class F>
static float timeit(F f, int reps = 20) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e9;
  for (int it = 0; it < reps; it++) {
    hipEventRecord(a);
    f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  return best * 1e3f;
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 100000000ull;
  const uint64_t n_keys = argc > 2 ? strtoull(argv[2], nullptr, 10) : 10000ull;
  int32_t* v;
  uint64_t *off, *out, *mask;
  uint32_t *wk, *zero, *word_key, *tile_cnt;
  hipMalloc(&v, n * 4 + 64);
  hipMalloc(&off, (n_keys + 1) * 8);
  hipMalloc(&out, (1u << 20) * 8 + 4096 * 8);
  const uint64_t n_waves = stencil_waves(n), n_tiles = stencil_tiles(n);
  hipMalloc(&wk, (n_waves + 1) * 4);
  hipMalloc(&zero, 4096 * 4);
  hipMalloc(&mask, 16 * (n / 64 + 2));
  hipMalloc(&word_key, 2 * ((n / 64 + 2 + 3) & ~3ull) * 4);
  hipMalloc(&tile_cnt, (n_waves + 1) * 4);
  hipLaunchKernelGGL(gen, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, v, n);
  hipLaunchKernelGGL(gen_off, dim3((uint32_t)((n_keys + 256) / 256)), dim3(256), 0, 0, off, n_keys, n);
  launch_wave_keys(off, n_keys, n, wk, zero, 4096, 0);
  hipDeviceSynchronize();
  StencilArgs a{};
  a.n_keys = n_keys;
  a.n_events = n;
  a.key_off = off;
  a.wave_key = wk;
  a.col[0] = a.col[1] = v;
  a.aligned = true;
  const int64_t lo[3] = {INT64_MIN, 4, 8}, hi[3] = {3, 7, INT64_MAX};
  for (int s = 0; s < 3; s++) {
    a.rs[s].lo[0] = a.rs[s].lo[1] = lo[s];
    a.rs[s].hi[0] = a.rs[s].hi[1] = hi[s];
  }
  a.words = reinterpret_cast<uint4*>(mask);
  a.group_cnt = zero;
  const double gb = n * 4.0 / 1e9;
  auto rep = [&](const char* name, float us) { printf("%-28s %8.1f us  %5.2f TB/s\n", name, us, gb / (us * 1e-6) / 1e3); };
  rep("rd (16 KB per wave)", timeit([&] { hipLaunchKernelGGL(rd, dim3((uint32_t)n_tiles), dim3(256), 0, 0, (const v4i*)v, n / 4, out); }));
  const uint64_t n_chunks = n_waves;
  a.n_chunk = n_chunks;
  const uint32_t nb_all = (uint32_t)((n_chunks + 3) / 4);
  rep("stencil_mask", timeit([&] { hipLaunchKernelGGL((stencil_mask<3, true, 1>), dim3(nb_all), dim3(256), 0, 0, a); }));
  a.m_key = (uint32_t*)out;  // (probe: the emit pass's outputs, sized for the synthetic stream's matches)
  uint32_t* pseq;
  uint64_t* tot;
  uint32_t* ovf;
  hipMalloc(&pseq, n * 3 * 4);
  hipMalloc(&tot, 8);
  hipMalloc(&ovf, 4);
  hipMalloc(&a.m_key, n * 4);
  a.p_seq = pseq;
  a.total = tot;
  a.out_cap = n;
  a.overflow = ovf;
  hipMemset(zero, 0, 4096 * 4);
  launch_stencil(3, a, true, 1, 0);  // (the counts the emit pass reads)
  hipDeviceSynchronize();
  rep("stencil_emit", timeit([&] {
        hipLaunchKernelGGL(stencil_emit<3>, dim3((uint32_t)((n_tiles + kEmW - 1) / kEmW)), dim3(256), 0, 0, a);
      }));
  rep("emit: loads + scans", timeit([&] { hipLaunchKernelGGL((emit_abl<3, 0>), dim3((uint32_t)((n_tiles + kEmW - 1) / kEmW)), dim3(256), 0, 0, a); }));
  rep("emit: + LDS staging", timeit([&] { hipLaunchKernelGGL((emit_abl<3, 1>), dim3((uint32_t)((n_tiles + kEmW - 1) / kEmW)), dim3(256), 0, 0, a); }));
  rep("emit: + writes", timeit([&] { hipLaunchKernelGGL((emit_abl<3, 2>), dim3((uint32_t)((n_tiles + kEmW - 1) / kEmW)), dim3(256), 0, 0, a); }));
  {
    uint64_t tt = 0;
    hipMemcpy(&tt, tot, 8, hipMemcpyDeviceToHost);
    printf("matches %llu\n", (unsigned long long)tt);
  }
  rep("mask + emit", timeit([&] {
        hipMemsetAsync(zero, 0, 4096 * 4);
        launch_stencil(3, a, true, 1, 0);
      }));
#define V2(SPW, PF, KEY)                                                                                        \
  rep("v2 SPW" #SPW " PF" #PF " KEY" #KEY, timeit([&] {                                                        \
        hipLaunchKernelGGL((v2<3, SPW, PF, KEY>), dim3((uint32_t)(n / (SPW * 256) / 4)), dim3(256), 0, 0, a, out); \
      }))
  V2(16, 1, 0);
  V2(16, 2, 0);
  V2(16, 4, 0);
  V2(16, 8, 0);
  V2(16, 2, 1);
  V2(16, 4, 1);
  V2(32, 2, 0);
  V2(32, 4, 0);
  V2(32, 4, 1);
  V2(64, 4, 0);
  V2(64, 4, 1);
  V2(64, 8, 1);
  return 0;
}
