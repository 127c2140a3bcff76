// stencil.hip — CEP_KIND_STENCIL: SEQ(p_0, ..., p_{m-1}) with every stage ONE + strict
// contiguity and total, state-free predicates and folds.
//
// For such queries the reference NFA (nfa/NFA.java) never branches, each run lives at most
// m events, and every run's buffer nodes are private; so the matches of a key's stream
// x_0..x_{n-1} are exactly the windows (i-m+1 .. i) with p_t(x_{i-m+1+t}) for all t,
// emitted in increasing i, each the walk (stage m-1, x_i), ..., (stage 0, x_{i-m+1})
// (proof: SURVEY Appendix A.5).  That is a 1-D stencil over the column:
// HBM-bound, one pass.
//
// Layout.  A tile is 256 threads x 64 consecutive events; a thread reads its 64 int32 values
// with sixteen 16-B loads (plus the m-1 halo events), evaluates the m stage predicates into
// 64-bit masks and ANDs them shifted (match bit i = Π_x P_{m-1-x}(i-x)).  Key starts come
// from a bitmap built once per batch, so a window crossing a key start is masked with
// shifts, and a match's key is the tile's first key advanced by the key starts before it.
//
// Passes.  (1) stencil_mask streams the column once and writes one 64-bit match mask per 64
// events (1 bit/event) and a count per tile; (2) a single-block scan turns tile counts into
// output offsets; (3) stencil_emit reads the masks back (1/32 of the column's bytes) and
// writes the matches in order.  Nothing waits on another workgroup, so the streaming pass
// runs at HBM rate (a single-pass decoupled look-back was measured latency-bound here:
// rounds of co-resident tiles look back through each other, profiles/README.md).
#include <hip/hip_runtime.h>

#include "cep_layout.h"
#include "nfa_device.h"
#include "stencil_args.h"

namespace cep {

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int kStThreads = 256;
constexpr int kStPer = 64;  // events per thread (one 64-bit mask)
constexpr uint64_t kStTile = (uint64_t)kStThreads * kStPer;

// ---------------------------------------------------------------- per-batch key index
// rank[k] = number of non-empty keys before k (two-level exclusive scan)
__global__ void __launch_bounds__(1024) nz_rank_blocks(const uint64_t* key_off, uint64_t n_keys, uint32_t* rank,
                                                       uint32_t* bsum) {
  __shared__ uint32_t s[1024];
  const uint64_t k = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  const uint32_t f = (k < n_keys && key_off[k + 1] > key_off[k]) ? 1u : 0u;
  s[threadIdx.x] = f;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const uint32_t y = threadIdx.x >= (unsigned)o ? s[threadIdx.x - o] : 0;
    __syncthreads();
    s[threadIdx.x] += y;
    __syncthreads();
  }
  if (k < n_keys) rank[k] = s[threadIdx.x] - f;
  if (threadIdx.x == 1023) bsum[blockIdx.x] = s[1023];
}

__global__ void __launch_bounds__(1024) nz_rank_top(uint32_t* bsum, uint64_t nb) {
  __shared__ uint32_t t[1024];
  const uint64_t per = (nb + 1023) / 1024;
  const uint64_t a = threadIdx.x * per, b = (a + per < nb) ? a + per : nb;
  uint32_t sum = 0;
  for (uint64_t i = a; i < b; i++) sum += bsum[i];
  t[threadIdx.x] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int i = 0; i < 1024; i++) {
      const uint32_t x = t[i];
      t[i] = acc;
      acc += x;
    }
  }
  __syncthreads();
  uint32_t o = t[threadIdx.x];
  for (uint64_t i = a; i < b; i++) {
    const uint32_t x = bsum[i];
    bsum[i] = o;
    o += x;
  }
}

// non-empty key k: nz_key[rank] = k, its start bit, and the rank of every tile whose first
// event lies inside it
__global__ void __launch_bounds__(256) key_index(const uint64_t* key_off, uint64_t n_keys, const uint32_t* rank,
                                                 const uint32_t* bsum, uint32_t* nz_key, uint64_t* bnd,
                                                 uint32_t* tile_rank, uint64_t n_tiles) {
  const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n_keys) return;
  const uint64_t s = key_off[k], e = key_off[k + 1];
  if (s == e) return;
  const uint32_t r = rank[k] + bsum[k / 1024];
  nz_key[r] = (uint32_t)k;
  atomicOr((unsigned long long*)&bnd[s / 64], 1ull << (s % 64));
  for (uint64_t t = (s + kStTile - 1) / kStTile; t * kStTile < e && t < n_tiles; t++) tile_rank[t] = r;
}

// ---------------------------------------------------------------- the stencil
__device__ __forceinline__ uint64_t mix64s(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ bool in_range(int64_t v, int64_t lo, int64_t hi) { return v >= lo && v <= hi; }

// Pass 1 layout.  A wave owns kStWave consecutive events and reads them with 16-B loads in
// which lane l holds events 4l..4l+3 of a 256-event step: every load instruction covers
// 1 KiB contiguous (fully coalesced).  Per step a lane evaluates the M stage predicates
// into 4-bit nibbles; the window needs the M-1 <= 7 events before the nibble, i.e. the
// nibbles of lanes l-1 and l-2 (cross-lane shuffles) or, for lanes 0-1, of lanes 62-63 of
// the previous step (wave-uniform carries).  Key starts come the same way from the bitmap.
constexpr int kStWave = kStTile / (kStThreads / 64);  // 4096 events per wave
constexpr int kStSteps = kStWave / 256;               // 16 load steps per wave

template <int M, bool RANGE, int NCOL>
struct StEval {
  int32_t lo[M][2], hi[M][2];
  __device__ __forceinline__ explicit StEval(const StencilArgs& A) {
    if (RANGE) {
      // int32 bounds (a range outside int32 is clamped: empty stays empty)
#pragma unroll
      for (int s = 0; s < M; s++)
#pragma unroll
        for (int c = 0; c < 2; c++) {
          const int64_t l = A.rs[s].lo[c], h = A.rs[s].hi[c];
          lo[s][c] = l < INT32_MIN ? INT32_MIN : (l > INT32_MAX ? INT32_MAX : (int32_t)l);
          hi[s][c] = h > INT32_MAX ? INT32_MAX : (h < INT32_MIN ? INT32_MIN : (int32_t)h);
          if (l > INT32_MAX || h < INT32_MIN || l > h) {
            lo[s][c] = 1;
            hi[s][c] = 0;
          }
        }
    }
  }
  // stage bits of one event into bit `bit` of P[s]
  __device__ __forceinline__ void range(int32_t x0, int32_t x1, uint32_t* P, int bit) const {
#pragma unroll
    for (int s = 0; s < M; s++) {
      bool ok = x0 >= lo[s][0] && x0 <= hi[s][0];
      if (NCOL > 1) ok = ok && x1 >= lo[s][1] && x1 <= hi[s][1];
      P[s] |= (ok ? 1u : 0u) << bit;
    }
  }
  __device__ __forceinline__ void one(const StencilArgs& A, uint64_t p, uint32_t* P, int bit) const {
    if (p >= A.n_events) return;
    if (RANGE) {
      range(A.col[0][p], A.col[NCOL - 1][p], P, bit);
    } else {
      EvalIn in{&A.cols, A.q->field_type, A.ts, p, nullptr, 0, 0, true};
      for (int s = 0; s < M; s++) {
        bool rn;
        int ee = 0;
        if (interp(A.code, A.prog[s], in, &rn, &ee) != 0) P[s] |= 1u << bit;  // total: never throws
      }
    }
  }
};

template <int M, bool RANGE, int NCOL>
__global__ void __launch_bounds__(kStThreads) stencil_mask(StencilArgs A) {
  constexpr int H = M - 1;  // events a window reaches back
  __shared__ uint32_t s_cnt[kStThreads / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t wbase = (uint64_t)blockIdx.x * kStTile + (uint64_t)wv * kStWave;
  const StEval<M, RANGE, NCOL> ev(A);
  // carries: nibbles of the 8 events before the step (c1: -4..-1, c2: -8..-5), wave-uniform
  uint32_t c1[M], c2[M];
  uint32_t bc1 = 0, bc2 = 0;
  {
    uint32_t P[M];
#pragma unroll
    for (int s = 0; s < M; s++) P[s] = 0;
    if (H > 0 && lane < 8 && wbase >= (uint64_t)(8 - lane)) ev.one(A, wbase - 8 + lane, P, 0);
#pragma unroll
    for (int s = 0; s < M; s++) {
      const uint64_t b = __ballot(P[s] & 1u);
      c2[s] = (uint32_t)b & 0xF;
      c1[s] = (uint32_t)(b >> 4) & 0xF;
    }
    if (H > 0 && wbase >= 8) {  // key-start bits of events wbase-8 .. wbase-1 (wbase % 64 == 0)
      const uint64_t w = A.bnd[wbase / 64 - 1];
      bc2 = (uint32_t)(w >> 56) & 0xF;
      bc1 = (uint32_t)(w >> 60) & 0xF;
    }
  }
  uint32_t cnt = 0;
#pragma unroll 4
  for (int q = 0; q < kStSteps; q++) {
    const uint64_t e0 = wbase + (uint64_t)q * 256 + (uint64_t)lane * 4;
    uint32_t P[M];
#pragma unroll
    for (int s = 0; s < M; s++) P[s] = 0;
    if (RANGE && A.aligned && e0 + 4 <= A.n_events) {
      const v4i x = __builtin_nontemporal_load(reinterpret_cast<const v4i*>(A.col[0] + e0));
      v4i y = x;
      if (NCOL > 1) y = __builtin_nontemporal_load(reinterpret_cast<const v4i*>(A.col[1] + e0));
      ev.range(x.x, y.x, P, 0);
      ev.range(x.y, y.y, P, 1);
      ev.range(x.z, y.z, P, 2);
      ev.range(x.w, y.w, P, 3);
    } else if (e0 < A.n_events) {
#pragma unroll
      for (int i = 0; i < 4; i++) ev.one(A, e0 + i, P, i);
    }
    uint32_t B = 0;
    if (H > 0 && e0 < A.n_events) B = (uint32_t)(A.bnd[e0 / 64] >> (e0 % 64)) & 0xF;
    // 12-bit windows: [11:8] this nibble, [7:4] the 4 events before, [3:0] the 4 before that
    uint32_t match = 0xF;
#pragma unroll
    for (int s = 0; s < M; s++) {
      uint32_t w = P[s] << 8;
      if (H > 0) {
        const uint32_t u1 = __shfl_up(P[s], 1, 64), u2 = __shfl_up(P[s], 2, 64);
        const uint32_t p1 = lane >= 1 ? u1 : c1[s];
        const uint32_t p2 = lane >= 2 ? u2 : (lane == 1 ? c1[s] : c2[s]);
        w |= (p1 << 4) | p2;
        c2[s] = __shfl(P[s], 62, 64);
        c1[s] = __shfl(P[s], 63, 64);
      }
      // stage s sits at offset -(M-1-s) from the window's last event
      match &= w >> (8 - (M - 1 - s));
    }
    if (H > 0) {
      const uint32_t u1 = __shfl_up(B, 1, 64), u2 = __shfl_up(B, 2, 64);
      const uint32_t b1 = lane >= 1 ? u1 : bc1;
      const uint32_t b2 = lane >= 2 ? u2 : (lane == 1 ? bc1 : bc2);
      const uint32_t bw = (B << 8) | (b1 << 4) | b2;
      // a key start at any of the window's last M-1 events (not its first) kills it
      uint32_t sm = 0;
#pragma unroll
      for (int x = 0; x < H; x++) sm |= bw << x;
      match &= ~(sm >> 8);
      bc2 = __shfl(B, 62, 64);
      bc1 = __shfl(B, 63, 64);
    }
    match &= 0xF;
    if (e0 + 4 > A.n_events) match &= e0 >= A.n_events ? 0u : ((1u << (A.n_events - e0)) - 1);
    cnt += __popc(match);
    // 16 lanes -> one 64-bit mask word
    uint64_t word = (uint64_t)match << (4 * (lane & 15));
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) word |= __shfl_xor(word, o, 64);
    if ((lane & 15) == 0 && e0 < A.n_events) A.mask[e0 / 64] = word;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off, 64);
  if (lane == 0) s_cnt[wv] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) A.tile_cnt[blockIdx.x] = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
}

// exclusive scan of the tile counts (one block; ~n_tiles/1024 sequential per thread)
__global__ void __launch_bounds__(1024) stencil_scan(const uint32_t* cnt, uint64_t n, uint64_t* off, uint64_t* total) {
  __shared__ uint64_t s[1024];
  const uint64_t per = (n + 1023) / 1024;
  const uint64_t a = threadIdx.x * per, b = (a + per < n) ? a + per : n;
  uint64_t sum = 0;
  for (uint64_t i = a; i < b; i++) sum += cnt[i];
  s[threadIdx.x] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const uint64_t y = threadIdx.x >= (unsigned)o ? s[threadIdx.x - o] : 0;
    __syncthreads();
    s[threadIdx.x] += y;
    __syncthreads();
  }
  uint64_t acc = s[threadIdx.x] - sum;
  for (uint64_t i = a; i < b; i++) {
    off[i] = acc;
    acc += cnt[i];
  }
  if (threadIdx.x == 1023) *total = s[1023];
}

template <int M>
__global__ void __launch_bounds__(kStThreads) stencil_emit(StencilArgs A) {
  __shared__ uint32_t s_wsum[kStThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint64_t t = blockIdx.x;
  const uint64_t p0 = t * kStTile + (uint64_t)tid * kStPer;
  uint64_t match = 0, B = 0;
  if (p0 < A.n_events) {
    match = A.mask[p0 / 64];
    B = A.bnd[p0 / 64];
  }
  const uint64_t Bk = (tid == 0) ? (B & ~1ull) : B;  // key starts after the tile's first event
  const uint32_t cnt = (uint32_t)__popcll(match), bc = (uint32_t)__popcll(Bk);
  // block exclusive scan of (matches, key starts), packed 16|16 (each <= 16384 per tile)
  const uint32_t packed = (cnt << 16) | bc;
  uint32_t incl = packed;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) s_wsum[wv] = incl;
  __syncthreads();
  uint32_t woff = 0;
#pragma unroll
  for (int w = 0; w < kStThreads / 64; w++)
    if (w < wv) woff += s_wsum[w];
  const uint32_t excl = woff + incl - packed;
  uint64_t o = A.tile_off[t] + (excl >> 16);
  const uint32_t rank0 = A.tile_rank[t] + (excl & 0xFFFF);
  uint32_t cur_rank = 0xFFFFFFFFu, key = 0;
  uint64_t kstart = 0;
  while (match) {
    const int i = __builtin_ctzll(match);
    match &= match - 1;
    const uint64_t p = p0 + i;
    const uint32_t rk = rank0 + (uint32_t)__popcll(Bk & (i == 63 ? ~0ull : ((2ull << i) - 1)));
    if (rk != cur_rank) {
      cur_rank = rk;
      key = A.nz_key[rk];
      kstart = A.key_off[key];
    }
    const uint32_t seq = (uint32_t)(p - kstart);
    if (o < A.out_cap) {
      A.m_key[o] = key;
#pragma unroll
      for (int x = 0; x < M; x++) A.p_seq[o * M + x] = seq - x;
    } else {
      atomicOr(A.overflow, 1u);
    }
    o++;
  }
}

// ---------------------------------------------------------------- host launchers
hipError_t launch_key_index(const uint64_t* key_off, uint64_t n_keys, uint64_t n_events, uint32_t* rank,
                            uint32_t* bsum, uint32_t* nz_key, uint64_t* bnd, uint32_t* tile_rank,
                            hipStream_t st) {
  const uint64_t n_tiles = (n_events + kStTile - 1) / kStTile;
  if (n_keys == 0 || n_tiles == 0) return hipSuccess;
  const uint64_t nb = (n_keys + 1023) / 1024;
  hipLaunchKernelGGL(nz_rank_blocks, dim3((uint32_t)nb), dim3(1024), 0, st, key_off, n_keys, rank, bsum);
  hipLaunchKernelGGL(nz_rank_top, dim3(1), dim3(1024), 0, st, bsum, nb);
  hipLaunchKernelGGL(key_index, dim3((uint32_t)((n_keys + 255) / 256)), dim3(256), 0, st, key_off, n_keys, rank, bsum,
                     nz_key, bnd, tile_rank, n_tiles);
  return hipGetLastError();
}

template <int M, bool RANGE, int NCOL>
static hipError_t launch_one(const StencilArgs& a, uint64_t n_tiles, hipStream_t st) {
  hipLaunchKernelGGL((stencil_mask<M, RANGE, NCOL>), dim3((uint32_t)n_tiles), dim3(kStThreads), 0, st, a);
  hipLaunchKernelGGL(stencil_scan, dim3(1), dim3(1024), 0, st, a.tile_cnt, n_tiles, a.tile_off, a.total);
  hipLaunchKernelGGL(stencil_emit<M>, dim3((uint32_t)n_tiles), dim3(kStThreads), 0, st, a);
  return hipGetLastError();
}

template <int M>
static hipError_t launch_m(const StencilArgs& a, bool range, int ncol, uint64_t n_tiles, hipStream_t st) {
  if (range && ncol == 1) return launch_one<M, true, 1>(a, n_tiles, st);
  if (range) return launch_one<M, true, 2>(a, n_tiles, st);
  return launch_one<M, false, 1>(a, n_tiles, st);
}

hipError_t launch_stencil(int m, const StencilArgs& a, bool range, int ncol, hipStream_t st) {
  const uint64_t n_tiles = (a.n_events + kStTile - 1) / kStTile;
  if (n_tiles == 0) return hipSuccess;
  switch (m) {
    case 1: return launch_m<1>(a, range, ncol, n_tiles, st);
    case 2: return launch_m<2>(a, range, ncol, n_tiles, st);
    case 3: return launch_m<3>(a, range, ncol, n_tiles, st);
    case 4: return launch_m<4>(a, range, ncol, n_tiles, st);
    case 5: return launch_m<5>(a, range, ncol, n_tiles, st);
    case 6: return launch_m<6>(a, range, ncol, n_tiles, st);
    case 7: return launch_m<7>(a, range, ncol, n_tiles, st);
    case 8: return launch_m<8>(a, range, ncol, n_tiles, st);
  }
  return hipErrorInvalidValue;
}

uint64_t stencil_tiles(uint64_t n_events) { return (n_events + kStTile - 1) / kStTile; }

}  // namespace cep
