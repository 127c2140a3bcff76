// stencil.hip — CEP_KIND_STENCIL: SEQ(p_0, ..., p_{m-1}) with every stage ONE + strict
// contiguity and total, state-free predicates.
//
// For such queries the reference NFA (nfa/NFA.java) never branches, each run lives at most
// m events, and every run's buffer nodes are private; so the matches of a key's stream
// x_0..x_{n-1} are exactly the windows (i-m+1 .. i) with p_t(x_{i-m+1+t}) for all t,
// emitted in increasing i, each the walk (stage m-1, x_i), ..., (stage 0, x_{i-m+1})
// (proof: SURVEY Appendix A.5).  That is a 1-D stencil over the column:
// HBM-bound, one pass.
//
// Layout: tile = 256 threads x 16 consecutive events.  A thread reads its 16 int32 values
// with four 16-B loads (plus the previous vector for the m-1 halo), evaluates the m stage
// predicates as bit vectors, and ANDs them shifted (match bit i = Π_t P_{m-1-t}(i-t)).
// Key boundaries come from the CSR offsets (first key of each tile precomputed).  Output
// order is deterministic: a per-tile decoupled look-back (8-B status granules, agent scope)
// gives each tile its global output offset in a single pass.
#include <hip/hip_runtime.h>

#include "cep_layout.h"
#include "nfa_device.h"

namespace cep {

constexpr int kStTile = 4096;  // events per tile
constexpr int kStThreads = 256;
constexpr int kStPer = 16;     // events per thread

// tile -> first key: key k writes every tile whose first event lies inside it
__global__ void __launch_bounds__(256) tile_first_key(const uint64_t* key_off, uint64_t n_keys, uint32_t* tile_key,
                                                      uint64_t n_tiles) {
  const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n_keys) return;
  const uint64_t s = key_off[k], e = key_off[k + 1];
  if (s == e) return;
  for (uint64_t t = (s + kStTile - 1) / kStTile; t * kStTile < e && t < n_tiles; t++) tile_key[t] = (uint32_t)k;
}

__device__ __forceinline__ uint64_t mix64s(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ bool in_range(int64_t v, int64_t lo, int64_t hi) { return v >= lo && v <= hi; }

template <int M, bool RANGE, int NCOL>
__global__ void __launch_bounds__(kStThreads) stencil_kernel(StencilArgs A) {
  constexpr int HV = 8;        // halo values loaded before p0 (two 16-B vectors)
  constexpr int H = M - 1;     // halo events a window needs
  constexpr int kBnd = kStTile + HV + 1;
  __shared__ uint32_t s_tile;
  __shared__ unsigned long long s_excl;
  __shared__ uint32_t s_bnd[kBnd];   // key starts, relative to tile_lo - HV (sorted)
  __shared__ uint32_t s_bkey[kBnd];
  __shared__ uint32_t s_wk[kStThreads / 64], s_wi[kStThreads / 64];
  __shared__ uint32_t s_wsum[kStThreads / 64];
  __shared__ unsigned long long s_dig[kStThreads / 64];

  const int tid = threadIdx.x;
  if (tid == 0) s_tile = atomicAdd(A.tile_counter, 1u);
  __syncthreads();
  const uint64_t t = s_tile;
  const uint64_t n_tiles = (A.n_events + kStTile - 1) / kStTile;
  const uint64_t tile_lo = t * kStTile;
  const uint64_t tile_hi = tile_lo + kStTile < A.n_events ? tile_lo + kStTile : A.n_events;
  const int64_t rel0 = (int64_t)tile_lo - HV;

  // issue this thread's column loads first: they do not depend on the key boundaries
  const uint64_t p0 = tile_lo + (uint64_t)tid * kStPer;  // first event of this thread
  int32_t v[NCOL][kStPer + HV];
  if (RANGE && p0 < tile_hi) {
#pragma unroll
    for (int c = 0; c < NCOL; c++) {
      const int32_t* col = A.col[c];
      if (p0 + kStPer <= A.n_events) {
        const int4* src = reinterpret_cast<const int4*>(col + p0);
#pragma unroll
        for (int q = 0; q < kStPer / 4; q++) {
          const int4 x = src[q];
          v[c][HV + 4 * q + 0] = x.x;
          v[c][HV + 4 * q + 1] = x.y;
          v[c][HV + 4 * q + 2] = x.z;
          v[c][HV + 4 * q + 3] = x.w;
        }
      } else {
#pragma unroll
        for (int i = 0; i < kStPer; i++) v[c][HV + i] = (p0 + i < A.n_events) ? col[p0 + i] : 0;
      }
      if (H > 0) {
        if (p0 >= (uint64_t)HV) {
          const int4* src = reinterpret_cast<const int4*>(col + p0 - HV);
#pragma unroll
          for (int q = (HV - H) / 4; q < HV / 4; q++) {
            const int4 x = src[q];
            v[c][4 * q + 0] = x.x; v[c][4 * q + 1] = x.y; v[c][4 * q + 2] = x.z; v[c][4 * q + 3] = x.w;
          }
        } else {
#pragma unroll
          for (int i = 0; i < HV; i++) v[c][i] = (p0 + i >= (uint64_t)HV) ? col[p0 + i - HV] : 0;
        }
      }
    }
  }

  // starts of the non-empty keys k0.. that begin before tile_hi (k0 = the key holding
  // tile_lo), compacted into LDS cooperatively: at most kStTile + 1 entries
  const int lane = tid & 63, wv = tid >> 6;
  const uint32_t k0 = A.tile_key[t];
  uint32_t nb = 0;
  for (uint64_t kb = k0;; kb += kStThreads) {
    const uint64_t k = kb + tid;
    const bool have = k < A.n_keys;
    uint64_t s = 0, e = 0;
    if (have) {
      s = A.key_off[k];
      e = A.key_off[k + 1];
    }
    const bool inr = have && s < tile_hi;
    const bool keep = inr && (e > s || k == k0);
    const uint64_t bk = __ballot(keep), bi = __ballot(inr);
    if (lane == 0) {
      s_wk[wv] = (uint32_t)__popcll(bk);
      s_wi[wv] = (uint32_t)__popcll(bi);
    }
    __syncthreads();
    uint32_t off = nb, tot = 0, toti = 0;
    for (int w = 0; w < kStThreads / 64; w++) {
      if (w < wv) off += s_wk[w];
      tot += s_wk[w];
      toti += s_wi[w];
    }
    if (keep) {
      const uint32_t idx = off + (uint32_t)__popcll(bk & ((1ull << lane) - 1));
      const int64_t r = (int64_t)s - rel0;
      s_bnd[idx] = r < 0 ? 0u : (uint32_t)r;
      s_bkey[idx] = (uint32_t)k;
    }
    nb += tot;
    __syncthreads();
    if (toti < (uint32_t)kStThreads) break;
  }

  uint32_t P[M];  // bit b: event p0 - H + b satisfies stage predicate
#pragma unroll
  for (int s = 0; s < M; s++) P[s] = 0;
  uint32_t valid = 0;
  if (p0 < tile_hi) {
    if (RANGE) {
#pragma unroll
      for (int b = 0; b < kStPer + H; b++) {
        const int i = HV - H + b;
        const int64_t p = (int64_t)p0 - H + b;
        if (p < 0 || (uint64_t)p >= A.n_events) continue;
        valid |= 1u << b;
#pragma unroll
        for (int s = 0; s < M; s++) {
          bool ok = in_range(v[0][i], A.rs[s].lo[0], A.rs[s].hi[0]);
          if (NCOL > 1) ok = ok && in_range(v[NCOL - 1][i], A.rs[s].lo[1], A.rs[s].hi[1]);
          P[s] |= (ok ? 1u : 0u) << b;
        }
      }
    } else {
      for (int b = 0; b < kStPer + H; b++) {
        const int64_t p = (int64_t)p0 - H + b;
        if (p < 0 || (uint64_t)p >= A.n_events) continue;
        valid |= 1u << b;
        EvalIn in;
        in.cols = &A.cols;
        in.ftype = A.q->field_type;
        in.ts = A.ts;
        in.pos = (uint64_t)p;
        in.W = nullptr;
        in.wnull = 0;
        in.curr = 0;
        in.curr_null = true;
        for (int s = 0; s < M; s++) {
          bool rn;
          int ee = 0;
          const bool ok = interp(A.code, A.prog[s], in, &rn, &ee) != 0;  // total: never throws
          P[s] |= (ok ? 1u : 0u) << b;
        }
      }
    }
  }
  // a key start strictly inside a window kills it: the window ending at bit e covers bits
  // e-H..e, so a start at bit d kills the windows ending at d .. d+H-1.
  uint32_t kill = 0;
  uint32_t kb = 0;  // index of the last key start <= the thread's first window event
  {
    const int64_t lo = (int64_t)p0 - H - rel0;  // bit 0 of this thread, relative to rel0
    uint32_t a = 0, b = nb;                     // upper_bound(lo) - 1
    while (a < b) {
      const uint32_t mid = (a + b) >> 1;
      if ((int64_t)s_bnd[mid] <= lo) a = mid + 1;
      else b = mid;
    }
    kb = a > 0 ? a - 1 : 0;
    for (uint32_t i = a; i < nb; i++) {
      const int64_t d = (int64_t)s_bnd[i] - lo;
      if (d >= kStPer + H) break;
#pragma unroll
      for (int x = 0; x < H; x++) kill |= (1u << d) << x;
    }
  }
  uint32_t match = valid;
#pragma unroll
  for (int x = 0; x < M; x++) match &= P[M - 1 - x] << x;  // stage M-1-x at offset -x
  match &= ~kill;
  match >>= H;  // bit i -> event p0 + i
  if (p0 >= tile_hi) match = 0;
  match &= (kStPer >= 32) ? 0xFFFFFFFFu : ((1u << kStPer) - 1);
  const uint32_t cnt = __popc(match);

  // block exclusive scan of counts
  uint32_t incl = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) s_wsum[wv] = incl;
  __syncthreads();
  uint32_t woff = 0, agg = 0;
  for (int w = 0; w < kStThreads / 64; w++) {
    if (w < wv) woff += s_wsum[w];
    agg += s_wsum[w];
  }
  // decoupled look-back for the tile's global offset, one wavefront reading 64 predecessor
  // status granules per step: it stops at the nearest inclusive prefix and sums the
  // aggregates in between, spinning only while a nearer predecessor has not published
  if (wv == 0) {
    unsigned long long excl = 0;
    if (lane == 0)
      __hip_atomic_store(&A.status[t], ((t == 0 ? 2ull : 1ull) << 62) | agg, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    if (t > 0) {
      int64_t base = (int64_t)t - 1;
      uint32_t spins = 0;
      for (;;) {
        const int64_t idx = base - lane;
        const unsigned long long s =
            idx >= 0 ? __hip_atomic_load(&A.status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                     : (2ull << 62);  // before tile 0: inclusive prefix 0
        const uint32_t flag = (uint32_t)(s >> 62);
        const uint64_t inc = __ballot(flag == 2), zero = __ballot(flag == 0);
        const int first = inc ? __builtin_ctzll(inc) : 64;
        const uint64_t upto = first >= 63 ? ~0ull : ((2ull << first) - 1);  // lanes 0..first
        if (zero & upto) {
          // predecessors took their tickets earlier, so they are resident and will publish;
          // the bound only turns a bug into a reported error instead of a hang
          if (++spins > (1u << 22)) {
            if (lane == 0) atomicOr(A.overflow, 2u);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        unsigned long long v = ((upto >> lane) & 1) ? (s & ((1ull << 62) - 1)) : 0;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
        excl += __shfl(v, 0, 64);
        if (first < 64) break;
        base -= 64;
      }
      if (lane == 0)
        __hip_atomic_store(&A.status[t], (2ull << 62) | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) {
      s_excl = excl;
      if (t == n_tiles - 1) *A.total = excl + agg;
    }
  }
  __syncthreads();
  uint64_t o = s_excl + woff + (incl - cnt);
  unsigned long long dsum = 0;
  while (match) {
    const int i = __builtin_ctz(match);
    match &= match - 1;
    const uint64_t p = p0 + i;
    const int64_t pr = (int64_t)p - rel0;
    while (kb + 1 < nb && (int64_t)s_bnd[kb + 1] <= pr) kb++;
    const uint32_t key = s_bkey[kb];
    const uint32_t seq = (uint32_t)(p - A.key_off[key]);
    if (o < A.out_cap) {
      A.m_key[o] = key;
#pragma unroll
      for (int x = 0; x < M; x++) A.p_seq[o * M + x] = seq - x;
    } else {
      atomicOr(A.overflow, 1u);
    }
    uint64_t h = mix64s(0x9E3779B97F4A7C15ull ^ ((uint64_t)key << 32) ^ seq);
#pragma unroll
    for (int x = 0; x < M; x++) h = mix64s(h ^ (((uint64_t)A.stage_name[x] << 32) | (seq - x)));
    dsum += h;
    o++;
  }
  // digest: wave reduce then one atomic per block
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) dsum += __shfl_down(dsum, off, 64);
  if (lane == 0) s_dig[wv] = dsum;
  __syncthreads();
  if (tid == 0) {
    unsigned long long d = 0;
    for (int w = 0; w < kStThreads / 64; w++) d += s_dig[w];
    if (d) atomicAdd(A.digest, d);
  }
}

hipError_t launch_tile_first_key(const uint64_t* key_off, uint64_t n_keys, uint32_t* tile_key, uint64_t n_events,
                                 hipStream_t st) {
  const uint64_t n_tiles = (n_events + kStTile - 1) / kStTile;
  if (n_keys == 0 || n_tiles == 0) return hipSuccess;
  hipLaunchKernelGGL(tile_first_key, dim3((uint32_t)((n_keys + 255) / 256)), dim3(256), 0, st, key_off, n_keys,
                     tile_key, n_tiles);
  return hipGetLastError();
}

template <int M>
static hipError_t launch_m(const StencilArgs& a, bool range, int ncol, uint64_t n_tiles, hipStream_t st) {
  if (range && ncol == 1)
    hipLaunchKernelGGL((stencil_kernel<M, true, 1>), dim3((uint32_t)n_tiles), dim3(kStThreads), 0, st, a);
  else if (range)
    hipLaunchKernelGGL((stencil_kernel<M, true, 2>), dim3((uint32_t)n_tiles), dim3(kStThreads), 0, st, a);
  else
    hipLaunchKernelGGL((stencil_kernel<M, false, 1>), dim3((uint32_t)n_tiles), dim3(kStThreads), 0, st, a);
  return hipGetLastError();
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
