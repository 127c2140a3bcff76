// partition.hip — arrival-order batches -> the key-partitioned (CSR) layout the matchers read.
//
// The reference's processor receives records one at a time in arrival order
// (CEPProcessor.process, CEPProcessor.java:155-163) and each key's NFA sees that key's records
// in that order.  A batch handed over in arrival order (one key id per event) is
// partitioned on the device: a stable LSD radix sort of (key, arrival index) pairs by key
// (rocPRIM through hipCUB), key_off by a binary search per key over the sorted keys, then one
// gather per column.
// Stability is what keeps every key's events in arrival order.  All passes are HBM-bound.
//
// Also the synthetic arrival-order stream of the bench/tests: the CSR stream of
// workloads.generate interleaved round-robin, arrival order = (index within key, key).
#include <hip/hip_runtime.h>


#include "cep_internal.h"
#include "kernel_args.h"

namespace cep {

__global__ void __launch_bounds__(256) iota_u32(uint32_t* v, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) v[i] = (uint32_t)i;
}

// ---- stable LSD counting sort of (key, arrival index) by key, hand-written -------------
// Digits of <= 8 bits (256 bins): a 20-bit key space (1M keys) is three passes.  Per pass:
//   rs_hist     per tile of 8192 events, a digit histogram in LDS -> hist[bin * T + tile]
//   scan_u32    exclusive scan of hist (bin-major, tile-minor): each (bin, tile)'s first slot
//   rs_scatter  per tile: each wave ranks its events within their digit with ballots (one
//               ballot per digit bit; peers = the lanes whose digits agree) and per-wave digit
//               counters in LDS; the tile is then sorted by digit in LDS and written out bin run
//               by bin run, so consecutive lanes store consecutive words (coalesced).
// Stability: within a wave by round then lane, across waves by the prefix, across tiles by
// the scan order - every key's events keep arrival order.  The first pass reads the caller's
// key array (and range-checks it) and makes the arrival index from the position; the last
// writes the sorted keys and the permutation.
constexpr int kRsThreads = 256, kRsRounds = 32, kRsWaves = kRsThreads / 64;
constexpr int kRsRoundsMin = 8;  // the smallest tile ($CEP_PART_ROUNDS, partition only)
constexpr int kRsMaxBits = 8;
constexpr uint32_t kRsBins = 1u << kRsMaxBits;

// (kRsHistTiles tiles per block, each with its own LDS histogram: 16-B loads, a quarter of the
// workgroups; one tile per block read the keys at ~3.1 TB/s)
constexpr int kRsHistTiles = 4;
template <bool FIRST, bool INV, int R = kRsRounds>
__global__ void __launch_bounds__(kRsThreads) rs_hist(const uint32_t* __restrict__ keys, uint64_t n, uint64_t n_keys,
                                                      int shift, int bits, uint32_t* hist, uint64_t T, unsigned* bad) {
  static_assert(R % 4 == 0, "16-B loads");
  __shared__ uint32_t h[kRsHistTiles][kRsBins];
  const uint32_t bins = 1u << bits, mask = bins - 1;
  for (uint32_t d = threadIdx.x; d < kRsHistTiles * kRsBins; d += kRsThreads) (&h[0][0])[d] = 0;
  __syncthreads();
  bool oob = false;
  const bool aligned = (reinterpret_cast<uintptr_t>(keys) & 15) == 0;  // (a caller's key array may not be)
  auto add = [&](int t, uint32_t k0) {
    const uint32_t k = (FIRST && INV) ? ~k0 : k0;
    if (FIRST && !INV && k >= n_keys) oob = true;
    atomicAdd(&h[t][(k >> shift) & mask], 1u);
  };
#pragma unroll
  for (int t = 0; t < kRsHistTiles; t++) {
    const uint64_t tile = (uint64_t)blockIdx.x * kRsHistTiles + t;
    const uint64_t t0 = tile * ((uint64_t)kRsThreads * R);
#pragma unroll
    for (int r = 0; r < R / 4; r++) {
      const uint64_t i = t0 + ((uint64_t)r * kRsThreads + threadIdx.x) * 4;
      if (aligned && i + 4 <= n) {
        const uint4 v = *reinterpret_cast<const uint4*>(keys + i);
        add(t, v.x);
        add(t, v.y);
        add(t, v.z);
        add(t, v.w);
      } else {
        for (uint64_t e = i; e < n && e < i + 4; e++) add(t, keys[e]);
      }
    }
  }
  if (FIRST && oob) atomicOr(bad, 1u);
  __syncthreads();
  for (int t = 0; t < kRsHistTiles; t++) {
    const uint64_t tile = (uint64_t)blockIdx.x * kRsHistTiles + t;
    if (tile >= T) break;
    for (uint32_t d = threadIdx.x; d < bins; d += kRsThreads) hist[(uint64_t)d * T + tile] = h[t][d];
  }
}

template <bool FIRST, bool INV, int R = kRsRounds>
__global__ void __launch_bounds__(kRsThreads) rs_scatter(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                         uint64_t n, int shift, int bits,
                                                         const uint32_t* __restrict__ off, uint64_t T, uint32_t* kout,
                                                         uint32_t* vout) {
  __shared__ uint32_t cnt[kRsWaves][kRsBins];  // per-wave digit counts -> the waves' first local slots
  __shared__ uint32_t lstart[kRsBins], gbase[kRsBins];
  constexpr uint32_t kTile = (uint32_t)kRsThreads * R;
  __shared__ uint32_t sk[kTile], sv[kTile];  // the tile sorted by digit
  const uint32_t bins = 1u << bits, mask = bins - 1;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint32_t d = threadIdx.x; d < kRsBins; d += kRsThreads)
#pragma unroll
    for (int x = 0; x < kRsWaves; x++) cnt[x][d] = 0;
  __syncthreads();
  const uint64_t t0 = (uint64_t)blockIdx.x * kTile;
  const uint32_t tn = (uint32_t)(n - t0 < kTile ? n - t0 : kTile);
  // this wave's events: a contiguous quarter of the tile, 64 per round
  const uint32_t e0 = w * (kTile / kRsWaves);
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t key[R], val[R], rank[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const uint32_t i = e0 + (uint32_t)r * 64 + lane;
    key[r] = i < tn ? ((FIRST && INV) ? ~kin[t0 + i] : kin[t0 + i]) : 0u;
    val[r] = i < tn ? (FIRST ? (uint32_t)(t0 + i) : vin[t0 + i]) : 0u;
  }
#pragma unroll
  for (int r = 0; r < R; r++) {
    const bool valid = e0 + (uint32_t)r * 64 + lane < tn;
    const uint32_t d = (key[r] >> shift) & mask;
    uint64_t peers = __ballot(valid);
    for (int b = 0; b < bits; b++) {
      const uint64_t bb = __ballot(valid && ((d >> b) & 1u));
      peers &= ((d >> b) & 1u) ? bb : ~bb;
    }
    uint32_t base = 0;
    if (valid) base = cnt[w][d];  // every lane reads before the leader writes (one wave, in order)
    rank[r] = base + (uint32_t)__popcll(peers & lt);
    if (valid && (peers & lt) == 0) cnt[w][d] = base + (uint32_t)__popcll(peers);
  }
  __syncthreads();
  // tile-local bin starts (exclusive scan of the bin totals, one wave), then per wave
  if (w == 0) {
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < kRsBins; c0 += 64) {
      const uint32_t d = c0 + lane;
      uint32_t t = 0;
#pragma unroll
      for (int x = 0; x < kRsWaves; x++) t += cnt[x][d];
      uint32_t s2 = t;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(s2, o, 64);
        if (lane >= (uint32_t)o) s2 += y;
      }
      const uint32_t ex = carry + s2 - t;
      lstart[d] = ex;
      uint32_t run = ex;
#pragma unroll
      for (int x = 0; x < kRsWaves; x++) {
        const uint32_t c = cnt[x][d];
        cnt[x][d] = run;
        run += c;
      }
      gbase[d] = d < bins ? off[(uint64_t)d * T + blockIdx.x] : 0u;
      carry += __shfl(s2, 63, 64);
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; r++) {
    if (e0 + (uint32_t)r * 64 + lane < tn) {
      const uint32_t p = cnt[w][(key[r] >> shift) & mask] + rank[r];
      sk[p] = key[r];
      sv[p] = val[r];
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < tn; i += kRsThreads) {
    const uint32_t k = sk[i], d = (k >> shift) & mask;
    const uint32_t g = gbase[d] + (i - lstart[d]);
    kout[g] = k;
    vout[g] = sv[i];
  }
}

// key_off[k] = first position of a key >= k in the sorted keys (binary search per key)
__global__ void __launch_bounds__(256) key_offsets(const uint32_t* __restrict__ sorted, uint64_t n, uint64_t n_keys,
                                                   uint64_t* key_off) {
  const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (k > n_keys) return;
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) / 2;
    if (sorted[mid] < k) lo = mid + 1;
    else hi = mid;
  }
  key_off[k] = lo;
}

// CSR position p <- arrival index perm[p], for every column (4- or 8-byte values) and ts.
// Tiled by key group (round 4; it replaced a position-order gather whose scattered reads ran
// ~22.6 ms for 1e9 events against ~7 ms): a block owns 32 consecutive keys and walks
// their events 64 at a time.  Per chunk: each wave reads 8 of the keys' next 64 permutation
// entries (one contiguous 256 B per key) into LDS; then every thread gathers with lanes laid
// key-minor - lane l reads key (l mod 32)'s event - so one load instruction touches the 32
// keys' events of the same index, which sit next to each other when keys arrive interleaved
// (one 128-B line for a 4-byte column instead of 32); the values go back through LDS and each
// wave writes its keys' 64 positions contiguously.  Any permutation is gathered exactly; the
// tiling only decides which loads run together.
constexpr int kTrKeys = 32, kTrChunk = 64;
__global__ void __launch_bounds__(256) gather_cols_tr(const uint32_t* __restrict__ perm, const uint64_t* key_off,
                                                      uint64_t n_keys, int nf, Cols in, Cols out, uint32_t wide_mask,
                                                      const int64_t* ts_in, int64_t* ts_out) {
  __shared__ uint32_t s_src[kTrKeys][kTrChunk];
  __shared__ uint64_t s_val[kTrKeys][kTrChunk + 1];  // (+1: the key-minor stores spread over banks)
  __shared__ uint64_t s_off[kTrKeys + 1];
  const uint64_t k0 = (uint64_t)blockIdx.x * kTrKeys;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid <= kTrKeys) s_off[tid] = key_off[k0 + tid < n_keys ? k0 + tid : n_keys];
  __syncthreads();
  uint64_t most = 0;
  for (int k = 0; k < kTrKeys; k++) most = s_off[k + 1] - s_off[k] > most ? s_off[k + 1] - s_off[k] : most;
  const int nk_cols = nf + (ts_in ? 1 : 0);
  for (uint64_t c0 = 0; c0 < most; c0 += kTrChunk) {
    // the chunk's permutation entries: wave w, keys 8w .. 8w+7, lane = event (every load in
    // flight before the first LDS store: the scheduler would wait on each in turn)
    uint32_t src[kTrKeys / 4];
#pragma unroll
    for (int i = 0; i < kTrKeys / 4; i++) {
      const int k = w * (kTrKeys / 4) + i;
      const uint64_t j = c0 + (uint64_t)lane;
      src[i] = s_off[k] + j < s_off[k + 1] ? perm[s_off[k] + j] : 0u;
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < kTrKeys / 4; i++) s_src[w * (kTrKeys / 4) + i][lane] = src[i];
    __syncthreads();
    for (int f = 0; f < nk_cols; f++) {
      const bool is_ts = f == nf;
      const bool wide = is_ts || ((wide_mask >> f) & 1u);
      // gather, key-minor: thread t reads key t mod 32, events t / 32 + 8 r (all 8 loads in
      // flight before the LDS stores)
      uint64_t v[kTrChunk / 8];
      const int k = tid % kTrKeys;
      // (loads without a branch - a position past the key's events reads event 0 and is dropped -
      // so they issue back to back: under a branch each waited for the one before)
      uint32_t sj[kTrChunk / 8];
#pragma unroll
      for (int r = 0; r < kTrChunk / 8; r++) {
        const int j = tid / kTrKeys + 8 * r;
        sj[r] = s_off[k] + c0 + (uint64_t)j < s_off[k + 1] ? s_src[k][j] : 0u;
      }
      if (wide) {  // (block-uniform)
        const int64_t* col = is_ts ? ts_in : (const int64_t*)in.p[f];
#pragma unroll
        for (int r = 0; r < kTrChunk / 8; r++) v[r] = (uint64_t)col[sj[r]];
      } else {
        const uint32_t* col = (const uint32_t*)in.p[f];
#pragma unroll
        for (int r = 0; r < kTrChunk / 8; r++) v[r] = col[sj[r]];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < kTrChunk / 8; r++) s_val[tid % kTrKeys][tid / kTrKeys + 8 * r] = v[r];
      __syncthreads();
#pragma unroll
      for (int i = 0; i < kTrKeys / 4; i++) {
        const int k = w * (kTrKeys / 4) + i;
        const uint64_t p = s_off[k] + c0 + (uint64_t)lane;
        if (p < s_off[k + 1]) {
          if (is_ts) ts_out[p] = (int64_t)s_val[k][lane];
          else if (wide) ((int64_t*)out.p[f])[p] = (int64_t)s_val[k][lane];
          else ((int32_t*)out.p[f])[p] = (int32_t)(uint32_t)s_val[k][lane];
        }
      }
      __syncthreads();
    }
  }
}

static int key_bits(uint64_t n_keys) {
  int b = 1;
  while (b < 32 && (1ull << b) < n_keys) b++;
  return b;
}

static uint64_t rs_tiles(uint64_t n, int rounds = kRsRounds) {
  const uint64_t t = (uint64_t)kRsThreads * rounds;
  return std::max<uint64_t>(1, (n + t - 1) / t);
}

// Device scratch of lsd_sort: bytes needed for n keys of `bits` bits (histograms and their
// scan, one (key, value) ping-pong pair per intermediate pass), for the smaller tile.
// (the histogram scan's own scratch last: no allocation on the sort's path)
static size_t lsd_scratch_bytes(uint64_t n, int bits) {
  const int passes = (bits + kRsMaxBits - 1) / kRsMaxBits;
  const uint64_t h = (uint64_t)(1u << kRsMaxBits) * rs_tiles(n, kRsRoundsMin);
  const uint64_t mid = passes > 1 ? (uint64_t)(passes > 2 ? 2 : 1) * 8 * std::max<uint64_t>(n, 1) : 0;
  return 4 * (2 * h + 256) + mid + 4 * scan_u32_scratch(h) + 1024;
}

// Stable sort of n u32 keys (`bits` significant bits; inv: by ~key, i.e. descending) ->
// sorted keys (complemented when inv) and the source index of each output position.
// check_keys > 0: keys >= check_keys set *bad.
template <int R>
static hipError_t lsd_sort_r(const uint32_t* key, uint64_t n, int bits, bool inv, uint64_t check_keys,
                             uint32_t* sorted_keys, uint32_t* perm, void* scratch, size_t scratch_bytes, unsigned* bad,
                             hipStream_t st) {
  if (!n) return hipSuccess;
  const int passes = (bits + kRsMaxBits - 1) / kRsMaxBits;
  const int width = (bits + passes - 1) / passes;
  const uint64_t T = rs_tiles(n, R);
  if (lsd_scratch_bytes(n, bits) > scratch_bytes) return hipErrorInvalidValue;
  uint32_t* hist = (uint32_t*)scratch;
  uint32_t* hoff = hist + ((uint64_t)1 << width) * T;
  // (the ping-pong pairs sit past the smaller tile's histograms: the same place for either tile)
  uint32_t* mid = (uint32_t*)((char*)scratch + 4 * (2 * (uint64_t)(1u << kRsMaxBits) * rs_tiles(n, kRsRoundsMin) + 256));
  uint32_t *mk[2] = {mid, mid + 2 * n}, *mv[2] = {mid + n, mid + 3 * n};
  const uint64_t mid_words = passes > 1 ? (uint64_t)(passes > 2 ? 2 : 1) * 2 * std::max<uint64_t>(n, 1) : 0;
  uint32_t* stmp = mid + mid_words;  // (lsd_scratch_bytes: the scan's scratch after the pairs)
  const uint32_t *ik = key, *iv = nullptr;
  const dim3 g((uint32_t)T), gh((uint32_t)((T + kRsHistTiles - 1) / kRsHistTiles)), b(kRsThreads);
  hipError_t e = hipSuccess;
  for (int p = 0; p < passes; p++) {
    const int shift = p * width, w = std::min(width, bits - shift);
    const bool last = p == passes - 1;
    uint32_t* ok = last ? sorted_keys : mk[p & 1];
    uint32_t* ov = last ? perm : mv[p & 1];
    const uint64_t nk = check_keys ? check_keys : ~0ull;
    if (p > 0) hipLaunchKernelGGL((rs_hist<false, false, R>), gh, b, 0, st, ik, n, nk, shift, w, hist, T, bad);
    else if (inv) hipLaunchKernelGGL((rs_hist<true, true, R>), gh, b, 0, st, ik, n, nk, shift, w, hist, T, bad);
    else hipLaunchKernelGGL((rs_hist<true, false, R>), gh, b, 0, st, ik, n, nk, shift, w, hist, T, bad);
    if ((e = scan_u32(hist, hoff, ((uint64_t)1 << w) * T, stmp, st)) != hipSuccess) return e;
    if (p > 0) hipLaunchKernelGGL((rs_scatter<false, false, R>), g, b, 0, st, ik, iv, n, shift, w, hoff, T, ok, ov);
    else if (inv) hipLaunchKernelGGL((rs_scatter<true, true, R>), g, b, 0, st, ik, iv, n, shift, w, hoff, T, ok, ov);
    else hipLaunchKernelGGL((rs_scatter<true, false, R>), g, b, 0, st, ik, iv, n, shift, w, hoff, T, ok, ov);
    ik = ok;
    iv = ov;
  }
  return hipGetLastError();
}

static hipError_t lsd_sort(const uint32_t* key, uint64_t n, int bits, bool inv, uint64_t check_keys,
                           uint32_t* sorted_keys, uint32_t* perm, void* scratch, size_t scratch_bytes, unsigned* bad,
                           hipStream_t st, int rounds = kRsRounds) {
  if (rounds == 8) return lsd_sort_r<8>(key, n, bits, inv, check_keys, sorted_keys, perm, scratch, scratch_bytes, bad, st);
  if (rounds == 12)
    return lsd_sort_r<12>(key, n, bits, inv, check_keys, sorted_keys, perm, scratch, scratch_bytes, bad, st);
  if (rounds == 24)
    return lsd_sort_r<24>(key, n, bits, inv, check_keys, sorted_keys, perm, scratch, scratch_bytes, bad, st);
  if (rounds == 16)
    return lsd_sort_r<16>(key, n, bits, inv, check_keys, sorted_keys, perm, scratch, scratch_bytes, bad, st);
  return lsd_sort_r<kRsRounds>(key, n, bits, inv, check_keys, sorted_keys, perm, scratch, scratch_bytes, bad, st);
}

// Device scratch of partition(): bytes needed for n events over n_keys keys.
size_t partition_scratch_bytes(uint64_t n, uint64_t n_keys) { return lsd_scratch_bytes(n, key_bits(n_keys)); }

// arrival-order batch -> key_off[n_keys + 1], perm[n] (arrival index of each CSR position),
// columns in CSR order.  scratch: partition_scratch_bytes; sorted_keys: n u32.
hipError_t partition(const uint32_t* key, uint64_t n, uint64_t n_keys, int nf, Cols in, Cols out, uint32_t wide_mask,
                     const int64_t* ts_in, int64_t* ts_out, uint64_t* key_off, uint64_t* cnt, uint32_t* perm,
                     uint32_t* sorted_keys, uint32_t* idx, void* scratch, size_t scratch_bytes, unsigned* bad,
                     hipStream_t st, int rounds) {
  (void)cnt;
  (void)idx;
  hipError_t e =
      lsd_sort(key, n, key_bits(n_keys), false, n_keys, sorted_keys, perm, scratch, scratch_bytes, bad, st, rounds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(key_offsets, dim3((uint32_t)((n_keys + 256) / 256)), dim3(256), 0, st, sorted_keys, n, n_keys,
                     key_off);
  if (n)
    hipLaunchKernelGGL(gather_cols_tr, dim3((uint32_t)((n_keys + kTrKeys - 1) / kTrKeys)), dim3(256), 0, st, perm, key_off,
                       n_keys, nf, in, out, wide_mask, ts_in, ts_out);
  return hipGetLastError();
}

// keys by estimated work, longest first (the NFA's lane order, session.cpp): a stable LSD sort
// by ~est, so equal estimates keep key order
// A work estimate as a 16-bit sort key, monotone in est: exact below 2048, else the exponent and the
// 11 bits below the leading one (relative step 2^-11).  The lane order only groups like work into
// waves; two radix passes instead of four (a streamed batch of 1M keys: ~0.15 ms less).
__global__ void __launch_bounds__(256) est_key16(const uint32_t* __restrict__ est, uint32_t* __restrict__ q, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t x = est[i];
  if (x < 2048u) {
    q[i] = x;
  } else {
    const uint32_t e = 31u - (uint32_t)__builtin_clz(x);  // 11..31
    q[i] = ((e - 10u) << 11) | ((x >> (e - 11u)) & 0x7FFu);
  }
}

// the scratch sort_keys_by_work needs for n keys, (re)allocated if `tmp` is smaller (the
// caller does this before its timed interval)
hipError_t sort_keys_scratch(uint64_t n, void*& tmp, size_t& tmp_bytes) {
  const size_t need = lsd_scratch_bytes(n, 16);
  if (need > tmp_bytes) {
    if (tmp) (void)hipFree(tmp);
    tmp = nullptr;
    tmp_bytes = 0;
    hipError_t e = hipMalloc(&tmp, need);
    if (e != hipSuccess) return e;
    tmp_bytes = need;
  }
  return hipSuccess;
}

hipError_t sort_keys_by_work(const uint32_t* est, uint32_t* est_sorted, uint32_t* key16, uint32_t* order,
                             uint64_t n, void*& tmp, size_t& tmp_bytes, hipStream_t st) {
  const hipError_t e = sort_keys_scratch(n, tmp, tmp_bytes);
  if (e != hipSuccess) return e;
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(est_key16, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, est, key16, n);
  return lsd_sort(key16, n, 16, true, 0, est_sorted, order, tmp, tmp_bytes, nullptr, st);
}

}  // namespace cep
