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
// Layout.  A tile is 4 waves x 4096 consecutive events.  A wave streams its events with 16-B
// loads (lane l holds events 4l..4l+3 of a 256-event step), evaluates the m stage predicates
// straight into scalar ballot words and ANDs them shifted (match bit i = Π_x P_{m-1-x}(i-x));
// the windows reaching back before the wave and those crossing a key start are settled after
// the loop on natural 64-event words (key starts from key_off around the wave's first key,
// wave_keys), and a match's key is its word's first key advanced over the key starts.
//
// Passes.  (1) stencil_mask streams the column once and writes one 64-bit match word per 64
// events (1 bit/event), the word's key and sequence number, and adds each wave's match count to
// its stencil_emit block's counter; (2) stencil_emit sums the counters of the blocks before its
// own, reads the words back (1/32 of the column's bytes) and writes the matches in order.  No
// tile waits on another.  (A single pass
// with a decoupled look-back over the tile counts was measured slower: 126.7 us against 112.6
// for the two passes at round 5's start, profiles/r05/ - a tile waits for every tile before
// it, ~24 look-back round trips deep within one round of co-resident tiles.)
#include <hip/hip_runtime.h>

#include <type_traits>

#include "cep_layout.h"
#include "dewey.h"
#include "interp.h"
#include "java.h"
#include "stencil_args.h"

namespace cep {

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int kStThreads = 256;
constexpr int kStPer = 64;  // events per thread (one 64-bit mask)
constexpr uint64_t kStTile = (uint64_t)kStThreads * kStPer;

// ---------------------------------------------------------------- per-batch key index
constexpr int kStWave = kStTile / (kStThreads / 64);  // 4096 events per wave of stencil_mask
constexpr int kWkInline = 16;  // wave starts a thread writes itself; longer keys: the block

// wave_key[w] = the key holding event w * kStWave (wave starts inside key k: ceil(s/W) ..
// ceil(e/W) - 1; empty keys hold none).  A thread per key; a key spanning more than kWkInline
// wave starts is written by its whole block (a single key of the whole stream stays parallel).
// (It also zeroes the batch's counters, `zero[0..n_zero)`, which the mask pass accumulates
// into after it: one launch fewer per batch than a separate memset.)
__global__ void __launch_bounds__(256) wave_keys(const uint64_t* key_off, uint64_t n_keys, uint64_t n_waves,
                                                 uint32_t* wave_key, uint32_t* zero, uint32_t n_zero) {
  __shared__ uint32_t s_big[256];
  __shared__ uint32_t s_nbig;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n_zero; i += (uint64_t)gridDim.x * 256) zero[i] = 0;
  if (threadIdx.x == 0) s_nbig = 0;
  __syncthreads();
  const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (k < n_keys) {
    const uint64_t s = key_off[k], e = key_off[k + 1];
    const uint64_t w0 = (s + kStWave - 1) / kStWave;
    uint64_t w1 = (e + kStWave - 1) / kStWave;
    w1 = w1 < n_waves ? w1 : n_waves;
    if (w1 > w0 + kWkInline) {
      s_big[atomicAdd(&s_nbig, 1u)] = (uint32_t)k;
    } else {
      for (uint64_t w = w0; w < w1; w++) wave_key[w] = (uint32_t)k;
    }
  }
  __syncthreads();
  const uint32_t nbig = s_nbig;
  for (uint32_t i = 0; i < nbig; i++) {
    const uint32_t kk = s_big[i];
    const uint64_t w0 = (key_off[kk] + kStWave - 1) / kStWave;
    uint64_t w1 = (key_off[kk + 1] + kStWave - 1) / kStWave;
    w1 = w1 < n_waves ? w1 : n_waves;
    for (uint64_t w = w0 + threadIdx.x; w < w1; w += 256) wave_key[w] = kk;
  }
}

// ---------------------------------------------------------------- the stencil
__device__ __forceinline__ uint64_t mix64s(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ bool in_range(int64_t v, int64_t lo, int64_t hi) { return v >= lo && v <= hi; }

// bit m of a 16-bit value -> bit 4 m
__device__ __forceinline__ uint64_t spread4(uint32_t x16) {
  uint64_t x = x16;
  x = (x | (x << 24)) & 0x000000FF000000FFull;
  x = (x | (x << 12)) & 0x000F000F000F000Full;
  x = (x | (x << 6)) & 0x0303030303030303ull;
  x = (x | (x << 3)) & 0x1111111111111111ull;
  return x;
}

// Pass 1 layout.  A wave owns kStWave consecutive events and reads them with 16-B loads in
// which lane l holds events 4l..4l+3 of a 256-event step: every load instruction covers
// 1 KiB contiguous (fully coalesced).  Per step the M stage predicates go straight into scalar
// ballot words and the windows are ANDs of shifted words (stage s sits M-1-s events back).
constexpr int kStSteps = kStWave / 256;               // 16 load steps per wave

template <int M, bool RANGE, int NCOL>
struct StEval {
  int32_t lo[M][2], hi[M][2];
  uint32_t span[M][2];
  bool never = false;  // an empty range: no stage-s event, no match (the slow path handles it)
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
          // lo <= x <= hi  <=>  (uint)(x - lo) <= (uint)(hi - lo): one subtract and one
          // compare, both vector ops (no scalar AND of two compare masks)
          span[s][c] = (uint32_t)hi[s][c] - (uint32_t)lo[s][c];
          if (c < NCOL && lo[s][c] > hi[s][c]) never = true;
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
  // stage s over the 4 events of a step: W[k] = ballot word of event 4 l + k.  Every
  // operation is a vector op whose result lands in scalar registers (the compare mask)
  __device__ __forceinline__ bool in1(int s, int c, int32_t v) const {
    return (uint32_t)v - (uint32_t)lo[s][c] <= span[s][c];
  }
  __device__ __forceinline__ void ballot4(int s, const v4i x, const v4i y, uint64_t* W) const {
    if (NCOL == 1) {
      W[0] = __builtin_amdgcn_ballot_w64(in1(s, 0, x.x));
      W[1] = __builtin_amdgcn_ballot_w64(in1(s, 0, x.y));
      W[2] = __builtin_amdgcn_ballot_w64(in1(s, 0, x.z));
      W[3] = __builtin_amdgcn_ballot_w64(in1(s, 0, x.w));
    } else {
      W[0] = __builtin_amdgcn_ballot_w64(in1(s, 0, x.x)) & __builtin_amdgcn_ballot_w64(in1(s, 1, y.x));
      W[1] = __builtin_amdgcn_ballot_w64(in1(s, 0, x.y)) & __builtin_amdgcn_ballot_w64(in1(s, 1, y.y));
      W[2] = __builtin_amdgcn_ballot_w64(in1(s, 0, x.z)) & __builtin_amdgcn_ballot_w64(in1(s, 1, y.z));
      W[3] = __builtin_amdgcn_ballot_w64(in1(s, 0, x.w)) & __builtin_amdgcn_ballot_w64(in1(s, 1, y.w));
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

// What the mask phase leaves a wave (kStWave events from wbase), per lane, for its natural
// 64-event word (events ws .. ws + 63, ws = wbase + 64 lane):
struct WaveMask {
  uint64_t nat;   // bit i: a match (a window of M events of one key) ends at event ws + i
  uint64_t bw;    // bit i: a key starts at event ws + i
  uint32_t wkey;  // the key holding event ws (the largest key whose offset is <= ws)
  uint64_t wks;   // that key's first event
};

// The mask phase of one wave.  The steps' loads are double-buffered (one step in flight while
// the other computes) and the step loop carries nothing but the stage words of the previous
// step: the windows that reach back before the wave (the first M-1 ending in it) and the
// windows crossing a key start are settled after the loop, on the natural words, with vector
// work.  (This keeps the loop's scalar registers down - 58 instead of 106, 8 waves per SIMD
// instead of 6 - and the pass at ~75 us for 1e8 events instead of ~90: profiles/r05/.)
template <int M, bool RANGE, int NCOL>
__device__ __forceinline__ void wave_mask(const StencilArgs& A, const uint64_t wbase, const int lane, WaveMask& out) {
  constexpr int H = M - 1;              // events a window reaches back
  const StEval<M, RANGE, NCOL> ev(A);
  const bool fast = RANGE && A.aligned && wbase + kStWave <= A.n_events && !ev.never;
  // The fast path's first step is requested before anything else: the key-start words and
  // the seed events below are dependent round trips
  const v4i* c0 = reinterpret_cast<const v4i*>(A.col[0] + wbase) + lane;
  const v4i* c1 = reinterpret_cast<const v4i*>(A.col[NCOL - 1] + wbase) + lane;
  v4i xa = {0, 0, 0, 0}, ya = {0, 0, 0, 0};
  if (fast) {
    xa = __builtin_nontemporal_load(c0);
    ya = NCOL > 1 ? __builtin_nontemporal_load(c1) : xa;
  }
  // the key holding the wave's first event (wave_keys)
  const uint64_t n_waves = (A.n_events + kStWave - 1) / kStWave;  // n_events >= 1: the tile exists
  const uint64_t wi = wbase / kStWave;
  const uint32_t k0 = A.wave_key[wi < n_waves ? wi : n_waves - 1];
  // the seed events wbase - H .. wbase + H - 1 (lane j < 2H: event wbase - H + j): the windows
  // ending at the wave's first H events, settled after the loop
  const int64_t sp = (int64_t)wbase - H + lane;
  const bool sv = H > 0 && lane < 2 * H && sp >= 0 && (uint64_t)sp < A.n_events;
  int32_t sx0 = 0, sx1 = 0;
  if (RANGE && sv) {
    sx0 = A.col[0][sp];
    sx1 = A.col[NCOL - 1][sp];
  }
  // Key starts in [wbase - 8, wend): lanes read key_off[k0 - 8 + 64 c + lane] (the 8 keys
  // before k0 may start among the 8 events before the wave) and a wave-uniform loop visits
  // the starts in range, in key order.  bw: this lane's start bits, pkb: starts among the 8
  // events before the wave (bit x: event wbase - 8 + x), wkey: the key holding event ws (for
  // stencil_emit: the largest key whose offset is <= it; empty keys share their successor's
  // offset and lose to it).
  const uint64_t wend = wbase + kStWave < A.n_events ? wbase + kStWave : A.n_events;
  const uint64_t lo = wbase >= 8 ? wbase - 8 : 0;
  const uint64_t ws = wbase + (uint64_t)lane * 64;
  uint64_t bw = 0;
  uint32_t pkb = 0, wkey = k0;
  uint64_t wks = 0;  // wkey's first event (stencil_emit: sequence numbers without key_off)
  if (wbase < A.n_events) {
    for (int64_t i0 = (int64_t)k0 - 8;; i0 += 64) {
      const int64_t i = i0 + lane;
      const bool valid = i >= 0 && (uint64_t)i < A.n_keys;
      const uint64_t sj = valid ? A.key_off[i] : 0;
      if (i0 == (int64_t)k0 - 8)  // (lane 8 of the first chunk read k0's offset)
        wks = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(sj >> 32), 8) << 32) |
              (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)sj, 8);
      uint64_t inr = __ballot(valid && sj >= lo && sj < wend);
      while (inr) {
        const int j = __builtin_ctzll(inr);
        inr &= inr - 1;
        const uint64_t sjj = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(sj >> 32), j) << 32) |
                             (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)sj, j);
        if (sjj >= wbase) {
          if (((sjj - wbase) >> 6) == (uint64_t)lane) bw |= 1ull << (sjj & 63);
        } else {
          pkb |= 1u << (uint32_t)(sjj - (wbase - 8));
        }
        if (sjj <= ws) {
          wkey = (uint32_t)(i0 + j);
          wks = sjj;
        }
      }
      const uint64_t s63 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(sj >> 32), 63) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)sj, 63);
      if (!(i0 + 64 < (int64_t)A.n_keys && s63 < wend)) break;  // no key after this chunk starts in range
    }
  }
  // Ballot words of the previous step (bit l of W[s][k] = stage s holds at event 4l + k),
  // zero before the wave's first step: windows reaching back before the wave are settled
  // below from the seed events
  uint64_t pW[M][4];
#pragma unroll
  for (int s = 0; s < M; s++)
#pragma unroll
    for (int k = 0; k < 4; k++) pW[s][k] = 0;
  uint64_t myword = 0;  // ballot layout: word k of step q for lane 4q + k
  // step q of the wave: x/y hold its 4 events per lane on the fast path (FAST: a
  // std::integral_constant, so each loop below gets its own straight-line body)
  auto step = [&](const int q, const v4i x, const v4i y, auto fast_c) {
    constexpr bool FAST = decltype(fast_c)::value;
    const uint64_t e0 = wbase + (uint64_t)q * 256 + (uint64_t)lane * 4;
    // stage words of this step (wave-uniform, scalar registers)
    uint64_t W[M][4];
    if (FAST) {
#pragma unroll
      for (int s = 0; s < M; s++) ev.ballot4(s, x, y, W[s]);
    } else {
      uint32_t P[M];
#pragma unroll
      for (int s = 0; s < M; s++) P[s] = 0;
      if (RANGE && A.aligned && e0 + 4 <= A.n_events) {
        const v4i xs = __builtin_nontemporal_load(reinterpret_cast<const v4i*>(A.col[0] + e0));
        v4i ys = xs;
        if (NCOL > 1) ys = __builtin_nontemporal_load(reinterpret_cast<const v4i*>(A.col[1] + e0));
        ev.range(xs.x, ys.x, P, 0);
        ev.range(xs.y, ys.y, P, 1);
        ev.range(xs.z, ys.z, P, 2);
        ev.range(xs.w, ys.w, P, 3);
      } else if (e0 < A.n_events) {  // events past the end stay 0: no window can end there
#pragma unroll
        for (int i = 0; i < 4; i++) ev.one(A, e0 + i, P, i);
      }
#pragma unroll
      for (int s = 0; s < M; s++)
#pragma unroll
        for (int k = 0; k < 4; k++) W[s][k] = __builtin_amdgcn_ballot_w64((P[s] >> k) & 1u);
    }
    // word k: windows ending at events 4l + k.  Stage s sits o = M-1-s events back: event
    // 4l + k - o is word (k - o) mod 4, `cr` lanes back (bits shifted up, the previous
    // step's top bits carried in).
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
    // lane 4q + k keeps word k (vector compare + select: no scalar work)
    const int lrel = lane - 4 * q;
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (lrel == k) myword = m[k];
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int s = 0; s < M; s++) pW[s][k] = W[s][k];
  };
  if (fast) {
    // two one-step buffers: while one step computes, the other's load is in flight.  The
    // loads are unconditional (the last pair re-reads its own step): a load under a branch
    // makes the waitcnt pass drain every outstanding load before the first use.
    v4i xb, yb;
#pragma unroll 1
    for (int q = 0; q < kStSteps; q += 2) {
      xb = __builtin_nontemporal_load(c0 + (q + 1) * 64);
      yb = NCOL > 1 ? __builtin_nontemporal_load(c1 + (q + 1) * 64) : xb;
      step(q, xa, ya, std::true_type{});
      const int qn = q + 2 < kStSteps ? q + 2 : q;
      xa = __builtin_nontemporal_load(c0 + qn * 64);
      ya = NCOL > 1 ? __builtin_nontemporal_load(c1 + qn * 64) : xa;
      step(q + 1, xb, yb, std::true_type{});
    }
  } else {
    const v4i z = {0, 0, 0, 0};
    for (int q = 0; q < kStSteps; q++) step(q, z, z, std::false_type{});
  }
  // natural words: events wbase + 256 q + 64 r + i (q = lane / 4, r = lane % 4) are bits
  // 16 r .. 16 r + 15 of the ballot words of step q, held by lanes 4q .. 4q + 3
  uint64_t nat = 0;
  {
    const int q4 = lane & ~3, r16 = 16 * (lane & 3);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint64_t wk = __shfl(myword, q4 + k, 64);
      nat |= spread4((uint32_t)(wk >> r16) & 0xFFFFu) << k;
    }
  }
  if (H > 0) {
    // the windows ending at events wbase + i, i < H (they reach back before the wave): stage
    // bits of the seed events, bit j of S[s] = stage s holds at event wbase - H + j; the window
    // ending at wbase + i holds iff bit i + s of S[s] is set for every s
    uint32_t P[M];
#pragma unroll
    for (int s = 0; s < M; s++) P[s] = 0;
    if (sv) {
      if constexpr (RANGE) ev.range(sx0, sx1, P, 0);
      else ev.one(A, (uint64_t)sp, P, 0);
    }
    uint64_t seed = wbase >= (uint64_t)H ? (1ull << H) - 1ull : 0ull;
#pragma unroll
    for (int s = 0; s < M; s++) seed &= __ballot(P[s] & 1u) >> s;
    if (lane == 0) nat |= seed;
    // a key start at any of a window's last M-1 events (offsets 0 .. M-2) kills it: the start
    // bits spread over the H events after them, carried across words (lane 0: the starts among
    // the 8 events before the wave)
    // (the shuffle outside the select: a permute reading an inactive lane returns 0)
    const uint64_t up = __shfl_up(bw, 1, 64);
    const uint64_t pw = lane == 0 ? (uint64_t)pkb << 56 : up;
    uint64_t kill = bw;
#pragma unroll
    for (int o = 1; o < H; o++) kill |= (bw << o) | (pw >> (64 - o));
    nat &= ~kill;
  }
  if (ws >= A.n_events) nat = 0;  // (the seed bits of a wave past the end)
  out.nat = nat;
  out.bw = bw;
  out.wkey = wkey;
  out.wks = wks;
}

// stencil_emit's block: kEmW mask tiles; the mask pass counts matches per emit block
constexpr int kEmW = 4;
constexpr uint64_t kStGroupChunks = kEmW * (kStTile / kStWave);  // chunks per group count: an emit block's

// Pass 1: per 4096-event chunk (a wave) the mask phase, its natural words, their keys and
// sequence numbers, and the match count per kStGroupChunks chunks (one stencil_emit block's
// span: its offset is the sum of the counts before it).  Each wave adds its own count: no
// block-wide barrier ties four waves together, and a counter takes 16 waves' atomics (probe,
// profiles/r05/: for 1e8 events the mask phase alone 65.4 us, with the three word stores 76.6,
// with a block-wide tile count and an atomic per 64 tiles 84.4; an atomic per wave into
// counters of 256 waves 156).  (A launch of resident waves looping over the chunks, so a
// chunk's stores overlap the next chunk's loads, measured 142 us: the loop's scalar state spills.)

template <int M, bool RANGE, int NCOL>
__global__ void __launch_bounds__(kStThreads) stencil_mask(StencilArgs A) {
  // wv through readfirstlane: the compiler cannot see that threadIdx.x >> 6 is wave-uniform,
  // and everything derived from it (the fast-path branch, the ballot words) would go to VGPRs
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t chunk = (uint64_t)blockIdx.x * (kStThreads / 64) + wv;
  if (chunk >= A.n_chunk) return;  // (wave-uniform; no barrier below)
  const uint64_t wbase = chunk * kStWave;
  WaveMask o;
  wave_mask<M, RANGE, NCOL>(A, wbase, lane, o);
  const uint64_t ws = wbase + (uint64_t)lane * 64;
  // (bit 31: a key starts inside the word after its first event - stencil_emit walks key_off
  // there; elsewhere a match's sequence number is word_seq + its offset in the word)
  if (ws < A.n_events)  // one 16-B store per word (three separate word arrays cost 2-3 us more)
    A.words[ws / 64] = uint4{(uint32_t)o.nat, (uint32_t)(o.nat >> 32), o.wkey | ((o.bw & ~1ull) ? 0x80000000u : 0u),
                             (uint32_t)(ws - o.wks)};
  // matches of the chunk: popcount of each lane's word, summed over the wave
  uint32_t cnt = (uint32_t)__popcll(o.nat);
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) cnt += __shfl_xor(cnt, d, 64);
  if (lane == 0 && cnt) atomicAdd(A.group_cnt + chunk / kStGroupChunks, cnt);  // (no return value)
}

// Pass 2: a thread per kEmW consecutive 64-event words (a block: kEmW mask tiles), the block's
// offset from the group and tile counts, a block scan for the threads' offsets.  A match's key
// is its word's first key advanced over the key offsets it passes.  (One word per
// thread ran 6104 blocks for 1e8 events, three rounds of resident blocks each paying a load
// and a store round trip: ~18 us; kEmW words per thread issue their loads together and the
// grid fits the chip in one round.)
constexpr uint32_t kEmStage = 3072;  // matches staged in LDS (24 KB: 6 blocks per CU)

template <int M>
__global__ void __launch_bounds__(kStThreads) stencil_emit(StencilArgs A) {
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

// ---------------------------------------------------------------- host launchers
hipError_t launch_wave_keys(const uint64_t* key_off, uint64_t n_keys, uint64_t n_events, uint32_t* wave_key,
                            uint32_t* zero, uint32_t n_zero, hipStream_t st) {
  const uint64_t n_waves = (n_events + kStWave - 1) / kStWave;
  if (n_keys == 0 || n_waves == 0) return hipMemsetAsync(zero, 0, 4ull * n_zero, st);
  hipLaunchKernelGGL(wave_keys, dim3((uint32_t)((n_keys + 255) / 256)), dim3(256), 0, st, key_off, n_keys, n_waves,
                     wave_key, zero, n_zero);
  return hipGetLastError();
}

uint64_t stencil_waves(uint64_t n_events) { return (n_events + kStWave - 1) / kStWave; }

template <int M, bool RANGE, int NCOL>
static hipError_t launch_one(const StencilArgs& a, uint64_t n_tiles, hipStream_t st) {
  // (a separate build for the whole fast-path chunks, without the slow path's code and
  // registers, measured the same - 79.5 against 79.6 us for 1e8 events - and cost a launch)
  StencilArgs b = a;
  b.n_chunk = (a.n_events + kStWave - 1) / kStWave;
  hipLaunchKernelGGL((stencil_mask<M, RANGE, NCOL>), dim3((uint32_t)((b.n_chunk + 3) / 4)), dim3(kStThreads), 0, st, b);
  hipLaunchKernelGGL(stencil_emit<M>, dim3((uint32_t)((n_tiles + kEmW - 1) / kEmW)), dim3(kStThreads), 0, st, a);
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
