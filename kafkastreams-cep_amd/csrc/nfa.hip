// nfa.hip — the general NFA matching kernel (CEP_KIND_NFA) and its output compaction.
//
// One lane = one key = one reference NFA (nfa/NFA.java).  A 64-lane wavefront advances 64
// keys in lockstep over their CSR event columns; each lane runs the reference's per-event
// algorithm exactly (queue order, edge order, Dewey versions, buffer refcounts and
// predecessor removal, fold timing), which is what makes the emitted match sets bit-exact.
//
//   per event j of key k                                   reference
//   ------------------------------------------------------ -----------------------------------
//   pop the |Q| runs present at event start, step each     NFA.matchPattern          :94-109
//   step = evaluate(level 0) + begin re-add                NFA.matchPattern(ctx)    :139-160
//   evaluate: edges, PROCEED chain (iterative), branch,    NFA.evaluate             :162-250
//             folds on unwind
//   dead run -> walk_remove (GC only)                      NFA.removePattern        :117-123
//   finals -> walk_remove emitting the Sequence            NFA.matchConstruction    :111-115
//   put / put(begin) / branch / peek(remove)               KVSharedVersionedBuffer :80-171
//
// State lives in HBM: the run FIFO is a per-key ring of Rec, buffer nodes and predecessor
// pointers come from global pools (chunked per lane), matches stream into per-key chained
// output chunks that the compaction kernels turn into flat, key-ordered arrays.
#include <hip/hip_runtime.h>

#include "cep_layout.h"
#include "dewey.h"
#include "interp.h"
#include "java.h"
#include "nfa_lane.h"

namespace cep {

// Bytecode-interpreter policy (AOT tier): walks the DevQuery stage table and evaluates the
// predicate/aggregate programs with interp().  NFA.evaluate's recursion over PROCEED edges
// (nfa/NFA.java:162-250) is unrolled into a level stack: edges in order on the way down,
// branch records and folds on the way back up (the recursion's return order).
template <int F>
struct InterpQ {
  const DevQuery& q;
  const uint32_t* code;
  const NfaArgs& A;
  bool quiet;
  uint32_t begin_stage;
  static constexpr bool kBeginReg = false;  // quiet is only known at run time here
  static constexpr bool kFold32 = false;     // fold slots hold any state type
  static constexpr uint32_t kRingLds = 0;    // LDS holds the DevQuery and bytecode: queues in HBM
  struct EvT {};                             // the programs read the columns themselves

  __device__ InterpQ(const DevQuery& qq, const uint32_t* c, const NfaArgs& a) : q(qq), code(c), A(a) {
    begin_stage = q.begin_stage;
    const DevStage& b = q.st[begin_stage];
    quiet = b.n_edges == 1 && b.e[0].op == OP_BEGIN;
  }
  __device__ __forceinline__ uint32_t stage_sk(uint32_t sw) const {
    return (sw & kRecEps) ? ((sw >> 8) & 0xFF) : q.st[sw & 0xFF].sk;
  }
  __device__ __forceinline__ uint16_t sk_name(uint32_t sk) const { return q.sk_name[sk]; }
  __device__ __forceinline__ void set_query(uint32_t) {}  // one query per interpreter launch

  template <class LaneT>
  __device__ bool begin_pred(LaneT& lane) {
    const DevEdge E = q.st[begin_stage].e[0];
    if (E.prog == kProgTrue) return true;
    int64_t W[F];
    EvalIn in{&A.cols, q.field_type, A.ts, lane.base + lane.j, W, (1u << F) - 1, 0, true};
    bool rn;
    int ee = 0;
    const int64_t r = interp(code, E.prog, in, &rn, &ee);
    if (ee) lane.err = ee;
    return r != 0;
  }

  __device__ __forceinline__ void load_ev(EvT&, uint64_t) const {}

  template <class LaneT>
  __device__ uint32_t begin_scan(LaneT& lane, uint32_t j0, uint32_t lim) {
    for (uint32_t p = j0; p < lim; p++) {
      lane.j = p;
      const bool hit = begin_pred(lane);
      if (lane.err || hit) return p;
    }
    return lim;
  }

  // NFA.matchPattern(ctx) :139-160.  Returns the number of records produced; -1 on error.
  template <class LaneT>
  __device__ int step(LaneT& lane, const Rec<F>& c) {
    int64_t W[F];
#pragma unroll
    for (int s = 0; s < F; s++) W[s] = c.fold[s];
    uint32_t wnull = c.nullmask;
    const uint32_t top = c.stage;
    const bool top_eps = top & kRecEps;
    const uint32_t top_sk = stage_sk(top);
    const uint32_t j = lane.j;
    int produced = 0;
    int same_seq = -1;  // slot of the (single) output record that keeps this run's sequence id

    uint8_t lv_cur[kMaxStages + 1];
    uint8_t lv_prev[kMaxStages + 1];
    uint8_t lv_zeros[kMaxStages + 1];
    uint8_t lv_flags[kMaxStages + 1];  // 1 branching ctx, 2 br, 4 consumed, 8 ignored
    int L = 0;
    lv_cur[0] = (uint8_t)(top & 0xFF);
    lv_prev[0] = kNoSk;
    lv_zeros[0] = 0;
    lv_flags[0] = (top & kRecBranch) ? 1 : 0;

    EvalIn in{&A.cols, q.field_type, A.ts, lane.base + j, W, wnull, 0, true};

    for (;;) {
      const bool eps = (L == 0) && top_eps;
      const uint32_t cur = lv_cur[L];
      const uint32_t cur_sk = eps ? top_sk : q.st[cur].sk;
      Dewey ver = c.ver;
      for (int z = 0; z < lv_zeros[L]; z++)
        if (!dw_add_stage(ver)) { lane.err = KE_CAPACITY; return -1; }
      uint32_t proceed_target = CEP_NONE;
      if (eps) {
        proceed_target = cur;  // epsilon: single PROCEED(true) -> target (Stage.java:42-46)
      } else {
        const DevStage& S = q.st[cur];
        uint32_t matched = 0;
        for (int e = 0; e < S.n_edges; e++) {  // matchEdgesAndGet :267-273 (all edges first)
          bool hit = true;
          if (S.e[e].prog != kProgTrue) {
            bool rn;
            int ee = 0;
            const int64_t r = interp(code, S.e[e].prog, in, &rn, &ee);
            if (ee) { lane.err = ee; return -1; }
            hit = r != 0;
          }
          if (hit) matched |= 1u << e;
        }
        uint32_t ops = 0;
        for (int e = 0; e < S.n_edges; e++)
          if (matched & (1u << e)) ops |= 1u << S.e[e].op;
        const bool hasP = ops & (1u << OP_PROCEED), hasT = ops & (1u << OP_TAKE);
        const bool hasI = ops & (1u << OP_IGNORE), hasB = ops & (1u << OP_BEGIN);
        const bool br = (hasP && hasT) || (hasI && hasT) || (hasI && hasB) || (hasI && hasP);  // :280-289
        if (br) lv_flags[L] |= 2;
        for (int e = 0; e < S.n_edges; e++) {
          if (!(matched & (1u << e))) continue;
          const DevEdge E = S.e[e];
          if (E.op == OP_PROCEED) {
            proceed_target = E.target;
          } else if (E.op == OP_TAKE) {
            if (!br) {  // newEpsilonState(current, current), same run
              const int r = lane.push_rec(kRecEps | (cur_sk << 8) | cur, j, CEP_NONE, ver);
              if (r < 0) return -1;
              same_seq = r;
              produced++;
              lane.put_link(cur_sk, lv_prev[L], c.event, c.ev_first, ver);
            } else {
              Dewey v2 = ver;
              if (!dw_add_run(v2)) { lane.err = KE_CAPACITY; return -1; }
              lane.put_link(cur_sk, lv_prev[L], c.event, c.ev_first, v2);
            }
            if (lane.err) return -1;
            lv_flags[L] |= 4;
          } else if (E.op == OP_BEGIN) {
            lane.put_link(cur_sk, lv_prev[L], c.event, c.ev_first, ver);
            if (lane.err) return -1;
            uint32_t sw = kRecEps | (cur_sk << 8) | E.target;
            if (q.st[E.target].type == ST_FINAL) sw |= kRecFinal;
            const int r = lane.push_rec(sw, j, CEP_NONE, ver);
            if (r < 0) return -1;
            same_seq = r;
            produced++;
            lv_flags[L] |= 4;
          } else {  // IGNORE: re-add the context record (top stage/event, this level's version)
            if (!br) {
              const int r = lane.push_rec((top & ~(kRecBranch | kRecFinal)) | ((lv_flags[L] & 1) ? kRecBranch : 0),
                                          c.event, c.ev_first, ver);
              if (r < 0) return -1;
              same_seq = r;
              produced++;
            }
            lv_flags[L] |= 8;
          }
        }
      }
      if (proceed_target == CEP_NONE) break;
      // PROCEED: addStage unless the target is the same stage key or the run is branching
      const uint32_t tsk = q.st[proceed_target].sk;
      const bool branching = lv_flags[L] & 1;
      const bool add = (tsk != cur_sk) && !branching;
      if (L + 1 > kMaxStages) { lane.err = KE_CAPACITY; return -1; }
      lv_cur[L + 1] = (uint8_t)proceed_target;
      lv_prev[L + 1] = (uint8_t)cur_sk;
      lv_zeros[L + 1] = lv_zeros[L] + (add ? 1 : 0);
      lv_flags[L + 1] = (add ? 0 : (branching ? 1 : 0));
      L++;
    }

    // unwind: branch records and folds, deepest level first (recursion return order)
    for (int l = L; l >= 0; l--) {
      const uint8_t fl = lv_flags[l];
      if (!(fl & 6)) continue;
      const uint32_t cur = lv_cur[l];  // a real stage: epsilons never branch or consume
      const DevStage& S = q.st[cur];
      Dewey ver = c.ver;
      for (int z = 0; z < lv_zeros[l]; z++) dw_add_stage(ver);
      if (fl & 2) {  // isBranching :231-246
        if (lv_prev[l] == kNoSk) { lane.err = KE_NPE; return -1; }  // newEpsilonState(null, ...)
        Dewey v2 = ver;
        if (!dw_add_run(v2)) { lane.err = KE_CAPACITY; return -1; }
        const int r = (fl & 8) ? lane.push_rec(kRecEps | kRecBranch | ((uint32_t)lv_prev[l] << 8) | cur, c.event,
                                             c.ev_first, v2)
                             : lane.push_rec(kRecEps | kRecBranch | ((uint32_t)lv_prev[l] << 8) | cur, j,
                                             CEP_NONE, v2);
        if (r < 0) return -1;
        uint32_t nm = (1u << F) - 1;  // fresh sequence: only this stage's aggregates are copied
        int64_t fv[F];
#pragma unroll
        for (int s = 0; s < F; s++) fv[s] = 0;
        for (int a = 0; a < S.n_aggs; a++) {
          const uint32_t s = S.agg_state[a];
          if (!((wnull >> s) & 1u)) {
#pragma unroll
            for (int t = 0; t < F; t++)
              if ((uint32_t)t == s) fv[t] = W[t];
            nm &= ~(1u << s);
          }
        }
        lane.set_folds(r, fv, nm);
        produced++;
        lane.walk_branch(lv_prev[l], c.event, c.ev_first, ver);
        if (lane.err) return -1;
      }
      if (fl & 4) {  // evaluateAggregates :259-265, declaration order
        for (int a = 0; a < S.n_aggs; a++) {
          const uint32_t s = S.agg_state[a];
          in.curr = W[s];
          in.curr_null = (wnull >> s) & 1u;
          bool rn;
          int ee = 0;
          const int64_t v = interp(code, S.agg_prog[a], in, &rn, &ee);
          if (ee) { lane.err = ee; return -1; }
          W[s] = v;
          wnull = rn ? (wnull | (1u << s)) : (wnull & ~(1u << s));
        }
      }
    }
    if (same_seq >= 0) lane.set_folds(same_seq, W, wnull);
    // begin state re-added with a new run (:148-157)
    if (!top_eps && q.st[top & 0xFF].type == ST_BEGIN) {
      Dewey v = c.ver;
      if (produced > 0 && !dw_add_run(v)) { lane.err = KE_CAPACITY; return -1; }
      if (!lane.readd_begin(top & 0xFF, v)) return -1;
      produced++;
    }
    return produced;
  }
};

template <int F>
__global__ void __launch_bounds__(256) nfa_kernel(NfaArgs A) {
  extern __shared__ uint32_t smem[];
  DevQuery* qs = reinterpret_cast<DevQuery*>(smem);
  uint32_t* code_s = smem + (sizeof(DevQuery) + 3) / 4;
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(A.q);
    for (uint32_t i = threadIdx.x; i < sizeof(DevQuery) / 4; i += blockDim.x) smem[i] = src[i];
  }
  __syncthreads();
  const uint32_t code_len = qs->code_len;
  for (uint32_t i = threadIdx.x; i < code_len; i += blockDim.x) code_s[i] = A.code[i];
  __syncthreads();
  InterpQ<F> q(*qs, code_s, A);
  run_key<F>(A, q);
}

// ---------------------------------------------------------------- compaction
// exclusive scans of per-key match / pair counts (two-level: block sums, then offsets)
__global__ void __launch_bounds__(256) count_blocks(const KeyState* ks, uint64_t n, uint64_t* bsum_m,
                                                    uint64_t* bsum_p) {
  __shared__ uint64_t sm[256], sp[256];
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  sm[threadIdx.x] = i < n ? ks[i].n_matches : 0;
  sp[threadIdx.x] = i < n ? ks[i].n_pairs : 0;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      sm[threadIdx.x] += sm[threadIdx.x + s];
      sp[threadIdx.x] += sp[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    bsum_m[blockIdx.x] = sm[0];
    bsum_p[blockIdx.x] = sp[0];
  }
}

// single block: in-place exclusive scan of nb block sums (sequential chunks per thread)
__global__ void __launch_bounds__(1024) scan_blocks(uint64_t* bm, uint64_t* bp, uint64_t nb, uint64_t* totals) {
  __shared__ uint64_t tm[1024], tp[1024];
  const uint64_t per = (nb + 1023) / 1024;
  const uint64_t a = threadIdx.x * per, b = (a + per < nb) ? a + per : nb;
  uint64_t sm = 0, sp = 0;
  for (uint64_t i = a; i < b; i++) { sm += bm[i]; sp += bp[i]; }
  tm[threadIdx.x] = sm;
  tp[threadIdx.x] = sp;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t am = 0, ap = 0;
    for (int t = 0; t < 1024; t++) {
      uint64_t xm = tm[t], xp = tp[t];
      tm[t] = am;
      tp[t] = ap;
      am += xm;
      ap += xp;
    }
    totals[0] = am;
    totals[1] = ap;
  }
  __syncthreads();
  uint64_t om = tm[threadIdx.x], op = tp[threadIdx.x];
  for (uint64_t i = a; i < b; i++) {
    uint64_t xm = bm[i], xp = bp[i];
    bm[i] = om;
    bp[i] = op;
    om += xm;
    op += xp;
  }
}

// per key: walk the output chain and write flat arrays; digest = Σ hash(match)
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// a key whose output chain is long: scattered by a whole wave (scatter_heavy)
struct HeavyKey {
  uint32_t key, pad;
  uint64_t mo, po;  // its first match / pair index in the flat arrays
};
// (a key from 64 pairs on: config 3's matching keys hold ~25-50; the per-thread walk of them
// scattered its writes across lanes - 0.87 ms against 0.23 + 0.26 ms this way, cfg 3; from
// 16 pairs on and twice the waves 0.19 + 0.38)
constexpr uint32_t kHeavyPairs = 64;

__global__ void __launch_bounds__(256) scatter_matches(const KeyState* ks, uint64_t n, const uint64_t* bsum_m,
                                                       const uint64_t* bsum_p, const uint32_t* out,
                                                       uint32_t* m_key, uint32_t* m_emit, uint64_t* m_off,
                                                       uint32_t* p_seq, uint16_t* p_stage,
                                                       const uint64_t* totals, HeavyKey* heavy, uint32_t* n_heavy) {
  __shared__ uint64_t sm[256], sp[256];
  const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint32_t nm = k < n ? ks[k].n_matches : 0, npairs = k < n ? ks[k].n_pairs : 0;
  sm[threadIdx.x] = nm;
  sp[threadIdx.x] = npairs;
  __syncthreads();
  // block-local exclusive scan (Hillis-Steele over 256)
  for (int s = 1; s < 256; s <<= 1) {
    uint64_t xm = threadIdx.x >= (unsigned)s ? sm[threadIdx.x - s] : 0;
    uint64_t xp = threadIdx.x >= (unsigned)s ? sp[threadIdx.x - s] : 0;
    __syncthreads();
    sm[threadIdx.x] += xm;
    sp[threadIdx.x] += xp;
    __syncthreads();
  }
  uint64_t mo = bsum_m[blockIdx.x] + sm[threadIdx.x] - nm;
  uint64_t po = bsum_p[blockIdx.x] + sp[threadIdx.x] - npairs;
  if (k == 0) m_off[totals[0]] = totals[1];
  if (nm == 0) return;
  if (npairs >= kHeavyPairs) {  // a wave per heavy key, next launch
    heavy[atomicAdd(n_heavy, 1u)] = HeavyKey{(uint32_t)k, 0, mo, po};
    return;
  }
  // The key's chain is read 16 words (four 16-B loads issued together) at a time into this
  // thread's LDS window: one memory round trip per 16 words instead of one per word (a heavy
  // key's chain holds millions of words).  Chunks are 1 KiB aligned; word 255 links the next.
  __shared__ uint32_t win_s[256 * 16];
  uint32_t* win = win_s + threadIdx.x * 16;
  uint32_t chunk = ks[k].out_first, pos = 0, wi = 16;
  auto next = [&]() -> uint32_t {
    if (pos == kOutChunkWords - 1) {  // the link is the window's last word
      chunk = win[15];
      pos = 0;
      wi = 16;
    }
    if (wi == 16) {
      const uint4* src = reinterpret_cast<const uint4*>(out + (uint64_t)chunk * kOutChunkWords + pos);
      const uint4 a = src[0], b = src[1], c = src[2], d = src[3];
      uint4* dst = reinterpret_cast<uint4*>(win);
      dst[0] = a;
      dst[1] = b;
      dst[2] = c;
      dst[3] = d;
      wi = 0;
    }
    pos++;
    return win[wi++];
  };
  for (uint32_t m = 0; m < nm; m++) {
    const uint32_t emit = next();
    const uint32_t np = next();
    m_key[mo] = (uint32_t)k;
    m_emit[mo] = emit;
    m_off[mo] = po;
    for (uint32_t i = 0; i < np; i++) {
      const uint32_t s = next();
      const uint32_t st = next();
      p_seq[po] = s;
      p_stage[po] = (uint16_t)st;
      po++;
    }
    mo++;
  }
}

// jobs to re-run: KE_RETRY -> cap_list, KE_CONFLICT -> conf_list (any order: jobs are
// independent); counts[0..1] their lengths.  (Streams: KE_WIDEN -> conf_list, the keys to
// continue; a stream never reports KE_CONFLICT)
__global__ void __launch_bounds__(256) collect_retry(const KeyState* ks, uint64_t n, uint32_t* cap_list,
                                                     uint32_t* conf_list, uint32_t* counts) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int e = ks[i].err;
  if (e == KE_RETRY) cap_list[atomicAdd(counts, 1u)] = (uint32_t)i;
  else if (e == KE_CONFLICT || e == KE_WIDEN) conf_list[atomicAdd(counts + 1, 1u)] = (uint32_t)i;
}

// One wave per heavy key: the chain is read a whole 1 KiB chunk per wave load (each lane 16 B =
// chunk words 4 lane .. 4 lane + 3), the next chunk's load issued before the current one is
// parsed.  The parse walks the chunk by SEGMENTS, wave-uniformly: a run of pair words (seq,
// stage, seq, ...) is written by all lanes at once, each lane its own words (their pair index
// follows from the segment's start), and only the match headers [emit, n_pairs] are read one
// word at a time (broadcast from their lane).  A heavy key's matches are long (hundreds of
// pairs), so most chunks are one segment: the old word-by-word parse cost ~255 dependent steps
// per chunk (config 5's heavy variants spent ~2.5 s per 125k-key batch there).
__device__ __forceinline__ uint32_t chunk_word(const uint4& cur, uint32_t i) {
  const uint32_t c = i & 3;
  const uint32_t v = c == 0 ? cur.x : c == 1 ? cur.y : c == 2 ? cur.z : cur.w;  // uniform select
  return __shfl(v, (int)(i >> 2), 64);
}

__global__ void __launch_bounds__(256) scatter_heavy(const KeyState* ks, const HeavyKey* heavy, const uint32_t* n_heavy,
                                                     const uint32_t* out, uint32_t* m_key, uint32_t* m_emit,
                                                     uint64_t* m_off, uint32_t* p_seq, uint16_t* p_stage) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nh = *n_heavy;
  for (uint32_t h = blockIdx.x * 4 + (threadIdx.x >> 6); h < nh; h += gridDim.x * 4) {
    const HeavyKey hk = heavy[h];
    const KeyState st = ks[hk.key];
    uint64_t mo = hk.mo;
    uint64_t pn = hk.po;  // the pair whose seq word comes next (or, after an odd count, is open)
    uint64_t words = 2ull * st.n_matches + 2ull * st.n_pairs;  // [emit, np, (seq, stage) x np] per match
    uint32_t chunk = st.out_first;
    uint4 cur = reinterpret_cast<const uint4*>(out + (uint64_t)chunk * kOutChunkWords)[lane];
    int hdr = 0;        // header words still expected: 0 emit next (when rem == 0), 1 np next
    uint64_t rem = 0;   // pair words left in the current match
    while (words) {
      const uint32_t link = __shfl(cur.w, 63, 64);  // word 255
      const uint32_t here = words > kOutChunkWords - 1 ? kOutChunkWords - 1 : (uint32_t)words;
      uint4 nxt = cur;
      if (words > here) nxt = reinterpret_cast<const uint4*>(out + (uint64_t)link * kOutChunkWords)[lane];
      uint32_t p = 0;
      while (p < here) {
        if (rem == 0) {  // a header word
          const uint32_t w = chunk_word(cur, p);
          if (hdr == 0) {
            if (lane == 0) {
              m_key[mo] = hk.key;
              m_emit[mo] = w;
              m_off[mo] = pn;
            }
            mo++;
            hdr = 1;
          } else {
            rem = 2ull * w;
            hdr = 0;
          }
          p++;
          continue;
        }
        // a segment of pair words: chunk words [p, p + len)
        const uint32_t len = (uint32_t)(rem < (uint64_t)(here - p) ? rem : (uint64_t)(here - p));
        const uint32_t odd = (uint32_t)(rem & 1);  // the segment starts with a stage word (its seq was earlier)
#pragma unroll
        for (int c = 0; c < 4; c++) {
          const uint32_t i = lane * 4 + c;
          if (i >= p && i < p + len) {
            const uint32_t v = c == 0 ? cur.x : c == 1 ? cur.y : c == 2 ? cur.z : cur.w;
            const uint32_t d = i - p;
            if (odd && d == 0) {
              p_stage[pn - 1] = (uint16_t)v;
            } else {
              const uint32_t e = d - odd;
              const uint64_t pair = pn + (e >> 1);
              if (e & 1) p_stage[pair] = (uint16_t)v;
              else p_seq[pair] = v;
            }
          }
        }
        pn += (len - odd + 1) >> 1;  // the seq words of the segment open their pairs
        rem -= len;
        p += len;
      }
      words -= here;
      cur = nxt;
    }
  }
}

// order-independent checksum of the flat match arrays (tests/gpu_helpers.py, bench.py and
// multi-GPU all-gather): Σ_match mix(mix(C ^ key << 32 ^ emit) ^ (stage << 32 | seq) ...),
// the same function as workloads.match_digest.  Fixed arity (m_emit == nullptr): match i's
// pairs are p_seq[i m .. i m + m) with stage names `names`, emit = its first pair.
struct DigestNames {
  uint16_t v[8];
};

__global__ void __launch_bounds__(256) digest_matches(uint64_t n, uint32_t arity, DigestNames names,
                                                      const uint32_t* m_key, const uint32_t* m_emit,
                                                      const uint64_t* m_off, const uint32_t* p_seq,
                                                      const uint16_t* p_stage, unsigned long long* out) {
  __shared__ unsigned long long sd[4];
  unsigned long long dsum = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    uint64_t h;
    if (arity) {
      const uint32_t* ps = p_seq + i * arity;
      h = mix64(0x9E3779B97F4A7C15ull ^ ((uint64_t)m_key[i] << 32) ^ ps[0]);
      for (uint32_t x = 0; x < arity && x < 8; x++) h = mix64(h ^ (((uint64_t)names.v[x] << 32) | ps[x]));
    } else {
      h = mix64(0x9E3779B97F4A7C15ull ^ ((uint64_t)m_key[i] << 32) ^ m_emit[i]);
      for (uint64_t p = m_off[i]; p < m_off[i + 1]; p++) h = mix64(h ^ (((uint64_t)p_stage[p] << 32) | p_seq[p]));
    }
    dsum += h;
  }
  for (int off = 32; off > 0; off >>= 1) dsum += __shfl_down(dsum, off, 64);
  if ((threadIdx.x & 63) == 0) sd[threadIdx.x >> 6] = dsum;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long d = sd[0] + sd[1] + sd[2] + sd[3];
    if (d) atomicAdd(out, d);
  }
}

// ---------------------------------------------------------------- host launchers
template <int F>
static hipError_t launch_nfa_t(const NfaArgs& a, uint64_t nslots, uint32_t code_len, hipStream_t st) {
  const uint32_t blocks = (uint32_t)((nslots + 255) / 256);
  const size_t shm = ((sizeof(DevQuery) + 3) / 4 + code_len) * 4;
  hipLaunchKernelGGL(nfa_kernel<F>, dim3(blocks), dim3(256), shm, st, a);
  return hipGetLastError();
}

hipError_t launch_nfa(int F, const NfaArgs& a, uint64_t nslots, uint32_t code_len, hipStream_t st) {
  if (nslots == 0) return hipSuccess;
  switch (F) {
    case 0: case 1: case 2: return launch_nfa_t<2>(a, nslots, code_len, st);
    case 3: case 4: return launch_nfa_t<4>(a, nslots, code_len, st);
    default: return launch_nfa_t<8>(a, nslots, code_len, st);
  }
}

uint64_t walkq_size(uint64_t n_slots, uint32_t wcap, uint32_t plog) { return walkq_bytes(n_slots, wcap, plog); }

uint64_t ring_size(int F, uint64_t n_slots, uint32_t rcap) {
  return ring_bytes(F <= 2 ? 2 : (F <= 4 ? 4 : 8), n_slots, rcap);
}

hipError_t launch_compact(const KeyState* ks, uint64_t n_keys, uint64_t* bsum_m, uint64_t* bsum_p,
                          uint64_t* totals, hipStream_t st) {
  const uint64_t nb = (n_keys + 255) / 256;
  if (nb == 0) return hipSuccess;
  hipLaunchKernelGGL(count_blocks, dim3((uint32_t)nb), dim3(256), 0, st, ks, n_keys, bsum_m, bsum_p);
  hipLaunchKernelGGL(scan_blocks, dim3(1), dim3(1024), 0, st, bsum_m, bsum_p, nb, totals);
  return hipGetLastError();
}

uint64_t scatter_heavy_bytes(uint64_t n_keys) { return sizeof(HeavyKey) * (n_keys + 1) + 16; }

// heavy_scratch: scatter_heavy_bytes(n_keys), its first word the heavy-key count (zeroed here)
hipError_t launch_scatter(const KeyState* ks, uint64_t n_keys, const uint64_t* bsum_m, const uint64_t* bsum_p,
                          const uint32_t* out, uint32_t* m_key, uint32_t* m_emit, uint64_t* m_off,
                          uint32_t* p_seq, uint16_t* p_stage, const uint64_t* totals, void* heavy_scratch,
                          hipStream_t st) {
  const uint64_t nb = (n_keys + 255) / 256;
  if (nb == 0) return hipSuccess;
  uint32_t* n_heavy = static_cast<uint32_t*>(heavy_scratch);
  HeavyKey* heavy = reinterpret_cast<HeavyKey*>(static_cast<char*>(heavy_scratch) + 16);
  hipError_t e = hipMemsetAsync(n_heavy, 0, sizeof(uint32_t), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(scatter_matches, dim3((uint32_t)nb), dim3(256), 0, st, ks, n_keys, bsum_m, bsum_p, out,
                     m_key, m_emit, m_off, p_seq, p_stage, totals, heavy, n_heavy);
  hipLaunchKernelGGL(scatter_heavy, dim3(4096), dim3(256), 0, st, ks, heavy, n_heavy, out, m_key, m_emit, m_off,
                     p_seq, p_stage);
  return hipGetLastError();
}

hipError_t launch_collect_retry(const KeyState* ks, uint64_t n, uint32_t* cap_list, uint32_t* conf_list,
                                uint32_t* counts, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(collect_retry, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, ks, n, cap_list, conf_list,
                     counts);
  return hipGetLastError();
}

hipError_t launch_digest(uint64_t n, uint32_t arity, const uint16_t* names, const uint32_t* m_key,
                         const uint32_t* m_emit, const uint64_t* m_off, const uint32_t* p_seq,
                         const uint16_t* p_stage, unsigned long long* out, hipStream_t st) {
  if (n == 0) return hipSuccess;
  DigestNames nm{};
  for (uint32_t x = 0; x < arity && x < 8; x++) nm.v[x] = names[x];
  const uint64_t want = (n + 255) / 256;
  const uint32_t blocks = (uint32_t)(want < 1024 ? want : 1024);
  hipLaunchKernelGGL(digest_matches, dim3(blocks), dim3(256), 0, st, n, arity, nm, m_key, m_emit, m_off, p_seq,
                     p_stage, out);
  return hipGetLastError();
}

}  // namespace cep
