// nfa_coop.h — wave-cooperative record steps (north_star: "wavefront ballot/prefix-scan to
// compact runs, allocate buffer versions and emit matches").
//
// The per-lane engine (nfa_lane.h) gives each lane one key and steps the key's queued records
// one after another, so at every event the wave runs max(records over its lanes) iterations of
// the record loop while most lanes idle (config 3: 1.28 records per lane-event, ~2.3 loop
// iterations per wave-event; a lone heavy key steps its ~3.4 records serially).  Here the
// records of all keys of the wave at their current events are laid out flat, key after key in
// lane order, and stepped in pages of 64: lane l of page p steps flat record 64p + l, whoever
// owns it.  A record's step (NFA.java:139-250, the generated policy) needs nothing from the
// other records of its event - predicates and folds read the record's own fold slots, Dewey
// versions are the record's own - except through the ordered side effects, which the step
// records here instead of performing (RecCtx):
//
//   side effect (reference)                     resolution (wave-wide, in record order)
//   ------------------------------------------  ------------------------------------------------
//   output records (matchPattern's list, the     segmented prefix sum of the records produced:
//     re-queued runs in order, :99-107)            slots in the owning key's next queue
//   put() of (stage key, event j)                per stage key a ballot of the putting lanes: the
//     (KVSharedVersionedBuffer.java:80-128):       key's first putter makes the node (or appends
//     node made by the first putter, pointers      to the one an earlier page made), every putter
//     appended in put order                        takes a pointer, linked to the next putter's
//   buffer walks (branch, removePattern), in     segmented prefix sum: slots in the key's walk
//     order (deferred, nfa_lane.h)                 queue, in record order
//   the first exception of the event             ballot: the key's first erring record; records
//     (process() throws, nothing after it)         after it in the key take no effect
//   put()'s conflict stamp (nfa_lane.h)          the key's walk count before the record
//
// A key's records are consecutive lanes of a page (a key spanning pages continues in the
// next, its per-key state carried in the owner lane), so "earlier in the key" is "lower lane
// of the same segment".  Each record's own effects come in a fixed order - its puts before its
// walks (evaluate's PROCEED recursion puts at every level before any level's branch walk) -
// so a put's stamp is the key's walk count before the record.  Exactness of each resolution
// against the reference's sequential order: DESIGN.md §2.2.11.
//
// Used when the query qualifies (compile.cpp sets JitQ::kCoop): the begin run lives in
// registers (kBeginReg) and is stepped by its owner after the pages; no queued record puts the
// begin stage's key; the stage keys one record can put at an event are distinct (so a key's
// puts of one stage key come from different records); the per-record action counts fit the
// capture (kCoopP/O/W).  Otherwise, and for kernel groups, the per-lane loop runs.
#pragma once


namespace cep {

constexpr uint32_t kTok = 0xFFFFFFF0u;  // a put's node as returned to the step: kTok | put slot

// ---- cross-lane helpers.  Convergent: every lane of the wave calls them.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const uint32_t lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(v, o, 64);
    if (lane >= (uint32_t)o) v += y;
  }
  return v;
}
// lanes [0, l)
__device__ __forceinline__ uint64_t lanes_below(uint32_t l) { return l >= 64 ? ~0ull : ((1ull << l) - 1ull); }
// lanes [lo, hi)
__device__ __forceinline__ uint64_t lanes_range(uint32_t lo, uint32_t hi) {
  return hi <= lo ? 0ull : (lanes_below(hi) & ~lanes_below(lo));
}
__device__ __forceinline__ uint32_t low_lane(uint64_t m, uint32_t dflt) { return m ? (uint32_t)__builtin_ctzll(m) : dflt; }
__device__ __forceinline__ uint32_t high_lane(uint64_t m, uint32_t dflt) { return m ? 63u - (uint32_t)__builtin_clzll(m) : dflt; }

// node (sk, event of the chain `first`); CEP_NONE when absent or deleted (Lane::lookup)
__device__ __forceinline__ uint32_t node_lookup(const NfaArgs& A, uint32_t sk, uint32_t first) {
  for (uint32_t i = first; i != CEP_NONE;) {
    CEP_STAT(6);
    const v4u q1 = reinterpret_cast<const v4u*>(A.nodes + i)[1];  // {same_next, meta, lk, -}
    if ((q1.y & 0xFF) == sk) return (q1.y & 0x100) ? i : CEP_NONE;
    i = q1.x;
  }
  return CEP_NONE;
}

// The step's side effects, recorded in program order (the Lane interface the generated step
// calls: put_link, push_rec, set_folds, walk_branch, readd_begin, j, ev, err).  Slots are
// written through compile-time indices (the `k == n` selects) so the capture stays in
// registers.  More actions than the capture holds: KE_RETRY (the key is re-run per lane).
template <int F, class Q>
struct RecCtx {
  using EvT = typename Q::EvT;
  static constexpr int kP = Q::kCoopP, kO = Q::kCoopO, kW = Q::kCoopW;
  const NfaArgs& A;
  EvT ev;
  uint32_t j = 0;
  uint64_t base = 0;
  int err = KE_OK;
  uint32_t np = 0, no = 0, nw = 0;
  uint32_t p_sk[kP], p_prev[kP], p_node[kP];
  Dewey p_ver[kP];
  uint32_t o_stage[kO], o_event[kO], o_ef[kO], o_node[kO], o_nm[kO];
  Dewey o_ver[kO];
  int64_t o_fold[kO][F];
  uint32_t w_word[kW], w_ev[kW], w_first[kW];
  Dewey w_ver[kW];

  __device__ explicit RecCtx(const NfaArgs& a) : A(a) {}

  // put(curr, currEvent, prev, prevEvent, version)  KVSharedVersionedBuffer.java:80-97: the
  // predecessor lookup (and its exceptions) here, the node and pointer at resolution
  __device__ __forceinline__ uint32_t put_link(uint32_t sk, uint32_t prev_sk, uint32_t prev_ev, uint32_t prev_first,
                                               const Dewey& v, uint32_t hint_sk = kNoSk, uint32_t hint = CEP_NONE) {
    uint32_t p = CEP_NONE;  // put(begin) (:117-128): no predecessor
    if (prev_sk != kNoSk) {
      if (prev_ev == CEP_NONE) {  // prevEvent.topic on a null Event
        err = KE_NPE;
        return CEP_NONE;
      }
      p = (hint != CEP_NONE && prev_sk == hint_sk) ? hint : node_lookup(A, prev_sk, prev_first);
      if (p == CEP_NONE) {  // "Cannot find predecessor event"
        err = KE_ILLEGAL_STATE;
        return CEP_NONE;
      }
    }
    if (np >= (uint32_t)kP) {
      err = KE_RETRY;
      return CEP_NONE;
    }
    const Dewey vp = dw_pin(v);
#pragma unroll
    for (int k = 0; k < kP; k++)
      if ((uint32_t)k == np) {
        p_sk[k] = sk;
        p_prev[k] = p;
        p_ver[k] = vp;
        p_node[k] = CEP_NONE;
      }
    return kTok | np++;
  }

  __device__ __forceinline__ int push_rec(uint32_t stage, uint32_t event, uint32_t ev_first, const Dewey& ver,
                                          uint32_t node = CEP_NONE, bool = false) {
    if (no >= (uint32_t)kO) {
      err = KE_RETRY;
      return -1;
    }
    const uint32_t ef = (event == j && ev_first == CEP_NONE) ? kPending : ev_first;
    const Dewey vp = dw_pin(ver);
#pragma unroll
    for (int k = 0; k < kO; k++)
      if ((uint32_t)k == no) {
        o_stage[k] = stage;
        o_event[k] = event;
        o_ef[k] = ef;
        o_node[k] = node;
        o_ver[k] = vp;
        o_nm[k] = (1u << F) - 1;
#pragma unroll
        for (int s = 0; s < F; s++) o_fold[k][s] = 0;
      }
    return (int)no++;
  }

  __device__ __forceinline__ void set_folds(int slot, const int64_t* v, uint32_t nm) {
#pragma unroll
    for (int k = 0; k < kO; k++)
      if (k == slot) {
        o_nm[k] = nm;
#pragma unroll
        for (int s = 0; s < F; s++) o_fold[k][s] = v[s];
      }
  }

  __device__ __forceinline__ void walk(uint32_t flags, uint32_t sk, uint32_t ev_, uint32_t first, const Dewey& v,
                                       uint32_t hint) {
    CEP_STAT(2);
    if (hint != CEP_NONE) {
      flags |= kWalkHint;
      first = hint;
    }
    if (nw >= (uint32_t)kW) {
      err = KE_RETRY;
      return;
    }
    const Dewey vp = dw_pin(v);
#pragma unroll
    for (int k = 0; k < kW; k++)
      if ((uint32_t)k == nw) {
        w_word[k] = sk | (flags << 8);
        w_ev[k] = ev_;
        w_first[k] = first;
        w_ver[k] = vp;
      }
    nw++;
  }
  __device__ __forceinline__ void walk_branch(uint32_t sk, uint32_t ev_, uint32_t first, const Dewey& v,
                                             uint32_t hint = CEP_NONE) {
    walk(kWalkBranch, sk, ev_, first, v, hint);
  }
  __device__ __forceinline__ void walk_remove(uint32_t sk, uint32_t ev_, uint32_t first, const Dewey& v, bool emit,
                                             uint32_t hint = CEP_NONE) {
    walk(emit ? kWalkEmit : 0u, sk, ev_, first, v, hint);
  }
  // (queued records are never the begin stage's: the begin run lives in its owner's registers)
  __device__ __forceinline__ bool readd_begin(uint32_t, const Dewey&) {
    err = KE_RETRY;
    return false;
  }
};

}  // namespace cep
