// nfa_lane.h — one key's reference NFA on one GPU lane: run FIFO, shared versioned buffer,
// match output, and the per-event driver.  The stage logic (NFA.evaluate) is a policy `Q`:
// the bytecode interpreter (nfa.hip) or per-query generated code compiled by hipRTC (jit.cpp).
//
//   per event j of key k                                   reference
//   ------------------------------------------------------ -----------------------------------
//   pop the |Q| runs present at event start, step each     NFA.matchPattern          :94-109
//   dead run -> walk_remove (GC only)                      NFA.removePattern        :117-123
//   finals -> walk_remove emitting the Sequence            NFA.matchConstruction    :111-115
//   put / put(begin) / branch / peek(remove)               KVSharedVersionedBuffer :80-171
//
// Policy interface (Q):
//   uint32_t stage_sk(uint32_t stage_word)   stage key of a record's stage (Stage.equals identity)
//   uint16_t sk_name(uint32_t sk)            stage-name id of a stage key (output)
//   int step(Lane&, const Rec<F>&)           NFA.matchPattern(ctx): records produced, -1 on error
//   bool quiet                               the begin stage has a single BEGIN edge
//   uint32_t begin_stage                     its stage index
//   bool begin_pred(Lane&)                   its predicate on event j with all-null folds
//   bool kBeginReg                           keep the begin run in registers (needs quiet)
//
// Run queue layout.  The queue a key holds between events is double-buffered: the records
// of event j are read from one half (slots 0..count-1) and the records they produce are
// written to the other (slots 0..), which becomes the queue of event j+1.  The halves of
// the 64 keys of a wavefront are interleaved at 16-B granularity, so lanes touching the
// same (half, slot, quad) - the common case, the queue loop runs in lockstep - form one
// fully coalesced 1 KiB access.  A record is kQuads quads: header {stage | Dewey pairs << 24,
// event, ev_first, Dewey length}, the Dewey (value, count) pairs two per quad (only quads
// holding live pairs are read or written), then {nullmask, -, fold0, fold1, ...}.
//
// When the begin stage has a single BEGIN edge (kBeginReg) the begin run, always the last
// record of the queue (NFA.java:148-157 re-adds it after its own outputs), lives in
// registers as its single Dewey digit: the ring holds live runs only.
#pragma once
#include "dewey.h"

namespace cep {

constexpr uint32_t kNoSk = 0xFF;
constexpr uint32_t kPending = 0xFFFFFFFEu;  // ev_first of a record created at the current event
constexpr uint32_t kQuietChunk = 16;        // events a runs-free lane may skip per driver step

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <int F>
struct RecLayout {
  static constexpr int kDwQuads = (kDeweyPairs + 1) / 2;
  static constexpr int kFoldQuads = (2 + 2 * F + 3) / 4;
  static constexpr int kQuads = 1 + kDwQuads + kFoldQuads;
};

// bytes of double-buffered run queues for n_slots lanes of rcap records
__host__ __device__ inline uint64_t ring_bytes(int F, uint64_t n_slots, uint32_t rcap) {
  const int quads = 1 + (kDeweyPairs + 1) / 2 + (2 + 2 * F + 3) / 4;
  return ((n_slots + 63) / 64) * 64ull * 2ull * rcap * quads * 16ull;
}

template <int F, class Q>
struct Lane {
  using Lay = RecLayout<F>;
  static constexpr bool kBeginReg = Q::kBeginReg;
  const NfaArgs& A;
  Q& q;
  uint32_t key;
  uint64_t base;
  uint32_t j = 0;  // current event (sequence number within the key)
  v4u* rb;         // this lane's quad 0 of half 0, slot 0 (stride 64 quads)
  uint32_t half = 0, count = 0, ocount = 0;  // input half, its records, records written
  uint32_t bdig = 1;                         // kBeginReg: the begin run's version "bdig"
  uint32_t pending = 0, n_final = 0;  // records of this event awaiting ev_first / finals queued
  uint32_t ncur = 0, nend = 0, pcur = 0, pend = 0;
  uint32_t ochunk = CEP_NONE, opos = 0;
  uint32_t cur_first = CEP_NONE;  // node chain of event j
  int err = KE_OK;
  uint32_t n_matches = 0, n_pairs = 0, out_first = CEP_NONE;

  __device__ Lane(const NfaArgs& a, Q& qq) : A(a), q(qq) {}

  __device__ __forceinline__ v4u* QP(uint32_t h, uint32_t slot, int quad) const {
    return rb + ((uint64_t)(h * A.rcap + slot) * Lay::kQuads + quad) * 64;
  }

  // ---------------------------------------------------------------- records
  __device__ __forceinline__ void load(uint32_t h, uint32_t slot, Rec<F>& r) const {
    const v4u hd = *QP(h, slot, 0);
    r.stage = hd.x & 0x00FFFFFFu;
    r.event = hd.y;
    r.ev_first = hd.z;
    r.ver.n = hd.x >> 24;
    r.ver.len = hd.w;
#pragma unroll
    for (int k = 0; k < Lay::kDwQuads; k++) {
      v4u d = {0, 0, 0, 0};
      if ((uint32_t)(2 * k) < r.ver.n) d = *QP(h, slot, 1 + k);
      r.ver.v[2 * k] = (int32_t)d.x;
      r.ver.c[2 * k] = d.y;
      if (2 * k + 1 < kDeweyPairs) {
        r.ver.v[2 * k + 1] = (int32_t)d.z;
        r.ver.c[2 * k + 1] = d.w;
      }
    }
    uint32_t w[Lay::kFoldQuads * 4];
#pragma unroll
    for (int k = 0; k < Lay::kFoldQuads; k++) {
      const v4u d = *QP(h, slot, 1 + Lay::kDwQuads + k);
      w[4 * k] = d.x;
      w[4 * k + 1] = d.y;
      w[4 * k + 2] = d.z;
      w[4 * k + 3] = d.w;
    }
    r.nullmask = w[0];
#pragma unroll
    for (int s = 0; s < F; s++) r.fold[s] = (int64_t)(((uint64_t)w[3 + 2 * s] << 32) | w[2 + 2 * s]);
  }

  __device__ __forceinline__ void store_head(uint32_t h, uint32_t slot, uint32_t stage, uint32_t event,
                                             uint32_t ev_first, const Dewey& ver0) {
    const Dewey ver = dw_pin(ver0);
    *QP(h, slot, 0) = v4u{stage | (ver.n << 24), event, ev_first, ver.len};
#pragma unroll
    for (int k = 0; k < Lay::kDwQuads; k++)
      if ((uint32_t)(2 * k) < ver.n)
        *QP(h, slot, 1 + k) = v4u{(uint32_t)ver.v[2 * k], ver.c[2 * k],
                                  2 * k + 1 < kDeweyPairs ? (uint32_t)ver.v[2 * k + 1] : 0u,
                                  2 * k + 1 < kDeweyPairs ? ver.c[2 * k + 1] : 0u};
  }

  __device__ __forceinline__ void store_folds(uint32_t h, uint32_t slot, const int64_t* v, uint32_t nm) {
    uint32_t w[Lay::kFoldQuads * 4];
#pragma unroll
    for (int i = 0; i < Lay::kFoldQuads * 4; i++) w[i] = 0;
    w[0] = nm;
#pragma unroll
    for (int s = 0; s < F; s++) {
      w[2 + 2 * s] = (uint32_t)(uint64_t)v[s];
      w[3 + 2 * s] = (uint32_t)((uint64_t)v[s] >> 32);
    }
#pragma unroll
    for (int k = 0; k < Lay::kFoldQuads; k++)
      *QP(h, slot, 1 + Lay::kDwQuads + k) = v4u{w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]};
  }

  __device__ __forceinline__ void copy_rec(uint32_t h, uint32_t from, uint32_t to) {
#pragma unroll
    for (int k = 0; k < Lay::kQuads; k++) *QP(h, to, k) = *QP(h, from, k);
  }

  // Appends an output record (header + version) and returns its slot, -1 when the queue is
  // full.  ev_first of a record whose event is the current one is only known once the
  // event's nodes exist: marked pending, patched after the event.  Folds: set_folds.
  __device__ __forceinline__ int push_rec(uint32_t stage, uint32_t event, uint32_t ev_first, const Dewey& ver) {
    if (ocount >= A.rcap) {
      err = KE_CAPACITY;
      return -1;
    }
    const uint32_t slot = ocount++;
    uint32_t ef = ev_first;
    if (event == j && ev_first == CEP_NONE) {
      ef = kPending;
      pending++;
    }
    store_head(half ^ 1u, slot, stage, event, ef, ver);
    if (stage & kRecFinal) n_final++;
    return (int)slot;
  }

  __device__ __forceinline__ void set_folds(int slot, const int64_t* v, uint32_t nm) {
    store_folds(half ^ 1u, (uint32_t)slot, v, nm);
  }

  // the begin run re-added after its outputs (NFA.java:148-157); `stage` is the begin stage
  __device__ __forceinline__ bool readd_begin(uint32_t stage, const Dewey& v) {
    if (kBeginReg) {
      bdig = (uint32_t)v.v[0];  // a begin run's version is a single digit
      return true;
    }
    const int r = push_rec(stage, CEP_NONE, CEP_NONE, v);
    if (r < 0) return false;
    int64_t z[F];
#pragma unroll
    for (int s = 0; s < F; s++) z[s] = 0;
    set_folds(r, z, (1u << F) - 1);
    return true;
  }

  // ---------------------------------------------------------------- buffer nodes
  __device__ __forceinline__ uint32_t lookup(uint32_t sk, uint32_t first) {
    for (uint32_t i = first; i != CEP_NONE;) {
      const Node& n = A.nodes[i];
      if ((n.meta & 0xFF) == sk) return (n.meta & 0x100) ? i : CEP_NONE;
      i = n.same_next;
    }
    return CEP_NONE;
  }

  __device__ __forceinline__ uint32_t new_node(uint32_t sk) {
    const uint32_t i = pool_take(A.node_pool, ncur, nend);
    if (i == CEP_NONE) {
      err = KE_CAPACITY;
      return CEP_NONE;
    }
    Node& n = A.nodes[i];
    n.event = j;
    n.refs = 1;
    n.head = n.tail = CEP_NONE;
    n.same_next = cur_first;
    n.meta = sk | 0x100;
    cur_first = i;
    return i;
  }

  __device__ __forceinline__ void append_pred(uint32_t node, uint32_t prev, const Dewey& v) {
    const uint32_t p = pool_take(A.pred_pool, pcur, pend);
    if (p == CEP_NONE) {
      err = KE_CAPACITY;
      return;
    }
    Pred& e = A.preds[p];
    e.prev = prev;
    e.next = CEP_NONE;
    e.removed = 0;
    dw_store(e.ver, v);
    Node& n = A.nodes[node];
    if (n.head == CEP_NONE) n.head = p;
    else A.preds[n.tail].next = p;
    n.tail = p;
    n.meta += 1u << 16;
  }

  // put(stage, evt, version)  KVSharedVersionedBuffer.java:117-128 (overwrites)
  __device__ __forceinline__ void put_begin(uint32_t sk, const Dewey& v) {
    uint32_t c = lookup(sk, cur_first);
    if (c == CEP_NONE) {
      c = new_node(sk);
      if (err) return;
    } else {
      Node& n = A.nodes[c];
      n.refs = 1;
      n.head = n.tail = CEP_NONE;
      n.meta = sk | 0x100;
    }
    append_pred(c, CEP_NONE, v);
  }

  // put(curr, currEvent, prev, prevEvent, version)  :80-97;  prev_sk == kNoSk: put(begin)
  __device__ __forceinline__ void put_link(uint32_t sk, uint32_t prev_sk, uint32_t prev_ev, uint32_t prev_first,
                           const Dewey& v) {
    if (prev_sk == kNoSk) {
      put_begin(sk, v);
      return;
    }
    if (prev_ev == CEP_NONE) {  // prevEvent.topic on a null Event
      err = KE_NPE;
      return;
    }
    const uint32_t p = lookup(prev_sk, prev_first);
    if (p == CEP_NONE) {  // "Cannot find predecessor event"
      err = KE_ILLEGAL_STATE;
      return;
    }
    uint32_t c = lookup(sk, cur_first);
    if (c == CEP_NONE) {
      c = new_node(sk);
      if (err) return;
    }
    append_pred(c, p, v);
  }

  // TimedKeyValue.getPointerByVersion  TimedKeyValue.java:83-92
  __device__ __forceinline__ uint32_t first_compat(uint32_t node, const Dewey& walker) {
    for (uint32_t p = A.nodes[node].head; p != CEP_NONE; p = A.preds[p].next) {
      const Pred& e = A.preds[p];
      if (e.removed) continue;
      if (dw_compatible(walker, e.ver)) return p;
    }
    return CEP_NONE;
  }

  // branch  :99-110
  __device__ __forceinline__ void walk_branch(uint32_t sk, uint32_t ev, uint32_t first, const Dewey& v) {
    if (ev == CEP_NONE) {
      err = KE_NPE;
      return;
    }
    uint32_t s = lookup(sk, first);
    Dewey w = dw_pin(v);
    for (;;) {
      if (s == CEP_NONE || !(A.nodes[s].meta & 0x100)) {
        err = KE_NPE;
        return;
      }
      A.nodes[s].refs += 1;
      const uint32_t p = first_compat(s, w);
      if (p == CEP_NONE) return;
      const uint32_t nx = A.preds[p].prev;
      if (nx == CEP_NONE) return;
      w = dw_pin(A.preds[p].ver);  // a value, not a pointer into the pool
      s = nx;
    }
  }

  // ---------------------------------------------------------------- output stream
  __device__ __forceinline__ uint64_t out_put(uint32_t w) {
    if (ochunk == CEP_NONE || opos == kOutChunkWords - 1) {
      const uint32_t c = atomicAdd(A.out_pool.top, 1u);
      if (c >= A.out_pool.cap) {
        err = KE_CAPACITY;
        return 0;
      }
      if (ochunk == CEP_NONE) out_first = c;
      else A.out[(uint64_t)ochunk * kOutChunkWords + kOutChunkWords - 1] = c;
      ochunk = c;
      opos = 0;
    }
    const uint64_t a = (uint64_t)ochunk * kOutChunkWords + opos++;
    A.out[a] = w;
    return a;
  }

  // peek(stage, event, version, remove=true)  :143-171; emit = match construction
  __device__ __forceinline__ void walk_remove(uint32_t sk, uint32_t ev, uint32_t first, const Dewey& v, bool emit) {
    if (ev == CEP_NONE) {
      err = KE_NPE;
      return;
    }
    uint32_t s = lookup(sk, first);
    Dewey w = dw_pin(v);
    uint64_t npair_addr = 0;
    uint32_t np = 0;
    if (emit) {
      out_put(j);
      npair_addr = out_put(0);
      if (err) return;
    }
    for (;;) {
      if (s == CEP_NONE) {
        err = KE_NPE;
        return;
      }
      Node& n = A.nodes[s];
      const uint32_t meta = n.meta;
      if (!(meta & 0x100)) {
        err = KE_NPE;
        return;
      }
      const int32_t left = n.refs == 0 ? 0 : n.refs - 1;
      n.refs = left;
      if (left == 0 && (meta >> 16) <= 1) n.meta = meta & ~0x100u;  // store.delete
      if (emit) {
        out_put(n.event);
        out_put(q.sk_name(meta & 0xFF));
        np++;
        if (err) return;
      }
      const uint32_t p = first_compat(s, w);
      if (p == CEP_NONE) break;
      if (left == 0) {  // removePredecessor(pointer)
        A.preds[p].removed = 1;
        n.meta -= 1u << 16;
      }
      const uint32_t nx = A.preds[p].prev;
      if (nx == CEP_NONE) break;
      w = dw_pin(A.preds[p].ver);  // a value, not a pointer into the pool
      s = nx;
    }
    if (emit) {
      A.out[npair_addr] = np;
      n_matches++;
      n_pairs += np;
    }
  }

  // ---------------------------------------------------------------- one event
  __device__ __forceinline__ void event(bool begin_hit) {
    cur_first = CEP_NONE;
    pending = 0;
    n_final = 0;
    ocount = 0;
    const uint32_t n = count;
    for (uint32_t i = 0; i < n; i++) {
      Rec<F> c;
      load(half, i, c);
      const int produced = q.step(*this, c);
      if (err) return;
      if (produced == 0) {  // removePattern
        walk_remove(q.stage_sk(c.stage), c.event, c.ev_first, c.ver, false);
        if (err) return;
      }
    }
    // the begin run, last in the queue: its predicate runs after every other record's
    // (an exception from it must not pre-empt theirs)
    if (kBeginReg && !begin_hit) {
      begin_hit = q.begin_pred(*this);
      if (err) return;
    }
    if (kBeginReg && begin_hit) {
      Rec<F> b;
      b.stage = q.begin_stage;
      b.event = CEP_NONE;
      b.ev_first = CEP_NONE;
      b.nullmask = (1u << F) - 1;
#pragma unroll
      for (int s = 0; s < F; s++) b.fold[s] = 0;
      dw_init(b.ver, (int32_t)bdig);
      q.step(*this, b);
      if (err) return;
    }
    const uint32_t oh = half ^ 1u;
    half = oh;
    count = ocount;
    // records created at this event learn the node chain of the event
    if (pending) {
      for (uint32_t i = 0; i < count; i++) {
        v4u* hp = QP(oh, i, 0);
        if ((*hp).z == kPending) (*hp).z = cur_first;
      }
    }
    if (!n_final) return;
    // matchConstruction: finals in order, then drop them from the queue
    const uint32_t m0 = n_matches, p0 = n_pairs;
    uint32_t w = 0;
    for (uint32_t i = 0; i < count; i++) {
      const v4u hd = *QP(oh, i, 0);
      if (hd.x & kRecFinal) {
        Rec<F> r;
        load(oh, i, r);
        walk_remove(q.stage_sk(r.stage), r.event, r.ev_first, r.ver, true);
        if (err) {  // nothing of this event is forwarded
          n_matches = m0;
          n_pairs = p0;
          return;
        }
      } else {
        if (w != i) copy_rec(oh, i, w);
        w++;
      }
    }
    count = w;
  }

  // ---------------------------------------------------------------- the key's stream
  // Lanes of a wavefront advance in lockstep; a lane whose queue holds only the begin run
  // (whose single BEGIN edge did not match) is in the reference's quiet state: an event
  // that fails the begin predicate changes nothing (the begin run is re-added with the same
  // version, NFA.java:149-157), so the lane tests up to kQuietChunk events per step.
  __device__ __forceinline__ bool only_begin() const {
    if (kBeginReg) return count == 0;
    if (count != 1) return false;
    return ((*QP(half, 0, 0)).x & 0x00FFFFFFu) == q.begin_stage;
  }

  __device__ __forceinline__ void run(uint32_t n, uint32_t* err_seq) {
    uint32_t jj = 0;
    while (jj < n) {
      bool hit = false, known = false;
      (void)hit;
      if (q.quiet && only_begin()) {
        const uint32_t lim = (n - jj > kQuietChunk) ? jj + kQuietChunk : n;
        for (; jj < lim; jj++) {
          j = jj;
          hit = q.begin_pred(*this);
          if (err || hit) break;
        }
        if (err) {
          *err_seq = jj;
          return;
        }
        if (!hit) continue;
        known = true;
      }
      j = jj;
      event(known);  // known: the quiet scan already found the begin predicate true
      if (err) {
        *err_seq = jj;
        return;
      }
      jj++;
    }
  }
};

// Driver shared by the AOT and JIT kernels: slot -> key, initial state, stream, KeyState.
template <int F, class Q>
__device__ __forceinline__ void run_key(const NfaArgs& A, Q& q) {
  const uint64_t slot = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nslots = A.key_list ? A.n_list : A.n_keys;
  if (slot >= nslots) return;
  const uint32_t key = A.key_list ? A.key_list[slot] : (uint32_t)slot;
  Lane<F, Q> L(A, q);
  L.key = key;
  L.base = A.key_off[key];
  const uint32_t n = (uint32_t)(A.key_off[key + 1] - L.base);
  L.rb = reinterpret_cast<v4u*>(A.rings) +
         (slot / 64) * (2ull * A.rcap * RecLayout<F>::kQuads * 64) + (slot % 64);
  // NFA.initComputationStates :74-81 — the begin stage, version 1, sequence 1
  L.bdig = 1;
  L.half = 0;
  L.count = 0;
  if (!Lane<F, Q>::kBeginReg) {
    Dewey v;
    dw_init(v, 1);
    L.ocount = 0;
    L.half = 1;  // push_rec writes the other half: half 0
    L.readd_begin(q.begin_stage, v);
    L.half = 0;
    L.count = 1;
  }
  uint32_t err_seq = 0;
  L.run(n, &err_seq);
  KeyState& ks = A.ks[key];
  ks.n_matches = L.n_matches;
  ks.n_pairs = L.n_pairs;
  ks.out_first = L.out_first;
  ks.err = L.err;
  ks.err_seq = err_seq;
  if (L.err == KE_CAPACITY) atomicAdd(A.n_capacity_err, 1u);
}

}  // namespace cep
