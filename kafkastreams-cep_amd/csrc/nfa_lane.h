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
#pragma once
#include "dewey.h"

namespace cep {

constexpr uint32_t kNoSk = 0xFF;
constexpr uint32_t kPending = 0xFFFFFFFEu;  // ev_first of a record created at the current event
constexpr uint32_t kQuietChunk = 16;        // events a runs-free lane may skip per driver step

template <int F, class Q>
struct Lane {
  const NfaArgs& A;
  Q& q;
  uint32_t key;
  uint64_t base;
  uint32_t j = 0;  // current event (sequence number within the key)
  Rec<F>* ring;
  uint32_t head = 0, count = 0;
  uint32_t pending = 0, n_final = 0;  // records of this event awaiting ev_first / finals queued
  uint32_t ncur = 0, nend = 0, pcur = 0, pend = 0;
  uint32_t ochunk = CEP_NONE, opos = 0;
  uint32_t cur_first = CEP_NONE;  // node chain of event j
  int err = KE_OK;
  uint32_t n_matches = 0, n_pairs = 0, out_first = CEP_NONE;

  __device__ Lane(const NfaArgs& a, Q& qq) : A(a), q(qq) {}

  __device__ __forceinline__ Rec<F>& R(uint32_t i) { return ring[i % A.rcap]; }

  // ---------------------------------------------------------------- records
  // Appends an output record; the caller fills it.  ev_first of a record whose event is the
  // current one is only known once the event's nodes exist: marked pending, patched later.
  __device__ __forceinline__ Rec<F>* push_rec(uint32_t stage, uint32_t event, uint32_t ev_first,
                                              const Dewey& ver) {
    if (count >= A.rcap) {
      err = KE_CAPACITY;
      return nullptr;
    }
    Rec<F>* r = &R(head + count);
    count++;
    r->stage = stage;
    r->event = event;
    if (event == j && ev_first == CEP_NONE) {
      r->ev_first = kPending;
      pending++;
    } else {
      r->ev_first = ev_first;
    }
    r->ver = ver;
    if (stage & kRecFinal) n_final++;
    return r;
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
    e.ver = v;
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
    Dewey w = v;
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
      w = A.preds[p].ver;
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
    Dewey w = v;
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
      w = A.preds[p].ver;
      s = nx;
    }
    if (emit) {
      A.out[npair_addr] = np;
      n_matches++;
      n_pairs += np;
    }
  }

  // ---------------------------------------------------------------- one event
  __device__ __forceinline__ void event() {
    cur_first = CEP_NONE;
    pending = 0;
    n_final = 0;
    const uint32_t n = count;
    for (uint32_t i = 0; i < n; i++) {
      const Rec<F> c = R(head);
      head++;
      count--;
      const int produced = q.step(*this, c);
      if (err) return;
      if (produced == 0) {  // removePattern
        walk_remove(q.stage_sk(c.stage), c.event, c.ev_first, c.ver, false);
        if (err) return;
      }
    }
    // records created at this event learn the node chain of the event
    if (pending) {
      for (uint32_t i = 0; i < count; i++) {
        Rec<F>& r = R(head + i);
        if (r.ev_first == kPending) r.ev_first = cur_first;
      }
    }
    if (!n_final) return;
    // matchConstruction: finals in order, then drop them from the queue
    const uint32_t m0 = n_matches, p0 = n_pairs;
    uint32_t w = 0;
    for (uint32_t i = 0; i < count; i++) {
      const Rec<F> r = R(head + i);
      if (r.stage & kRecFinal) {
        walk_remove(q.stage_sk(r.stage), r.event, r.ev_first, r.ver, true);
        if (err) {  // nothing of this event is forwarded
          n_matches = m0;
          n_pairs = p0;
          return;
        }
      } else {
        if (w != i) R(head + w) = r;
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
  __device__ __forceinline__ void run(uint32_t n, uint32_t* err_seq) {
    uint32_t jj = 0;
    while (jj < n) {
      if (q.quiet && count == 1 && R(head).stage == q.begin_stage) {
        const uint32_t lim = (n - jj > kQuietChunk) ? jj + kQuietChunk : n;
        bool hit = false;
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
      }
      j = jj;
      event();
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
  L.ring = reinterpret_cast<Rec<F>*>(A.rings) + slot * A.rcap;
  {  // NFA.initComputationStates :74-81 — the begin stage, version 1, sequence 1
    Rec<F>& r = L.ring[0];
    r.stage = q.begin_stage;
    r.event = CEP_NONE;
    r.ev_first = CEP_NONE;
    r.nullmask = (1u << F) - 1;
    dw_init(r.ver, 1);
    L.head = 0;
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
