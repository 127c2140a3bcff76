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
//   EvT                                      the event fields the query reads (registers)
//   void load_ev(EvT&, uint64_t pos)         loads them for CSR position pos
//   uint32_t stage_sk(uint32_t stage_word)   stage key of a record's stage (Stage.equals identity)
//   uint16_t sk_name(uint32_t sk)            stage-name id of a stage key (output)
//   int step(Lane&, const Rec<F>&)           NFA.matchPattern(ctx) on L.ev: records produced, -1 on error
//   bool quiet                               the begin stage has a single BEGIN edge
//   uint32_t begin_stage                     its stage index
//   bool begin_pred(Lane&)                   its predicate on L.ev with all-null folds
//   void set_query(uint32_t qi)              the lane's query within the launch (group kernels)
//   uint32_t begin_scan(Lane&, j0, lim)      first position in [j0, lim) where begin_pred is
//                                            true or throws (L.err set), else lim
//   bool kBeginReg                           keep the begin run in registers (needs quiet)
//   bool kFold32                             every fold state is a 32-bit int
//
// Run queue layout.  The queue a key holds between events is double-buffered: the records
// of event j are read from one half (slots 0..count-1) and the records they produce are
// written to the other (slots 0..), which becomes the queue of event j+1.  The halves of
// the 64 keys of a wavefront are interleaved at 16-B granularity, so lanes touching the
// same (half, slot, quad) - the common case, the queue loop runs in lockstep - form one
// fully coalesced 1 KiB access.  A record is kQuads quads: header {stage | Dewey pairs << 24,
// event, ev_first, node hint}, the Dewey (value, count) pairs two per quad (only quads
// holding live pairs are read or written), then {nullmask, -, fold0, fold1, ...} (64-bit
// slots) or {nullmask, fold0, fold1, ...} when every fold state is an int (kFold32).
// A record created at event j does not know the node chain of j until the event ends; it is
// written with ev_first = kPending and resolved when it is next loaded (event j+1, or the
// final-match pass of event j itself).  Node hint: the buffer node (source stage key, event)
// of the record, known when the step that made the record put that node (TAKE, BEGIN) or
// copied from the record it continues (IGNORE).  With deferred walks no node is deleted
// between two flushes, so put()'s predecessor lookup takes the hint without a memory round
// trip; a flush clears the hints of the queued records (and walks in place never use them).
// The Dewey length is not stored: it is the sum of the pair counts.
//
// LDS slots (Q::kRingLds = RL > 0).  The first RL slots of each half live in LDS instead of
// HBM: their header quad, first Dewey quad and fold quads (the quads every record uses); the
// remaining Dewey quads (pairs 2.., rare) stay at the slot's HBM position.  A lane whose queue
// holds at most RL records between events - most lanes at most events - then never touches
// HBM for its run queue.  The slot index of the queue loop is wave-uniform (lanes iterate
// i = 0, 1, ... in lockstep), so the LDS/HBM choice does not diverge there.  LDS is per
// launch: a streaming session spills the LDS slots of a key's queue to their HBM positions
// when the batch ends and reloads them when the next batch starts.
//
// When the begin stage has a single BEGIN edge (kBeginReg) the begin run, always the last
// record of the queue (NFA.java:148-157 re-adds it after its own outputs), lives in
// registers as its single Dewey digit: the ring holds live runs only.
//
// Deferred walks (A.defer).  The buffer walks - branch (refs++ along a path), removePattern
// and match extraction (peek with remove) - are pointer chases of O(path) dependent loads.
// Run in place, a lane walking stalls the 63 others.  Instead each walk is queued (in
// order) and the wave drains all queues together in one loop where every lane advances its
// own walk by one node per iteration, so the wave pays for the longest queue, not the sum.
// This is exact because the per-event work between a walk and its deferred execution never
// observes a walk's effects: walks change refcounts, predecessor lists and live bits of
// nodes of events before the walk's own event; the step only appends to nodes of the
// current event and reads older nodes through put()'s predecessor lookup, which checks the
// live bit.  That one read is checked: a lookup made while walks are queued stamps the node
// with the number of walks queued so far and appends (node, that number, event) to the lane's
// put log.  A walk that deletes a node stamped after the walk was queued is exactly the
// reference's "Cannot find predecessor event" (KVSharedVersionedBuffer.java:86-89): the node
// is gone when the first put made after the walk looks it up, and nothing between the two
// reads that node (nodes are only created at the current event; steps read older nodes only
// through put()).  So the walk completes, the put log names that first put (its event and
// walk count), the walks queued before it still run in order (their matches and exceptions
// come first), and the key stops with IllegalState at the put's event - the result of
// running the walks in place, without a re-run.  (A put log that would overflow mid-event
// falls back to KE_CONFLICT: the key is re-run with walks in place, session.cpp.)  Errors keep
// their reference order: a walk's exception precedes anything the step did after queueing it.
#pragma once
#include "dewey.h"

// Work counters for the CPU lane build (tests/lane_cpu, CEP_LANE_STATS); nothing on the GPU.
#ifdef CEP_LANE_STATS
extern uint64_t cep_lane_stats[10];  // events, records, walks, walk nodes, pred scans, flushes, chain steps, flush iters, exact conflicts, twin writes saved
// every walk node (job key, the walk's event, the node, walk flags, the walker's version on
// arrival): which extraction hops retrace a branch walk of the same event (tests/lane_cpu)
void cep_lane_hop(uint32_t key, uint32_t t, uint32_t node, uint32_t flags, const cep::Dewey& w);
#define CEP_HOP(k, t, s, f, w) cep_lane_hop(k, t, s, f, w)
#define CEP_STAT(i) (cep_lane_stats[i]++)
#else
#define CEP_STAT(i) ((void)0)
#define CEP_HOP(k, t, s, f, w) ((void)0)
#endif

// Time split of a launch (measurement builds only: $CEP_PROF at query compile, NfaArgs.prof):
// per wave, shader-clock cycles in each part of the job loop, summed over waves by lane 0.
//   0 walk drains mid-job   1 quiet skip (bitmap / scan)   2 record loop (steps, lookups, puts)
//   3 begin run             4 finals + queue swap          5 final drain
//   6 waves                 7 whole run()                  8 loop iterations   9 records stepped
//   10 lane-events (event() entered)                        11 walk nodes
//   12 max over waves of the wave's lifetime (cycles)       13 the same in wall-clock ticks (100 MHz)
#ifdef CEP_PROF
#define CEP_PT(v) const uint64_t v = clock64()
#define CEP_PACC(i, d) (prof[i] += (d))
#define CEP_LPACC(L, i, d) ((L).prof[i] += (d))
#else
#define CEP_PT(v) ((void)0)
#define CEP_PACC(i, d) ((void)0)
#define CEP_LPACC(L, i, d) ((void)0)
#endif

namespace cep {

constexpr uint32_t kNoSk = 0xFF;
constexpr uint32_t kPending = 0xFFFFFFFEu;  // ev_first of a record created at the current event
#ifndef CEP_QUIET_CHUNK
#define CEP_QUIET_CHUNK 16
#endif
// partial drains (flush(may_stop)): 1 on, 0 off, 2 every flush stops as soon as it may (tests)
#ifndef CEP_PARTIAL_DRAIN
#define CEP_PARTIAL_DRAIN 1
#endif
#ifndef CEP_WALK_FLUSH
#define CEP_WALK_FLUSH 24
#endif
#ifndef CEP_JOB_DRAIN
#define CEP_JOB_DRAIN 1
#endif
#ifndef CEP_WALK_COMPAT2
#define CEP_WALK_COMPAT2 0
#endif
// Fused branch + extraction walks (deferred walks).  A TAKE+PROCEED branch at a stage followed by
// the final it forwards (NFA.java:231-246, then :111-115) queues a branch walk W_b from (stage,
// event) and, in the finals pass of the same event, the final's extraction W_e from its new node
// N_f, whose pointer leads back to W_b's start with W_b's version: from there both walk the same
// path (a walk's choice of predecessor reads pointer versions and removed flags, which a branch
// walk never changes and an extraction changes only behind itself), W_b adding 1 to every
// node's refs and W_e taking 1 off.  When W_e directly follows W_b in the lane's queue (no walk
// between them could observe W_b's counts), W_b is skipped and W_e, from W_b's start node on,
// leaves refs as they are - deleting a node and removing its pointer exactly when the sequence
// would (refs 0 before W_b).  W_e's first hop touches N_f alone, which W_b never reads, so it
// commutes with W_b.  A failure W_b would meet (a dead node) W_e meets at the same node and
// event; the key stops there either way and its unwound buffer is never read.  Measured on the
// CPU lane build (profiles/r06/hops): 96-97 % of extraction hops retrace a branch walk of the
// same event, half of all walk hops (config 3's README query and config 5's 64 queries).
#ifndef CEP_WALK_FUSE
#define CEP_WALK_FUSE CEP_WALK_COMPAT2
#endif
constexpr uint32_t kQuietChunk = CEP_QUIET_CHUNK;  // events a runs-free lane scans per driver step
constexpr int kJobDrain = CEP_JOB_DRAIN;  // lanes at a job's end that make the wave drain its walks
constexpr uint32_t kWalkFlush = CEP_WALK_FLUSH;    // a queue this long drains the wave's walk queues
constexpr int kWalkQuads = 2 + (kLayoutPairs + 1) / 2;  // {sk|flags|n, ev, first, len} pairs {t}
constexpr uint32_t kWalkEmit = 1, kWalkBranch = 2;
constexpr uint32_t kWalkFused = 16;  // (runtime only) an extraction past the start of the branch walk it absorbed
// the entry's `first` field holds the walk's start node itself (the record's node hint, live
// when the walk was queued - an epsilon record's hint is its node of (stage key, event)): no
// lookup at the walk's start.  Exact: no node is taken from the pool during a flush, so a
// start node deleted by an earlier walk of the flush is found dead (NPE) by walk_node, as the
// lookup would find none.
constexpr uint32_t kWalkHint = 8;
// put-log entries per lane ({node, walks queued, event, -}), after each 64 lanes' walk queues
// in A.walks (the log's address is the walk queue's plus a launch constant); the wave drains
// its walks before an event could overflow it.  A.plog entries per lane, sized by the host from
// the run-queue capacity (put_log_entries): every put one event can log fits twice over.
// (put_log_entries, cep_layout.h)
// The narrow build of a query (compile.cpp) leaves the put log out - the registers it costs
// spill there - and reports a conflict as KE_CONFLICT: the key is re-run in the wide build,
// which resolves it.  (Default: on.)
#ifndef CEP_PUT_LOG
#define CEP_PUT_LOG 1
#endif
// Walks in place (A.defer == 0): the wide build's re-runs after a put log overflowed, and the
// interpreter's.  The narrow and stream builds are never launched with A.defer == 0 (session.cpp:
// their re-runs and continuations take the wide build) and leave the path out: inlined into
// every walk site of the step, its dead code alone made the record loop spill 15 VGPRs at the
// 168-VGPR budget of 3 waves per SIMD (with it out: 163 VGPRs, none spilled).  (Launched with
// A.defer == 0 anyway, such a build defers: exact, a conflict re-runs the job in the wide build.)
#ifndef CEP_WALK_IN_PLACE
#define CEP_WALK_IN_PLACE 1
#endif
// a value every active lane of the wave holds (the compiler then branches on it with the scalar
// unit); the CPU lane build runs lanes one at a time and takes the lane's own
#ifndef CEP_UNIFORM
#define CEP_UNIFORM(x) ((uint32_t)__builtin_amdgcn_readfirstlane((int)(x)))
#endif
// a Dewey version outgrowing the pairs this build holds: the narrow build (fewer than 6)
// re-runs the job in the wide one (a retry); the wide build's limit is final
#ifndef CEP_STREAM_STOP
#define CEP_STREAM_STOP 0
#endif
constexpr int32_t kDwFull = kDeweyPairs >= 6 ? KE_CAPACITY : CEP_STREAM_STOP ? KE_WIDEN : KE_RETRY;

// may_alias: quads of Node/Pred are also read and written field by field (Node::refs, ...);
// without it TBAA lets the compiler reorder the two views of the same bytes
typedef uint32_t v4u __attribute__((ext_vector_type(4), may_alias));
// LDS-typed quads: a load from LDS and one from HBM of the same shape in the two arms of a
// branch must not be merged into one flat load through a pointer select (the compiler
// would otherwise do exactly that); distinct address spaces cannot be merged.
#ifndef CEP_LDS_AS
#define CEP_LDS_AS __attribute__((address_space(3)))
#endif
typedef CEP_LDS_AS v4u lds_v4u;

// Twin slots.  A record that a step re-adds unchanged (an IGNORE without a new stage: the
// reference re-adds the same object, NFA.java:225) at the slot it was read from already sits,
// word for word, in the other queue half if it sat there two events ago: header bit kTwin of a
// stored record says "the other half's copy of this slot is the same record", kTwinT says "and
// that copy's kTwin is set".  The record's write is then reduced to its header (kTwin) or
// dropped (kTwin and kTwinT).  Only HBM slots (the LDS slots are cheap to write) - config 4's
// ~20 runs a key holds were read and rewritten every event (54x its algorithmic
// bytes).  A copy's flags are read only when the copy is an event's input, and an event's
// input half was its previous event's output half, whose every slot in use was written or
// kept with the guarantee; anything that changes a record in place (clear_hints, the finals'
// compaction) clears them.
constexpr uint32_t kTwin = 1u << 23, kTwinT = 1u << 22;
constexpr uint32_t kInPend = 1u << 16;  // (Lane::in_info only)
constexpr uint32_t kStageMask = 0x003FFFFFu;  // the stage word bits of a stored header's x

// W32: every fold state is a 32-bit int (one word per slot, the query's own choice)
template <int F, bool W32 = false>
struct RecLayout {
  static constexpr int kDwQuads = (kLayoutPairs + 1) / 2;  // (memory)
  static constexpr int kDwRegQuads = (kDeweyPairs + 1) / 2;  // the quads a version in registers fills
  static constexpr int kFoldQuads = W32 ? (1 + F + 3) / 4 : (2 + 2 * F + 3) / 4;
  static constexpr int kQuads = 1 + kDwQuads + kFoldQuads;
  // quads of an LDS slot: header, Dewey quad 0, folds
  static constexpr int kLdsQuads = 2 + kFoldQuads;
  __host__ __device__ static constexpr bool in_lds(int quad) { return quad <= 1 || quad > kDwQuads; }
  __host__ __device__ static constexpr int lds_quad(int quad) { return quad <= 1 ? quad : quad - (kDwQuads - 1); }
};

// LDS slots per queue half for a record layout: 192 B of LDS per lane (48 KiB per 256-lane
// block keeps 3 blocks = 3 waves per SIMD resident), at most 2 slots
// ($CEP_RING_LDS_SLOTS at query compile: measurement runs)
template <class Lay>
__host__ __device__ constexpr int ring_lds_slots() {
#ifdef CEP_RING_LDS_SLOTS
  return CEP_RING_LDS_SLOTS;
#else
  return (192 / (2 * 16 * Lay::kLdsQuads)) < 2 ? (192 / (2 * 16 * Lay::kLdsQuads)) : 2;
#endif
}

// bytes of double-buffered run queues for n_slots lanes of rcap records (64-bit folds: the
// larger layout, so one allocation serves every query)
__host__ __device__ inline uint64_t ring_bytes(int F, uint64_t n_slots, uint32_t rcap) {
  const int quads = 1 + (kLayoutPairs + 1) / 2 + (2 + 2 * F + 3) / 4;
  return ((n_slots + 63) / 64) * 64ull * 2ull * rcap * quads * 16ull;
}

// bytes of deferred-walk queues for n_slots lanes of wcap walks and their put logs (plog entries)
__host__ __device__ inline uint64_t walkq_bytes(uint64_t n_slots, uint32_t wcap, uint32_t plog) {
  return ((n_slots + 63) / 64) * 64ull * ((uint64_t)wcap * kWalkQuads + plog) * 16ull;
}
// quads per 64 lanes of that allocation
__host__ __device__ inline uint64_t walkq_group_quads(uint32_t wcap, uint32_t plog) {
  return ((uint64_t)wcap * kWalkQuads + plog) * 64;
}

template <int F, class Q>
struct Lane {
  using Lay = RecLayout<F, Q::kFold32>;
  using EvT = typename Q::EvT;
  static constexpr bool kBeginReg = Q::kBeginReg;
  static constexpr uint32_t kRL = Q::kRingLds;  // LDS slots per half (0: all HBM)
  const NfaArgs& A;
  Q& q;
  uint32_t key;
  uint64_t base;      // CSR position of sequence number 0 (base + j = event j's position)
  uint32_t j0 = 0;    // sequence number of the batch's first event of the key
  uint32_t n_ev = 0;  // events of the key in this batch
  uint32_t j = 0;     // current event (sequence number within the key's stream)
  EvT ev;             // fields of event ev_pos
  uint32_t ev_pos = CEP_NONE;
  v4u* rb;  // this lane's quad 0 of half 0, slot 0 (stride 64 quads)
  lds_v4u* lr;  // LDS slots: this lane's quad 0 of half 0, slot 0 (stride 64 quads)
  v4u* wb;  // this lane's walk queue, slot 0 quad 0 (stride 64 quads), then its put log
  uint32_t half = 0, count = 0, ocount = 0;  // input half, its records, records written
  uint32_t bdig = 1;                         // kBeginReg: the begin run's version "bdig"
  uint32_t n_final = 0;                      // finals queued at this event
  uint32_t ncur = 0, nend = 0, pcur = 0, pend = 0;
  uint32_t ochunk = CEP_NONE, opos = 0;
  uint32_t ocur = 0, oend = 0;  // output chunks in hand (kept across the jobs of a persistent lane)
  // twin slots: the record being stepped (its slot, its stored head quad) and a re-add of it
  // whose head write waits for its folds
  // in_info: its Dewey length (bits 0-15; a longer one never matches) | its stored twin flags |
  // kInPend (stored ev_first kPending)
  uint32_t in_slot = CEP_NONE, pend_slot = CEP_NONE, in_info = 0;
  uint32_t cur_first = CEP_NONE;  // node chain of event j
  uint32_t pf_ev = CEP_NONE;      // node chain of the previous event (resolves kPending)
  int err = KE_OK;
  uint32_t err_seq = 0;
  uint32_t n_matches = 0, n_pairs = 0, out_first = CEP_NONE;
  // deferred walks
  uint32_t wq_n = 0;  // queued
  uint32_t wq_h = 0;  // queue slot of the oldest (the queue is a ring of wcap slots)
  uint32_t opc = 0;   // walks queued since the key started (walk ids)
  uint32_t pl_n = 0;  // put-log entries since the last flush
  uint32_t wt_last = CEP_NONE, wm0 = 0, wp0 = 0;  // event of the last walk run, counts before it
  uint32_t stop_j = CEP_NONE;  // CEP_STREAM_STOP: the event the key stopped before (KE_WIDEN)
#ifdef CEP_PROF
  unsigned long long prof[14] = {};  // the time split (see CEP_PROF above), this wave / lane
  // lane 0 adds the wave's cycles, the lane counters summed over the wave
  __device__ void prof_flush() {
    for (int i = 9; i < 12; i++)
      for (int o = 32; o > 0; o >>= 1) prof[i] += __shfl_xor(prof[i], o, 64);
    if ((threadIdx.x & 63) == 0) {
      for (int i = 0; i < 12; i++) atomicAdd(A.prof + i, prof[i]);
      atomicMax(A.prof + 12, prof[12]);
      atomicMax(A.prof + 13, prof[13]);
    }
  }
#endif

  __device__ Lane(const NfaArgs& a, Q& qq) : A(a), q(qq) {}

  __device__ __forceinline__ v4u* QP(uint32_t h, uint32_t slot, int quad) const {
    return rb + ((uint64_t)(h * A.rcap + slot) * Lay::kQuads + quad) * 64;
  }
  __device__ __forceinline__ v4u* WQ(uint32_t i, int quad) const {
    return wb + ((uint64_t)i * kWalkQuads + quad) * 64;
  }
  // the slot of the i-th queued walk
  __device__ __forceinline__ uint32_t wq_slot(uint32_t i) const {
    const uint32_t q = wq_h + i;
    return q >= A.wcap ? q - A.wcap : q;
  }
  __device__ __forceinline__ v4u* PL(uint32_t i) const { return wb + ((uint64_t)A.wcap * kWalkQuads + i) * 64; }
  // put-log entries one event may add at most (its records' puts): the wave drains before
  __device__ __forceinline__ uint32_t plog_margin() const {
    return 2 * A.rcap + 4 < A.plog / 2 ? 2 * A.rcap + 4 : A.plog / 2;
  }
  __device__ __forceinline__ lds_v4u* LQ(uint32_t h, uint32_t slot, int lq) const {
    return lr + ((h * kRL + slot) * Lay::kLdsQuads + lq) * 64;
  }
  // quad `quad` (compile-time) of a queue slot, from LDS or HBM
  __device__ __forceinline__ bool lds_slot(uint32_t slot, int quad) const {
    return kRL > 0 && Lay::in_lds(quad) && slot < kRL;
  }
  // quad `quad` of a slot every active lane of the wave reads at once (the queue loops): the
  // LDS-or-HBM choice on the scalar unit
  __device__ __forceinline__ v4u rd_u(uint32_t h, uint32_t slot, int quad) const {
    if (kRL > 0 && Lay::in_lds(quad) && CEP_UNIFORM(slot) < kRL) return *LQ(h, slot, Lay::lds_quad(quad));
    return *QP(h, slot, quad);
  }
  __device__ __forceinline__ v4u rd(uint32_t h, uint32_t slot, int quad) const {
    if (lds_slot(slot, quad)) return *LQ(h, slot, Lay::lds_quad(quad));
    return *QP(h, slot, quad);
  }
  __device__ __forceinline__ void wr(uint32_t h, uint32_t slot, int quad, const v4u& v) const {
    if (lds_slot(slot, quad)) *LQ(h, slot, Lay::lds_quad(quad)) = v;
    else *QP(h, slot, quad) = v;
  }
  // streaming: the LDS slots of the queue (half `half`, `count` records) <-> their HBM positions
  __device__ __forceinline__ void lds_spill(bool to_hbm) {
    for (uint32_t s = 0; s < kRL && s < count; s++) {
#pragma unroll
      for (int k = 0; k < Lay::kQuads; k++)
        if (Lay::in_lds(k)) {
          if (to_hbm) *QP(half, s, k) = *LQ(half, s, Lay::lds_quad(k));
          else *LQ(half, s, Lay::lds_quad(k)) = *QP(half, s, k);
        }
    }
  }

  // ---------------------------------------------------------------- records
  // `pf`: node chain that resolves a pending ev_first (the event the record was made at)
  // (`slot` is wave-uniform at every call - the queue loops step record i of every lane together -
  // so one scalar branch picks LDS or HBM for all of the record's quads and their loads go out
  // together: a choice per quad on a slot the compiler takes for divergent cost a wait each)
  __device__ __forceinline__ void load(uint32_t h, uint32_t slot, Rec<F>& r, uint32_t pf, v4u* raw = nullptr) const {
    const bool lds = kRL > 0 && CEP_UNIFORM(slot) < kRL;
    v4u hd, d0, fqs[Lay::kFoldQuads];
    if (lds) {
      hd = *LQ(h, slot, 0);
      d0 = *LQ(h, slot, 1);
#pragma unroll
      for (int k = 0; k < Lay::kFoldQuads; k++) fqs[k] = *LQ(h, slot, Lay::lds_quad(1 + Lay::kDwQuads + k));
    } else {
      hd = *QP(h, slot, 0);
      d0 = *QP(h, slot, 1);
#pragma unroll
      for (int k = 0; k < Lay::kFoldQuads; k++) fqs[k] = *QP(h, slot, 1 + Lay::kDwQuads + k);
    }
    if (raw) *raw = hd;
    r.stage = hd.x & kStageMask;
    r.event = hd.y;
    r.ev_first = hd.z == kPending ? pf : hd.z;
    r.node = hd.w;
    r.ver.n = hd.x >> 24;
#pragma unroll
    for (int k = 0; k < Lay::kDwRegQuads; k++) {
      // (pairs past the first two: HBM at every slot, and only when the version has them)
      v4u dq = d0;
      if (k > 0) dq = (uint32_t)(2 * k) < r.ver.n ? *QP(h, slot, 1 + k) : v4u{0, 0, 0, 0};
      r.ver.v[2 * k] = (int32_t)dq.x;
      r.ver.c[2 * k] = dq.y;
      if (2 * k + 1 < kDeweyPairs) {
        r.ver.v[2 * k + 1] = (int32_t)dq.z;
        r.ver.c[2 * k + 1] = dq.w;
      }
    }
    uint32_t len = 0;  // DeweyVersion.length(): the digits of every pair
#pragma unroll
    for (int k = 0; k < kDeweyPairs; k++)
      if ((uint32_t)k < r.ver.n) len += r.ver.c[k];
    r.ver.len = len;
    uint32_t w[Lay::kFoldQuads * 4];
#pragma unroll
    for (int k = 0; k < Lay::kFoldQuads; k++) {
      const v4u fq = fqs[k];
      w[4 * k] = fq.x;
      w[4 * k + 1] = fq.y;
      w[4 * k + 2] = fq.z;
      w[4 * k + 3] = fq.w;
    }
    r.nullmask = w[0];
#pragma unroll
    for (int s = 0; s < F; s++)
      r.fold[s] = Q::kFold32 ? (int64_t)(int32_t)w[1 + s] : (int64_t)(((uint64_t)w[3 + 2 * s] << 32) | w[2 + 2 * s]);
  }

  __device__ __forceinline__ void store_head(uint32_t h, uint32_t slot, uint32_t stage, uint32_t event,
                                             uint32_t ev_first, const Dewey& ver0, uint32_t node, uint32_t flags = 0) {
    const Dewey ver = dw_pin(ver0);
    // the header and the first pairs: one branch for both (LDS slot or HBM), then pairs past the
    // first two (HBM at every slot)
    const v4u q0 = v4u{stage | flags | (ver.n << 24), event, ev_first, node};
    const v4u q1 = v4u{(uint32_t)ver.v[0], ver.c[0], 1 < kDeweyPairs ? (uint32_t)ver.v[1 < kDeweyPairs ? 1 : 0] : 0u,
                       1 < kDeweyPairs ? ver.c[1 < kDeweyPairs ? 1 : 0] : 0u};
    if (kRL > 0 && slot < kRL) {
      *LQ(h, slot, 0) = q0;
      *LQ(h, slot, 1) = q1;
    } else {
      *QP(h, slot, 0) = q0;
      *QP(h, slot, 1) = q1;
    }
#pragma unroll
    for (int k = 1; k < Lay::kDwRegQuads; k++)
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
      if (Q::kFold32) {
        w[1 + s] = (uint32_t)(uint64_t)v[s];
      } else {
        w[2 + 2 * s] = (uint32_t)(uint64_t)v[s];
        w[3 + 2 * s] = (uint32_t)((uint64_t)v[s] >> 32);
      }
    }
    if (kRL > 0 && slot < kRL) {
#pragma unroll
      for (int k = 0; k < Lay::kFoldQuads; k++)
        *LQ(h, slot, Lay::lds_quad(1 + Lay::kDwQuads + k)) = v4u{w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]};
    } else {
#pragma unroll
      for (int k = 0; k < Lay::kFoldQuads; k++)
        *QP(h, slot, 1 + Lay::kDwQuads + k) = v4u{w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]};
    }
  }

  // (a record moved to another slot: its twin flags do not hold there; `from` is wave-uniform:
  // the finals' compaction steps slot i of every lane together)
  __device__ __forceinline__ void copy_rec(uint32_t h, uint32_t from, uint32_t to) {
#pragma unroll
    for (int k = 0; k < Lay::kQuads; k++) {
      v4u q4 = rd_u(h, from, k);
      if (k == 0) q4.x &= ~(kTwin | kTwinT);
      wr(h, to, k, q4);
    }
  }

  // Appends an output record (header + version) and returns its slot, -1 when the queue is
  // full.  ev_first of a record whose event is the current one is only known once the
  // event's nodes exist: kPending, resolved at its next load.  Folds: set_folds.
  // `keep`: a non-consuming re-add of the record being stepped (IGNORE, NFA.java:225): its folds
  // are the record's own, and with its own version (the same Dewey length: on this path the
  // version is the record's with zero or more addStage digits) and head it is the same record -
  // at its own HBM slot, the twin slots spare its rewrite (header above).
  __device__ __forceinline__ int push_rec(uint32_t stage, uint32_t event, uint32_t ev_first, const Dewey& ver,
                                          uint32_t node = CEP_NONE, bool keep = false) {
#if CEP_STREAM_STOP && defined(CEP_TEST_WIDEN)
    // (tests/lane_cpu: stops at pseudo-random records mid-event, after earlier records' puts,
    // pushes and walks, so the undo and the continuation are exercised on every query)
    if (A.carry && ev_pos == j && ((j * 2654435761u) ^ (key * 40503u) ^ (ocount * 97u)) % CEP_TEST_WIDEN == 0) {
      err = KE_WIDEN;
      return -1;
    }
#endif
    if (ocount >= A.rcap) {
      err = KE_RETRY;
      if (A.full) atomicOr(A.full, 1u);
      return -1;
    }
    const uint32_t slot = ocount++;
    const uint32_t ef = (event == j && ev_first == CEP_NONE) ? kPending : ev_first;
    if (stage & kRecFinal) n_final++;
    // (on the keep path the stage word, event and node hint are the record's own - sw is its
    // stage word with its own branching flag - so the head differs from the stored one only
    // when the stored ev_first was kPending: in_info bit kInPend)
    if (keep && slot == in_slot && slot >= kRL && (in_info & kInPend) == 0 && ver.len == (in_info & 0xFFFFu)) {
      if (!(in_info & kTwin)) {  // the output copy is stale: written whole, marked the input's twin
        store_head(half ^ 1u, slot, stage, event, ef, ver, node, kTwin);
        return (int)slot;
      }
      // the output copy already holds it: at most its header's flags, never its folds
      CEP_STAT(9);
      pend_slot = slot;
      if (!(in_info & kTwinT))
        wr(half ^ 1u, slot, 0, v4u{stage | kTwin | kTwinT | (ver.n << 24), event, ef, node});
      return (int)slot;
    }
    store_head(half ^ 1u, slot, stage, event, ef, ver, node);
    return (int)slot;
  }

  __device__ __forceinline__ void set_folds(int slot, const int64_t* v, uint32_t nm) {
    if ((uint32_t)slot == pend_slot) {  // a kept twin: its folds are in place (push_rec)
      pend_slot = CEP_NONE;
      return;
    }
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
  // A node's first predecessor lives in its own slot of A.preds0 (same index as the node,
  // pred id kPred0 | node); later ones come from the predecessor pool.  A walk step then
  // reads the node and its first predecessor with four independent 16-B loads - one memory
  // round trip per node instead of three (node -> pointer -> its version).
  __device__ __forceinline__ v4u* NQ(uint32_t i, int k) const { return reinterpret_cast<v4u*>(A.nodes + i) + k; }
  __device__ __forceinline__ Pred& PR(uint32_t p) const {
    return (p & kPred0) ? A.preds0[p & ~kPred0] : A.preds[p];
  }
  __device__ __forceinline__ v4u* PQ(uint32_t p, int k) const { return reinterpret_cast<v4u*>(&PR(p)) + k; }

  // node (sk, event of the chain); CEP_NONE when absent or deleted.  (Pool quads are read as
  // 16-B vectors; v4u is may_alias, so the field writes of the same bytes stay ordered.)
  __device__ __forceinline__ uint32_t lookup(uint32_t sk, uint32_t first) {
    for (uint32_t i = first; i != CEP_NONE;) {
      CEP_STAT(6);
      const v4u q1 = *NQ(i, 1);  // {same_next, meta, lk, -}
      if ((q1.y & 0xFF) == sk) return (q1.y & 0x100) ? i : CEP_NONE;
      i = q1.x;
    }
    return CEP_NONE;
  }

  __device__ __forceinline__ void write_pred(uint32_t p, uint32_t prev, const Dewey& v0, uint32_t next = CEP_NONE) {
    const Dewey v = dw_pin(v0);
    *PQ(p, 0) = v4u{prev, next, v.n << 8, v.len};
#pragma unroll
    for (int k = 0; k < (kDeweyPairs + 1) / 2; k++)
      if ((uint32_t)(2 * k) < v.n)
        *PQ(p, 1 + k) = v4u{(uint32_t)v.v[2 * k], v.c[2 * k],
                            2 * k + 1 < kDeweyPairs ? (uint32_t)v.v[2 * k + 1] : 0u,
                            2 * k + 1 < kDeweyPairs ? v.c[2 * k + 1] : 0u};
  }

  // a new node at event j holding one predecessor (prev, v) in its first-pred slot: both
  // written as whole quads
  __device__ __forceinline__ uint32_t new_node(uint32_t sk, uint32_t prev, const Dewey& v) {
    const uint32_t i = pool_take(A.node_pool, ncur, nend);
    if (i == CEP_NONE) {
      err = KE_RETRY;
      return CEP_NONE;
    }
    const uint32_t p = kPred0 | i;
    write_pred(p, prev, v);
    *NQ(i, 0) = v4u{j, 1u, p, p};
    *NQ(i, 1) = v4u{cur_first, sk | 0x100u | (1u << 16), 0u, key};
    cur_first = i;
    return i;
  }

  // appends (prev, v) to an existing node of event j
  __device__ __forceinline__ void append_pred(uint32_t node, uint32_t prev, const Dewey& v) {
    const uint32_t p = pool_take(A.pred_pool, pcur, pend);
    if (p == CEP_NONE) {
      err = KE_RETRY;
      return;
    }
    // (both quads of the node read together, written whole: it is a node of the current event,
    // which no queued walk reads before the next flush)
    const v4u q0 = *NQ(node, 0), q1 = *NQ(node, 1);  // {event, refs, head, tail}, {same_next, meta, lk, key}
    write_pred(p, prev, v);
    if (q0.z != CEP_NONE) PR(q0.w).next = p;
    *NQ(node, 0) = v4u{q0.x, q0.y, q0.z == CEP_NONE ? p : q0.z, p};
    *NQ(node, 1) = v4u{q1.x, q1.y + (1u << 16), q1.z, q1.w};
  }

  // put(stage, evt, version)  KVSharedVersionedBuffer.java:117-128 (overwrites)
  __device__ __forceinline__ uint32_t put_begin(uint32_t sk, const Dewey& v) {
    const uint32_t c = lookup(sk, cur_first);
    if (c == CEP_NONE) return new_node(sk, CEP_NONE, v);
    // a new TimedKeyValue with one pointer: the node's first-pred slot, rewritten (the node is
    // of the current event: no queued walk can read its old pointers)
    const uint32_t p = kPred0 | c;
    write_pred(p, CEP_NONE, v);
    Node& n = A.nodes[c];
    n.refs = 1;
    n.head = p;
    n.tail = p;
    n.meta = sk | 0x100u | (1u << 16);
    return c;
  }

  // put(curr, currEvent, prev, prevEvent, version)  :80-97;  prev_sk == kNoSk: put(begin).
  // (hint_sk, hint): the putting record's node hint; returns the node of (sk, j) (CEP_NONE
  // on an error)
  __device__ __forceinline__ uint32_t put_link(uint32_t sk, uint32_t prev_sk, uint32_t prev_ev, uint32_t prev_first,
                                               const Dewey& v, uint32_t hint_sk = kNoSk, uint32_t hint = CEP_NONE) {
    if (prev_sk == kNoSk) return put_begin(sk, v);
    if (prev_ev == CEP_NONE) {  // prevEvent.topic on a null Event
      err = KE_NPE;
      return CEP_NONE;
    }
    uint32_t p;
    if (A.defer && hint != CEP_NONE && prev_sk == hint_sk) p = hint;
    else p = lookup(prev_sk, prev_first);
    if (p == CEP_NONE) {  // "Cannot find predecessor event"
      err = KE_ILLEGAL_STATE;
      return CEP_NONE;
    }
#if CEP_PUT_LOG
    if (A.defer && wq_n > 0) {  // found live while walks are queued: stamp and log (conflict check)
      if (pl_n >= A.plog) {         // (only an event with more puts than plog_margin())
        err = A.carry ? KE_CAPACITY : KE_CONFLICT;
        return CEP_NONE;
      }
      A.nodes[p].lk = opc;
      *PL(pl_n++) = v4u{p, opc, j, 0u};
    }
#else
    // found live after `opc` queued walks (conflict check; only a walk queued before this put
    // can conflict with it: none is when the queue is empty)
    if (A.defer && wq_n > 0) A.nodes[p].lk = opc;
#endif
    const uint32_t c = lookup(sk, cur_first);
    if (c == CEP_NONE) return new_node(sk, p, v);
    append_pred(c, p, v);
    return c;
  }

  // a flush (walks may delete nodes): the queued records' node hints no longer hold
  __device__ __forceinline__ void clear_hints() {
    for (uint32_t i = 0; i < count; i++) {
      v4u hd = rd_u(half, i, 0);
      if (hd.w != CEP_NONE) {
        hd.w = CEP_NONE;
        hd.x &= ~(kTwin | kTwinT);  // (changed in place: no longer its twin's copy)
        wr(half, i, 0, hd);
      }
    }
  }

  // TimedKeyValue.getPointerByVersion  TimedKeyValue.java:83-92, from the node's list head:
  // the first live pointer whose version the walker is compatible with; its key and version
  // come back in prev / ver
  // `pre`/`pre0`/`pre1`: the two first quads of pointer `pre`, already loaded (a walk step's
  // node's first-pred slot)
  // `pflags` (optional): the chosen pointer's flags word, as loaded
  __device__ __forceinline__ uint32_t first_compat(uint32_t head, const Dewey& walker, uint32_t& prev, Dewey& ver,
                                                   uint32_t pre = CEP_NONE, v4u pre0 = v4u{0, 0, 0, 0},
                                                   v4u pre1 = v4u{0, 0, 0, 0}, bool* same = nullptr,
                                                   uint32_t* pflags = nullptr) {
    for (uint32_t p = head; p != CEP_NONE;) {
      CEP_STAT(4);
      v4u e0 = pre0, d1 = pre1;
      if (p != pre) {  // the pointer and its first Dewey quad, loaded together
        e0 = *PQ(p, 0);
        d1 = *PQ(p, 1);
      }
      const uint32_t fl = e0.z, nxt = e0.y;
      if (!(fl & 1u)) {
        // the pointer's version is the walker's own (a run's chain: the common case):
        // compatible, and the walker keeps its version (*same)
        const uint32_t en = (fl >> 8) & 0xFF;
        if (same && en <= 2 && en == walker.n && e0.w == walker.len &&
            (en < 1 || ((int32_t)d1.x == walker.v[0] && d1.y == walker.c[0])) &&
            (en < 2 || ((int32_t)d1.z == walker.v[1] && d1.w == walker.c[1]))) {
          prev = e0.x;
          *same = true;
          if (pflags) *pflags = fl;
          return p;
        }
        if (en <= 2 && walker.n <= 2) {  // both short: compare straight from the quad
          if (dw_compat2(walker.n, walker.len, walker.v[0], walker.c[0], walker.v[1], walker.c[1], en, e0.w,
                         en >= 1 ? (int32_t)d1.x : 0, en >= 1 ? d1.y : 0u, en >= 2 ? (int32_t)d1.z : 0,
                         en >= 2 ? d1.w : 0u)) {
            prev = e0.x;
            Dewey e;
            dw_init(e, en >= 1 ? (int32_t)d1.x : 0);
            e.n = en;
            e.len = e0.w;
            e.c[0] = en >= 1 ? d1.y : 0u;
            e.v[1] = en >= 2 ? (int32_t)d1.z : 0;
            e.c[1] = en >= 2 ? d1.w : 0u;
            ver = dw_pin(e);
            if (pflags) *pflags = fl;
            return p;
          }
          p = nxt;
          continue;
        }
        Dewey e;
        e.n = en;
        e.len = e0.w;
#pragma unroll
        for (int k = 0; k < (kDeweyPairs + 1) / 2; k++) {
          v4u d = k == 0 ? d1 : v4u{0, 0, 0, 0};
          if (k > 0 && (uint32_t)(2 * k) < e.n) d = *PQ(p, 1 + k);
          if (k == 0 && e.n == 0) d = v4u{0, 0, 0, 0};
          e.v[2 * k] = (int32_t)d.x;
          e.c[2 * k] = d.y;
          if (2 * k + 1 < kDeweyPairs) {
            e.v[2 * k + 1] = (int32_t)d.z;
            e.c[2 * k + 1] = d.w;
          }
        }
        if (dw_compatible(walker, e)) {
          prev = e0.x;
          ver = dw_pin(e);
          if (pflags) *pflags = fl;
          return p;
        }
      }
      p = nxt;
    }
    return CEP_NONE;
  }

  // ---------------------------------------------------------------- output stream
  __device__ __forceinline__ uint64_t out_put(uint32_t w) {
    if (ochunk == CEP_NONE || opos == kOutChunkWords - 1) {
      // chunks come from the lane's range in hand, refilled A.out_pool.chunk at a time: one
      // atomic on the pool's single counter per range (a chunk per atomic serialised ~26M
      // same-address atomics per config-5 batch)
      const uint32_t c = pool_take(A.out_pool, ocur, oend);
      if (c == CEP_NONE) {
        err = KE_RETRY;
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

  // two words (a pair's event id and stage name): one chunk check, two stores
  __device__ __forceinline__ void out_put2(uint32_t w0, uint32_t w1) {
    if (ochunk != CEP_NONE && opos + 2 <= kOutChunkWords - 1) {
      uint32_t* d = A.out + (uint64_t)ochunk * kOutChunkWords + opos;
      d[0] = w0;
      d[1] = w1;
      opos += 2;
      return;
    }
    out_put(w0);
    out_put(w1);
  }

  // ---------------------------------------------------------------- walks
  // branch  KVSharedVersionedBuffer.java:99-110;  peek(remove=true)  :143-171 (emit: the
  // match construction's Sequence).  In place when !A.defer, else queued (see the header).
  __device__ __forceinline__ void walk(uint32_t flags, uint32_t sk, uint32_t ev, uint32_t first, const Dewey& v0,
                                      uint32_t hint = CEP_NONE) {
    CEP_STAT(2);
    if (CEP_WALK_IN_PLACE && !A.defer) {  // (in place: hints are not kept valid)
      walk_now(flags, sk, ev, first, v0, j);
      return;
    }
    if (hint != CEP_NONE) {
      flags |= kWalkHint;
      first = hint;
    }
    if (wq_n >= A.wcap) {  // more walks in one event than the queue holds: re-run in place
      err = A.carry ? KE_CAPACITY : KE_CONFLICT;  // (a stream cannot re-run: session.cpp sizes it)
      return;
    }
    const Dewey v = dw_pin(v0);
    const uint32_t q = wq_slot(wq_n);
    *WQ(q, 0) = v4u{sk | (flags << 8) | (v.n << 24), ev, first, v.len};
#pragma unroll
    for (int k = 0; k < (kDeweyPairs + 1) / 2; k++)
      if ((uint32_t)(2 * k) < v.n)
        *WQ(q, 1 + k) = v4u{(uint32_t)v.v[2 * k], v.c[2 * k],
                            2 * k + 1 < kDeweyPairs ? (uint32_t)v.v[2 * k + 1] : 0u,
                            2 * k + 1 < kDeweyPairs ? v.c[2 * k + 1] : 0u};
    reinterpret_cast<uint32_t*>(WQ(q, kWalkQuads - 1))[0] = j;
    wq_n++;
    opc++;
  }
  // `hint`: the node (sk, ev) when the caller knows it (a record's node hint), else CEP_NONE
  __device__ __forceinline__ void walk_branch(uint32_t sk, uint32_t ev, uint32_t first, const Dewey& v,
                                             uint32_t hint = CEP_NONE) {
    walk(kWalkBranch, sk, ev, first, v, hint);
  }
  __device__ __forceinline__ void walk_remove(uint32_t sk, uint32_t ev, uint32_t first, const Dewey& v, bool emit,
                                             uint32_t hint = CEP_NONE) {
    walk(emit ? kWalkEmit : 0u, sk, ev, first, v, hint);
  }

  // a walk of event t threw: nothing of event t is forwarded, the key stops at t
  __device__ __forceinline__ void walk_fail(int code, uint32_t t) {
    err = code;
    err_seq = t;
    n_matches = wm0;
    n_pairs = wp0;
  }

  __device__ __forceinline__ void walk_begin(uint32_t t) {
    if (t != wt_last) {
      wt_last = t;
      wm0 = n_matches;
      wp0 = n_pairs;
    }
  }

  // A walk step's reads: the node and its first-pred slot, four independent 16-B loads (one
  // memory round trip)
  struct WalkPre {
    v4u n0, n1, f0, f1;  // {event, refs, head, tail}, {same_next, meta, lk, key}, first pointer quads 0-1
  };
  // (both addresses are materialised before the first load: otherwise the compiler computes
  // the second address into registers the first load is still writing and waits for it
  // in between - two round trips instead of one)
  __device__ __forceinline__ void walk_load(uint32_t s, WalkPre& P) const {
    const v4u* na = NQ(s, 0);
    const v4u* pa = reinterpret_cast<const v4u*>(A.preds0 + s);
    asm volatile("" : "+v"(na), "+v"(pa));
    typedef __attribute__((address_space(1))) const v4u gv4u;  // the pools are global memory
    const gv4u* gn = (const gv4u*)na;
    const gv4u* gp = (const gv4u*)pa;
    P.n0 = gn[0];
    P.n1 = gn[1];
    P.f0 = gp[0];
    P.f1 = gp[1];
    // (all four in flight before the step branches on any: otherwise the compiler sinks the
    // pointer loads into the live-node branch, a second dependent round trip per hop)
    asm volatile("" : "+v"(P.n0), "+v"(P.n1), "+v"(P.f0), "+v"(P.f1));
  }

  // One node of a walk at node s with walker version w.  Returns false when the walk ends (or
  // fails); s/w advance to the next node otherwise.  `wid`: the walk's id (deferred).
  // (Prefetching the next node ahead of this step's stores was measured: 4 % on the heavy
  // walk bench, but 16 more live VGPRs across the drain loop cost cfg 3's kernel 11 % in
  // spills; the step loads its own node.)
  // the put-log entry of the first put after walk `wid` that found node `s` live (CEP_NONE: none)
  __device__ __forceinline__ uint32_t first_put_after(uint32_t s, uint32_t wid) const {
    for (uint32_t i = 0; i < pl_n; i++) {
      const v4u e = *PL(i);
      if (e.x == s && e.y > wid) return i;
    }
    return CEP_NONE;
  }

  // `conf` (deferred walks): set to the node when its delete conflicts with a later put
  __device__ __forceinline__ bool walk_node(uint32_t flags, uint32_t& s, Dewey& w, uint32_t t, uint32_t wid,
                                            uint32_t& np, uint32_t& conf) {
    if (s == CEP_NONE) {
      walk_fail(KE_NPE, t);
      return false;
    }
    CEP_STAT(3);
    CEP_HOP(key, t, s, flags, w);
    CEP_PACC(11, 1);
    Node& n = A.nodes[s];
    WalkPre P;
    walk_load(s, P);
    const v4u n0 = P.n0, n1 = P.n1, f0 = P.f0, f1 = P.f1;
    const uint32_t ev_s = n0.x, head = n0.z, lk = n1.z, cur = s;
    uint32_t meta = n1.y;
    if (!(meta & 0x100)) {
      walk_fail(KE_NPE, t);
      return false;
    }
    const int32_t refs = (int32_t)n0.y;
    int32_t left = 1, nrefs;
    bool del = false;
    if (flags & kWalkBranch) {
      nrefs = refs + 1;
    } else {
      // (fused: the skipped branch walk's +1 and this walk's -1 - refs stays, left = refs)
      left = (flags & kWalkFused) ? refs : refs == 0 ? 0 : refs - 1;
      nrefs = left;
      if (left == 0 && (meta >> 16) <= 1) {  // store.delete
        if (A.defer && lk > wid) {  // a put made after this walk was queued found the node live:
#if CEP_PUT_LOG
          // in the reference the first such put throws (header); the walk itself completes, the
          // drain loop finds that put (fewer live registers there than in the step)
          conf = s;
#else
          walk_fail(KE_CONFLICT, t);  // (the narrow build: the key is re-run in the wide one)
          return false;
#endif
        }
        del = true;
      }
    }
    uint32_t nx = CEP_NONE, pfl = 0, p;
    Dewey nv;
    bool same = false;
    const uint32_t en = (f0.z >> 8) & 0xFF;
    const int32_t bv0 = en >= 1 ? (int32_t)f1.x : 0, bv1 = en >= 2 ? (int32_t)f1.z : 0;
    const uint32_t bc0 = en >= 1 ? f1.y : 0u, bc1 = en >= 2 ? f1.w : 0u;
#if CEP_WALK_COMPAT2
    // kernel groups (config 5: walk-heavy jobs): any compatible short version of the first
    // pointer takes the straight-line step
    bool fast = head == (kPred0 | cur) && !(f0.z & 1u) && en <= 2 && w.n <= 2;
    same = fast && en == w.n && f0.w == w.len && (en < 1 || (bv0 == w.v[0] && bc0 == w.c[0])) &&
           (en < 2 || (bv1 == w.v[1] && bc1 == w.c[1]));
    if (fast && !same) fast = dw_compat2(w.n, w.len, w.v[0], w.c[0], w.v[1], w.c[1], en, f0.w, bv0, bc0, bv1, bc1);
    if (fast && !same) {
      dw_init(nv, bv0);
      nv.n = en;
      nv.len = f0.w;
      nv.c[0] = bc0;
      nv.v[1] = bv1;
      nv.c[1] = bc1;
    }
#else
    // single queries: only the exact version (fewer live registers in the drain loop: the
    // wider test cost cfg 3's kernel ~11 % in spills)
    same = head == (kPred0 | cur) && !(f0.z & 1u) && en <= 2 && en == w.n && f0.w == w.len &&
           (en < 1 || (bv0 == w.v[0] && bc0 == w.c[0])) && (en < 2 || (bv1 == w.v[1] && bc1 == w.c[1]));
    const bool fast = same;
#endif
    if (fast) {
      // the common step, straight-line: the node's first pointer is live and carries the
      // walker's own version (a run's chain) - first_compat's answer without its loop
      // (first_compat compares other short versions from the quad, dw_compat2)
      p = kPred0 | cur;
      nx = f0.x;
      pfl = f0.z;
    } else {
      p = first_compat(head, w, nx, nv, kPred0 | cur, f0, f1, &same, &pfl);
    }
    const bool more = p != CEP_NONE && nx != CEP_NONE;
    n.refs = nrefs;
    if (del) meta &= ~0x100u;
    if (p != CEP_NONE && left == 0) {  // removePredecessor(pointer)
      PR(p).flags = pfl | 1u;
      meta -= 1u << 16;
    }
    if (del || (p != CEP_NONE && left == 0)) n.meta = meta;
    if (!(flags & kWalkBranch) && (flags & kWalkEmit)) {
      out_put2(ev_s, q.sk_name(meta & 0xFF));
      np++;
      if (err) {
        walk_fail(err, t);
        return false;
      }
    }
    if (!more) return false;
    if (!same) w = nv;  // a value, not a pointer into the pool
    s = nx;
    return true;
  }

  __device__ __forceinline__ bool walk_start(uint32_t flags, uint32_t sk, uint32_t ev, uint32_t first, uint32_t t,
                                             uint32_t& s, uint64_t& npa, uint32_t& np) {
    walk_begin(t);
    if (ev == CEP_NONE) {
      walk_fail(KE_NPE, t);
      return false;
    }
    s = (flags & kWalkHint) ? first : lookup(sk, first);
    np = 0;
    if (flags & kWalkEmit) {
      out_put(t);
      npa = out_put(0);
      if (err) {
        walk_fail(err, t);
        return false;
      }
    }
    return true;
  }

  __device__ __forceinline__ void walk_end(uint32_t flags, uint64_t npa, uint32_t np) {
    if (flags & kWalkEmit) {
      A.out[npa] = np;
      n_matches++;
      n_pairs += np;
    }
  }

  __device__ __forceinline__ void walk_now(uint32_t flags, uint32_t sk, uint32_t ev, uint32_t first, const Dewey& v,
                                           uint32_t t) {
    uint32_t s = CEP_NONE, np = 0;
    uint64_t npa = 0;
    if (!walk_start(flags, sk, ev, first, t, s, npa, np)) return;
    Dewey w = dw_pin(v);
    uint32_t conf = CEP_NONE;  // (in place: no conflicts)
    while (walk_node(flags, s, w, t, 0, np, conf)) {
    }
    if (!err) walk_end(flags, npa, np);
  }

  // Drains this lane's queue in order.  Called by every lane of the wave at once (convergent:
  // the loop's cross-lane operations see every lane; `part` false: this lane takes part with
  // nothing to walk): the loop gives each lane one node per iteration, starting its next walk
  // as soon as one ends.
  // `may_stop` (partial drain): once at most half the lanes that had walks are still walking,
  // this lane starts no further walk while fewer than kWalkFlush remain queued - the rest stay
  // queued, in order, for a later flush (the wave goes back to its events instead of waiting
  // for the longest queue).  Exact as any deferral: the put stamps and the put log cover the
  // walks still queued (the log keeps the entries they can conflict with).
  __device__ __forceinline__ void flush(bool may_stop = false, bool part = true) {
    CEP_STAT(5);
    if (part && wq_n) {  // this lane's walks may delete its nodes (no other lane's can)
      clear_hints();
    }
    const uint32_t id0 = opc - wq_n;
    uint32_t i = 0, s = CEP_NONE, t = 0, flags = 0, np = 0;
    uint64_t npa = 0;
    Dewey w;
    dw_init(w, 0);
    bool active = false, draining = part;
#if CEP_WALK_FUSE
    uint32_t fuse_at = CEP_NONE;  // the absorbed branch walk's start node (the fused mode from there)
#endif
    uint32_t cut = CEP_NONE;   // put-log entry of the first put a walk's delete makes throw
    uint32_t conf = CEP_NONE;  // the node of this step's conflicting delete
#if CEP_PARTIAL_DRAIN == 1
    const uint32_t n_start = (uint32_t)__popcll(__ballot(part && wq_n > 0));
#endif
    for (;;) {
      const uint64_t in = __ballot(draining);  // the lanes still draining
      if (!in) break;
#if CEP_PARTIAL_DRAIN == 1
      const bool stop = may_stop && 2 * (uint32_t)__popcll(in) <= n_start;
#elif CEP_PARTIAL_DRAIN == 2
      const bool stop = may_stop;
#else
      const bool stop = false;
#endif
      if (!draining) continue;
      if (!active) {
        // (walks queued after the first put a conflict makes throw never run)
        if (i >= wq_n || err || (cut != CEP_NONE && id0 + i >= PL(cut)->y)) {
          draining = false;
          continue;
        }
        // (no partial stop once a conflict was found: every walk queued before that put runs
        // first, as in the reference, before the key stops at the put's event)
        if (stop && cut == CEP_NONE && wq_n - i < kWalkFlush) {
          draining = false;
          continue;
        }
        const uint32_t qs = wq_slot(i);
        const v4u h = *WQ(qs, 0);
        flags = (h.x >> 8) & 0xFF;
        w.n = h.x >> 24;
        w.len = h.w;
#pragma unroll
        for (int k = 0; k < (kDeweyPairs + 1) / 2; k++) {
          // (quad 0 with the header: an entry's version has a pair)
          v4u d = {0, 0, 0, 0};
          if (k == 0 || (uint32_t)(2 * k) < w.n) d = *WQ(qs, 1 + k);
          w.v[2 * k] = (int32_t)d.x;
          w.c[2 * k] = d.y;
          if (2 * k + 1 < kDeweyPairs) {
            w.v[2 * k + 1] = (int32_t)d.z;
            w.c[2 * k + 1] = d.w;
          }
        }
        w = dw_pin(w);
        t = reinterpret_cast<const uint32_t*>(WQ(qs, kWalkQuads - 1))[0];
        i++;
        v4u hs = h;
#if CEP_WALK_FUSE
        fuse_at = CEP_NONE;
        // a branch walk directly followed by an extraction of the same event that retraces it
        // (CEP_WALK_FUSE above): skip it, the extraction absorbs it from its start node on
        if ((flags & kWalkBranch) && i < wq_n && (cut == CEP_NONE || id0 + i < PL(cut)->y)) {
          const uint32_t qe = wq_slot(i);
          const v4u he = *WQ(qe, 0);
          const uint32_t fe = (he.x >> 8) & 0xFF;
          if ((fe & (kWalkEmit | kWalkBranch | kWalkHint)) == (kWalkEmit | kWalkHint) &&
              reinterpret_cast<const uint32_t*>(WQ(qe, kWalkQuads - 1))[0] == t) {
            const uint32_t sb = (flags & kWalkHint) ? h.z : lookup(h.x & 0xFF, h.z);
            Dewey we;
            we.n = he.x >> 24;
            we.len = he.w;
#pragma unroll
            for (int k = 0; k < (kDeweyPairs + 1) / 2; k++) {
              v4u d = {0, 0, 0, 0};
              if (k == 0 || (uint32_t)(2 * k) < we.n) d = *WQ(qe, 1 + k);
              we.v[2 * k] = (int32_t)d.x;
              we.c[2 * k] = d.y;
              if (2 * k + 1 < kDeweyPairs) {
                we.v[2 * k + 1] = (int32_t)d.z;
                we.c[2 * k + 1] = d.w;
              }
            }
            we = dw_pin(we);
            const uint32_t nf = he.z;  // N_f (the final record's node hint)
            const v4u f0 = *NQ(nf, 0), f1 = *NQ(nf, 1);
            if (sb != CEP_NONE && (f1.y & 0x100)) {
              uint32_t nx = CEP_NONE;
              Dewey nv;
              bool same = false;
              const uint32_t p = first_compat(f0.z, we, nx, nv, CEP_NONE, v4u{0, 0, 0, 0}, v4u{0, 0, 0, 0}, &same);
              if (p != CEP_NONE && nx == sb && dw_equal(same ? we : nv, w)) {
                fuse_at = sb;
                flags = fe;
                w = we;
                hs = he;
                i++;
              }
            }
          }
        }
#endif
        if (!walk_start(flags, hs.x & 0xFF, hs.y, hs.z, t, s, npa, np)) {
          draining = false;
          continue;
        }
        active = true;
      }
      CEP_STAT(7);
#if CEP_WALK_FUSE
      if (s == fuse_at && s != CEP_NONE) {
        flags |= kWalkFused;
        fuse_at = CEP_NONE;
      }
#endif
      const bool more = walk_node(flags, s, w, t, id0 + i - 1, np, conf);
      if (conf != CEP_NONE) {
        const uint32_t k = first_put_after(conf, id0 + i - 1);
        conf = CEP_NONE;
        if (k == CEP_NONE) {  // (a stamp without its log entry: never; re-run to be safe)
          walk_fail(A.carry ? KE_CAPACITY : KE_CONFLICT, t);
          draining = false;
          continue;
        }
        CEP_STAT(8);
        if (cut == CEP_NONE || PL(k)->y < PL(cut)->y) cut = k;  // (the earliest such put)
      }
      if (!more) {
        if (err) {
          draining = false;
          continue;
        }
        walk_end(flags, npa, np);
        active = false;
      }
    }
    if (!part) return;
    if (cut != CEP_NONE && !err) {  // IllegalState at that put's event: its matches dropped
      const uint32_t ce = PL(cut)->z;
      if (wt_last == ce) {
        n_matches = wm0;
        n_pairs = wp0;
      }
      err = KE_ILLEGAL_STATE;
      err_seq = ce;
    }
    if (i < wq_n && !err) {  // a partial drain: walks [i, wq_n) stay queued
      wq_h = wq_slot(i);
      wq_n -= i;
      // the put-log entries a remaining walk (id >= id0 + i) can conflict with: put id > walk id
      uint32_t k = 0;
      for (uint32_t e = 0; e < pl_n; e++) {
        const v4u x = *PL(e);
        if (x.y > id0 + i) {
          if (k != e) *PL(k) = x;
          k++;
        }
      }
      pl_n = k;
      return;
    }
    pl_n = 0;
    wq_n = 0;
    wq_h = 0;
  }

  // ---------------------------------------------------------------- one event
  // event() = event_pre(), the records (event_records()), event_post(): the begin run, the
  // queue swap and the finals.
  EvT nev;             // the next event's fields, prefetched by event_pre (consumed at the next event)
  bool nmore = false;  // there is a next event

  __device__ __forceinline__ void event_pre() {
    CEP_STAT(0);
    CEP_PACC(10, 1);
    pf_ev = cur_first;  // node chain of the previous event: resolves kPending
    cur_first = CEP_NONE;
    n_final = 0;
    ocount = 0;
    // prefetch the next event's fields (consumed by the next event)
    nev = ev;
    nmore = j + 1 < j0 + n_ev;
    if (nmore) q.load_ev(nev, base + j + 1);
  }

  // the queued records, one after another (NFA.java:99-107)
  __device__ __forceinline__ void event_records() {
    const uint32_t n = count;
    for (uint32_t i = 0; i < n; i++) {
      Rec<F> c;
      CEP_STAT(1);
      v4u raw;
      load(half, i, c, pf_ev, &raw);
      in_slot = i;
      in_info = (c.ver.len & 0xFFFFu) | (raw.x & (kTwin | kTwinT)) | (raw.z == kPending ? kInPend : 0u);
      const int produced = q.step(*this, c);
      in_slot = CEP_NONE;
      if (err) return;
      CEP_PACC(9, 1);
      if (produced == 0) {  // removePattern
        walk_remove(q.stage_sk(c.stage), c.event, c.ev_first, c.ver, false, (c.stage & kRecEps) ? c.node : CEP_NONE);
        if (err) return;
      }
    }
  }

  __device__ __forceinline__ void event_post(bool begin_hit) {
    CEP_PT(te1);
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
      b.node = CEP_NONE;
      b.nullmask = (1u << F) - 1;
#pragma unroll
      for (int s = 0; s < F; s++) b.fold[s] = 0;
      dw_init(b.ver, (int32_t)bdig);
      q.step(*this, b);
      if (err) return;
    }
    CEP_PT(te2);
    CEP_PACC(3, te2 - te1);
    const uint32_t oh = half ^ 1u;
    half = oh;
    count = ocount;
    if (nmore) {
      ev = nev;
      ev_pos = j + 1;
    }
    if (!n_final) {
      CEP_PT(te3);
      CEP_PACC(4, te3 - te2);
      return;
    }
    // matchConstruction: finals in order, then drop them from the queue
    uint32_t w = 0;
    for (uint32_t i = 0; i < count; i++) {
      const v4u hd = rd_u(oh, i, 0);
      if (hd.x & kRecFinal) {
        Rec<F> r;
        load(oh, i, r, cur_first);
        walk_remove(q.stage_sk(r.stage), r.event, r.ev_first, r.ver, true, (r.stage & kRecEps) ? r.node : CEP_NONE);
        if (err) return;
      } else {
        if (w != i) copy_rec(oh, i, w);
        w++;
      }
    }
    count = w;
    CEP_PT(te4);
    CEP_PACC(4, te4 - te2);
  }

  __device__ __forceinline__ void event(bool begin_hit) {
    CEP_PT(te0);
    event_pre();
    event_records();
    CEP_PT(te9);
    CEP_PACC(2, te9 - te0);
    if (err) return;
    event_post(begin_hit);
  }

  // ---------------------------------------------------------------- the key's stream
  // Lanes of a wavefront advance in lockstep; a lane whose queue holds only the begin run
  // (whose single BEGIN edge did not match) is in the reference's quiet state: an event
  // that fails the begin predicate changes nothing (the begin run is re-added with the same
  // version, NFA.java:149-157), so the lane tests kQuietChunk events per step with their
  // loads issued together.
  __device__ __forceinline__ bool only_begin() const {
    if (kBeginReg) return count == 0;
    if (count != 1) return false;
    return (rd(half, 0, 0).x & kStageMask) == q.begin_stage;
  }

  // ---------------------------------------------------------------- the job's event loop
  // tick() runs one step of the loop over the key's events (the quiet skip or one event);
  // false once the events are over (jj == jn) or the step threw (pa_err).  finish() is the
  // final drain of the deferred walks, after which err holds the job's outcome: a walk's
  // exception precedes a step exception queued after it (the reference's order).
  uint32_t jj = 0, jn = 0;  // next event, end
  int pa_err = KE_OK;       // an exception of the per-event step (walks queued before it go first)
  uint32_t pa_seq = 0;

  // tick_pre: the quiet skip, then this tick's event: 2 an event at jj (j set, its fields
  // loaded; `known`: the begin predicate already found true), 1 no event this tick (a quiet
  // chunk scanned), 0 the events are over or the quiet scan threw (pa_err).
  __device__ __forceinline__ int tick_pre(bool& known) {
    CEP_PT(tq0);
    known = false;
    if (q.quiet && A.bhits && only_begin()) {
      // the next event whose begin predicate holds or throws, 64 positions per word;
      // event() evaluates the predicate there itself (its exception, in order)
      uint64_t p = base + jj;
      uint64_t w = A.bhits[p >> 6] >> (p & 63);
      while (!w) {
        jj += 64 - (uint32_t)(p & 63);
        if (jj >= jn) break;
        p = base + jj;
        w = A.bhits[p >> 6];
      }
      if (jj >= jn) {
        jj = jn;
        return 0;
      }
      jj += (uint32_t)__builtin_ctzll(w);
      if (jj >= jn) {
        jj = jn;
        return 0;
      }
    } else if (q.quiet && only_begin()) {
      const uint32_t lim = (jn - jj > kQuietChunk) ? jj + kQuietChunk : jn;
      const uint32_t h = q.begin_scan(*this, jj, lim);
      if (err) {
        pa_err = err;
        pa_seq = h;
        return 0;
      }
      if (h >= lim) {
        jj = lim;
        return jj < jn ? 1 : 0;
      }
      jj = h;
      known = true;  // the scan already found the begin predicate true
    }
    CEP_PT(tq1);
    CEP_PACC(1, tq1 - tq0);
    j = jj;
    if (ev_pos != jj) {
      q.load_ev(ev, base + jj);
      ev_pos = jj;
    }
    return 2;
  }

  // after the event at jj: false once the events are over or the step threw (pa_err)
  __device__ __forceinline__ bool tick_post() {
    if (err) {
      pa_err = err;
      pa_seq = jj;
      return false;
    }
    jj++;
    return jj < jn;
  }

  __device__ __forceinline__ bool tick() {
    bool known = false;
    const int st = tick_pre(known);
    if (st != 2) return st == 1;
#if CEP_STREAM_STOP
    const uint32_t wq0 = wq_n;
    event(known);
    if (err == KE_WIDEN) {
      stop_event(wq0);
      return false;
    }
#else
    event(known);
#endif
    return tick_post();
  }

#if CEP_STREAM_STOP
  // The stream build's versions outgrew 3 pairs at event j (kDwFull): the key stops BEFORE j, as
  // the previous event left it, and the wide build continues it from j (run_key, session.cpp).
  // What event j did so far is undone - no walk runs inside an event, so it touched only:
  //  - the walks it queued: dropped (ids reused: the continuation queues the same ones);
  //  - the nodes of (_, j) it made or rewrote (its chain, cur_first): dead, unreachable from
  //    any record or pointer of an older event; cur_first back to event j - 1's chain;
  //  - records written to the other queue half: never read (half and count stay), but a twin
  //    slot there (kTwin) may have been overwritten: the input records' twin flags are cleared;
  //  - stamps and put-log entries of the puts that found a node live: kept.  The stop's drain
  //    (run: the walks queued before j) then finds the conflicts the reference would throw at j
  //    (IllegalState at a put of j that precedes the overflowing record), and a stamp left for
  //    the continuation is the one its identical put writes again (same walks queued before it).
  __device__ __forceinline__ void stop_event(uint32_t wq0) {
    opc -= wq_n - wq0;
    wq_n = wq0;
    for (uint32_t i = cur_first; i != CEP_NONE;) {
      v4u n1 = *NQ(i, 1);
      const uint32_t nx = n1.x;
      n1.y &= ~0x100u;
      *NQ(i, 1) = n1;
      i = nx;
    }
    cur_first = pf_ev;
    for (uint32_t i = 0; i < count; i++) {
      v4u hd = rd(half, i, 0);
      if (hd.x & (kTwin | kTwinT)) {
        hd.x &= ~(kTwin | kTwinT);
        wr(half, i, 0, hd);
      }
    }
    stop_j = j;
    err = KE_OK;
  }
#endif

  // the step's exception, after the final drain found nothing earlier (drained: flush() ran)
  __device__ __forceinline__ void finish_err() {
    if (!err && pa_err != KE_OK) {
      err = pa_err;
      err_seq = pa_seq;
    }
  }

  // the whole key in one go (streaming sessions and single queries: one key per lane and
  // launch).  Convergent: every lane of the wave takes each iteration (a lane whose events are
  // over idles in it, as SIMT execution would mask it), so the flushes' cross-lane operations
  // see the whole wave.
  __device__ __forceinline__ void run() {
    CEP_PT(tr0);
#ifdef CEP_PROF
    const uint64_t tw0 = wall_clock64();
#endif
    jj = j0;
    jn = j0 + n_ev;
    pa_err = KE_OK;
    bool more = jj < jn;
    while (__any(more)) {
      CEP_PACC(8, more ? 1 : 0);
      CEP_PT(tf0);
      if (A.defer && __any(more && (wq_n >= kWalkFlush || pl_n + plog_margin() > A.plog))) {
        flush(pl_n + plog_margin() <= A.plog, more);
        if (more && err) more = false;  // a walk threw: the key stops there
      }
      CEP_PT(tf1);
      CEP_PACC(0, tf1 - tf0);
      if (more) more = tick();
    }
    CEP_PT(tr1);
    // the final drain, every lane of the wave together (lanes whose walk threw mid-stream take
    // part with nothing to walk)
    const bool fin = pa_err != KE_OK || !err;
    if (fin) err = KE_OK;
    flush(false, fin);
    if (fin) finish_err();
#ifdef CEP_PROF
    CEP_PT(tr2);
    CEP_PACC(5, tr2 - tr1);
    CEP_PACC(6, 1);
    CEP_PACC(7, tr2 - tr0);
    prof[12] = tr2 - tr0;
    prof[13] = wall_clock64() - tw0;
    if (A.prof) prof_flush();
#endif
  }

  // a fresh job: key `k`'s events of this batch from the NFA's initial state
  // (NFA.initComputationStates :74-81 — the begin stage, version 1, sequence 1).  The pool
  // chunks in hand (ncur/nend, pcur/pend) stay with the lane.
  __device__ __forceinline__ void begin_job(uint32_t k) {
    key = k;
    base = A.key_off[k];
    n_ev = (uint32_t)(A.key_off[k + 1] - base);
    j0 = 0;
    j = 0;
    ev_pos = CEP_NONE;
    half = 0;
    count = 0;
    ocount = 0;
    bdig = 1;
    n_final = 0;
    ochunk = CEP_NONE;
    opos = 0;
    cur_first = CEP_NONE;
    err = KE_OK;
    err_seq = 0;
    n_matches = n_pairs = 0;
    out_first = CEP_NONE;
    wq_n = 0;
    wq_h = 0;
    opc = 0;
    pl_n = 0;
    wt_last = CEP_NONE;
    wm0 = wp0 = 0;
    jj = 0;
    jn = n_ev;
    pa_err = KE_OK;
    pa_seq = 0;
    if (!kBeginReg) {
      Dewey v;
      dw_init(v, 1);
      half = 1;  // push_rec writes the other half: half 0
      readd_begin(q.begin_stage, v);
      half = 0;
      count = 1;
    }
  }
};

// job index -> (query, key) job id: explicit (retries) or query-minor over the lane order
__device__ __forceinline__ uint64_t job_id(const NfaArgs& A, uint64_t idx) {
  if (A.jobs) return A.jobs[idx];
  const uint32_t nq = A.n_q ? A.n_q : 1;
  const uint64_t rank = idx / nq;
  const uint32_t qi = (uint32_t)(idx % nq);
  return (uint64_t)qi * A.n_keys + (A.order ? A.order[rank] : rank);
}

// Persistent lanes (per-batch sessions).  The launch has about as many lanes as fit the chip;
// each lane runs job after job, claiming the next ones from a global counter, so a wave no
// longer waits for its slowest lane's key before taking new work: the lanes of a wave stay
// busy until the job list runs dry.  Jobs are claimed in list order - keys by estimated work,
// longest first (cep_nfa_est), queries interleaved - so the longest jobs start first.  Claims
// are wave-wide: one atomic per claiming round, the idle lanes taking consecutive jobs.  The
// deferred walks are drained wave-wide as before, and whenever a lane's job has reached its
// last event (its final drain); only then is the job's KeyState written.
template <int F, class Q>
__device__ __forceinline__ void run_jobs(const NfaArgs& A, Q& q, v4u* lds) {
  const uint64_t slot = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63;
  Lane<F, Q> L(A, q);
  L.rb = reinterpret_cast<v4u*>(A.rings) + (slot / 64) * (2ull * A.rcap * Lane<F, Q>::Lay::kQuads * 64) + lane;
  L.wb = reinterpret_cast<v4u*>(A.walks) + (slot / 64) * walkq_group_quads(A.wcap, A.plog) + lane;
  if (Lane<F, Q>::kRL > 0)  // (kRL == 0: never dereferenced)
    L.lr = (lds_v4u*)lds + (threadIdx.x / 64) * (2 * Lane<F, Q>::kRL * Lane<F, Q>::Lay::kLdsQuads * 64) + lane;
  bool has = false, drained = false;
  int phase = 0;  // 0 events, 1 final drain pending, 2 done
  uint64_t job = 0;
  // the wave's claimed job indices [wnext, wend) (wave-uniform): one atomic on the launch's
  // single counter per kClaim jobs instead of one per claiming round (lanes finish jobs one
  // at a time, so rounds mostly hand out a single job)
  constexpr uint32_t kClaim = 128;
  uint64_t wnext = 0, wend = 0;
  CEP_PT(tr0);
#ifdef CEP_PROF
  const uint64_t tw0 = wall_clock64();
#endif
  for (;;) {
    CEP_LPACC(L, 8, 1);
    const uint64_t need = __ballot(!has && !drained);
    if (need) {
      if (wnext == wend) {
        const int leader = __ffsll((unsigned long long)need) - 1;
        uint32_t first = 0;
        if ((int)lane == leader) first = atomicAdd(A.job_next, kClaim);
        wnext = __shfl(first, leader, 64);
        wend = wnext + kClaim;
      }
      const uint32_t cnt = (uint32_t)__popcll(need);
      const uint32_t take = (uint64_t)cnt < wend - wnext ? cnt : (uint32_t)(wend - wnext);
      const uint32_t rank = (uint32_t)__popcll(need & ((1ull << lane) - 1ull));
      if (!has && !drained && rank < take) {  // the others take theirs at the next round
        const uint64_t idx = wnext + rank;
        if (idx < A.n_jobs) {
          job = job_id(A, idx);
          q.set_query((uint32_t)(job / A.n_keys));
          L.begin_job((uint32_t)(job % A.n_keys));
          has = true;
          phase = L.jn > 0 ? 0 : (A.defer ? 1 : 2);
        } else {
          drained = true;
        }
      }
      wnext += take;
    }
    if (!__any(has)) break;
    // drain when a queue is long, when kJobDrain lanes wait for their final drain, or when no
    // lane has events left to run (the finished lanes' drains batched into one flush)
    const uint64_t ending = __ballot(has && phase == 1);
    CEP_PT(tf0);
    if (A.defer && (__any(has && (L.wq_n >= kWalkFlush || L.pl_n + L.plog_margin() > A.plog)) ||
                    (ending && (__popcll(ending) >= kJobDrain || !__any(has && phase == 0))))) {
      // every lane of the wave together (lanes without a queue leave at once); lanes at their
      // job's end drain all of theirs
      L.flush(has && phase == 0 && L.pl_n + L.plog_margin() <= A.plog);
      if (has && phase == 0 && L.err) phase = 2;  // a walk threw mid-job: the job stops there
      if (has && phase == 1) {
        L.finish_err();
        phase = 2;
      }
    }
    CEP_PT(tf1);
    CEP_LPACC(L, 0, tf1 - tf0);
    if (has && phase == 0 && !L.tick()) {
      // the events are over (or a step threw): the remaining walks drain at the next flush
      L.err = KE_OK;
      phase = 1;
      if (!A.defer) {
        L.finish_err();
        phase = 2;
      }
    }
    if (has && phase == 2) {
      KeyState& ks = A.ks[job];
      ks.n_matches = L.n_matches;
      ks.n_pairs = L.n_pairs;
      ks.out_first = L.out_first;
      ks.err = L.err;
      ks.err_seq = L.err_seq;
      if (L.err == KE_RETRY || L.err == KE_CONFLICT) atomicAdd(A.n_capacity_err, 1u);
      L.wq_n = 0;
      has = false;
    }
  }
#ifdef CEP_PROF
  CEP_PT(tr1);
  CEP_LPACC(L, 6, 1);
  CEP_LPACC(L, 7, tr1 - tr0);
  L.prof[12] = tr1 - tr0;
  L.prof[13] = wall_clock64() - tw0;
  if (A.prof) L.prof_flush();
#endif
}

// Driver shared by the AOT and JIT kernels: slot -> key, initial or carried state, the
// batch's events of the key, KeyState (and KeyCarry for the next batch of a stream).
#ifndef CEP_PERSIST_LANES
#define CEP_PERSIST_LANES 1
#endif
template <int F, class Q>
__device__ __forceinline__ void run_key(const NfaArgs& A, Q& q, v4u* lds = nullptr) {
#if CEP_PERSIST_LANES
  if (A.job_next) {  // per-batch sessions: persistent lanes over the job list
    run_jobs<F>(A, q, lds);
    return;
  }
#endif
  const uint64_t slot = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // A lane without a job stays in its wave with no events (has false): the wave-wide loops
  // read every lane of the wave, so none may have left.
  bool has = true;
  uint64_t job = 0;
  if (A.jobs) {
    if (slot >= A.n_jobs) has = false;
    else job = A.jobs[slot];
  } else {
    const uint32_t nq = A.n_q ? A.n_q : 1;
    const uint64_t w = slot / 64;
    // spread: the heaviest W keys (lane order) lead one wave each, the next W are their lanes 1,
    // ...; odd lanes take their row in reverse (wave 0's lane 1 is the row's lightest key), so
    // the waves of the heaviest keys carry the lightest neighbours
    const uint64_t l = slot % 64;
    uint64_t rank;
    if (A.spread && w >= A.spread) {  // (the grid's last block past the W waves: idle)
      rank = ~0ull;
    } else if (A.spread) {
      const uint64_t W = A.spread;
      rank = l * W + ((l & 1) ? W - 1 - w : w);
    } else if (A.spread_iso && w < A.spread_iso) {  // (lane order) the heaviest ranks alone
      rank = l == 0 ? w : ~0ull;
    } else if (A.spread_iso) {
      rank = A.spread_iso + (w - A.spread_iso) * 64 + l;
    } else {
      rank = (w / nq) * 64 + l;
    }
    if (rank >= A.n_keys) has = false;
    else job = (w % nq) * A.n_keys + (A.order ? A.order[rank] : rank);
  }
  if (!__any(has)) return;  // (the whole wave)
  const uint32_t qi = (uint32_t)(job / A.n_keys);
  const uint32_t key = (uint32_t)(job % A.n_keys);
  q.set_query(qi);
  Lane<F, Q> L(A, q);
  L.key = key;
  L.n_ev = has ? (uint32_t)(A.key_off[key + 1] - A.key_off[key]) : 0u;
  // a stream's run queue lives at its key's position (kept from batch to batch whatever lane
  // order the batch runs in); a per-batch launch's at the lane's slot (coalesced)
  const uint64_t rslot = A.carry ? job : slot;
  L.rb = reinterpret_cast<v4u*>(A.rings) +
         (rslot / 64) * (2ull * A.rcap * Lane<F, Q>::Lay::kQuads * 64) + (rslot % 64);
  L.wb = reinterpret_cast<v4u*>(A.walks) + (slot / 64) * walkq_group_quads(A.wcap, A.plog) + (slot % 64);
  if (Lane<F, Q>::kRL > 0)  // (kRL == 0: never dereferenced)
    L.lr = (lds_v4u*)lds + (threadIdx.x / 64) * (2 * Lane<F, Q>::kRL * Lane<F, Q>::Lay::kLdsQuads * 64) + (threadIdx.x % 64);
  KeyState& ks = A.ks[job];
  KeyCarry* kc = (A.carry && has) ? A.carry + job : nullptr;
  if (kc && kc->live && kc->err) {  // stopped by an exception: stays stopped
    ks.n_matches = ks.n_pairs = 0;
    ks.out_first = CEP_NONE;
    ks.err = kc->err;
    ks.err_seq = kc->err_seq;
    has = false;
    kc = nullptr;
    L.n_ev = 0;
  }
  uint32_t bseq = 0;  // sequence number of the batch's first event of the key
  if (kc && kc->live) {  // the key's NFA as the previous batch (or this batch's stop) left it
    L.j0 = kc->seq;
    bseq = L.j0;
    if (A.widen) {  // continue a key the stream build stopped (KE_WIDEN) at its event kc->seq
      bseq = kc->bseq;
      L.n_ev -= L.j0 - bseq;
      L.n_matches = ks.n_matches;
      L.n_pairs = ks.n_pairs;
      L.out_first = ks.out_first;
      L.ochunk = ks.ochunk;
      L.opos = ks.opos;
    }
    L.half = kc->half;
    L.count = kc->count;
    L.bdig = kc->bdig;
    L.cur_first = kc->cur_first;
    L.ncur = kc->ncur;
    L.nend = kc->nend;
    L.pcur = kc->pcur;
    L.pend = kc->pend;
    L.opc = kc->opc;
    L.lds_spill(false);  // the queue's first slots back into LDS
  } else {
    // NFA.initComputationStates :74-81 — the begin stage, version 1, sequence 1
    L.bdig = 1;
    L.half = 0;
    L.count = 0;
    if (!Lane<F, Q>::kBeginReg && has) {
      Dewey v;
      dw_init(v, 1);
      L.ocount = 0;
      L.half = 1;  // push_rec writes the other half: half 0
      L.readd_begin(q.begin_stage, v);
      L.half = 0;
      L.count = 1;
    }
  }
  L.base = has ? A.key_off[key] - bseq : 0;
  L.run();
  if (!has) return;
  ks.n_matches = L.n_matches;
  ks.n_pairs = L.n_pairs;
  ks.out_first = L.out_first;
  ks.err = L.err;
  ks.err_seq = L.err_seq;
  const bool stopped = L.stop_j != CEP_NONE && !L.err;  // (its drain threw: stopped for good)
  if (stopped) {
    ks.err = KE_WIDEN;
    ks.ochunk = L.ochunk;
    ks.opos = L.opos;
  }
  if (L.err == KE_RETRY || L.err == KE_CONFLICT || stopped) atomicAdd(A.n_capacity_err, 1u);
  if (kc) {
    if (!L.err) L.lds_spill(true);  // LDS ends with the launch: the queue continues from HBM
    kc->live = 1;
    kc->seq = stopped ? L.stop_j : L.j0 + L.n_ev;
    kc->bseq = bseq;
    kc->half = L.half;
    kc->count = L.count;
    kc->bdig = L.bdig;
    kc->cur_first = L.cur_first;
    kc->ncur = L.ncur;
    kc->nend = L.nend;
    kc->pcur = L.pcur;
    kc->pend = L.pend;
    kc->opc = L.opc;
    kc->err = L.err;
    kc->err_seq = L.err_seq;
  }
}

}  // namespace cep
