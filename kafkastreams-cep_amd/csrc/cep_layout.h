// cep_layout.h — device data layout shared by the host compiler and the HIP kernels.
//
// One reference NFA per key.  The reference keeps, per NFA (nfa/NFA.java:50-56):
//   a FIFO of ComputationStage run records      -> a per-key ring of Rec in HBM
//   KVSharedVersionedBuffer nodes + predecessor  -> pooled Node / Pred entries in HBM,
//     lists, keyed (stage name, type, offset)       found through a per-event node chain
//   ValueStore fold values keyed (state, run seq) -> inline fold registers in Rec
//   DeweyVersion int[]                           -> run-length encoded (value, count) pairs
// Layout rationale and the proofs behind the inline folds / node chains: DESIGN.md §3.
#pragma once
#include <stdint.h>

#define CEP_NONE 0xFFFFFFFFu

namespace cep {

constexpr int kMaxStages = 32;     // compiled stages per query (2m+1 for m patterns)
constexpr int kMaxStageKeys = 32;  // distinct (name, type) pairs
constexpr int kMaxFields = 16;
constexpr int kMaxStates = 8;      // fold state names per query (MAXF)
constexpr int kMaxAggs = 8;        // folds per pattern
constexpr int kMaxStack = 16;      // interpreter stack depth
// RLE pairs per Dewey version (overflow -> CEP_KEY_CAPACITY).  A generated kernel may be
// compiled with fewer ($CEP_DEWEY_PAIRS, measurement runs); host-side sizes always use 6.
#ifndef CEP_DEWEY_PAIRS
#define CEP_DEWEY_PAIRS 6
#endif
constexpr int kDeweyPairs = CEP_DEWEY_PAIRS;
// Pairs the memory layout has room for (run records, predecessor pointers, walk queue
// entries): a stream's state outlives a launch, so the stream build (3 pairs in registers,
// session.cpp) keeps the wide build's layout and a key it stops continues in the wide build.
#ifndef CEP_LAYOUT_PAIRS
#define CEP_LAYOUT_PAIRS CEP_DEWEY_PAIRS
#endif
constexpr int kLayoutPairs = CEP_LAYOUT_PAIRS;
static_assert(kLayoutPairs >= kDeweyPairs, "the layout holds every pair in registers");
constexpr int kMaxStencil = 8;     // stages of a CEP_KIND_STENCIL query (stencil.hip instantiations)

enum StateType : uint8_t { ST_BEGIN = 0, ST_NORMAL = 1, ST_FINAL = 2 };
enum EdgeOp : uint8_t { OP_BEGIN = 0, OP_TAKE = 1, OP_PROCEED = 2, OP_IGNORE = 3 };
// KE_CONFLICT: a deferred walk would have changed what the step saw, or one event queued more
// walks than the queue holds (nfa_lane.h); internal, the key is re-run with walks in place.  KE_RETRY: a resource of the launch ran out (run
// queue, walk queue, node / predecessor / output pool); internal, the key is re-run with more.
// KE_CAPACITY: a hard limit (Dewey RLE pairs, stage depth): final.  A KE_RETRY left after the
// last re-run is reported as KE_CAPACITY.  KE_WIDEN (streams, internal): the stream build's
// versions outgrew 3 pairs at an event; the key stopped before it and the wide build continues it
// (nfa_lane.h stop_event, session.cpp run_nfa).
enum KeyErr : int32_t {
  KE_OK = 0, KE_NPE = 1, KE_ILLEGAL_STATE = 2, KE_ARITH = 3, KE_CAPACITY = 16, KE_CONFLICT = 17, KE_RETRY = 18,
  KE_WIDEN = 19
};

constexpr uint16_t kProgTrue = 0xFFFF;

struct DevEdge {
  uint8_t op;
  uint8_t target;  // stage index (0xFF: none, IGNORE)
  uint16_t prog;   // predicate program offset in code[], kProgTrue = constant true
};

struct DevStage {
  uint8_t sk;      // interned (name, type) — Stage.equals / StateKey identity
  uint8_t type;    // StateType
  uint8_t n_edges;
  uint8_t n_aggs;
  DevEdge e[3];    // edge order [BEGIN|TAKE, IGNORE?, PROCEED?] (StatesFactory.java:80-107)
  uint16_t agg_state[kMaxAggs];
  uint16_t agg_prog[kMaxAggs];
};

struct DevQuery {
  uint32_t n_stages, n_sk, n_states, n_fields;
  uint32_t begin_stage;  // StatesFactory.make's last element (the only BEGIN stage)
  uint32_t code_len;     // words
  uint8_t sk_type[kMaxStageKeys];
  uint16_t sk_name[kMaxStageKeys];
  uint8_t field_type[kMaxFields];  // 1 int, 2 long, 3 double
  uint8_t state_type[kMaxStates];
  DevStage st[kMaxStages];
};

// ---- Dewey version, run-length encoded: digits = v[0] x c[0], v[1] x c[1], ...
struct Dewey {
  uint32_t n;    // pairs in use
  uint32_t len;  // number of digits (DeweyVersion.length())
  int32_t v[kDeweyPairs];
  uint32_t c[kDeweyPairs];
};

// ---- run record (ComputationStage, nfa/ComputationStage.java:29-157)
// stage word: [7:0] stage index (real) or epsilon target; [15:8] stage key; bit16 epsilon;
// bit17 branching flag.  Epsilon stages (Stage.newEpsilonState) are (source key, target).
constexpr uint32_t kRecEps = 1u << 16;
constexpr uint32_t kRecBranch = 1u << 17;
constexpr uint32_t kRecFinal = 1u << 18;  // transient: forwarding to $final (in-step only)

template <int F>
struct Rec {
  uint32_t stage;
  uint32_t event;     // sequence number of the run's last event within the key, CEP_NONE = null
  uint32_t ev_first;  // head of the node chain of `event` (CEP_NONE: none / pending)
  uint32_t node;      // the node (source stage key, event) when known and valid (nfa_lane.h), else CEP_NONE
  uint32_t nullmask;  // bit s: fold state s is null
  Dewey ver;
  int64_t fold[F];
};

// ---- buffer node (TimedKeyValue + its StackEventKey, nfa/buffer/impl/TimedKeyValue.java)
// Two 16-B quads, read and written as vectors: {event, refs, head, tail}, {same_next, meta, lk, key}
struct alignas(16) Node {
  uint32_t event;      // sequence number within key
  int32_t refs;        // TimedKeyValue.refs
  uint32_t head, tail; // predecessor list (Pred indices), insertion order
  uint32_t same_next;  // next node created at the same event (lookup chain)
  uint32_t meta;       // [7:0] stage key, bit8 live, [31:16] live predecessor count
  uint32_t lk;         // walks queued when put() last found this node live (deferred walks)
  uint32_t key;        // the key (job key) whose NFA made the node (cep_live_floor)
};

// pointer ids: kPred0 | node = the node's first-pointer slot (preds0[node]), else the pool
constexpr uint32_t kPred0 = 0x80000000u;

// ---- predecessor pointer (TimedKeyValue.Pointer): (version, key|null).  Four quads:
// {prev, next, removed | pairs << 8, Dewey length}, then the Dewey (value, count) pairs,
// two per quad (only quads holding live pairs are written or read)
struct alignas(16) Pred {
  uint32_t prev;   // node index of the key, CEP_NONE = null key
  uint32_t next;   // next Pred of the node, CEP_NONE = end
  uint32_t flags;  // bit0 removed, [15:8] Dewey pairs in use
  uint32_t len;
  uint32_t pair[2 * kLayoutPairs];  // v0, c0, v1, c1, ...
};

// ---- per-key NFA state carried from one batch to the next (streaming sessions): what the
// reference keeps in its NFA between process() calls (nfa/NFA.java:50-56) besides the run
// records (the ring) and the buffer (the pools)
struct KeyCarry {
  uint32_t live;       // 1 once the key's NFA exists (initComputationStates done)
  uint32_t seq;        // events consumed so far = sequence number of the next event
  uint32_t half, count;
  uint32_t bdig;       // begin run's version digit (kBeginReg)
  uint32_t cur_first;  // node chain of the last event (resolves its records' kPending)
  uint32_t ncur, nend, pcur, pend;  // pool chunks in hand
  uint32_t opc;        // walks queued so far (deferred-walk ids)
  int32_t err;         // sticky: the exception that stopped the key
  uint32_t err_seq;
  uint32_t bseq;       // KE_WIDEN: sequence number of the batch's first event of the key
  uint32_t west;       // lane order: the key's running work estimate (cep_nfa_est, compile.cpp)
  uint32_t pad;
};

// ---- per-key state kept between kernel phases
struct KeyState {
  uint32_t n_matches;
  uint32_t n_pairs;
  uint32_t out_first;  // first output chunk (CEP_NONE: no output)
  int32_t err;
  uint32_t err_seq;
  uint32_t ochunk, opos;  // KE_WIDEN: where the key's output continues
  uint32_t pad;
};

constexpr uint32_t kOutChunkWords = 256;  // output stream chunk (last word links the next)

// ---- interpreter bytecode (u32 words): op in [7:0], argument in [31:16]
enum Bc : uint8_t {
  BC_END = 0,
  BC_PUSH32,   // + 1 word (sign-extended)
  BC_PUSH64,   // + 2 words (lo, hi)
  BC_FIELD,    // arg field
  BC_TS,
  BC_SGET,     // arg state, nullable
  BC_SGETOR,   // arg state, pops the default
  BC_CURR,     // nullable
  BC_UNBOX,    // NPE if top is null
  BC_ARITH,    // arg = op(0 add,1 sub,2 mul,3 div,4 rem) | type << 4
  BC_NEG,      // arg type
  BC_CAST,     // arg = from | to << 4
  BC_CMP,      // arg = op(0 lt,1 le,2 gt,3 ge,4 eq,5 ne) | type << 4
  BC_NOT,
  BC_JF,       // arg = target word: top false -> jump keeping it, else pop
  BC_JT,       // arg = target word: top true -> jump keeping it, else pop
};

// put-log entries per lane of the deferred-walk queues (nfa_lane.h): every put one event can
// log (2 * rcap + 4 for rcap records) fits twice over, at least kPutLogMin
constexpr uint32_t kPutLogMin = 256;
__host__ __device__ inline uint32_t put_log_entries(uint32_t rcap) {
  const uint64_t need = 2ull * (2ull * rcap + 4);
  return need > kPutLogMin ? (uint32_t)need : kPutLogMin;
}

// lanes per key of the work-estimate kernel (compile.cpp cep_nfa_est; session.cpp sizes its grid
// with the same function): a power of two at least the bitmap words a mean key spans, 4..64.  A
// key's words are read one per lane, so a wave per key left most lanes idle on short keys (a
// streamed batch: ~100 events, 2-3 words per key)
__host__ __device__ inline uint32_t est_lanes(uint64_t n_events, uint64_t n_keys) {
  const uint64_t words = (n_keys ? n_events / n_keys : 0) / 64 + 2;
  uint32_t g = 4;
  while (g < 64 && g < words) g <<= 1;
  return g;
}

}  // namespace cep
