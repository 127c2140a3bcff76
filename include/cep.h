/* cep.h — C ABI of libcep.so, the MI355X-native CEP matcher.
 *
 * This is the drop-in boundary for the reference's hot path.  The reference runs one
 * NFA inside a Kafka Streams Processor and is driven record by record:
 *
 *   new CEPProcessor<>(pattern[, inMemory])            CEPProcessor.java:71-84
 *   CEPProcessor.init(ProcessorContext)                CEPProcessor.java:88-108
 *   CEPProcessor.process(K, V) -> context.forward(null, Sequence) per match
 *                                                      CEPProcessor.java:155-163
 *   NFA.matchPattern(K, V, long) -> List<Sequence>     nfa/NFA.java:94-109
 *   StatesFactory.make(Pattern) -> List<Stage>         pattern/StatesFactory.java:41-63
 *
 * Here a query (the serialised Pattern chain with its where/fold lambdas lowered to a
 * typed IR, see "Query IR" below) is compiled once (cep_query_compile ~ StatesFactory.make),
 * a session holds the per-key NFA state on one GPU (~ CEPProcessor.init + NFA), and records
 * arrive as key-partitioned column batches (cep_push_batch ~ a run of process() calls);
 * matches come back as flat arrays (cep_poll_matches ~ the forwarded Sequences).
 *
 * Semantics: one reference NFA per key ("key" = independent stream), results
 * bit-exact with the reference on the same inputs, including its exceptions, which are
 * reported per key (cep_key_errors) instead of killing the stream thread.
 *
 * Threading: a session is used from one thread at a time (the reference's Processor is
 * single-threaded too); sessions are independent.  All functions return CEP_OK (0) or a
 * negative CEP_E_* status; cep_last_error() has the message (thread-local).
 */
#ifndef CEP_H_
#define CEP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CEP_ABI_VERSION 1

/* ---- status codes ---- */
#define CEP_OK 0
#define CEP_E_INVALID (-1)   /* bad argument */
#define CEP_E_HIP (-2)       /* HIP runtime error */
#define CEP_E_NOMEM (-3)     /* device allocation failed */
#define CEP_E_COMPILE (-4)   /* query compile error (see cep_query_compile) */
#define CEP_E_STATE (-5)     /* call out of order */

/* ---- per-key error codes: the reference exception that would escape process() ---- */
#define CEP_KEY_OK 0
#define CEP_KEY_NPE 1            /* NullPointerException (null fold unboxing, H2/H3 walks, ...) */
#define CEP_KEY_ILLEGAL_STATE 2  /* IllegalStateException "Cannot find predecessor event"
                                    (nfa/buffer/impl/KVSharedVersionedBuffer.java:86-89) */
#define CEP_KEY_ARITHMETIC 3     /* ArithmeticException (integer / or % by zero in a lambda) */
#define CEP_KEY_CAPACITY 16      /* this build only: a per-key limit (live runs, Dewey width,
                                    buffer pools) was exceeded; never silent */
#define CEP_KEY_CONFLICT 17      /* internal: a deferred buffer walk would have changed what a
                                    later step saw; such keys are re-run with walks in place and
                                    the code never reaches the caller */

/* ---- compile-time errors, returned in cep_query_info.compile_error ---- */
#define CEP_COMPILE_NPE 1              /* pattern ending in a Kleene/optional stage (StatesFactory:102) */
#define CEP_COMPILE_ILLEGAL_ARGUMENT 4 /* a pattern without where() (Stage.java:159) */

/* ---- Query IR (produced by kafkastreams-cep_amd/pattern.py Pattern.to_ir) ----
 * little-endian; str = u16 length + UTF-8 bytes
 *   "CEPQ" u32 version(=1)
 *   u16 n_fields  { u8 type; str name }      event columns (type: 1=int 2=long 3=double)
 *   u16 n_states  { u8 type; str name }      fold states (boxed Integer/Long/Double)
 *   u16 n_names   { str name }               distinct stage names (output stage ids index this)
 *   u16 n_patterns, first to last:
 *       u16 name; u8 cardinality (0 ONE,1 OPTIONAL,2 ZERO_OR_MORE,3 ONE_OR_MORE);
 *       u8 strategy (0 STRICT,1 SKIP_TIL_NEXT,2 SKIP_TIL_ANY); u8 has_window; i64 window_ms;
 *       u8 has_pred; [expr]; u16 n_aggs { u16 state; expr }
 *   expr (prefix): u8 op, then
 *     01 CONST_I32 i32 | 02 CONST_I64 i64 | 03 CONST_F64 f64 | 04 CONST_BOOL u8
 *     05 FIELD u16 | 06 TS | 07 STATE_GET u16 (nullable) | 08 STATE_GET_OR u16 expr(default)
 *     09 CURR (nullable; fold only)
 *     10 ADD 11 SUB 12 MUL 13 DIV 14 REM: u8 type, expr, expr   (Java int/long/double rules)
 *     15 NEG u8 type expr | 18 CAST u8 from u8 to expr
 *     20 LT 21 LE 22 GT 23 GE 24 EQ 25 NE: u8 operand type, expr, expr
 *     30 AND expr expr | 31 OR expr expr | 32 NOT expr   (short-circuit, left first)
 *   Operands are already promoted (explicit CASTs); a nullable operand is unboxed where used.
 */

typedef struct cep_query cep_query;
typedef struct cep_session cep_session;

typedef struct {
  uint32_t n_patterns;
  uint32_t n_stages;      /* compiled stages incl. $final and ONE_OR_MORE wrappers */
  uint32_t n_names;       /* stage-name ids 0..n_names-1 used in match output */
  uint32_t n_fields;
  uint32_t n_states;
  uint32_t kind;          /* CEP_KIND_* : which kernel runs this query */
  uint32_t arity;         /* CEP_KIND_STENCIL: events per match (else 0) */
  int32_t compile_error;  /* 0, CEP_COMPILE_NPE or CEP_COMPILE_ILLEGAL_ARGUMENT */
} cep_query_info;

#define CEP_KIND_NFA 0      /* general NFA kernel (runs, shared versioned buffer, folds) */
#define CEP_KIND_STENCIL 1  /* proven specialisation: all stages ONE + strict, total
                               state-free predicates, distinct names */

/* Compile a serialised Pattern chain.  On a reference compile-time exception the call
 * still succeeds and info.compile_error says which (sessions then refuse the query). */
int cep_query_compile(const uint8_t* ir, size_t n, cep_query** out);
int cep_query_info_get(const cep_query* q, cep_query_info* info);
/* stage name of id `name_id` (UTF-8, NUL-terminated, owned by the query) */
const char* cep_query_stage_name(const cep_query* q, uint32_t name_id);
void cep_query_destroy(cep_query* q);
/* The generated C++ of the query's NFA step (what CEP_TIER_JIT compiles), owned by the query. */
const char* cep_query_jit_source(const cep_query* q);
/* Compile the query's JIT kernel into the on-disk code-object cache without a GPU
 * ($CEP_JIT_CACHE, default <libcep.so dir>/jit_cache); sessions then load it directly.  A
 * cache hit refreshes the entry's mtime (stale entries can be pruned by age). */
int cep_jit_precompile(const cep_query* q, double* compile_s);
/* The same for the kernel groups a session over these queries would launch (cep_opts.no_groups
 * = 0): one code object per group of queries that differ only in literals. */
int cep_jit_precompile_group(const cep_query* const* queries, int n_queries, double* compile_s);
/* Kernel group `group` of a session over these queries: its members (query indices), the
 * generated source and the per-query literal table (members x n_literals, row-major).  Arrays
 * are owned by the library until the next call on this thread.  CEP_E_INVALID past the last
 * group.  (Introspection: which queries share a launch, and what it compiles.) */
int cep_query_group_plan(const cep_query* const* queries, int n_queries, int group, const char** source,
                         uint32_t* n_members, const int32_t** members, uint32_t* n_literals,
                         const int64_t** literals);

#define CEP_TIER_JIT 0     /* NFA queries run their own kernel, generated and compiled by hipRTC */
#define CEP_TIER_INTERP 1  /* NFA queries run the precompiled bytecode-interpreter kernel */

typedef struct {
  int device;             /* HIP device ordinal */
  int force_nfa;          /* 1: run CEP_KIND_STENCIL queries on the general NFA kernel */
  int tier;               /* CEP_TIER_JIT (default) or CEP_TIER_INTERP */
  uint32_t max_runs;      /* live runs per key (0 = default 32); retried x8 on overflow */
  double pool_factor;     /* buffer pool size per event of the batch (0 = default) */
  int streaming;          /* 1: a key's NFA state carries over from one batch to the next (its
                             events in consecutive batches are one stream, sequence numbers
                             continue; every batch has the same n_keys); 0: every batch starts
                             every key from the initial state */
  int no_groups;          /* 1: every NFA query runs its own launch.  0 (default): in a per-batch
                             JIT session, queries that differ only in literal values (config 5's
                             64 variants) run as one kernel launch, lanes = (query, key), reading
                             the batch's columns once for all of them */
} cep_opts;

int cep_session_create(const cep_query* const* queries, int n_queries, const cep_opts* opts,
                       cep_session** out);
void cep_session_destroy(cep_session* s);

#define CEP_MEM_HOST 0
#define CEP_MEM_DEVICE 1

/* A key-partitioned (CSR) column batch: events of key k are positions
 * key_off[k] .. key_off[k+1]-1, in arrival order.  cols[f] holds n_events values of the
 * IR field type f.  ts may be NULL (timestamps are not read by WITHIN in the reference:
 * its windows never prune).  Buffer lifetime: see cep_push_batch. */
typedef struct {
  uint64_t n_keys;
  uint64_t n_events;
  const uint64_t* key_off;  /* [n_keys + 1] (NULL for an arrival-order batch) */
  const void* const* cols;  /* [n_fields] */
  const int64_t* ts;        /* [n_events] or NULL */
  int memory;               /* CEP_MEM_HOST or CEP_MEM_DEVICE */
  /* Arrival-order batch: instead of key_off, the key (< n_keys) of every event, the events
   * and cols/ts in the order the records arrived (a run of CEPProcessor.process calls).  The
   * batch is partitioned on the device (stable: each key keeps its arrival order);
   * cep_batch_layout gives the resulting CSR layout and the arrival index of each position. */
  const uint32_t* arrival_key;  /* [n_events] or NULL */
} cep_batch;

/* Runs every query of the session over the batch: a run of process() calls per key.  In a
 * streaming session (cep_opts.streaming) the batch continues each key's stream where the
 * previous batch left it (run queue, shared buffer, folds, sequence numbers); otherwise every
 * batch starts every key from the NFA's initial state.  A streaming session cannot re-run a
 * key: one that hits a limit (CEP_KEY_CAPACITY: size max_runs for the query) stops there,
 * like a key whose query threw; its buffer walks run in place (no CEP_KEY_CONFLICT), and
 * stencil-kind queries run on the NFA kernel.
 * Buffer lifetime.  CEP_MEM_HOST batches are copied to the device before the call returns:
 * their buffers are borrowed for the call only.  CEP_MEM_DEVICE batches are read in place:
 * NFA batches finish before the call returns, but stencil-kind queries and the watermark
 * run asynchronously on the session stream, so a device batch stays borrowed until the next
 * result call on the session (cep_poll_matches, cep_match_digest, cep_key_errors,
 * cep_watermark, cep_last_timing/stats, cep_timing_totals), the next push, cep_sync or
 * cep_session_destroy returns. */
int cep_push_batch(cep_session* s, const cep_batch* b);

/* Streaming sessions: every key back to the NFA's initial state (NFA.initComputationStates,
 * nfa/NFA.java:74-81) - run queues, buffer nodes and sequence numbers dropped, device
 * allocations kept for the next stream.  A no-op for per-batch sessions (every batch starts
 * fresh there). */
int cep_session_reset(cep_session* s);

/* Layout of the last batch as the matchers saw it: key_off [n_keys + 1] and, for an
 * arrival-order batch, arrival_index [n_events] (the arrival position of each CSR position;
 * NULL for a CSR batch).  Arrays live in `memory` space until the next push/destroy.
 * partition_ms: device time of the partition (0 for a CSR batch). */
int cep_batch_layout(cep_session* s, int memory, const uint64_t** key_off, const uint32_t** arrival_index,
                     double* partition_ms);
int cep_sync(cep_session* s);

/* Matches of query `query` for the last batch, ordered by key then emission order (the
 * order the reference forwards them per key).  A match is the Sequence walk of
 * KVSharedVersionedBuffer.remove (nfa/buffer/impl/KVSharedVersionedBuffer.java:143-171):
 * pairs (stage name id, event) from the final event back to the first; events are given
 * as sequence numbers within the key (CSR position = key_off[key] + seq).
 * CEP_KIND_STENCIL queries return fixed-arity matches: pair_off/pair_stage are NULL,
 * match i owns pairs [i*arity, (i+1)*arity) with stage ids arity_stage[0..arity-1].
 * Arrays live in `memory` space and stay valid until the next push/poll/destroy. */
typedef struct {
  uint64_t n_matches;
  uint64_t n_pairs;
  uint32_t arity;                /* 0: variable-length (use pair_off) */
  const uint16_t* arity_stage;   /* host memory, [arity] (fixed-arity only) */
  const uint32_t* key;           /* [n_matches] */
  const uint32_t* emit_seq;      /* [n_matches] event whose arrival completed the match */
  const uint64_t* pair_off;      /* [n_matches + 1] or NULL */
  const uint32_t* pair_seq;      /* [n_pairs] */
  const uint16_t* pair_stage;    /* [n_pairs] or NULL */
  int memory;
} cep_matches;

int cep_poll_matches(cep_session* s, int query, int memory, cep_matches* out);

/* Per-key reference exceptions of the last batch: code[k] (CEP_KEY_*) and the sequence
 * number of the event whose processing threw (matches of earlier events are kept). */
int cep_key_errors(cep_session* s, int query, int32_t* code, uint32_t* seq, uint64_t n_keys);

/* Order-independent match checksum (Σ over matches of a 64-bit hash of key, emit and the
 * pair list) and count, computed on the device: what ranks all-gather over RCCL. */
int cep_match_digest(cep_session* s, int query, uint64_t* n_matches, uint64_t* checksum);

/* Largest timestamp of the last batch (INT64_MIN without ts): the rank-local watermark
 * that multi-GPU runs reduce with min. */
int cep_watermark(cep_session* s, int64_t* out);

/* Device time of the last batch, per query, from HIP events recorded on the session
 * stream (ms): the matching kernel launches (kernel_ms, `launches` of them: the NFA kernel
 * incl. capacity retries, or stencil_mask + stencil_emit) and the
 * setup/compaction kernels (aux_ms; 0 for a stencil batch, whose 4 us key-index pass is left
 * unbracketed: an event marker costs the stream about as much). */
/* ---- streaming-session snapshot / restore ----
 * The reference's persistent mode stores the NFA's run queue and buffer nodes after every
 * record (CEPProcessor.java:121-131,159-160; nfa/ComputationStageSerDe.java:53-125;
 * nfa/buffer/impl/TimedKeyValueSerDes.java:42-63) and reloads them in init().  Here the
 * complete per-key NFA state of a streaming session (cep_opts.streaming = 1) is one
 * versioned blob.  cep_session_snapshot(s, NULL, 0, &size) returns the size; with a buffer
 * of at least that size it writes the blob (the session is unchanged).  cep_session_restore
 * loads a blob into a streaming session created over the same queries and max_runs; the
 * next cep_push_batch continues every key's stream where the snapshot left it.  Blobs from
 * other queries, options or versions are rejected with CEP_E_INVALID before any change. */
int cep_session_snapshot(cep_session* s, void* buf, size_t cap, size_t* size);

/* Streaming sessions: floor[k] = the smallest sequence number of key k's events that a live
 * node of the query's shared buffer still holds (0xFFFFFFFF: none) - the only events a later
 * match of the key can contain (KVSharedVersionedBuffer.java:143-171 deletes a node when its
 * last reference is walked).  A host that keeps records to build Sequences may drop the older
 * ones.  floor is host memory [n_keys]; n_keys <= the session's key space. */
int cep_live_floor(cep_session* s, int query, uint32_t* floor, uint64_t n_keys);
int cep_session_restore(cep_session* s, const void* buf, size_t size);

int cep_last_timing(cep_session* s, int query, double* kernel_ms, double* aux_ms, uint32_t* launches);

/* The same device times summed over every batch since the last reset (reset != 0 zeroes
 * them after reading), and the number of batches.  Stencil batches return from
 * cep_push_batch without a host sync (pushes queue on the session stream); their event
 * pairs are read here and by every result call (poll, digest, timing, watermark), so a
 * caller can push many batches and time them all without stalling the pipeline. */
int cep_timing_totals(cep_session* s, int query, int reset, double* kernel_ms, double* aux_ms, uint64_t* batches);

/* Where the last batch's NFA work went, for query `query`'s kernel group (queries sharing a
 * launch report the same group figures; stencil queries report zeros but kernel_ms). */
typedef struct {
  uint32_t group;          /* kernel group of the query (-1 as u32: stencil) */
  uint32_t group_queries;  /* queries in that launch */
  double kernel_ms;        /* bitmap + lane order + matching launch + re-runs */
  double main_ms;          /* the matching launch (cep_nfa_jit / nfa_kernel) alone */
  double retry_ms;         /* re-runs of jobs that hit a capacity limit or a walk conflict
                              (streams: the wide build's continuation of stopped keys) */
  uint64_t retried_jobs;   /* (query, key) jobs re-run (streams: keys whose versions outgrew
                              the stream build's 3 pairs, continued by the wide build) */
  uint64_t nodes_used, preds_used, out_chunks_used;  /* buffer pools at the end of the batch */
  uint32_t launches;
  uint32_t allocs;         /* device allocations the last cep_push_batch made (0 once a session has
                              seen a batch of this shape: buffers and pools are reused) */
} cep_batch_stats;
int cep_last_stats(cep_session* s, int query, cep_batch_stats* out);

/* Lane-work balance of the last batch's NFA launch for query `query`'s group (north_star's
 * wave divergence figure): the per-key work estimate of cep_nfa_est (run-steps if every run
 * lived to the end) over waves of 64 consecutive lanes; a wave lasts as long as its busiest
 * lane, so sum over waves of (max / mean) tells how much of the launch is lane idling.
 * *ordered: sum_waves max / sum_waves mean in the launch's longest-first lane order;
 * *identity: the same for keys in index order (no lane order).  1.0 = perfectly balanced.
 * Computed on demand from the last batch (a 4-B-per-key download); CEP_E_INVALID when the
 * batch ran no estimate (stencil queries, streams, <= 64 keys). */
int cep_lane_balance(cep_session* s, int query, double* ordered, double* identity);

/* A shard of a device-resident CSR batch (multi-GPU key sharding): the events of the keys
 * sel_keys[0..n_sel) (indices into src_key_off) gathered into dst columns at dst_key_off
 * (the shard's own CSR offsets, [n_sel + 1]).  All arrays are device memory except the
 * pointer arrays and col_bytes (4 or 8 per column); src_ts/dst_ts may be NULL.  Which keys
 * a rank owns: kafkastreams-cep_amd/shard.py (Kafka's DefaultPartitioner). */
int cep_gather_keys(int device, uint64_t n_sel, const uint32_t* sel_keys, const uint64_t* src_key_off,
                    const uint64_t* dst_key_off, int n_cols, const uint32_t* col_bytes,
                    const void* const* src_cols, void* const* dst_cols, const int64_t* src_ts, int64_t* dst_ts);

const char* cep_last_error(void);
int cep_alloc_pinned(size_t bytes, void** out);
int cep_free_pinned(void* p);
int cep_device_alloc(int device, size_t bytes, void** out);
int cep_device_free(void* p);
int cep_memcpy(void* dst, const void* src, size_t bytes, int dst_memory, int src_memory);

/* ---- ingest: StockEvent JSON record values -> event columns (on the device) ----
 * Replaces the demo topology's value deserializer StockEventSerDe.JsonSerDeserializer.deserialize
 * (src/test/java/.../demo/StockEventSerDe.java:58-72: json-simple 1.1.1 JSONParser, then
 * new StockEvent((String) name, (Long) price, (Long) volume), demo/StockEvent.java:4-14), applied
 * to a whole batch of record values.  bytes: the values back to back; rec_off[n+1] (u64) their
 * offsets.  Per record: status[r] = 0 or the CEP_JSON_* exception deserialize() would throw;
 * price/volume columns (col_width 8 = the reference's long, 4 = the int32 columns the matcher
 * reads; a long that does not fit is CEP_JSON_NARROW); name_span[2r..2r+1] (optional) = byte
 * offset of the name's text within the record and its raw length (bit 31: the text holds
 * escapes), length 0xFFFFFFFF for a null/absent name.  Failed records get 0 in the columns.
 * All pointers are device memory; the launch is asynchronous on `stream` (hipStream_t, NULL =
 * the default stream). */
enum {
  CEP_JSON_OK = 0,
  CEP_JSON_PARSE = 1,      /* RuntimeException(ParseException): malformed record */
  CEP_JSON_CLASS_CAST = 2, /* ClassCastException: not an object, name not a String, price/volume not Long */
  CEP_JSON_NULL = 3,       /* NullPointerException: null record object, price/volume null or absent */
  CEP_JSON_NUMBER = 4,     /* NumberFormatException: an integer literal outside long */
  CEP_JSON_LEX = 5,        /* java.lang.Error from the scanner: an unknown string escape */
  CEP_JSON_NARROW = 6,     /* col_width 4 and price/volume outside int32 (no reference outcome) */
  CEP_JSON_DEPTH = 7       /* nesting deeper than 64 (this decoder's limit; the reference parses it) */
};
int cep_decode_stock_json(int device, const uint8_t* bytes, const uint64_t* rec_off, uint64_t n_records,
                          int col_width, void* price, void* volume, int32_t* status, uint32_t* name_span,
                          void* stream);

/* ---- [symbol] keying: the README query's `[symbol]` (README.md:19-28)
 * partitions the stream by StockEvent.name.  For a batch decoded by cep_decode_stock_json with
 * name spans: key_out[r] = index of record r's name among the batch's distinct names in order
 * of first appearance (the name compared as the Java String deserialize() builds: UTF-16 units
 * of the unescaped text; a null name is one symbol); records with status[r] != 0 (deserialize()
 * throws) get 0xFFFFFFFF.  *n_symbols = distinct names.  max_symbols sizes the hash table (more
 * distinct names fail the call).  A name holding malformed UTF-8 fails the call (CEP_E_INVALID),
 * as does a 64-bit hash collision between different names (checked, never merged).  All
 * arrays are device memory; n_records < 2^32; synchronous on `stream`. */
int cep_symbol_keys(int device, const uint8_t* bytes, const uint64_t* rec_off, const uint32_t* name_span,
                    const int32_t* status, uint64_t n_records, uint64_t max_symbols, uint32_t* key_out,
                    uint64_t* n_symbols, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CEP_H_ */
