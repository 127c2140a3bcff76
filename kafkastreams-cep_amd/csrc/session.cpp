// session.cpp — the C ABI (include/cep.h): query compile, sessions on one GPU, batch
// matching, result retrieval.  Host code; kernels live in nfa.hip / stencil.hip / partition.hip /
// ingest.hip / symbol.hip / shard.hip / watermark.hip (the synthetic generators of the bench
// and the tests are a separate library, synth_gen.hip -> libcep_synth.so).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "cep_internal.h"
#include "kernel_args.h"
#include "stencil_args.h"

using namespace cep;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define HIPCHECK(x)                                                                          \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess)                                                                    \
      throw HipError(std::string(#x) + ": " + hipGetErrorString(e_));                        \
  } while (0)

// A grow-only device buffer.
// $CEP_HOST_TRACE (measurement runs, Tuning.host_trace): device (re)allocations and push phases
// on stderr, ms.  Set when a session is created with the knob.
static bool g_host_trace = false;
static bool host_trace() { return g_host_trace; }
// device allocations made (DBuf ensure / grow_keep): cep_batch_stats.allocs counts a batch's
static thread_local uint32_t g_allocs = 0;
// $CEP_POISON=mask (measurement runs): the session's k-th device allocation (k < 64, bit k of
// the mask; -1: all) filled with 0xFF bytes (CEP_NONE words; $CEP_POISON_BYTE another byte), so a read of memory no kernel wrote is not hidden
// by a fresh allocation's zeros
// (thread_local like g_allocs: one session per thread, each thread's allocation index against its
// own base)
static thread_local uint64_t g_poison = 0;
static thread_local uint32_t g_poison_base = 0;
static thread_local int g_poison_byte = 0xFF;  // ($CEP_POISON_BYTE)
static bool poison_next() {
  const uint32_t k = g_allocs - g_poison_base;
  return k < 64 && ((g_poison >> k) & 1u);
}
// A copy on the session's own stream, waited for.  Session paths never use the null stream:
// it does not order with the sessions' hipStreamNonBlocking streams.
static void copy_sync(void* dst, const void* src, size_t n, hipMemcpyKind k, hipStream_t st) {
  HIPCHECK(hipMemcpyAsync(dst, src, n, k, st));
  HIPCHECK(hipStreamSynchronize(st));
}
static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct DBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void ensure(size_t n) {
    if (n <= bytes) return;
    const double t0 = host_trace() ? now_ms() : 0;
    struct Tr {
      double t0;
      size_t n;
      ~Tr() {
        if (host_trace()) std::fprintf(stderr, "cep_host alloc %zu B %.2f ms\n", n, now_ms() - t0);
      }
    } tr{t0, n};
    if (p) HIPCHECK(hipFree(p));
    p = nullptr;
    bytes = 0;
    const bool poison = poison_next();
    if (host_trace()) std::fprintf(stderr, "cep_host alloc #%u\n", g_allocs - g_poison_base);
    g_allocs++;
    n = std::max<size_t>(n, 256);
    if (hipMalloc(&p, n) != hipSuccess) {
      p = nullptr;
      throw std::bad_alloc();
    }
    if (poison) {  // (synchronous: the null stream does not order with the session's)
      HIPCHECK(hipMemset(p, g_poison_byte, n));
      HIPCHECK(hipDeviceSynchronize());
    }
    bytes = n;
  }
  // grow keeping the first `keep` bytes
  void grow_keep(size_t n, size_t keep, hipStream_t st) {
    if (n <= bytes) return;
    const double t0 = host_trace() ? now_ms() : 0;
    struct Tr {
      double t0;
      size_t n;
      ~Tr() {
        if (host_trace()) std::fprintf(stderr, "cep_host grow %zu B %.2f ms\n", n, now_ms() - t0);
      }
    } tr{t0, n};
    void* q = nullptr;
    const bool poison = poison_next();
    g_allocs++;
    if (hipMalloc(&q, n) != hipSuccess) throw std::bad_alloc();
    if (poison) {
      HIPCHECK(hipMemset(q, g_poison_byte, n));
      HIPCHECK(hipDeviceSynchronize());
    }
    if (p && keep) HIPCHECK(hipMemcpyAsync(q, p, std::min(keep, bytes), hipMemcpyDeviceToDevice, st));
    HIPCHECK(hipStreamSynchronize(st));
    if (p) HIPCHECK(hipFree(p));
    p = q;
    bytes = n;
  }
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
};

template <class T> struct HVec {  // host copy of a result array
  std::vector<T> v;
};

struct Scratch {  // small counters, one allocation
  uint32_t node_top, pred_top, out_top, n_cap_err;
  uint32_t tile_counter, overflow, n_retry_cap, n_retry_conflict;
  uint32_t job_next, full;  // full: NfaArgs.full
  uint64_t totals[2];
  uint64_t total;
  unsigned long long digest;
  unsigned long long wmax;
};

// A streaming session's per-query NFA state (cep_opts.streaming): every key's run queue,
// buffer pools and carried lane state persist from one batch to the next.
struct StreamState {
  DBuf rings, nodes, preds, preds0, carry, tops;  // tops: {node_top, pred_top} (device)
  uint64_t n_keys = 0, node_cap = 0, pred_cap = 0;
  uint32_t node_used = 0, pred_used = 0;  // pool tops after the last batch
  uint32_t rcap = 0;                      // run-queue slots per key (ring layout)
  uint64_t ring_bytes = 0;
  bool init = false;
};

struct QueryRt {
  const cep_query* q;
  int F = 2;
  DBuf d_q, d_code;
  int group = -1;   // kernel group (NFA path), -1: stencil
  uint32_t qi = 0;  // index within the group
  // results of the last batch (device)
  DBuf m_key, m_emit, m_off, p_seq, p_stage;
  DBuf ks;                      // stencil path: per-key state (all zero)
  const KeyState* ks_dev = nullptr;  // this query's KeyState[n_keys] (the group's slice or ks)
  uint64_t n_matches = 0, n_pairs = 0;
  unsigned long long digest = 0;
  bool digest_valid = false;  // computed on demand (cep_match_digest)
  uint32_t arity = 0;
  bool have = false;
  // host copies
  std::vector<uint32_t> h_key, h_emit, h_seq;
  std::vector<uint64_t> h_off;
  std::vector<uint16_t> h_stage;
  bool host_valid = false;
  float kernel_ms = 0;  // the matching kernel launches (a group's launches, shared by its queries)
  float aux_ms = 0;     // setup and compaction kernels of the same batch
  uint32_t launches = 0;
  StreamState st;
  // Stencil batches return without a host sync (pushes pipeline on the stream): the match
  // count comes back through pinned memory and each batch's event triple (setup start,
  // kernels start, end) goes into a ring, all read when a result is asked for (resolve()).
  static constexpr int kRing = 16;
  Scratch* h_sc = nullptr;  // pinned copy of the batch's counters
  Scratch* h_sc_dev = nullptr;  // its device address (stencil_emit writes the match count there)
  bool pending = false;
  hipEvent_t tev[kRing][3] = {};
  bool tev_used[kRing] = {};
  int tev_next = 0, tev_last = -1;
  uint64_t ks_zeroed = 0;  // stencil: KeyState entries known zero
  // every batch's timing since the last cep_timing_totals reset
  double acc_kernel_ms = 0, acc_aux_ms = 0;
  uint64_t acc_batches = 0;
  ~QueryRt() {
    for (auto& t : tev)
      for (auto& e : t)
        if (e) (void)hipEventDestroy(e);
    if (h_sc) (void)hipHostFree(h_sc);
  }
};

// Queries whose NFA kernels run as one launch (compile.cpp plan_groups): lanes are (query,
// key) jobs, wave W runs query W % Q on 64 keys, so the Q waves of a key group read its
// event columns together (one HBM read, L2 hits for the rest).
struct GroupRt {
  std::vector<int> members;
  int F = 2;
  hipModule_t mod = nullptr;  // JIT tier: the group's kernel (cep_nfa_jit), narrow Dewey build
  hipFunction_t fn = nullptr;
  hipModule_t mod_wide = nullptr;  // its wide build (compile.cpp generate_jit): re-runs, streams
  hipFunction_t fn_wide = nullptr;
  hipModule_t mod_stream = nullptr;  // streaming sessions: the stream build (jit_stream_source)
  hipFunction_t fn_stream = nullptr;
  uint32_t waves_cu = 0, waves_cu_wide = 0;  // resident waves per CU of fn / fn_wide (occupancy)
  uint32_t waves_cu_stream = 0;               // ... of fn_stream (streams run it)
  uint32_t walk_flush = 24;  // the drain threshold the group's kernels were compiled with
  hipFunction_t fn_est = nullptr;   // cep_nfa_est (begin stage = one BEGIN edge)
  hipFunction_t fn_bits = nullptr;  // cep_nfa_bits (the same queries): begin-hit bitmap
  double jit_compile_s = 0;
  DBuf kc;  // literal table, Q x nkc
  DBuf ks;  // KeyState[Q x n_keys]
  DBuf est, order, order_tmp, est_sorted;
  bool est_valid = false;  // the last batch ran cep_nfa_est + the lane order (cep_lane_balance)
  void* sort_tmp = nullptr;  // lane-order sort scratch
  size_t sort_tmp_bytes = 0;
  // pool use of the last batch (the next batch's pools are sized from it)
  uint64_t last_nodes = 0, last_preds = 0, last_out = 0;
  uint32_t rcap_hint = 0;  // run-queue slots per key: grown when a batch's queues overflowed
  uint64_t stream_widened = 0;  // keys the wide build continued (KE_WIDEN), over the session
  cep_batch_stats stats{};  // the last batch
  ~GroupRt() {
    if (mod) (void)hipModuleUnload(mod);
    if (mod_wide) (void)hipModuleUnload(mod_wide);
    if (mod_stream) (void)hipModuleUnload(mod_stream);
    if (sort_tmp) (void)hipFree(sort_tmp);
  }
};

}  // namespace

struct cep_session {
  int device = 0;
  cep_opts opts{};
  cep::Tuning tune{};  // measurement knobs, read once at creation (tuning.cpp)
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
  int cus = 256;  // compute units of the device (persistent-lane grids)
  std::vector<std::unique_ptr<QueryRt>> qs;
  std::vector<std::unique_ptr<GroupRt>> groups;
  // batch (device copies when the batch is host-resident)
  DBuf b_off, b_ts;
  DBuf b_cols[kMaxFields];
  uint64_t n_keys = 0, n_events = 0;
  const uint64_t* key_off = nullptr;
  const int64_t* ts = nullptr;
  Cols cols{};
  int64_t watermark = INT64_MIN;
  unsigned long long* h_wm = nullptr;  // pinned: the batch's max timestamp (read by resolve())
  bool wm_pending = false;
  bool wm_fold = false;  // this batch's watermark comes from the first group's bitmap/estimate passes
  DBuf wm_blocks;        // their per-block maxima
  // arrival-order batches: device copies of the input, the partitioned (CSR) batch
  DBuf a_keys, a_ts, p_off, p_cnt, p_ts, p_perm, p_sorted, p_idx, p_scratch;
  DBuf a_cols[kMaxFields], p_cols[kMaxFields];
  bool arrival = false;
  float partition_ms = 0;
  std::vector<uint64_t> h_off;
  std::vector<uint32_t> h_perm;
  bool layout_host_valid = false;
  // scratch
  DBuf heavy;  // heavy-key list of the output scatter
  DBuf rings, walks, nodes, preds, preds0, out, scratch, status, keylist, mask, bhits, retry_rings, bsum;
  DBuf prof;  // measurement runs ($CEP_PROF): the main launch's time split (nfa_lane.h)
  uint32_t last_allocs = 0;  // device allocations the last cep_push_batch made
};

namespace {

struct DeviceGuard {
  int prev = 0;
  explicit DeviceGuard(int d) {
    (void)hipGetDevice(&prev);
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DeviceGuard() { (void)hipSetDevice(prev); }
};

// a ring slot's timing into the query's totals (its events are waited for)
void ring_take(QueryRt& r, int i) {
  HIPCHECK(hipEventSynchronize(r.tev[i][2]));
  float a = 0, k = 0;  // (aux: the key-index pass is not bracketed, see run_stencil)
  HIPCHECK(hipEventElapsedTime(&k, r.tev[i][1], r.tev[i][2]));
  r.acc_kernel_ms += k;
  r.acc_aux_ms += a;
  r.acc_batches++;
  r.tev_used[i] = false;
  if (i == r.tev_last) {
    r.kernel_ms = k;
    r.aux_ms = a;
  }
}

// The host side of the last batch's asynchronous results (stencil counts and timing, the
// watermark): one stream sync, then the pinned copies are read.
void resolve(cep_session* s) {
  bool any = s->wm_pending;
  for (auto& r : s->qs) any = any || r->pending;
  if (!any) return;
  HIPCHECK(hipStreamSynchronize(s->stream));
  for (auto& rp : s->qs) {
    QueryRt& r = *rp;
    if (!r.pending) continue;
    for (int i = 0; i < QueryRt::kRing; i++)
      if (r.tev_used[i]) ring_take(r, i);
    r.pending = false;
    // (no overflow check: the output holds one match per event, the most a strict chain can
    // emit; stencil_emit still flags it on the device)
    r.n_matches = r.h_sc->total;
    r.n_pairs = r.n_matches * r.arity;
  }
  if (s->wm_pending) {
    s->watermark = (int64_t)(*s->h_wm ^ 0x8000000000000000ull);
    s->wm_pending = false;
  }
}

// Strict chains (stencil.hip): wave_keys, stencil_mask, stencil_emit; no host sync.
void run_stencil(cep_session* s, QueryRt& r) {
  const cep_query* q = r.q;
  const uint32_t m = q->info.arity;
  const uint64_t nk = s->n_keys;
  const uint64_t n_tiles = stencil_tiles(s->n_events);
  const uint64_t n_groups = n_tiles / 4 + 2;  // (a count per stencil_emit block: 4 tiles)
  s->status.ensure(sizeof(Scratch) + sizeof(uint32_t) * n_groups);               // counters + group counts
  s->mask.ensure(16 * (s->n_events / 64 + 2));                                   // a 16-B record per 64 events
  s->keylist.ensure(sizeof(uint32_t) * (stencil_waves(s->n_events) + 1));        // wave -> key
  // worst case one match per event
  const uint64_t cap = std::max<uint64_t>(s->n_events, 1);
  if (!r.h_sc) {
    HIPCHECK(hipHostMalloc((void**)&r.h_sc, sizeof(Scratch), hipHostMallocMapped));
    std::memset(r.h_sc, 0, sizeof(Scratch));
  }
  if (s->n_events == 0) {
    // launch_stencil launches nothing, so nothing writes this batch's count into the pinned
    // copy: zero it here, once an earlier batch's stencil_emit can no longer overwrite it
    HIPCHECK(hipStreamSynchronize(s->stream));
    r.h_sc->total = 0;
  }
  r.m_key.ensure(sizeof(uint32_t) * cap);
  r.p_seq.ensure(sizeof(uint32_t) * cap * m);
  if (!r.tev[0][0])
    for (auto& t : r.tev)
      for (auto& e : t) HIPCHECK(hipEventCreate(&e));
  const int slot = r.tev_next;
  if (r.tev_used[slot]) ring_take(r, slot);  // kRing batches back: long done
  r.tev_next = (slot + 1) % QueryRt::kRing;
  r.tev_last = slot;
  r.tev_used[slot] = true;

  Scratch* sc = s->status.as<Scratch>();
  StencilArgs a{};
  a.n_keys = nk;
  a.n_events = s->n_events;
  a.key_off = s->key_off;
  a.wave_key = s->keylist.as<uint32_t>();
  a.q = r.d_q.as<DevQuery>();
  a.code = r.d_code.as<uint32_t>();
  a.cols = s->cols;
  a.ts = s->ts;
  const bool range = q->stencilRange;
  for (int c = 0; c < 2; c++) a.col[c] = (const int32_t*)s->cols.p[q->rangeCols[c]];
  a.aligned = ((uintptr_t)a.col[0] % 16 == 0) && ((uintptr_t)a.col[1] % 16 == 0);
  for (uint32_t i = 0; i < m && i < (uint32_t)kMaxStencil; i++) {
    a.prog[i] = q->stencilProg[i];
    for (int c = 0; c < 2; c++) {
      a.rs[i].lo[c] = q->rangeLo[i][c];
      a.rs[i].hi[c] = q->rangeHi[i][c];
    }
  }
  for (uint32_t x = 0; x < m && x < (uint32_t)kMaxStencil; x++) a.stage_name[x] = q->arityStage[x];
  a.words = s->mask.as<uint4>();
  a.group_cnt = reinterpret_cast<uint32_t*>(sc + 1);
  a.m_key = r.m_key.as<uint32_t>();
  a.p_seq = r.p_seq.as<uint32_t>();
  a.total = &sc->total;
  a.out_cap = cap;
  a.overflow = &sc->overflow;
  if (!r.h_sc_dev) HIPCHECK(hipHostGetDevicePointer((void**)&r.h_sc_dev, r.h_sc, 0));
  a.total_host = &r.h_sc_dev->total;  // the emit pass writes the count straight to the host copy
  // No event before wave_keys: every marker packet costs the stream ~5 us between kernels
  // (4 % of this 0.12 ms step), so the 4 us key-index pass is not timed (aux_ms 0).
  // wave_keys also zeroes the counters (no memset launch); no D2H copy of them either
  HIPCHECK(launch_wave_keys(s->key_off, nk, s->n_events, s->keylist.as<uint32_t>(), reinterpret_cast<uint32_t*>(sc),
                            (uint32_t)((sizeof(Scratch) + sizeof(uint32_t) * n_groups) / 4), s->stream));
  HIPCHECK(hipEventRecord(r.tev[slot][1], s->stream));
  HIPCHECK(launch_stencil((int)m, a, range, q->nRangeCols, s->stream));
  HIPCHECK(hipEventRecord(r.tev[slot][2], s->stream));
  r.pending = true;
  r.launches = 2;  // stencil_mask + stencil_emit
  r.digest_valid = false;
  r.arity = m;
  // no per-key errors on this path: the predicates and folds are total
  if (r.ks_zeroed < nk) {
    r.ks.ensure(sizeof(KeyState) * std::max<uint64_t>(nk, 1));
    HIPCHECK(hipMemsetAsync(r.ks.p, 0, sizeof(KeyState) * nk, s->stream));
    r.ks_zeroed = nk;
  }
  r.ks_dev = r.ks.as<KeyState>();
}

// wide: the JIT kernel's wide Dewey build (re-runs, streaming sessions)
hipError_t launch_nfa_tier(GroupRt& g, const cep_query* q0, NfaArgs& a, uint64_t nslots, hipStream_t st,
                           bool wide) {
  if (!g.fn) return launch_nfa(g.F, a, nslots, q0->dev.code_len, st);
  if (nslots == 0) return hipSuccess;
  size_t size = sizeof(NfaArgs);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size, HIP_LAUNCH_PARAM_END};
  return hipModuleLaunchKernel(wide ? g.fn_wide : g.fn, (uint32_t)((nslots + 255) / 256), 1, 1, 256, 1, 1, 0, st,
                               nullptr, cfg);
}

hipError_t launch_fn(hipFunction_t fn, NfaArgs& a, uint64_t blocks, hipStream_t st) {
  size_t size = sizeof(NfaArgs);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size, HIP_LAUNCH_PARAM_END};
  return hipModuleLaunchKernel(fn, (uint32_t)blocks, 1, 1, 256, 1, 1, 0, st, nullptr, cfg);
}

constexpr uint64_t kPoolMax = 0xFFFFFFF0ull;   // output chunk ids are u32
constexpr uint64_t kNodeMax = 0x7FFFFFF0ull;   // node / pointer ids: 31 bits (kPred0 tags a node's slot)

// Runs a kernel group over the batch: the begin-hit bitmap and lane order, the matching
// launch, re-runs of the jobs that hit a capacity limit or a deferred-walk conflict, and the
// per-query compaction of the output chains into flat arrays.
void run_nfa(cep_session* s, GroupRt& g) {
  const uint64_t nk = s->n_keys;
  const uint64_t Q = g.members.size();
  const uint64_t jobs = Q * nk;
  QueryRt& r0 = *s->qs[g.members[0]];
  uint32_t rcap = s->opts.max_runs ? s->opts.max_runs : 32;
  const bool streaming0 = s->opts.streaming != 0;
  if (!streaming0) rcap = std::max(rcap, g.rcap_hint);  // (a stream's ring geometry is fixed)
  const double pf = s->opts.pool_factor > 0 ? s->opts.pool_factor : 0.0625;
  const bool streaming = s->opts.streaming != 0;  // (a streaming group holds one query)
  // Per-batch sessions run persistent lanes (nfa_lane.h run_jobs): a grid of about what the
  // chip holds at once (3 waves per SIMD), every lane claiming job after job.  Streams keep one
  // lane per key (their run queues live at the key's slot).
  // waves per CU of the JIT kernels (compile.cpp): the narrow build 3 per SIMD, the wide one
  // (streams, re-runs) 2; $CEP_RESIDENT_WAVES (per CU): measurement runs
  const uint64_t wn = g.waves_cu ? g.waves_cu : 12, ww = g.waves_cu_wide ? g.waves_cu_wide : 8;
  // (a stream runs the stream build when it has one: its own occupancy)
  const uint64_t wst = g.fn_stream && g.waves_cu_stream ? g.waves_cu_stream : ww;
  uint64_t waves_cu = streaming ? wst : wn, waves_cu_wide = ww;
  if (s->tune.resident_waves > 0) waves_cu = waves_cu_wide = s->tune.resident_waves;
  const uint64_t resident = (uint64_t)s->cus * waves_cu * 64;
  const uint64_t resident_wide = (uint64_t)s->cus * waves_cu_wide * 64;
  auto grid_for = [&](uint64_t n) { return std::min<uint64_t>((n + 255) / 256 * 256, resident); };
  auto grid_wide = [&](uint64_t n) { return std::min<uint64_t>((n + 255) / 256 * 256, resident_wide); };
  // $CEP_NO_PERSIST (measurement runs): one lane per job.  Single queries run one lane per key:
  // their longest-first lane order already balances the waves (persistent lanes cost cfg 3
  // ~35 %), and their narrow kernel is built without the persistent driver; groups mix light
  // and heavy queries.
  const bool persist = !streaming && !s->tune.no_persist && Q > 1;
  // An underfilled single-query launch (fewer waves than the chip holds: a shard of a
  // multi-GPU run, a small batch) is as long as its longest wave, whose length is its heaviest
  // key's chain of events times the wave's per-event cost; that cost grows with the number of
  // divergent lanes.  So its keys are spread over every wave slot the chip holds: the heaviest
  // keys lead one wave each, with lighter keys beside them ($CEP_NO_SPREAD: measurement runs).
  uint64_t spread = 0;
  // (odd lanes take their row of ranks reversed: the slowest world-8 shard 16.5 -> 15.6 ms)
  if (!persist && Q == 1 && nk > 64 && (nk + 63) / 64 < resident / 64 && !s->tune.no_spread)
    spread = std::min<uint64_t>(resident / 64, nk);
  // (a full launch spread over all its waves - every wave led by one of the heaviest keys with
  // lighter ones beside it - was measured: cfg 3 29.2 -> 48.8 ms, every wave pays the divergence;
  // so was isolating a spread launch's heaviest ranks in waves of their own: the slowest world-8
  // shard 15.4 -> 14.4-15.2 ms, within its spread - dropped in round 5)
  uint32_t iso = 0;
  // A stream launch bigger than the chip: its K heaviest keys (by the lane order's estimate) run
  // alone in their waves, the others 64 per wave in lane order.  A streamed batch lasts as long as
  // its heaviest wave, and a heavy key's wave otherwise pays its lighter neighbours' divergent
  // paths and drains too (streamed cfg 3, main launches: 61.3 -> 43.9 ms at K = 2048).  (The same
  // for a per-batch launch measured slower - 33.9 -> 36.9 ms at K = 2048: one launch of 1e9
  // events is throughput-bound - and was dropped in round 5.)  Only with a lane order to pick the
  // heaviest keys by (a begin stage with a single BEGIN edge has one): else the first keys by id
  // would each take a wave for nothing.
  const bool lane_order = g.fn_est && nk > 64 && !(streaming && s->tune.stream_no_order);
  if (streaming && !spread && lane_order && s->tune.stream_iso)
    iso = (uint32_t)std::min<uint64_t>(s->tune.stream_iso, nk / 2);
  const uint64_t slots = spread ? spread * 64
                         : iso  ? ((uint64_t)iso + (nk - iso + 63) / 64) * 64
                         : !persist ? ((nk + 63) / 64) * 64 * Q
                                    : grid_for(jobs);
  g.ks.ensure(sizeof(KeyState) * std::max<uint64_t>(jobs, 1));
  s->scratch.ensure(sizeof(Scratch));
  Scratch* sc = s->scratch.as<Scratch>();

  // Pools: nodes / preds / output chunks, shared by the group's jobs.  Sized from the last
  // batch's use when there is one (x1.5), else from pool_factor per event and query; a job
  // that runs out is re-run below with grown pools.
  // per-lane pool ranges: one atomic per range on each pool's counter.  Per-batch launches
  // (persistent lanes keep their ranges across jobs) take bigger ranges; streams hold a range
  // per key between batches, so theirs stay small
  uint32_t nchunk = streaming ? 16 : 64, ochunk = streaming ? 1 : 8;
  if (s->tune.node_chunk) nchunk = s->tune.node_chunk;  // (measurement runs)
  if (s->tune.out_chunk) ochunk = s->tune.out_chunk;
  const uint32_t pchunk = nchunk;
  const uint64_t ev_q = (uint64_t)((double)s->n_events * (double)Q);
  // (the last batch's pool tops already count the ranges lanes held at its end; the estimate
  // from pool_factor adds them: a steady stream of like batches never reallocates)
  uint64_t node_cap = std::max<uint64_t>((uint64_t)(pf * (double)ev_q) + 4096 + slots * nchunk,
                                         g.last_nodes * 3 / 2 + 4096);
  uint64_t pred_cap = std::max<uint64_t>((uint64_t)(pf * (double)ev_q) + 4096 + slots * pchunk,
                                         g.last_preds * 3 / 2 + 4096);
  uint64_t out_cap = std::max<uint64_t>((uint64_t)(pf * (double)ev_q * 2 / kOutChunkWords) + jobs / 64 + 1024 +
                                            slots * ochunk,
                                        g.last_out * 3 / 2 + 1024);
  node_cap = std::min<uint64_t>(node_cap, kNodeMax);
  pred_cap = std::min<uint64_t>(pred_cap, kNodeMax);
  out_cap = std::min<uint64_t>(out_cap, kPoolMax);  // chunk ids are u32, word addresses u64
  s->nodes.ensure(sizeof(Node) * node_cap);
  s->preds0.ensure(sizeof(Pred) * node_cap);
  s->preds.ensure(sizeof(Pred) * pred_cap);
  s->out.ensure(sizeof(uint32_t) * kOutChunkWords * out_cap);
  s->rings.ensure(ring_size(g.F, std::max<uint64_t>(slots, 1), rcap));
  // deferred walks a key can queue (nfa_lane.h drains at the compiled CEP_WALK_FLUSH, recorded
  // with the group; $CEP_WALK_CAP: tuning)
  // (a stream cannot re-run a key whose event overflows its queue: room for every walk one
  // event can queue - removePattern and branch walks of its records, one extraction per output
  // - beyond the drain threshold)
  uint32_t wcap = streaming ? std::max<uint32_t>(64, g.walk_flush + 3 * rcap) : 64;
  if (s->tune.walk_cap) wcap = s->tune.walk_cap;
  // put-log entries per lane: every put one event can log fits twice over (a stream turns a
  // put-log overflow into a sticky error, so it must never happen there)
  uint32_t plog = put_log_entries(rcap);
  s->walks.ensure(walkq_size(std::max<uint64_t>(slots, 1), wcap, plog));
  HIPCHECK(hipMemsetAsync(sc, 0, sizeof(Scratch), s->stream));

  NfaArgs a{};
  StreamState& S = r0.st;
  if (streaming) {
    if (!S.init) {
      S.n_keys = nk;
      S.carry.ensure(sizeof(KeyCarry) * std::max<uint64_t>(nk, 1));
      HIPCHECK(hipMemsetAsync(S.carry.p, 0, sizeof(KeyCarry) * std::max<uint64_t>(nk, 1), s->stream));
      S.tops.ensure(2 * sizeof(uint32_t));
      HIPCHECK(hipMemsetAsync(S.tops.p, 0, 2 * sizeof(uint32_t), s->stream));
      // a stream's run queues live at their key's position (nfa_lane.h run_key), whatever the
      // launch's slot count (an underfilled launch spreads its keys over more slots)
      S.rings.ensure(ring_size(g.F, std::max<uint64_t>(nk, 1), rcap));
      S.rcap = rcap;
      S.ring_bytes = ring_size(g.F, std::max<uint64_t>(nk, 1), rcap);
      S.init = true;
    } else if (nk != S.n_keys) {
      throw std::invalid_argument("the batches of a streaming session share one key space (n_keys)");
    }
    // a stream cannot re-run a key (its state moved on): size the pools for this batch on top
    // of what the stream already holds, generously (capacity errors would be final)
    const uint64_t add = s->n_events + nk * 2 * nchunk + 4096;
    const uint64_t nn = std::min<uint64_t>(S.node_used + add, kNodeMax);
    const uint64_t pn = std::min<uint64_t>(S.pred_used + add, kNodeMax);
    if (nn > S.node_cap) {
      const uint64_t c = std::min<uint64_t>(std::max<uint64_t>(nn, S.node_cap * 3 / 2), kNodeMax);
      S.nodes.grow_keep(sizeof(Node) * c, sizeof(Node) * S.node_used, s->stream);
      S.preds0.grow_keep(sizeof(Pred) * c, sizeof(Pred) * S.node_used, s->stream);
      // node slots past the used prefix start dead: pool chunks in hand hold slots no lane
      // has written yet, which cep_live_floor scans
      HIPCHECK(hipMemsetAsync(S.nodes.as<Node>() + S.node_used, 0, sizeof(Node) * (c - S.node_used), s->stream));
      S.node_cap = c;
    }
    if (pn > S.pred_cap) {
      const uint64_t c = std::min<uint64_t>(std::max<uint64_t>(pn, S.pred_cap * 3 / 2), kNodeMax);
      S.preds.grow_keep(sizeof(Pred) * c, sizeof(Pred) * S.pred_used, s->stream);
      S.pred_cap = c;
    }
    out_cap = std::max<uint64_t>(out_cap, std::min<uint64_t>(nk + s->n_events / 64 + 1024, kPoolMax));
    s->out.ensure(sizeof(uint32_t) * kOutChunkWords * out_cap);
  }
  a.q = r0.d_q.as<DevQuery>();
  a.code = r0.d_code.as<uint32_t>();
  a.n_keys = nk;
  a.key_off = s->key_off;
  a.cols = s->cols;
  a.ts = s->ts;
  a.rings = s->rings.p;
  a.rcap = rcap;
  a.walks = s->walks.p;
  a.wcap = wcap;
  a.plog = plog;
  a.defer = 1;
  a.n_q = (uint32_t)Q;
  a.spread = spread;
  a.spread_iso = iso;
  a.kc = g.kc.bytes ? g.kc.as<int64_t>() : nullptr;
  a.nodes = s->nodes.as<Node>();
  a.preds = s->preds.as<Pred>();
  a.preds0 = s->preds0.as<Pred>();
  a.out = s->out.as<uint32_t>();
  a.node_pool = Pool{&sc->node_top, (uint32_t)node_cap, nchunk};
  a.pred_pool = Pool{&sc->pred_top, (uint32_t)pred_cap, pchunk};
  a.out_pool = Pool{&sc->out_top, (uint32_t)out_cap, ochunk};
  a.ks = g.ks.as<KeyState>();
  a.n_capacity_err = &sc->n_cap_err;
  a.full = &sc->full;
  a.n_events = s->n_events;
  if (persist) {
    a.job_next = &sc->job_next;
    a.n_jobs = jobs;
  }
  if (streaming) {  // walks deferred too: a conflict resolves exactly without a re-run (nfa_lane.h)
    a.rings = S.rings.p;
    a.nodes = S.nodes.as<Node>();
    a.preds = S.preds.as<Pred>();
    a.preds0 = S.preds0.as<Pred>();
    a.carry = S.carry.as<KeyCarry>();
    a.node_pool = Pool{S.tops.as<uint32_t>(), (uint32_t)S.node_cap, nchunk};
    a.pred_pool = Pool{S.tops.as<uint32_t>() + 1, (uint32_t)S.pred_cap, pchunk};
  }

  float total_ms = 0;
  uint32_t launches = 0;
  const bool wm_here = s->wm_fold && &g == s->groups[0].get();
  // (every buffer of the timed interval below is allocated before its first event: an
  // allocation there would count its host time - hipFree synchronises - as kernel time)
  const uint64_t nb_bits = (s->n_events + 256 * kBitStrips - 1) / (256 * kBitStrips);
  if (g.fn_bits && s->n_events) {
    s->bhits.ensure(8 * ((s->n_events + 63) / 64));
    if (wm_here) s->wm_blocks.ensure(8 * nb_bits);
  }
  if (g.fn_est && nk > 64) {
    g.est.ensure(4 * nk);
    g.est_sorted.ensure(4 * nk);
    g.order.ensure(4 * nk);
    g.order_tmp.ensure(4 * nk);
    HIPCHECK(sort_keys_scratch(nk, g.sort_tmp, g.sort_tmp_bytes));
  }
  if (s->tune.prof) s->prof.ensure(16 * sizeof(unsigned long long));
  HIPCHECK(hipEventRecord(s->ev0, s->stream));
  if (g.fn_bits && s->n_events) {  // begin-hit bitmap: quiet lanes skip 64 events per load
    a.bhits = s->bhits.as<uint64_t>();
    const uint64_t nb = nb_bits;
    if (wm_here) {  // (run_nfa's scratch memset above cleared wmax)
      a.wm_blocks = s->wm_blocks.as<int64_t>();
      a.n_wm_blocks = nb;
      a.wmax = &sc->wmax;
    }
    HIPCHECK(launch_fn(g.fn_bits, a, nb, s->stream));
  }
  // Lane order: keys sorted by estimated work, longest first (cep_nfa_est, from the begin-hit bitmap), so a wave's 64
  // lanes carry similar work (a wave lasts as long as its longest lane) and the longest waves
  // start first.  (A stream's run queues live at the key's position, so its lanes too may run
  // in any order; its estimate adds the runs each key carries.)
  if (g.fn_est && nk > 64) {
    a.est = g.est.as<uint32_t>();
    a.est_blend = streaming && !s->tune.no_est_blend ? 1u : 0u;  // ($CEP_NO_EST_BLEND: measurement runs)
    const uint64_t eg = est_lanes(s->n_events, nk);  // lanes per key
    HIPCHECK(launch_fn(g.fn_est, a, (nk * eg + 255) / 256, s->stream));
    a.wmax = nullptr;  // (reduced once; wm_blocks stays set: no other kernel reads it)
    HIPCHECK(sort_keys_by_work(g.est.as<uint32_t>(), g.est_sorted.as<uint32_t>(), g.order_tmp.as<uint32_t>(),
                               g.order.as<uint32_t>(), nk, g.sort_tmp, g.sort_tmp_bytes, s->stream));
    a.order = g.order.as<uint32_t>();
    g.est_valid = true;
  } else {
    g.est_valid = false;
  }
  const bool prof = s->tune.prof;  // (the query must be compiled with it too)
  if (prof) {
    HIPCHECK(hipMemsetAsync(s->prof.p, 0, 16 * sizeof(unsigned long long), s->stream));
    a.prof = s->prof.as<unsigned long long>();
  }
  HIPCHECK(hipEventRecord(s->ev2, s->stream));
  // ($CEP_STREAM_NARROW: a stream on the narrow build - no put log, so a walk conflict is a sticky
  // error - and $CEP_STREAM_NO_ORDER: without the lane order; measurement runs only)
  const bool stream_narrow = s->tune.stream_narrow;
  if (streaming && s->tune.stream_no_order) a.order = nullptr;
  if (streaming && g.fn_stream) HIPCHECK(launch_fn(g.fn_stream, a, (slots + 255) / 256, s->stream));
  else HIPCHECK(launch_nfa_tier(g, r0.q, a, slots, s->stream, streaming && !stream_narrow));
  HIPCHECK(hipEventRecord(s->ev1, s->stream));
  launches++;
  Scratch h{};
  HIPCHECK(hipMemcpyAsync(&h, sc, sizeof h, hipMemcpyDeviceToHost, s->stream));
  uint32_t tops[2] = {0, 0};  // a stream's pool tops, read back with the counters (one wait)
  if (streaming) HIPCHECK(hipMemcpyAsync(tops, S.tops.p, sizeof tops, hipMemcpyDeviceToHost, s->stream));
  HIPCHECK(hipStreamSynchronize(s->stream));
  if (wm_here) s->watermark = (int64_t)(h.wmax ^ 0x8000000000000000ull);
  if (prof) {  // one line per launch on stderr: the counters of nfa_lane.h's CEP_PROF list
    unsigned long long pc[16];
    copy_sync(pc, s->prof.p, sizeof pc, hipMemcpyDeviceToHost, s->stream);
    std::fprintf(stderr, "cep_prof {\"jobs\": %llu, \"c\": [", (unsigned long long)jobs);
    for (int i = 0; i < 14; i++) std::fprintf(stderr, "%s%llu", i ? ", " : "", pc[i]);
    std::fprintf(stderr, "]}\n");
    a.prof = nullptr;
  }
  float ms = 0;
  HIPCHECK(hipEventElapsedTime(&ms, s->ev0, s->ev1));
  total_ms += ms;
  float main_ms = 0;  // the matching launch alone (before any continuation below)
  HIPCHECK(hipEventElapsedTime(&main_ms, s->ev2, s->ev1));
  uint32_t widened = 0;  // keys the wide build continued (streams), and its launch time
  float widen_ms = 0;
  if (streaming && g.fn_stream && h.n_cap_err > 0) {
    // keys the stream build stopped before an event their versions outgrew 3 pairs at
    // (KE_WIDEN): the wide build continues each from that event over the same state
    s->keylist.ensure(sizeof(uint32_t) * 2 * h.n_cap_err);
    uint32_t* cap_list = s->keylist.as<uint32_t>();
    uint32_t* widen_list = cap_list + h.n_cap_err;
    HIPCHECK(hipMemsetAsync(&sc->n_retry_cap, 0, 2 * sizeof(uint32_t), s->stream));
    HIPCHECK(launch_collect_retry(g.ks.as<KeyState>(), jobs, cap_list, widen_list, &sc->n_retry_cap, s->stream));
    uint32_t lens[2];
    HIPCHECK(hipMemcpyAsync(lens, &sc->n_retry_cap, sizeof lens, hipMemcpyDeviceToHost, s->stream));
    HIPCHECK(hipStreamSynchronize(s->stream));
    if (lens[1]) {
      a.jobs = widen_list;
      a.n_jobs = lens[1];
      a.widen = 1;
      a.order = nullptr;
      a.spread = 0;
      a.spread_iso = 0;
      HIPCHECK(hipEventRecord(s->ev0, s->stream));
      HIPCHECK(launch_nfa_tier(g, r0.q, a, lens[1], s->stream, true));
      HIPCHECK(hipEventRecord(s->ev1, s->stream));
      launches++;
      HIPCHECK(hipMemcpyAsync(&h, sc, sizeof h, hipMemcpyDeviceToHost, s->stream));
      HIPCHECK(hipStreamSynchronize(s->stream));
      HIPCHECK(hipEventElapsedTime(&widen_ms, s->ev0, s->ev1));
      total_ms += widen_ms;
      widened = lens[1];
      g.stream_widened += lens[1];
      a.jobs = nullptr;
      a.widen = 0;
    }
  }
  if (streaming) {  // no re-runs: a key that hit a limit keeps its error (sticky, reported)
    if (widened) copy_sync(tops, S.tops.p, sizeof tops, hipMemcpyDeviceToHost, s->stream);  // (moved on)
    S.node_used = (uint32_t)std::min<uint64_t>(tops[0], S.node_cap);
    S.pred_used = (uint32_t)std::min<uint64_t>(tops[1], S.pred_cap);
    h.n_cap_err = 0;
  }
  g.last_nodes = h.node_top;
  g.last_preds = h.pred_top;
  g.last_out = h.out_top;
  // a run queue overflowed: its jobs are re-run below, and the next batch starts with 4x the
  // slots (run queues past the LDS slots live in HBM: a bigger ring costs memory, not time),
  // the ring kept within 32 GiB
  if (!streaming && (h.full & 1u)) {
    uint32_t nr = rcap * 4;
    while (nr > rcap && ring_size(g.F, std::max<uint64_t>(slots, 1), nr) > (32ull << 30)) nr /= 2;
    g.rcap_hint = nr;
  }

  // Re-run the jobs that hit a capacity limit (with 8x the run queue and 4x every exhausted
  // pool; walks still deferred) and those whose deferred walks conflicted,
  // in the wide Dewey build (a narrow-build job whose version outgrew 3 pairs is a capacity
  // re-run too).
  // The job lists are collected on the device; only their lengths come back.
  g.stats = cep_batch_stats{};
  g.stats.group_queries = (uint32_t)Q;
  g.stats.main_ms = main_ms;
  g.stats.retried_jobs = widened;  // (streams: the keys the wide build continued)
  g.stats.retry_ms = widen_ms;
  if (s->tune.no_retry) h.n_cap_err = 0;  // (measurement runs: which keys a build cannot finish)
  for (int round = 0; h.n_cap_err > 0 && round < 8; round++) {
    const uint64_t nlist = h.n_cap_err;
    s->keylist.ensure(sizeof(uint32_t) * 2 * nlist);
    uint32_t* cap_list = s->keylist.as<uint32_t>();
    uint32_t* conf_list = cap_list + nlist;
    HIPCHECK(launch_collect_retry(g.ks.as<KeyState>(), jobs, cap_list, conf_list, &sc->n_retry_cap, s->stream));
    // grow every pool a job ran out of (indices of the used prefix stay valid)
    const bool node_full = h.node_top >= node_cap - nchunk, pred_full = h.pred_top >= pred_cap - pchunk;
    const bool out_full = (uint64_t)h.out_top + ochunk > out_cap;
    const uint64_t nn = node_full ? std::min<uint64_t>(node_cap * 4 + nlist * 64, kNodeMax) : node_cap;
    const uint64_t pn = pred_full ? std::min<uint64_t>(pred_cap * 4 + nlist * 64, kNodeMax) : pred_cap;
    const uint64_t on = out_full ? std::min<uint64_t>(out_cap * 4 + nlist, kPoolMax) : out_cap;
    s->nodes.grow_keep(sizeof(Node) * nn, sizeof(Node) * std::min<uint64_t>(h.node_top, node_cap), s->stream);
    s->preds0.grow_keep(sizeof(Pred) * nn, sizeof(Pred) * std::min<uint64_t>(h.node_top, node_cap), s->stream);
    s->preds.grow_keep(sizeof(Pred) * pn, sizeof(Pred) * std::min<uint64_t>(h.pred_top, pred_cap), s->stream);
    s->out.grow_keep(sizeof(uint32_t) * kOutChunkWords * on,
                     sizeof(uint32_t) * kOutChunkWords * std::min<uint64_t>(h.out_top, out_cap), s->stream);
    Scratch fix{};  // pool tops may have run past the caps; restart them at the old caps
    fix.node_top = (uint32_t)std::min<uint64_t>(h.node_top, node_cap);
    fix.pred_top = (uint32_t)std::min<uint64_t>(h.pred_top, pred_cap);
    fix.out_top = (uint32_t)std::min<uint64_t>(h.out_top, out_cap);
    uint32_t lens[2];
    HIPCHECK(hipMemcpyAsync(lens, &sc->n_retry_cap, sizeof lens, hipMemcpyDeviceToHost, s->stream));
    HIPCHECK(hipStreamSynchronize(s->stream));
    HIPCHECK(hipMemcpyAsync(sc, &fix, sizeof fix, hipMemcpyHostToDevice, s->stream));
    node_cap = nn;
    pred_cap = pn;
    out_cap = on;
    a.nodes = s->nodes.as<Node>();
    a.preds = s->preds.as<Pred>();
    a.preds0 = s->preds0.as<Pred>();
    a.out = s->out.as<uint32_t>();
    a.node_pool.cap = (uint32_t)node_cap;
    a.pred_pool.cap = (uint32_t)pred_cap;
    a.out_pool.cap = (uint32_t)out_cap;
    // a bigger run queue per retried job, its ring kept within 16 GiB
    rcap *= 8;
    // (re-runs take the wide build: its occupancy; the interpreter tier keeps the default)
    auto grid_re = [&](uint64_t n) { return g.fn ? grid_wide(n) : grid_for(n); };
    const uint64_t most = grid_re(std::max<uint64_t>(lens[0], lens[1]));
    // (the walk queues' put logs grow with rcap too: both within the cap)
    while (rcap > 32 && most &&
           ring_size(g.F, most, rcap) + walkq_size(most, wcap, put_log_entries(rcap)) > (16ull << 30))
      rcap /= 2;
    a.rcap = rcap;
    s->retry_rings.ensure(ring_size(g.F, std::max<uint64_t>(most, 1), rcap));
    plog = put_log_entries(rcap);
    a.plog = plog;
    s->walks.ensure(walkq_size(std::max<uint64_t>(most, 1), wcap, plog));  // (may move: re-read below)
    a.rings = s->retry_rings.p;
    a.walks = s->walks.p;
    a.order = nullptr;
    a.spread = 0;
    a.spread_iso = 0;
    HIPCHECK(hipEventRecord(s->ev0, s->stream));
    // capacity re-runs keep deferred walks; conflicts too (the wide build resolves them
    // exactly through its put log, nfa_lane.h), except after a put log overflowed: in place
    for (int k = 0; k < 2; k++) {
      if (!lens[k]) continue;
      a.defer = (k == 0 || round == 0) ? 1 : 0;
      a.jobs = k == 0 ? cap_list : conf_list;
      a.n_jobs = lens[k];
      a.job_next = &sc->job_next;  // re-runs always on persistent lanes
      HIPCHECK(hipMemsetAsync(&sc->job_next, 0, sizeof(uint32_t), s->stream));
      HIPCHECK(launch_nfa_tier(g, r0.q, a, grid_re(lens[k]), s->stream, true));
      launches++;
      g.stats.retried_jobs += lens[k];
    }
    HIPCHECK(hipEventRecord(s->ev1, s->stream));
    HIPCHECK(hipMemcpyAsync(&h, sc, sizeof h, hipMemcpyDeviceToHost, s->stream));
    HIPCHECK(hipStreamSynchronize(s->stream));
    HIPCHECK(hipEventElapsedTime(&ms, s->ev0, s->ev1));
    total_ms += ms;
    g.stats.retry_ms += ms;
    g.last_nodes = h.node_top;
    g.last_preds = h.pred_top;
    g.last_out = h.out_top;
  }

  g.stats.kernel_ms = total_ms;
  g.stats.launches = launches;
  g.stats.nodes_used = std::min<uint64_t>(h.node_top, node_cap);
  g.stats.preds_used = std::min<uint64_t>(h.pred_top, pred_cap);
  g.stats.out_chunks_used = std::min<uint64_t>(h.out_top, out_cap);
  // compaction per query: scans of per-key counts, then the scatter into flat arrays
  const uint64_t nb = (nk + 255) / 256;
  s->bsum.ensure(sizeof(uint64_t) * 2 * (nb + 1));
  uint64_t* bm = s->bsum.as<uint64_t>();
  uint64_t* bp = bm + nb + 1;
  for (uint64_t qi = 0; qi < Q; qi++) {
    QueryRt& r = *s->qs[g.members[qi]];
    const KeyState* ks = g.ks.as<KeyState>() + qi * nk;
    r.ks_dev = ks;
    HIPCHECK(hipEventRecord(s->ev0, s->stream));
    HIPCHECK(launch_compact(ks, nk, bm, bp, sc->totals, s->stream));
    uint64_t tot[2] = {0, 0};
    HIPCHECK(hipMemcpyAsync(tot, sc->totals, sizeof tot, hipMemcpyDeviceToHost, s->stream));
    HIPCHECK(hipStreamSynchronize(s->stream));
    r.n_matches = tot[0];
    r.n_pairs = tot[1];
    r.m_key.ensure(sizeof(uint32_t) * (tot[0] + 1));
    r.m_emit.ensure(sizeof(uint32_t) * (tot[0] + 1));
    r.m_off.ensure(sizeof(uint64_t) * (tot[0] + 1));
    r.p_seq.ensure(sizeof(uint32_t) * (tot[1] + 1));
    r.p_stage.ensure(sizeof(uint16_t) * (tot[1] + 1));
    s->heavy.ensure(scatter_heavy_bytes(nk));
    HIPCHECK(launch_scatter(ks, nk, bm, bp, s->out.as<uint32_t>(), r.m_key.as<uint32_t>(), r.m_emit.as<uint32_t>(),
                            r.m_off.as<uint64_t>(), r.p_seq.as<uint32_t>(), r.p_stage.as<uint16_t>(), sc->totals,
                            s->heavy.p, s->stream));
    if (nk == 0) HIPCHECK(hipMemsetAsync(r.m_off.p, 0, sizeof(uint64_t), s->stream));
    HIPCHECK(hipEventRecord(s->ev1, s->stream));
    HIPCHECK(hipStreamSynchronize(s->stream));
    HIPCHECK(hipEventElapsedTime(&ms, s->ev0, s->ev1));
    r.aux_ms = ms;  // compaction (count/scan/scatter)
    r.digest_valid = false;
    r.arity = 0;
    r.kernel_ms = total_ms;  // the group's matching launches
    r.launches = launches;
    r.acc_kernel_ms += r.kernel_ms;
    r.acc_aux_ms += r.aux_ms;
    r.acc_batches++;
  }
}

int guarded(const std::function<void()>& f) {
  try {
    f();
    return CEP_OK;
  } catch (HipError& e) {
    return fail(CEP_E_HIP, e.what());
  } catch (std::bad_alloc&) {
    return fail(CEP_E_NOMEM, "device allocation failed");
  } catch (std::exception& e) {
    return fail(CEP_E_INVALID, e.what());
  }
}

}  // namespace

extern "C" {

const char* cep_last_error(void) { return g_err.c_str(); }

int cep_query_compile(const uint8_t* ir, size_t n, cep_query** out) {
  if (!ir || !out) return fail(CEP_E_INVALID, "null argument");
  auto q = std::make_unique<cep_query>();
  try {
    compile_query(ir, n, q.get());
  } catch (std::exception& e) {
    return fail(CEP_E_COMPILE, e.what());
  }
  *out = q.release();
  return CEP_OK;
}

int cep_query_info_get(const cep_query* q, cep_query_info* info) {
  if (!q || !info) return fail(CEP_E_INVALID, "null argument");
  *info = q->info;
  return CEP_OK;
}

const char* cep_query_stage_name(const cep_query* q, uint32_t id) {
  if (!q || id >= q->names.size()) return nullptr;
  return q->names[id].c_str();
}

void cep_query_destroy(cep_query* q) { delete q; }

const char* cep_query_jit_source(const cep_query* q) { return q ? q->jitSource.c_str() : nullptr; }

int cep_jit_precompile(const cep_query* q, double* compile_s) {
  if (!q) return fail(CEP_E_INVALID, "null query");
  try {
    double w = 0;
    jit_code_object(q->jitSource, compile_s, true);
    jit_code_object(jit_wide_source(q->jitSource), &w, true);
    if (compile_s) *compile_s += w;
    jit_code_object(jit_stream_source(q->jitSource), &w, true);  // (streaming sessions over the query)
    if (compile_s) *compile_s += w;
  } catch (std::exception& e) {
    return fail(CEP_E_COMPILE, e.what());
  }
  return CEP_OK;
}

int cep_jit_precompile_group(const cep_query* const* queries, int n_queries, double* compile_s) {
  if (!queries || n_queries <= 0) return fail(CEP_E_INVALID, "need at least one query");
  std::vector<const cep_query*> qv;
  for (int i = 0; i < n_queries; i++) {
    if (!queries[i]) return fail(CEP_E_INVALID, "null query");
    if (!queries[i]->info.compile_error) qv.push_back(queries[i]);
  }
  if (compile_s) *compile_s = 0;
  try {
    for (auto& pl : plan_groups(qv)) {
      double t = 0, w = 0;
      jit_code_object(pl.source, &t, true);
      jit_code_object(jit_wide_source(pl.source), &w, true);
      if (compile_s) *compile_s += t + w;
    }
  } catch (std::exception& e) {
    return fail(CEP_E_COMPILE, e.what());
  }
  return CEP_OK;
}

int cep_query_group_plan(const cep_query* const* queries, int n_queries, int group, const char** source,
                         uint32_t* n_members, const int32_t** members, uint32_t* n_literals,
                         const int64_t** literals) {
  thread_local GroupPlan plan;
  thread_local std::vector<int32_t> mem;
  if (!queries || n_queries <= 0 || group < 0) return fail(CEP_E_INVALID, "bad argument");
  std::vector<const cep_query*> qv;
  std::vector<int> idx;
  for (int i = 0; i < n_queries; i++) {
    if (!queries[i]) return fail(CEP_E_INVALID, "null query");
    if (!queries[i]->info.compile_error) {
      qv.push_back(queries[i]);
      idx.push_back(i);
    }
  }
  try {
    auto plans = plan_groups(qv);
    if (group >= (int)plans.size()) return fail(CEP_E_INVALID, "no such group");
    plan = std::move(plans[group]);
  } catch (std::exception& e) {
    return fail(CEP_E_COMPILE, e.what());
  }
  mem.clear();
  for (int m : plan.members) mem.push_back(idx[m]);
  if (source) *source = plan.source.c_str();
  if (n_members) *n_members = (uint32_t)mem.size();
  if (members) *members = mem.data();
  if (n_literals) *n_literals = plan.nkc;
  if (literals) *literals = plan.table.data();
  return CEP_OK;
}

int cep_session_create(const cep_query* const* queries, int n_queries, const cep_opts* opts, cep_session** out) {
  if (!queries || n_queries <= 0 || !out) return fail(CEP_E_INVALID, "need at least one query");
  for (int i = 0; i < n_queries; i++) {
    if (!queries[i]) return fail(CEP_E_INVALID, "null query");
    if (queries[i]->info.compile_error)
      return fail(CEP_E_COMPILE, "query " + std::to_string(i) + " does not compile in the reference");
    if (queries[i]->info.n_fields != queries[0]->info.n_fields)
      return fail(CEP_E_INVALID, "queries of a session must share the event schema");
  }
  auto s = std::make_unique<cep_session>();
  if (opts) s->opts = *opts;
  s->tune = cep::tuning_from_env();  // (the only read of the measurement knobs: not per launch)
  if (s->tune.host_trace) g_host_trace = true;
  g_poison = s->tune.poison;
  g_poison_byte = s->tune.poison_byte;
  g_poison_base = g_allocs;
  for (int i = 0; i < n_queries; i++)
    if (queries[i]->windowed && s->opts.tier != CEP_TIER_JIT)
      return fail(CEP_E_INVALID, "semantic WITHIN runs on the JIT tier only");
  s->device = s->opts.device;
  int rc = guarded([&] {
    DeviceGuard g(s->device);
    HIPCHECK(hipSetDevice(s->device));
    HIPCHECK(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    HIPCHECK(hipDeviceGetAttribute(&s->cus, hipDeviceAttributeMultiprocessorCount, s->device));
    HIPCHECK(hipEventCreate(&s->ev0));
    HIPCHECK(hipEventCreate(&s->ev1));
    HIPCHECK(hipEventCreate(&s->ev2));
    for (int i = 0; i < n_queries; i++) {
      auto r = std::make_unique<QueryRt>();
      r->q = queries[i];
      r->F = queries[i]->F;  // fold slots of a run record (compile.cpp)
      r->d_q.ensure(sizeof(DevQuery));
      copy_sync(r->d_q.p, &queries[i]->dev, sizeof(DevQuery), hipMemcpyHostToDevice, s->stream);
      r->d_code.ensure(sizeof(uint32_t) * queries[i]->code.size());
      copy_sync(r->d_code.p, queries[i]->code.data(), sizeof(uint32_t) * queries[i]->code.size(),
                hipMemcpyHostToDevice, s->stream);
      s->qs.push_back(std::move(r));
    }
    // kernel groups: the JIT tier of a per-batch session runs queries that differ only in
    // literals as one launch (plan_groups); streams and the interpreter run one query each
    std::vector<int> nfa;
    for (int i = 0; i < n_queries; i++)
      if (queries[i]->info.kind == CEP_KIND_NFA || s->opts.force_nfa || s->opts.streaming) nfa.push_back(i);
    std::vector<GroupPlan> plans;
    if (s->opts.tier == CEP_TIER_JIT && !s->opts.streaming && !s->opts.no_groups) {
      std::vector<const cep_query*> qv;
      for (int i : nfa) qv.push_back(queries[i]);
      plans = plan_groups(qv);
      for (auto& pl : plans)
        for (int& m : pl.members) m = nfa[m];
    } else {
      for (int i : nfa) {
        GroupPlan pl;
        pl.members.push_back(i);
        pl.source = queries[i]->jitSource;
        plans.push_back(std::move(pl));
      }
    }
    for (auto& pl : plans) {
      auto g = std::make_unique<GroupRt>();
      g->members = pl.members;
      g->F = s->qs[pl.members[0]]->F;
      for (size_t k = 0; k < pl.members.size(); k++) {
        s->qs[pl.members[k]]->group = (int)s->groups.size();
        s->qs[pl.members[k]]->qi = (uint32_t)k;
      }
      {  // (the source's CEP_WALK_FLUSH: the value its kernels drain at, whatever the session's
         // environment says now - ADVICE r4)
        const size_t at = pl.source.find("#define CEP_WALK_FLUSH ");
        if (at != std::string::npos) g->walk_flush = (uint32_t)std::strtoul(pl.source.c_str() + at + 23, nullptr, 10);
      }
      if (s->opts.tier == CEP_TIER_JIT) {  // the group's own kernel, compiled by hipRTC
        std::vector<char> co = jit_code_object(pl.source, &g->jit_compile_s);
        HIPCHECK(hipModuleLoadData(&g->mod, co.data()));
        HIPCHECK(hipModuleGetFunction(&g->fn, g->mod, "cep_nfa_jit"));
        double w = 0;
        std::vector<char> cw = jit_code_object(jit_wide_source(pl.source), &w);
        g->jit_compile_s += w;
        HIPCHECK(hipModuleLoadData(&g->mod_wide, cw.data()));
        HIPCHECK(hipModuleGetFunction(&g->fn_wide, g->mod_wide, "cep_nfa_jit"));
        // streams run the stream build: 3-pair versions at 3 waves per SIMD, a key whose
        // versions outgrow them continued by the wide build (run_nfa)
        if (s->opts.streaming && !s->tune.stream_wide && !s->tune.stream_narrow) {
          std::vector<char> cs = jit_code_object(jit_stream_source(pl.source), &w);
          g->jit_compile_s += w;
          HIPCHECK(hipModuleLoadData(&g->mod_stream, cs.data()));
          HIPCHECK(hipModuleGetFunction(&g->fn_stream, g->mod_stream, "cep_nfa_jit"));
        }
        // the kernels' occupancy (waves per SIMD as compiled: 3 narrow, 2 wide or coop) sizes the
        // persistent and spread grids (run_nfa)
        int nb = 0;
        if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&nb, g->fn, 256, 0) == hipSuccess && nb > 0)
          g->waves_cu = (uint32_t)nb * 4;
        nb = 0;
        if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&nb, g->fn_wide, 256, 0) == hipSuccess && nb > 0)
          g->waves_cu_wide = (uint32_t)nb * 4;
        nb = 0;
        if (g->fn_stream && hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&nb, g->fn_stream, 256, 0) == hipSuccess &&
            nb > 0)
          g->waves_cu_stream = (uint32_t)nb * 4;
        if (pl.source.find("cep_nfa_est") != std::string::npos) {  // (a failed lookup would stick)
          HIPCHECK(hipModuleGetFunction(&g->fn_est, g->mod, "cep_nfa_est"));
          HIPCHECK(hipModuleGetFunction(&g->fn_bits, g->mod, "cep_nfa_bits"));
        }
      }
      if (pl.nkc) {
        g->kc.ensure(sizeof(int64_t) * pl.table.size());
        copy_sync(g->kc.p, pl.table.data(), sizeof(int64_t) * pl.table.size(), hipMemcpyHostToDevice, s->stream);
      }
      s->groups.push_back(std::move(g));
    }
  });
  if (rc) return rc;
  *out = s.release();
  return CEP_OK;
}

int cep_session_reset(cep_session* s) {
  if (!s) return fail(CEP_E_INVALID, "null session");
  return guarded([&] {
    DeviceGuard g(s->device);
    HIPCHECK(hipStreamSynchronize(s->stream));
    for (auto& r : s->qs) {
      StreamState& S = r->st;
      if (!S.init) continue;
      // KeyCarry.live = 0: each key restarts from the initial state at its next batch (its ring
      // slots are rewritten from scratch); empty pools
      HIPCHECK(hipMemsetAsync(S.carry.p, 0, sizeof(KeyCarry) * std::max<uint64_t>(S.n_keys, 1), s->stream));
      HIPCHECK(hipMemsetAsync(S.tops.p, 0, 2 * sizeof(uint32_t), s->stream));
      if (S.node_used) HIPCHECK(hipMemsetAsync(S.nodes.p, 0, sizeof(Node) * S.node_used, s->stream));
      S.node_used = S.pred_used = 0;
    }
    s->watermark = INT64_MIN;
    HIPCHECK(hipStreamSynchronize(s->stream));
  });
}

void cep_session_destroy(cep_session* s) {
  if (!s) return;
  {
    DeviceGuard g(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    s->groups.clear();
    s->qs.clear();
    if (s->h_wm) (void)hipHostFree(s->h_wm);
    if (s->ev0) (void)hipEventDestroy(s->ev0);
    if (s->ev1) (void)hipEventDestroy(s->ev1);
    if (s->ev2) (void)hipEventDestroy(s->ev2);
    if (s->stream) (void)hipStreamDestroy(s->stream);
  }
  delete s;
}

// arrival-order batch -> s->key_off / s->cols / s->ts in CSR order (partition.hip)
static void partition_batch(cep_session* s, const cep_batch* b) {
  const cep_query* q0 = s->qs[0]->q;
  const uint32_t nf = q0->info.n_fields;
  const uint64_t n = b->n_events, nk = b->n_keys;
  const uint32_t* keys = b->arrival_key;
  Cols in{}, out{};
  const int64_t* ts = b->ts;
  uint32_t wide = 0;
  for (uint32_t f = 0; f < nf; f++) wide |= (q0->dev.field_type[f] == 1 ? 0u : 1u) << f;
  if (b->memory != CEP_MEM_DEVICE) {
    s->a_keys.ensure(4 * std::max<uint64_t>(n, 1));
    if (n) HIPCHECK(hipMemcpyAsync(s->a_keys.p, keys, 4 * n, hipMemcpyHostToDevice, s->stream));
    keys = s->a_keys.as<uint32_t>();
    for (uint32_t f = 0; f < nf; f++) {
      const size_t esz = (wide >> f) & 1u ? 8 : 4;
      s->a_cols[f].ensure(esz * std::max<uint64_t>(n, 1));
      if (n) HIPCHECK(hipMemcpyAsync(s->a_cols[f].p, b->cols[f], esz * n, hipMemcpyHostToDevice, s->stream));
      in.p[f] = s->a_cols[f].p;
    }
    if (ts) {
      s->a_ts.ensure(8 * std::max<uint64_t>(n, 1));
      if (n) HIPCHECK(hipMemcpyAsync(s->a_ts.p, ts, 8 * n, hipMemcpyHostToDevice, s->stream));
      ts = s->a_ts.as<int64_t>();
    }
  } else {
    for (uint32_t f = 0; f < nf; f++) in.p[f] = b->cols[f];
  }
  for (uint32_t f = 0; f < nf; f++) {
    s->p_cols[f].ensure(((wide >> f) & 1u ? 8 : 4) * std::max<uint64_t>(n, 1));
    out.p[f] = s->p_cols[f].p;
  }
  if (ts) s->p_ts.ensure(8 * std::max<uint64_t>(n, 1));
  s->p_off.ensure(8 * (nk + 1));
  s->p_cnt.ensure(8 * (nk + 1));
  s->p_perm.ensure(4 * std::max<uint64_t>(n, 1));
  s->p_sorted.ensure(4 * std::max<uint64_t>(n, 1));
  s->p_idx.ensure(4 * std::max<uint64_t>(n, 1));
  const size_t sb = partition_scratch_bytes(n, nk);
  s->p_scratch.ensure(sb);
  s->scratch.ensure(sizeof(Scratch));
  Scratch* sc = s->scratch.as<Scratch>();
  HIPCHECK(hipMemsetAsync(&sc->overflow, 0, sizeof(uint32_t), s->stream));
  HIPCHECK(hipEventRecord(s->ev0, s->stream));
  HIPCHECK(partition(keys, n, nk, (int)nf, in, out, wide, ts, ts ? s->p_ts.as<int64_t>() : nullptr,
                     s->p_off.as<uint64_t>(), s->p_cnt.as<uint64_t>(), s->p_perm.as<uint32_t>(),
                     s->p_sorted.as<uint32_t>(), s->p_idx.as<uint32_t>(), s->p_scratch.p, sb, &sc->overflow,
                     s->stream, s->tune.part_rounds));
  HIPCHECK(hipEventRecord(s->ev1, s->stream));
  uint32_t bad = 0;
  HIPCHECK(hipMemcpyAsync(&bad, &sc->overflow, sizeof bad, hipMemcpyDeviceToHost, s->stream));
  HIPCHECK(hipStreamSynchronize(s->stream));
  HIPCHECK(hipEventElapsedTime(&s->partition_ms, s->ev0, s->ev1));
  if (bad) throw std::invalid_argument("arrival_key: a key id >= n_keys");
  s->key_off = s->p_off.as<uint64_t>();
  s->cols = out;
  s->ts = ts ? s->p_ts.as<int64_t>() : nullptr;
}

int cep_push_batch(cep_session* s, const cep_batch* b) {
  if (!s || !b || (!b->key_off && !b->arrival_key) || (!b->cols && b->n_events))
    return fail(CEP_E_INVALID, "null argument");
  if (b->n_keys >= 0xFFFFFFFFull || b->n_events >= 0xFFFFFFFFull)
    return fail(CEP_E_INVALID, "a batch holds < 2^32 keys and events (sequence numbers are u32)");
  if (b->arrival_key && b->n_events >= 0x80000000ull)
    return fail(CEP_E_INVALID, "an arrival-order batch holds < 2^31 events (split it)");
  const uint32_t allocs0 = g_allocs;
  const int rc = guarded([&] {
    DeviceGuard g(s->device);
    const cep_query* q0 = s->qs[0]->q;
    const uint32_t nf = q0->info.n_fields;
    s->n_keys = b->n_keys;
    s->n_events = b->n_events;
    for (auto& r : s->qs) {
      r->have = false;
      r->host_valid = false;
      r->pending = false;  // (its timing stays in the ring: still accumulated)
    }
    s->arrival = b->arrival_key != nullptr;
    s->partition_ms = 0;
    s->layout_host_valid = false;
    if (s->arrival) {
      const double t0 = host_trace() ? now_ms() : 0;
      partition_batch(s, b);
      if (host_trace()) std::fprintf(stderr, "cep_host partition %.2f ms\n", now_ms() - t0);
    } else if (b->memory == CEP_MEM_DEVICE) {
      s->key_off = b->key_off;
      for (uint32_t f = 0; f < nf; f++) s->cols.p[f] = b->cols[f];
      s->ts = b->ts;
    } else {
      s->b_off.ensure(sizeof(uint64_t) * (b->n_keys + 1));
      HIPCHECK(hipMemcpyAsync(s->b_off.p, b->key_off, sizeof(uint64_t) * (b->n_keys + 1), hipMemcpyHostToDevice,
                              s->stream));
      s->key_off = s->b_off.as<uint64_t>();
      for (uint32_t f = 0; f < nf; f++) {
        const size_t esz = q0->dev.field_type[f] == 1 ? 4 : 8;
        s->b_cols[f].ensure(esz * std::max<uint64_t>(b->n_events, 1));
        if (b->n_events)
          HIPCHECK(hipMemcpyAsync(s->b_cols[f].p, b->cols[f], esz * b->n_events, hipMemcpyHostToDevice, s->stream));
        s->cols.p[f] = s->b_cols[f].p;
      }
      if (b->ts) {
        s->b_ts.ensure(sizeof(int64_t) * std::max<uint64_t>(b->n_events, 1));
        HIPCHECK(hipMemcpyAsync(s->b_ts.p, b->ts, sizeof(int64_t) * b->n_events, hipMemcpyHostToDevice, s->stream));
        s->ts = s->b_ts.as<int64_t>();
      } else {
        s->ts = nullptr;
      }
      // host buffers are borrowed for the call only: the copies (truly asynchronous from pinned
      // memory) must be done before returning, even when only stencil work follows
      HIPCHECK(hipStreamSynchronize(s->stream));
    }
    // watermark.  When the batch runs an NFA group with a begin-hit bitmap and a lane order,
    // the max is folded into those passes (run_nfa: block maxima in cep_nfa_bits, reduced by
    // cep_nfa_est), which stream the batch anyway; otherwise its own pass over the timestamps
    s->watermark = INT64_MIN;
    s->wm_pending = false;
    s->wm_fold = s->ts && s->n_events && !s->groups.empty() && s->groups[0]->fn_bits && s->groups[0]->fn_est &&
                 s->n_keys > 64 && !s->tune.no_wm_fold;
    if (s->ts && s->n_events && !s->wm_fold) {  // read back with the batch's other results (resolve())
      s->scratch.ensure(sizeof(Scratch));
      Scratch* sc = s->scratch.as<Scratch>();
      if (!s->h_wm) HIPCHECK(hipHostMalloc((void**)&s->h_wm, sizeof(unsigned long long), hipHostMallocDefault));
      HIPCHECK(hipMemsetAsync(&sc->wmax, 0, sizeof(unsigned long long), s->stream));
      HIPCHECK(launch_max(s->ts, s->n_events, &sc->wmax, s->stream));
      HIPCHECK(hipMemcpyAsync(s->h_wm, &sc->wmax, sizeof(unsigned long long), hipMemcpyDeviceToHost, s->stream));
      s->wm_pending = true;
    }
    // persistent lanes claim job indices 128 at a time from a u32 counter (nfa_lane.h
    // run_jobs): every resident wave (at most 64 per CU) may claim up to 128 past the last job
    const uint64_t claim_slack = (uint64_t)s->cus * 64 * 128;
    if (s->groups.size() && (uint64_t)s->qs.size() * s->n_keys + claim_slack >= 0xFFFFFFFFull)
      throw std::invalid_argument("queries x keys of a batch must stay below 2^32 (job ids are u32)");
    for (auto& r : s->qs)  // a stream carries NFA state between batches: stencil queries run on the NFA there
      if (r->group < 0) run_stencil(s, *r);
    const double t0 = host_trace() ? now_ms() : 0;
    for (auto& g : s->groups) run_nfa(s, *g);
    if (host_trace()) std::fprintf(stderr, "cep_host run_nfa %.2f ms\n", now_ms() - t0);
    for (auto& r : s->qs) r->have = true;
  });
  s->last_allocs = g_allocs - allocs0;
  return rc;
}

int cep_batch_layout(cep_session* s, int memory, const uint64_t** key_off, const uint32_t** arrival_index,
                     double* partition_ms) {
  if (!s) return fail(CEP_E_INVALID, "null session");
  if (!s->key_off) return fail(CEP_E_STATE, "no batch has been pushed");
  return guarded([&] {
    DeviceGuard g(s->device);
    if (partition_ms) *partition_ms = s->partition_ms;
    if (memory == CEP_MEM_DEVICE) {
      if (key_off) *key_off = s->key_off;
      if (arrival_index) *arrival_index = s->arrival ? s->p_perm.as<uint32_t>() : nullptr;
      return;
    }
    if (!s->layout_host_valid) {
      s->h_off.resize(s->n_keys + 1);
      HIPCHECK(hipMemcpyAsync(s->h_off.data(), s->key_off, 8 * (s->n_keys + 1), hipMemcpyDeviceToHost, s->stream));
      s->h_perm.resize(s->arrival ? s->n_events : 0);
      if (s->arrival && s->n_events)
        HIPCHECK(hipMemcpyAsync(s->h_perm.data(), s->p_perm.p, 4 * s->n_events, hipMemcpyDeviceToHost, s->stream));
      HIPCHECK(hipStreamSynchronize(s->stream));
      s->layout_host_valid = true;
    }
    if (key_off) *key_off = s->h_off.data();
    if (arrival_index) *arrival_index = s->arrival ? s->h_perm.data() : nullptr;
  });
}

int cep_sync(cep_session* s) {
  if (!s) return fail(CEP_E_INVALID, "null session");
  return guarded([&] {
    DeviceGuard g(s->device);
    HIPCHECK(hipStreamSynchronize(s->stream));
  });
}

int cep_poll_matches(cep_session* s, int query, int memory, cep_matches* out) {
  if (!s || !out || query < 0 || query >= (int)s->qs.size()) return fail(CEP_E_INVALID, "bad argument");
  QueryRt& r = *s->qs[query];
  if (!r.have) return fail(CEP_E_STATE, "no batch has been pushed");
  return guarded([&] {
    DeviceGuard g(s->device);
    resolve(s);
    std::memset(out, 0, sizeof *out);
    out->n_matches = r.n_matches;
    out->n_pairs = r.n_pairs;
    out->arity = r.arity;
    out->arity_stage = r.arity ? r.q->arityStage.data() : nullptr;
    out->memory = memory;
    if (memory == CEP_MEM_DEVICE) {
      out->key = r.m_key.as<uint32_t>();
      out->emit_seq = r.arity ? nullptr : r.m_emit.as<uint32_t>();
      out->pair_off = r.arity ? nullptr : r.m_off.as<uint64_t>();
      out->pair_seq = r.p_seq.as<uint32_t>();
      out->pair_stage = r.arity ? nullptr : r.p_stage.as<uint16_t>();
      return;
    }
    if (!r.host_valid) {
      r.h_key.resize(r.n_matches);
      r.h_seq.resize(r.n_pairs);
      if (r.n_matches)
        HIPCHECK(hipMemcpyAsync(r.h_key.data(), r.m_key.p, 4 * r.n_matches, hipMemcpyDeviceToHost, s->stream));
      if (r.n_pairs)
        HIPCHECK(hipMemcpyAsync(r.h_seq.data(), r.p_seq.p, 4 * r.n_pairs, hipMemcpyDeviceToHost, s->stream));
      if (!r.arity) {
        r.h_emit.resize(r.n_matches);
        r.h_off.resize(r.n_matches + 1);
        r.h_stage.resize(r.n_pairs);
        if (r.n_matches)
          HIPCHECK(hipMemcpyAsync(r.h_emit.data(), r.m_emit.p, 4 * r.n_matches, hipMemcpyDeviceToHost, s->stream));
        HIPCHECK(hipMemcpyAsync(r.h_off.data(), r.m_off.p, 8 * (r.n_matches + 1), hipMemcpyDeviceToHost, s->stream));
        if (r.n_pairs)
          HIPCHECK(hipMemcpyAsync(r.h_stage.data(), r.p_stage.p, 2 * r.n_pairs, hipMemcpyDeviceToHost, s->stream));
      }
      HIPCHECK(hipStreamSynchronize(s->stream));
      r.host_valid = true;
    }
    out->key = r.h_key.data();
    out->pair_seq = r.h_seq.data();
    if (!r.arity) {
      out->emit_seq = r.h_emit.data();
      out->pair_off = r.h_off.data();
      out->pair_stage = r.h_stage.data();
    }
  });
}

int cep_key_errors(cep_session* s, int query, int32_t* code, uint32_t* seq, uint64_t n_keys) {
  if (!s || query < 0 || query >= (int)s->qs.size()) return fail(CEP_E_INVALID, "bad argument");
  QueryRt& r = *s->qs[query];
  if (!r.have) return fail(CEP_E_STATE, "no batch has been pushed");
  if (n_keys > s->n_keys) return fail(CEP_E_INVALID, "n_keys larger than the batch");
  return guarded([&] {
    DeviceGuard g(s->device);
    std::vector<KeyState> ks(n_keys);
    if (n_keys)
      HIPCHECK(hipMemcpyAsync(ks.data(), r.ks_dev, sizeof(KeyState) * n_keys, hipMemcpyDeviceToHost, s->stream));
    HIPCHECK(hipStreamSynchronize(s->stream));
    for (uint64_t k = 0; k < n_keys; k++) {  // (a resource limit left after the re-runs: capacity)
      if (code) code[k] = ks[k].err == KE_RETRY ? KE_CAPACITY : ks[k].err;
      if (seq) seq[k] = ks[k].err_seq;
    }
  });
}

int cep_match_digest(cep_session* s, int query, uint64_t* n_matches, uint64_t* checksum) {
  if (!s || query < 0 || query >= (int)s->qs.size()) return fail(CEP_E_INVALID, "bad argument");
  QueryRt& r = *s->qs[query];
  if (!r.have) return fail(CEP_E_STATE, "no batch has been pushed");
  return guarded([&] {
    DeviceGuard g0(s->device);
    resolve(s);
    if (checksum && !r.digest_valid) {
      DeviceGuard g(s->device);
      s->scratch.ensure(sizeof(Scratch));
      Scratch* sc = s->scratch.as<Scratch>();
      HIPCHECK(hipMemsetAsync(&sc->digest, 0, sizeof sc->digest, s->stream));
      HIPCHECK(launch_digest(r.n_matches, r.arity, r.arity ? r.q->arityStage.data() : nullptr,
                             r.m_key.as<uint32_t>(), r.m_emit.as<uint32_t>(), r.m_off.as<uint64_t>(),
                             r.p_seq.as<uint32_t>(), r.p_stage.as<uint16_t>(), &sc->digest, s->stream));
      HIPCHECK(hipMemcpyAsync(&r.digest, &sc->digest, sizeof r.digest, hipMemcpyDeviceToHost, s->stream));
      HIPCHECK(hipStreamSynchronize(s->stream));
      r.digest_valid = true;
    }
    if (n_matches) *n_matches = r.n_matches;
    if (checksum) *checksum = r.digest;
  });
}

int cep_watermark(cep_session* s, int64_t* out) {
  if (!s || !out) return fail(CEP_E_INVALID, "null argument");
  return guarded([&] {
    DeviceGuard g(s->device);
    resolve(s);
    *out = s->watermark;
  });
}

// ---- streaming-session snapshot / restore ----
// Stands for the reference's persistent mode: CEPProcessor keeps the NFA's run queue in a
// store, serialised with Kryo after every record (CEPProcessor.java:121-131,159-160;
// nfa/ComputationStageSerDe.java:53-125) and the buffer nodes in their own store
// (nfa/buffer/impl/TimedKeyValueSerDes.java:42-63).  Here the whole per-key state of every
// query of a streaming session - KeyCarry per key, the run-queue rings, the used prefix of the
// node/predecessor pools and the pool tops - is one versioned little-endian blob.  Restoring
// it into a fresh streaming session over the same queries and options continues every key's
// stream exactly (tests/test_gpu_parity.py::test_streaming_snapshot_restore).
namespace {
constexpr uint64_t kSnapMagic = 0x31504E5350454300ull;  // "\0CEPSNP1"
constexpr uint32_t kSnapVersion = 3;
// 2: a node's first pointer in its own slot (preds0).  3: a run record's header w field holds
// its node hint (was the Dewey length, now the sum of the pair counts), and Node quad 1's w
// field holds the key (cep_live_floor)

uint64_t query_fingerprint(const cep_query* q) {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](const void* p, size_t n) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
  };
  mix(q->code.data(), q->code.size() * sizeof(uint32_t));
  mix(q->jitSource.data(), q->jitSource.size());
  mix(&q->info.kind, sizeof q->info.kind);
  return h;
}

struct SnapQueryHdr {
  uint64_t fingerprint, n_keys, ring_bytes;
  uint32_t F, rcap, node_used, pred_used, init, pad;
};

uint64_t snap_size(const cep_session* s) {
  uint64_t n = 32;  // magic, version, n_queries, watermark, reserved
  for (auto& r : s->qs) {
    n += sizeof(SnapQueryHdr);
    const StreamState& S = r->st;
    if (S.init)
      n += sizeof(KeyCarry) * std::max<uint64_t>(S.n_keys, 1) + S.ring_bytes + (sizeof(Node) + sizeof(Pred)) * S.node_used +
           sizeof(Pred) * S.pred_used;
  }
  return n;
}
}  // namespace

int cep_session_snapshot(cep_session* s, void* buf, size_t cap, size_t* size) {
  if (!s || !size) return fail(CEP_E_INVALID, "null argument");
  if (!s->opts.streaming) return fail(CEP_E_STATE, "snapshot needs a streaming session (cep_opts.streaming)");
  const uint64_t need = snap_size(s);
  *size = (size_t)need;
  if (!buf) return CEP_OK;  // size query
  if (cap < need) return fail(CEP_E_INVALID, "snapshot buffer too small (see *size)");
  return guarded([&] {
    DeviceGuard g(s->device);
    HIPCHECK(hipStreamSynchronize(s->stream));
    uint8_t* o = static_cast<uint8_t*>(buf);
    const uint32_t nq = (uint32_t)s->qs.size();
    std::memset(o, 0, 32);
    std::memcpy(o, &kSnapMagic, 8);
    std::memcpy(o + 8, &kSnapVersion, 4);
    std::memcpy(o + 12, &nq, 4);
    std::memcpy(o + 16, &s->watermark, 8);
    o += 32;
    for (auto& r : s->qs) {
      const StreamState& S = r->st;
      SnapQueryHdr h{query_fingerprint(r->q), S.n_keys, S.ring_bytes, (uint32_t)r->F, S.rcap,
                     S.node_used, S.pred_used, S.init ? 1u : 0u, 0};
      std::memcpy(o, &h, sizeof h);
      o += sizeof h;
      if (!S.init) continue;
      auto d2h = [&](const void* src, uint64_t n) {
        if (n) copy_sync(o, src, n, hipMemcpyDeviceToHost, s->stream);
        o += n;
      };
      d2h(S.carry.p, sizeof(KeyCarry) * std::max<uint64_t>(S.n_keys, 1));
      d2h(S.rings.p, S.ring_bytes);
      d2h(S.nodes.p, sizeof(Node) * S.node_used);
      d2h(S.preds0.p, sizeof(Pred) * S.node_used);
      d2h(S.preds.p, sizeof(Pred) * S.pred_used);
    }
  });
}

int cep_live_floor(cep_session* s, int query, uint32_t* floor, uint64_t n_keys) {
  if (!s || !floor || query < 0 || query >= (int)s->qs.size()) return fail(CEP_E_INVALID, "bad argument");
  if (!s->opts.streaming) return fail(CEP_E_STATE, "cep_live_floor needs a streaming session (cep_opts.streaming)");
  QueryRt& r = *s->qs[query];
  const StreamState& S = r.st;
  if (S.init && n_keys > S.n_keys) return fail(CEP_E_INVALID, "n_keys larger than the session's key space");
  return guarded([&] {
    DeviceGuard g(s->device);
    if (!S.init || n_keys == 0) {
      for (uint64_t k = 0; k < n_keys; k++) floor[k] = 0xFFFFFFFFu;
      return;
    }
    DBuf out;
    out.ensure(4 * S.n_keys);
    HIPCHECK(launch_live_floor(S.nodes.as<Node>(), S.node_used, S.n_keys, out.as<uint32_t>(), s->stream));
    HIPCHECK(hipMemcpyAsync(floor, out.p, 4 * n_keys, hipMemcpyDeviceToHost, s->stream));
    HIPCHECK(hipStreamSynchronize(s->stream));
  });
}

int cep_session_restore(cep_session* s, const void* buf, size_t size) {
  if (!s || !buf) return fail(CEP_E_INVALID, "null argument");
  if (!s->opts.streaming) return fail(CEP_E_STATE, "restore needs a streaming session (cep_opts.streaming)");
  const uint8_t* p = static_cast<const uint8_t*>(buf);
  const uint8_t* end = p + size;
  uint64_t magic = 0;
  uint32_t ver = 0, nq = 0;
  if (size < 32) return fail(CEP_E_INVALID, "snapshot truncated");
  std::memcpy(&magic, p, 8);
  std::memcpy(&ver, p + 8, 4);
  std::memcpy(&nq, p + 12, 4);
  if (magic != kSnapMagic) return fail(CEP_E_INVALID, "not a cep snapshot");
  if (ver != kSnapVersion) return fail(CEP_E_INVALID, "unsupported snapshot version");
  if (nq != s->qs.size()) return fail(CEP_E_INVALID, "snapshot holds a different number of queries");
  int64_t wm = 0;
  std::memcpy(&wm, p + 16, 8);
  // validate everything before touching the session
  {
    const uint8_t* q = p + 32;
    for (auto& r : s->qs) {
      SnapQueryHdr h;
      if (q + sizeof h > end) return fail(CEP_E_INVALID, "snapshot truncated");
      std::memcpy(&h, q, sizeof h);
      q += sizeof h;
      if (h.fingerprint != query_fingerprint(r->q)) return fail(CEP_E_INVALID, "snapshot of a different query");
      if (!h.init) continue;
      const uint32_t rcap = s->opts.max_runs ? s->opts.max_runs : 32;
      if (h.rcap != rcap || h.F != (uint32_t)r->F || h.ring_bytes != ring_size(r->F, std::max<uint64_t>(h.n_keys, 1), rcap))
        return fail(CEP_E_INVALID, "snapshot taken with other session options (max_runs)");
      const uint64_t n = sizeof(KeyCarry) * std::max<uint64_t>(h.n_keys, 1) + h.ring_bytes +
                         (sizeof(Node) + sizeof(Pred)) * (uint64_t)h.node_used + sizeof(Pred) * (uint64_t)h.pred_used;
      if ((uint64_t)(end - q) < n) return fail(CEP_E_INVALID, "snapshot truncated");
      q += n;
    }
  }
  return guarded([&] {
    DeviceGuard g(s->device);
    HIPCHECK(hipStreamSynchronize(s->stream));
    const uint8_t* q = p + 32;
    for (auto& r : s->qs) {
      SnapQueryHdr h;
      std::memcpy(&h, q, sizeof h);
      q += sizeof h;
      StreamState& S = r->st;
      S.init = false;
      if (!h.init) continue;
      auto h2d = [&](DBuf& dst, uint64_t n) {
        dst.ensure(std::max<uint64_t>(n, 16));
        if (n) copy_sync(dst.p, q, n, hipMemcpyHostToDevice, s->stream);
        q += n;
      };
      S.n_keys = h.n_keys;
      S.rcap = h.rcap;
      S.ring_bytes = h.ring_bytes;
      h2d(S.carry, sizeof(KeyCarry) * std::max<uint64_t>(h.n_keys, 1));
      h2d(S.rings, h.ring_bytes);
      S.node_cap = std::max<uint64_t>(h.node_used, 1);
      S.pred_cap = std::max<uint64_t>(h.pred_used, 1);
      h2d(S.nodes, sizeof(Node) * (uint64_t)h.node_used);
      h2d(S.preds0, sizeof(Pred) * (uint64_t)h.node_used);
      h2d(S.preds, sizeof(Pred) * (uint64_t)h.pred_used);
      S.node_used = h.node_used;
      S.pred_used = h.pred_used;
      const uint32_t tops[2] = {h.node_used, h.pred_used};
      S.tops.ensure(2 * sizeof(uint32_t));
      copy_sync(S.tops.p, tops, sizeof tops, hipMemcpyHostToDevice, s->stream);
      S.init = true;
    }
    s->watermark = wm;
  });
}

int cep_last_timing(cep_session* s, int query, double* kernel_ms, double* aux_ms, uint32_t* launches) {
  if (!s || query < 0 || query >= (int)s->qs.size()) return fail(CEP_E_INVALID, "bad argument");
  return guarded([&] {
    DeviceGuard g(s->device);
    resolve(s);
    if (kernel_ms) *kernel_ms = s->qs[query]->kernel_ms;
    if (aux_ms) *aux_ms = s->qs[query]->aux_ms;
    if (launches) *launches = s->qs[query]->launches;
  });
}

int cep_timing_totals(cep_session* s, int query, int reset, double* kernel_ms, double* aux_ms, uint64_t* batches) {
  if (!s || query < 0 || query >= (int)s->qs.size()) return fail(CEP_E_INVALID, "bad argument");
  return guarded([&] {
    DeviceGuard g(s->device);
    resolve(s);
    QueryRt& r = *s->qs[query];
    for (int i = 0; i < QueryRt::kRing; i++)
      if (r.tev_used[i]) ring_take(r, i);
    if (kernel_ms) *kernel_ms = r.acc_kernel_ms;
    if (aux_ms) *aux_ms = r.acc_aux_ms;
    if (batches) *batches = r.acc_batches;
    if (reset) {
      r.acc_kernel_ms = r.acc_aux_ms = 0;
      r.acc_batches = 0;
    }
  });
}

int cep_last_stats(cep_session* s, int query, cep_batch_stats* out) {
  if (!s || !out || query < 0 || query >= (int)s->qs.size()) return fail(CEP_E_INVALID, "bad argument");
  return guarded([&] {
    DeviceGuard g(s->device);
    resolve(s);
    const QueryRt& r = *s->qs[query];
    if (r.group < 0) {
      *out = cep_batch_stats{};
      out->group = 0xFFFFFFFFu;
      out->kernel_ms = out->main_ms = r.kernel_ms;
      out->launches = r.launches;
      out->allocs = s->last_allocs;
      return;
    }
    *out = s->groups[r.group]->stats;
    out->group = (uint32_t)r.group;
    out->allocs = s->last_allocs;
  });
}

int cep_lane_balance(cep_session* s, int query, double* ordered, double* identity) {
  if (!s || !ordered || !identity || query < 0 || query >= (int)s->qs.size())
    return fail(CEP_E_INVALID, "bad argument");
  const QueryRt& r = *s->qs[query];
  if (r.group < 0) return fail(CEP_E_INVALID, "a stencil query has no lane order");
  GroupRt& g = *s->groups[r.group];
  const uint64_t nk = s->n_keys;
  if (!g.est_valid || nk <= 64 || g.est.bytes < 4 * nk) return fail(CEP_E_INVALID, "the last batch ran no work estimate");
  return guarded([&] {
    DeviceGuard dg(s->device);
    std::vector<uint32_t> est(nk), ord(nk), srt(nk);
    HIPCHECK(hipMemcpyAsync(est.data(), g.est.p, 4 * nk, hipMemcpyDeviceToHost, s->stream));
    HIPCHECK(hipMemcpyAsync(ord.data(), g.order.p, 4 * nk, hipMemcpyDeviceToHost, s->stream));
    HIPCHECK(hipStreamSynchronize(s->stream));
    for (uint64_t i = 0; i < nk; i++) srt[i] = ord[i] < nk ? est[ord[i]] : 0u;  // est in lane order
    auto balance = [&](const std::vector<uint32_t>& v) {
      double smax = 0, smean = 0;
      for (uint64_t w = 0; w < nk; w += 64) {
        const uint64_t e = std::min<uint64_t>(w + 64, nk);
        double mx = 0, sum = 0;
        for (uint64_t i = w; i < e; i++) {
          const double x = (double)v[i];
          mx = std::max(mx, x);
          sum += x;
        }
        smax += mx;
        smean += sum / (double)(e - w);
      }
      return smean > 0 ? smax / smean : 1.0;
    };
    *ordered = balance(srt);
    *identity = balance(est);
  });
}

int cep_gather_keys(int device, uint64_t n_sel, const uint32_t* sel_keys, const uint64_t* src_key_off,
                    const uint64_t* dst_key_off, int n_cols, const uint32_t* col_bytes,
                    const void* const* src_cols, void* const* dst_cols, const int64_t* src_ts, int64_t* dst_ts) {
  if (n_sel && (!sel_keys || !src_key_off || !dst_key_off || (n_cols && (!col_bytes || !src_cols || !dst_cols))))
    return fail(CEP_E_INVALID, "null argument");
  if (n_cols < 0 || n_cols > kMaxFields) return fail(CEP_E_INVALID, "1..16 columns");
  return guarded([&] {
    DeviceGuard g(device);
    HIPCHECK(hipSetDevice(device));
    HIPCHECK(gather_keys(n_sel, sel_keys, src_key_off, dst_key_off, n_cols, col_bytes, src_cols, dst_cols, src_ts,
                         dst_ts, nullptr));
    HIPCHECK(hipDeviceSynchronize());
  });
}

int cep_alloc_pinned(size_t bytes, void** out) {
  if (!out) return fail(CEP_E_INVALID, "null argument");
  return guarded([&] { HIPCHECK(hipHostMalloc(out, bytes, hipHostMallocDefault)); });
}

int cep_free_pinned(void* p) {
  return guarded([&] { HIPCHECK(hipHostFree(p)); });
}

int cep_device_alloc(int device, size_t bytes, void** out) {
  if (!out) return fail(CEP_E_INVALID, "null argument");
  return guarded([&] {
    DeviceGuard g(device);
    HIPCHECK(hipSetDevice(device));
    HIPCHECK(hipMalloc(out, std::max<size_t>(bytes, 256)));
  });
}

int cep_device_free(void* p) {
  return guarded([&] { HIPCHECK(hipFree(p)); });
}

int cep_memcpy(void* dst, const void* src, size_t bytes, int dst_memory, int src_memory) {
  hipMemcpyKind k = dst_memory == CEP_MEM_DEVICE ? (src_memory == CEP_MEM_DEVICE ? hipMemcpyDeviceToDevice
                                                                                  : hipMemcpyHostToDevice)
                                                 : (src_memory == CEP_MEM_DEVICE ? hipMemcpyDeviceToHost
                                                                                  : hipMemcpyHostToHost);
  // (a caller's copy of a session's device results: every stream's work on them done first - the
  // stencil path returns without a host sync, and the null stream does not order with the
  // sessions' non-blocking streams)
  return guarded([&] {
    HIPCHECK(hipDeviceSynchronize());
    HIPCHECK(hipMemcpy(dst, src, bytes, k));
  });
}

int cep_decode_stock_json(int device, const uint8_t* bytes, const uint64_t* rec_off, uint64_t n_records,
                          int col_width, void* price, void* volume, int32_t* status, uint32_t* name_span,
                          void* stream) {
  if (!rec_off || !price || !volume || !status || (!bytes && n_records))
    return fail(CEP_E_INVALID, "null argument");
  if (col_width != 4 && col_width != 8) return fail(CEP_E_INVALID, "col_width must be 4 or 8");
  return guarded([&] {
    DeviceGuard g(device);
    HIPCHECK(hipSetDevice(device));
    HIPCHECK(launch_decode_stock_json(bytes, rec_off, n_records, col_width, price, volume, status, name_span,
                                      (hipStream_t)stream));
  });
}

int cep_symbol_keys(int device, const uint8_t* bytes, const uint64_t* rec_off, const uint32_t* name_span,
                    const int32_t* status, uint64_t n_records, uint64_t max_symbols, uint32_t* key_out,
                    uint64_t* n_symbols, void* stream) {
  if (!rec_off || !name_span || !key_out || !n_symbols || (!bytes && n_records))
    return fail(CEP_E_INVALID, "null argument");
  if (n_records >= 0xFFFFFFFFull) return fail(CEP_E_INVALID, "n_records must be < 2^32");
  if (max_symbols == 0) max_symbols = n_records;
  uint32_t err = 0;
  int rc = guarded([&] {
    DeviceGuard g(device);
    HIPCHECK(hipSetDevice(device));
    HIPCHECK(symbol_keys(bytes, rec_off, name_span, status, n_records, max_symbols, key_out, n_symbols, &err,
                         (hipStream_t)stream));
  });
  if (rc) return rc;
  if (err & 1u) return fail(CEP_E_INVALID, "a record's name holds malformed UTF-8");
  // (the hash table holds at least 2 x max_symbols slots: err bit 2 only fires when it is
  // full, so the limit itself is checked on the count)
  if ((err & 2u) || *n_symbols > max_symbols) return fail(CEP_E_INVALID, "more distinct names than max_symbols");
  if (err & 4u) return fail(CEP_E_INVALID, "64-bit hash collision between two different names");
  return CEP_OK;
}

}  // extern "C"
