// CPU driver of a generated NFA kernel (test infrastructure): the host side of
// session.cpp run_nfa - pools, deferred-walk queues, capacity/conflict retries with walks in
// place - with the kernel run lane by lane, then the matches flattened in key order.
// Built per query by tests/lane_cpu.py with QUERY_SRC = the query's generated source.
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cstdint>
#include <algorithm>
#include <cstdlib>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include QUERY_SRC
#include "wave_emu.h"

thread_local LaneDim3 blockIdx, threadIdx, blockDim, gridDim;

static void wave_body(void* a) { cep_nfa_jit(*static_cast<cep::NfaArgs*>(a)); }
uint64_t cep_lane_stats[10];
extern "C" void lane_stats(uint64_t* out) { std::memcpy(out, cep_lane_stats, sizeof cep_lane_stats); }

// Walk hops by kind (nfa_lane.h CEP_HOP): branch, extraction (emit), extraction hops at a node
// a branch walk of the same key and event passed with the same walker version (the hops a
// fused branch + extraction walk would not repeat), remove-only.  Walks drain in queue order,
// so a key's walk events only grow: the key keeps the (node, version) set of its latest event.
namespace {
struct HopSet {
  uint32_t t = 0xFFFFFFFFu;
  std::unordered_set<uint64_t> seen;
};
std::unordered_map<uint32_t, HopSet> g_hop_keys;
uint64_t g_hops[4];
uint64_t ver_hash(const cep::Dewey& w) {
  uint64_t h = 1469598103934665603ull ^ w.len;
  for (uint32_t i = 0; i < w.n && i < (uint32_t)cep::kDeweyPairs; i++)
    h = (h ^ ((uint64_t)(uint32_t)w.v[i] << 32 | w.c[i])) * 1099511628211ull;
  return h;
}
}  // namespace
void cep_lane_hop(uint32_t key, uint32_t t, uint32_t node, uint32_t flags, const cep::Dewey& w) {
  HopSet& hs = g_hop_keys[key];
  if (hs.t != t) {
    hs.t = t;
    hs.seen.clear();
  }
  const uint64_t id = ((uint64_t)node << 32) ^ (ver_hash(w) & 0xFFFFFFFFull);
  if (flags & cep::kWalkBranch) {
    g_hops[0]++;
    hs.seen.insert(id);
  } else if (flags & cep::kWalkEmit) {
    g_hops[1]++;
    if (hs.seen.count(id)) g_hops[2]++;
  } else {
    g_hops[3]++;
  }
}
extern "C" void lane_hop_stats(uint64_t* out) { std::memcpy(out, g_hops, sizeof g_hops); }

namespace {
std::vector<uint32_t> g_key, g_emit, g_seq;
std::vector<uint64_t> g_off;
std::vector<uint16_t> g_stage;
std::vector<int32_t> g_err;
std::vector<uint32_t> g_err_seq;
}  // namespace

static void on_fault(int sig) {  // a lane bug: print where, then die
  void* bt[32];
  const int n = backtrace(bt, 32);
  backtrace_symbols_fd(bt, n, 2);
  _exit(128 + sig);
}

// a streaming session's state between lane_run calls (streaming != 0)
struct Stream {
  std::vector<cep::Node> nodes;
  std::vector<cep::Pred> preds, preds0;
  std::vector<cep::KeyCarry> carry;
  std::vector<cep::v4u> rings;
  uint32_t node_top = 0, pred_top = 0;
};
static Stream g_stream;
static bool g_bits_used = false;
extern "C" int lane_bits_used() { return g_bits_used; }

extern "C" void lane_stream_reset() { g_stream = Stream{}; }

// The wide build's continuation of keys the stream build stopped (KE_WIDEN, session.cpp
// run_nfa): another build of the same query (tests/lane_cpu.py loads both), run here over the
// launch's own arguments - the same rings, pools, carry and outputs.
typedef void (*ContFn)(void* args, uint64_t nslots);
static ContFn g_cont = nullptr;
extern "C" void lane_set_continuation(void* fn) { g_cont = reinterpret_cast<ContFn>(fn); }
extern "C" void lane_continue(void* args, uint64_t nslots) {
  cep::NfaArgs& a = *static_cast<cep::NfaArgs*>(args);
  blockDim.x = 256;
  if (std::getenv("CEP_LANE_WAVES")) {
    for (uint64_t s = 0; s < nslots; s += 64) emu::run_wave((unsigned)(s / 256), (unsigned)(s % 256), wave_body, &a);
  } else {
    for (uint64_t s = 0; s < nslots; s++) {
      blockIdx.x = (unsigned)(s / 256);
      threadIdx.x = (unsigned)(s % 256);
      cep_nfa_jit(a);
    }
  }
}
static uint64_t g_widened = 0;
extern "C" uint64_t lane_widened() { return g_widened; }

// the begin-hit bitmap (cep_nfa_bits), one position at a time; absent when the query's begin
// stage is not a single BEGIN edge (no bits kernel)
template <class A_>
static auto fill_bits(const A_& a, std::vector<uint64_t>& bits, int) -> decltype(begin_hit_at(a, 0), bool()) {
  for (uint64_t p = 0; p < a.n_events; p++)
    if (begin_hit_at(a, p)) bits[p >> 6] |= 1ull << (p & 63);
  return true;
}
template <class A_>
static bool fill_bits(const A_&, std::vector<uint64_t>&, long) { return false; }

extern "C" int lane_run(uint64_t nk, const uint64_t* key_off, const void* const* cols, int n_cols,
                        const int64_t* ts, uint32_t rcap, int defer, uint32_t* n_retried, int streaming,
                        int use_bits, uint32_t n_q, const int64_t* kc) {
  using namespace cep;
  signal(SIGSEGV, on_fault);
  std::memset(cep_lane_stats, 0, sizeof cep_lane_stats);
  std::memset(g_hops, 0, sizeof g_hops);
  g_hop_keys.clear();
  const uint64_t ne = key_off[nk];
  std::vector<Node> nodes_batch, *nodes_p = &nodes_batch;
  std::vector<Pred> preds_batch, *preds_p = &preds_batch, preds0_batch, *preds0_p = &preds0_batch;
  if (streaming) {  // pools persist; a fixed generous size for the tests' streams
    if (g_stream.carry.empty()) {
      g_stream.carry.assign(nk, KeyCarry{});
      g_stream.nodes.resize(1 << 20);
      g_stream.preds.resize(1 << 20);
      g_stream.preds0.resize(1 << 20);
      g_stream.rings.resize(ring_bytes(8, nk, rcap) / 16 + 64);
    }
    nodes_p = &g_stream.nodes;
    preds_p = &g_stream.preds;
    preds0_p = &g_stream.preds0;
  } else {
    nodes_batch.resize(ne * 4 + nk * 64 + 4096);
    preds_batch.resize(ne * 4 + nk * 64 + 4096);
    preds0_batch.resize(nodes_batch.size());
  }
  std::vector<Node>& nodes = *nodes_p;
  std::vector<Pred>& preds = *preds_p;
  std::vector<Pred>& preds0 = *preds0_p;
  // ($CEP_LANE_OUT_CHUNKS: a bigger output pool, for keys emitting more than ~2 pairs per event)
  uint64_t out_chunks = (ne + nk * 4 + 64) * 2;
  if (const char* e = std::getenv("CEP_LANE_OUT_CHUNKS")) out_chunks = std::max<uint64_t>(out_chunks, std::atoll(e));
  std::vector<uint32_t> out(out_chunks * kOutChunkWords);
  if (n_q == 0) n_q = 1;
  const uint64_t jobs = (uint64_t)n_q * nk;
  std::vector<KeyState> ks(jobs);
  // device pools are not cleared between batches: start from garbage, not zeros
  auto scribble = [](void* p, size_t n) {
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (size_t i = 0; i + 8 <= n; i += 8) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      std::memcpy((char*)p + i, &x, 8);
    }
  };
  if (!streaming) {
    scribble(nodes.data(), nodes.size() * sizeof(Node));
    scribble(preds.data(), preds.size() * sizeof(Pred));
    scribble(preds0.data(), preds0.size() * sizeof(Pred));
  }
  scribble(out.data(), out.size() * 4);
  uint32_t node_top = 0, pred_top = 0, out_top = 0, n_cap = 0, job_next = 0;
  NfaArgs a{};
  a.n_keys = nk;
  a.key_off = key_off;
  for (int f = 0; f < n_cols; f++) a.cols.p[f] = cols[f];
  a.ts = ts;
  a.nodes = nodes.data();
  a.preds = preds.data();
  a.preds0 = preds0.data();
  a.out = out.data();
  a.node_pool = Pool{streaming ? &g_stream.node_top : &node_top, (uint32_t)nodes.size(), 16};
  a.pred_pool = Pool{streaming ? &g_stream.pred_top : &pred_top, (uint32_t)preds.size(), 16};
  if (streaming) a.carry = g_stream.carry.data();
  a.out_pool = Pool{&out_top, (uint32_t)(out.size() / kOutChunkWords), 1};
  a.ks = ks.data();
  a.n_capacity_err = &n_cap;
  a.n_q = n_q;
  a.kc = kc;
  a.n_events = ne;
  std::vector<uint64_t> bits((ne + 63) / 64 + 1, 0);
  g_bits_used = use_bits && fill_bits(a, bits, 0);
  if (g_bits_used) a.bhits = bits.data();
  // persistent lanes (session.cpp): one "lane" claims every job in turn; streams: lane per key
  auto launch = [&](uint64_t nslots, uint32_t rc, int df) {
    // $CEP_LANE_NO_PERSIST: one lane per job, as session.cpp launches single queries
    if (!streaming && !std::getenv("CEP_LANE_NO_PERSIST")) {
      job_next = 0;
      a.job_next = &job_next;
      a.n_jobs = a.jobs ? a.n_jobs : jobs;
      nslots = 64;
    } else if (!streaming && a.jobs) {
      nslots = a.n_jobs;
    }
    std::vector<v4u> rings_batch;
    if (!streaming) {
      rings_batch.resize(ring_bytes(8, nslots, rc) / 16 + 64);
      scribble(rings_batch.data(), rings_batch.size() * 16);
    }
    const uint32_t wc = streaming ? std::max<uint32_t>(64, kWalkFlush + 3 * rc) : 64;  // (session.cpp run_nfa)
    const uint32_t pl = put_log_entries(rc);
    std::vector<v4u> walks(walkq_bytes(nslots, wc, pl) / 16 + 64);
    scribble(walks.data(), walks.size() * 16);
    a.rings = streaming ? g_stream.rings.data() : rings_batch.data();
    a.rcap = rc;
    a.walks = walks.data();
    a.wcap = wc;
    a.plog = pl;
    a.defer = (uint32_t)df;
    blockDim.x = 256;
    if (std::getenv("CEP_LANE_WAVES")) {  // whole 64-lane waves (wave_emu.h): cross-lane ops see every lane
      for (uint64_t s = 0; s < nslots; s += 64) emu::run_wave((unsigned)(s / 256), (unsigned)(s % 256), wave_body, &a);
    } else {
      for (uint64_t s = 0; s < nslots; s++) {
        blockIdx.x = (unsigned)(s / 256);
        threadIdx.x = (unsigned)(s % 256);
        cep_nfa_jit(a);
      }
    }
  };
  // $CEP_LANE_POOL: node/pred pools of that many entries for the first launch (as session.cpp
  // sizes them from the batch; the re-runs get the whole pools)
  if (const char* e = std::getenv("CEP_LANE_POOL")) {
    a.node_pool.cap = std::min<uint32_t>(a.node_pool.cap, (uint32_t)std::atol(e));
    a.pred_pool.cap = std::min<uint32_t>(a.pred_pool.cap, (uint32_t)std::atol(e));
  }
  // $CEP_LANE_SPREAD: the launch spread over W waves (session.cpp: underfilled launches): wave
  // w's lane l runs key l * W + w (odd lanes reversed), W = the value, waves past W idle
  if (const char* sp = std::getenv("CEP_LANE_SPREAD")) {
    if (n_q == 1) {
      a.spread = std::strtoull(sp, nullptr, 10);
    }
  }
  // (spread: three idle waves past the W, as the grid's last block can hold)
  if (const char* si = std::getenv("CEP_LANE_STREAM_ISO"); si && streaming && n_q == 1 && !a.spread) {
    // (session.cpp $CEP_STREAM_ISO: the first K keys alone in their waves, the rest 64 per wave)
    const uint64_t k = std::min<uint64_t>(std::strtoull(si, nullptr, 10), nk / 2);
    a.spread_iso = (uint32_t)k;
    launch((k + (nk - k + 63) / 64) * 64, rcap, defer);
    a.spread_iso = 0;
  } else {
    launch(a.spread ? (a.spread + 3) * 64 : ((nk + 63) / 64) * 64 * n_q, rcap, defer);  // (streams defer their walks too)
  }
  a.spread = 0;
  g_widened = 0;
  if (streaming) {  // keys the stream build stopped: continued by the wide build (g_cont)
    std::vector<uint32_t> list;
    for (uint64_t k = 0; k < jobs; k++)
      if (ks[k].err == KE_WIDEN) list.push_back((uint32_t)k);
    if (!list.empty()) {
      if (!g_cont) std::abort();  // (a stream build without its wide build)
      const uint32_t wc = std::max<uint32_t>(64, kWalkFlush + 3 * rcap);
      const uint32_t pl = put_log_entries(rcap);
      std::vector<v4u> walks(walkq_bytes(list.size(), wc, pl) / 16 + 64);
      scribble(walks.data(), walks.size() * 16);
      a.walks = walks.data();
      a.jobs = list.data();
      a.n_jobs = list.size();
      a.widen = 1;
      g_cont(&a, list.size());
      a.widen = 0;
      a.jobs = nullptr;
      g_widened = list.size();
    }
  }
  a.node_pool.cap = (uint32_t)nodes.size();
  a.pred_pool.cap = (uint32_t)preds.size();
  *n_retried = 0;
  for (int round = 0; !streaming && n_cap > 0 && round < 8; round++) {  // session.cpp run_nfa
    std::vector<uint32_t> list;
    for (uint64_t k = 0; k < jobs; k++)
      if (ks[k].err == KE_RETRY || ks[k].err == KE_CONFLICT) list.push_back((uint32_t)k);
    *n_retried += (uint32_t)list.size();
    n_cap = 0;
    // (session.cpp keeps the re-run rings within 16 GiB; here 2 GiB)
    if ((uint64_t)rcap * 8 * ((list.size() + 63) / 64 * 64) * 192 <= (2ull << 30)) rcap *= 8;
    std::vector<uint32_t> cap, conf;  // session.cpp: capacity re-runs keep deferred walks, conflicts walk in place
    for (uint32_t k : list) (ks[k].err == KE_RETRY ? cap : conf).push_back(k);
    for (int k = 0; k < 2; k++) {
      std::vector<uint32_t>& l = k == 0 ? cap : conf;
      if (l.empty()) continue;
      a.jobs = l.data();
      a.n_jobs = (uint32_t)l.size();
      launch(l.size(), rcap, k == 0 ? (streaming ? 0 : defer) : 0);
    }
  }
  g_key.clear(); g_emit.clear(); g_seq.clear(); g_off.assign(1, 0); g_stage.clear();
  g_err.resize(jobs); g_err_seq.resize(jobs);
  for (uint64_t k = 0; k < jobs; k++) {  // job k = query k / nk, key k % nk
    g_err[k] = ks[k].err == KE_RETRY ? KE_CAPACITY : ks[k].err;
    g_err_seq[k] = ks[k].err_seq;
    uint32_t chunk = ks[k].out_first, pos = 0;
    auto next = [&]() -> uint32_t {
      if (pos == kOutChunkWords - 1) {
        chunk = out[(uint64_t)chunk * kOutChunkWords + kOutChunkWords - 1];
        pos = 0;
      }
      return out[(uint64_t)chunk * kOutChunkWords + pos++];
    };
    for (uint32_t m = 0; m < ks[k].n_matches; m++) {
      g_key.push_back((uint32_t)k);
      g_emit.push_back(next());
      const uint32_t np = next();
      for (uint32_t i = 0; i < np; i++) {
        g_seq.push_back(next());
        g_stage.push_back((uint16_t)next());
      }
      g_off.push_back(g_seq.size());
    }
  }
  return 0;
}

extern "C" uint64_t lane_n_matches() { return g_key.size(); }
extern "C" uint64_t lane_n_pairs() { return g_seq.size(); }
extern "C" void lane_fetch(uint32_t* key, uint32_t* emit, uint64_t* off, uint32_t* seq, uint16_t* stage,
                           int32_t* err, uint32_t* err_seq) {
  std::memcpy(key, g_key.data(), 4 * g_key.size());
  std::memcpy(emit, g_emit.data(), 4 * g_emit.size());
  std::memcpy(off, g_off.data(), 8 * g_off.size());
  std::memcpy(seq, g_seq.data(), 4 * g_seq.size());
  std::memcpy(stage, g_stage.data(), 2 * g_stage.size());
  std::memcpy(err, g_err.data(), 4 * g_err.size());
  std::memcpy(err_seq, g_err_seq.data(), 4 * g_err_seq.size());
}
