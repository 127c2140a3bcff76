// tuning.cpp — the measurement knobs of libcep ($CEP_* environment variables), read in one
// place: at session creation (cep_session_create keeps a copy in the session) and, for the
// knobs compiled into a query's kernel, at query compile.  Nothing on the launch path reads
// the environment (tests/test_native_abi.py checks the sources).  Results never depend on
// these knobs.
#include <cstdlib>

#include "cep_internal.h"

namespace cep {

namespace {
bool flag(const char* name) { return std::getenv(name) != nullptr; }
long num(const char* name, long dflt) {
  const char* e = std::getenv(name);
  return e ? std::atol(e) : dflt;
}
}  // namespace

uint32_t tuning_walk_flush() {
  const long v = num("CEP_WALK_FLUSH", 24);
  return v > 0 ? (uint32_t)v : 24u;
}

Tuning tuning_from_env() {
  Tuning t;
  const long rw = num("CEP_RESIDENT_WAVES", 0);
  t.resident_waves = rw > 0 ? (uint32_t)rw : 0u;
  t.no_persist = flag("CEP_NO_PERSIST");
  t.spread = (int)num("CEP_SPREAD", 2);
  const long iso = num("CEP_ISOLATE", 0);
  t.isolate = iso > 0 ? (uint32_t)iso : 0u;
  const long nc = num("CEP_NODE_CHUNK", 0), oc = num("CEP_OUT_CHUNK", 0), wc = num("CEP_WALK_CAP", 0);
  t.node_chunk = nc > 0 ? (uint32_t)nc : 0u;
  t.out_chunk = oc > 0 ? (uint32_t)oc : 0u;
  t.walk_cap = wc > 0 ? (uint32_t)wc : 0u;
  t.walk_flush = tuning_walk_flush();
  t.job_map = (uint32_t)num("CEP_JOB_MAP", 0);
  t.prof = flag("CEP_PROF");
  t.stream_narrow = flag("CEP_STREAM_NARROW");
  t.stream_wide = flag("CEP_STREAM_WIDE");
  t.no_est_blend = flag("CEP_NO_EST_BLEND");
  {
    // (measured on cfg 3's arrival order, 1e9 events: 8192-event tiles 48.7 ms, 4096 42.4, 2048 55.8)
    const long r = num("CEP_PART_ROUNDS", 16);
    t.part_rounds = (r == 8 || r == 12 || r == 24 || r == 32) ? (int)r : 16;
    const long g = num("CEP_GATHER_PER", 0);
    t.gather_per = (g == 4 || g == 8 || g == 16) ? (int)g : 0;
  }
  // (measured on the streamed cfg 3, main launches of 10 batches: 0 61.3 ms, 64 56.3, 256 52.4,
  // 1024 46.8 (46.5, 46.4), 1536 44.8, 2048 43.9 (44.2, 43.7), 3072 46.0, 4096 47.1; profiles/r04/probes/streamiso)
  const long siso = num("CEP_STREAM_ISO", 2048);
  t.stream_iso = siso > 0 ? (uint32_t)siso : 0u;
  const long biso = num("CEP_BATCH_ISO", 0);
  t.batch_iso = biso > 0 ? (uint32_t)biso : 0u;
  const long solo = num("CEP_SOLO_KEYS", 0);
  t.solo_keys = solo > 0 ? (uint32_t)solo : 0u;
  t.stream_no_order = flag("CEP_STREAM_NO_ORDER");
  t.no_wm_fold = flag("CEP_NO_WM_FOLD");
  const long pf = num("CEP_STENCIL_PF", 0);
  t.stencil_pf = (pf == 1 || pf == 2 || pf == 4) ? (int)pf : 0;
  t.host_trace = flag("CEP_HOST_TRACE");
  return t;
}

}  // namespace cep
