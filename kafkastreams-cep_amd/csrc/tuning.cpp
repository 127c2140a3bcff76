// tuning.cpp — the measurement knobs of libcep ($CEP_* environment variables), read in one
// place: at session creation (cep_session_create keeps a copy in the session) and, for the
// knobs compiled into a query's kernel, at query compile.  Only the measurement build reads
// the environment (CEP_MEASURE: libcep_measure.so, Makefile `measure`); the release libcep.so
// runs the defaults and calls getenv for $CEP_JIT_CACHE alone (tests/test_native_abi.py).
// Most knobs change only launch geometry and timing; these change results and are for timing
// and diagnosis only: $CEP_NO_RETRY (keys keep their capacity / conflict error), $CEP_STREAM_PUTLOG=0
// and $CEP_STREAM_LAYOUT < 6 (inexact for streams), $CEP_POISON (buffer contents before first
// write), $CEP_DEWEY_PAIRS (fewer pairs: more keys re-run or fail).
#include <cstdlib>

#include "cep_internal.h"

namespace cep {

#ifdef CEP_MEASURE
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

void tuning_stream_build(int* pairs, int* layout, int* plog) {
  const long p = num("CEP_STREAM_PAIRS", 3), l = num("CEP_STREAM_LAYOUT", 6);
  *pairs = p > 0 && p < 6 ? (int)p : 3;
  *layout = l >= *pairs && l <= 6 ? (int)l : 6;
  *plog = num("CEP_STREAM_PUTLOG", 1) ? 1 : 0;
}

Tuning tuning_from_env() {
  Tuning t;
  const long rw = num("CEP_RESIDENT_WAVES", 0);
  t.resident_waves = rw > 0 ? (uint32_t)rw : 0u;
  t.no_persist = flag("CEP_NO_PERSIST");
  t.no_spread = flag("CEP_NO_SPREAD");
  t.no_retry = flag("CEP_NO_RETRY");
  const long nc = num("CEP_NODE_CHUNK", 0), oc = num("CEP_OUT_CHUNK", 0), wc = num("CEP_WALK_CAP", 0);
  t.node_chunk = nc > 0 ? (uint32_t)nc : 0u;
  t.out_chunk = oc > 0 ? (uint32_t)oc : 0u;
  t.walk_cap = wc > 0 ? (uint32_t)wc : 0u;
  t.prof = flag("CEP_PROF");
  t.stream_narrow = flag("CEP_STREAM_NARROW");
  t.stream_wide = flag("CEP_STREAM_WIDE");
  t.no_est_blend = flag("CEP_NO_EST_BLEND");
  {
    // (measured on cfg 3's arrival order, 1e9 events: 8192-event tiles 48.7 ms, 4096 42.4, 2048 55.8)
    const long r = num("CEP_PART_ROUNDS", 16);
    t.part_rounds = (r == 8 || r == 12 || r == 24 || r == 32) ? (int)r : 16;
  }
  // (measured on the streamed cfg 3, main launches of 10 batches: 0 61.3 ms, 64 56.3, 256 52.4,
  // 1024 46.8 (46.5, 46.4), 1536 44.8, 2048 43.9 (44.2, 43.7), 3072 46.0, 4096 47.1; profiles/r04/probes/streamiso)
  const long siso = num("CEP_STREAM_ISO", 2048);
  t.stream_iso = siso > 0 ? (uint32_t)siso : 0u;
  t.stream_no_order = flag("CEP_STREAM_NO_ORDER");
  t.no_wm_fold = flag("CEP_NO_WM_FOLD");
  t.host_trace = flag("CEP_HOST_TRACE");
  if (const char* v = std::getenv("CEP_POISON")) t.poison = std::strtoull(v, nullptr, 0);
  t.poison_byte = (int)num("CEP_POISON_BYTE", 0xFF);
  return t;
}
#else
uint32_t tuning_walk_flush() { return 24u; }
void tuning_stream_build(int*, int*, int*) {}
Tuning tuning_from_env() { return Tuning{}; }
#endif

}  // namespace cep
