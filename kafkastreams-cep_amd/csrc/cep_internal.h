// cep_internal.h — host-side structures of libcep.so (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../../include/cep.h"
#include "cep_layout.h"

namespace cep {

// 256-position strips per workgroup of the begin-hit bitmap kernel (compile.cpp cep_nfa_bits)
constexpr int kBitStrips = 16;
static_assert(kBitStrips % 4 == 0, "cep_nfa_bits covers a block's positions as kBitStrips / 4 strips of 1024");
struct ParsedQuery;
}

struct cep_query {
  cep_query_info info{};
  cep::DevQuery dev{};
  std::vector<uint32_t> code;
  std::vector<std::string> names, fieldNames, stateNames;
  // CEP_KIND_STENCIL
  std::vector<uint16_t> arityStage;   // walk order stage names
  std::vector<uint16_t> stencilProg;  // predicate program per pattern (first..last)
  bool stencilRange = false;          // every predicate is a conjunction of int ranges
  int rangeCols[2] = {0, 0};
  int nRangeCols = 0;
  int64_t rangeLo[8][2]{}, rangeHi[8][2]{};
  // semantic WITHIN (IR v2 flag): epsilon stages keep their source stage's
  // window, so runs expire (the reference's own WITHIN never prunes: parity mode)
  bool semantic = false;
  bool windowed = false;            // semantic and some stage has a window
  int F = 2;                        // fold slots of a run record (states + the start slot)
  std::string jitSource;  // per-query NFA step policy for hipRTC (jit.cpp)
  std::shared_ptr<cep::ParsedQuery> parsed;  // the parsed chain and stage build (plan_groups)
};

namespace cep {

void compile_query(const uint8_t* ir, size_t n, cep_query* q);

// queries sharing one kernel launch (compile.cpp plan_groups)
struct GroupPlan {
  std::vector<int> members;    // query indices, in session order
  std::string source;          // the group's JIT source
  uint32_t nkc = 0;            // literals per query in `table` (0: all compiled in)
  std::vector<int64_t> table;  // members.size() x nkc
};
std::vector<GroupPlan> plan_groups(const std::vector<const cep_query*>& qs);

// Measurement knobs ($CEP_* environment variables).  Read only by the measurement
// build (libcep_measure.so: CEP_MEASURE, Makefile `measure`), once, when a session is created
// (tuning.cpp) - never on the launch path - and kept in the session; the release build uses the
// defaults below.  Most change only the launch geometry and the time a batch takes; the few that
// change results (timing and diagnosis only) are listed in tuning.cpp's header.
struct Tuning {
  uint32_t resident_waves = 0;  // $CEP_RESIDENT_WAVES: waves per CU of the persistent grids (0: default)
  bool no_persist = false;      // $CEP_NO_PERSIST: one lane per job for kernel groups too
  bool no_spread = false;       // $CEP_NO_SPREAD: underfilled single-query launches not spread
  bool no_retry = false;        // $CEP_NO_RETRY: capacity / conflict re-runs skipped (their keys keep the error)
  uint32_t node_chunk = 0;      // $CEP_NODE_CHUNK: pool range per lane (0: default)
  uint32_t out_chunk = 0;       // $CEP_OUT_CHUNK
  uint32_t walk_cap = 0;        // $CEP_WALK_CAP: deferred walks per lane (0: default)
  bool prof = false;            // $CEP_PROF: print the kernel's time split (compiled in too)
  bool stream_narrow = false;   // $CEP_STREAM_NARROW: streams on the narrow build
  int part_rounds = 16;         // $CEP_PART_ROUNDS (8, 12, 16, 24, 32): events per thread of the partition's sort tiles
  uint32_t stream_iso = 2048;   // $CEP_STREAM_ISO: a stream's heaviest keys alone in their waves (0: off)
  bool no_est_blend = false;    // $CEP_NO_EST_BLEND: a stream's lane order from this batch alone
  bool stream_wide = false;     // $CEP_STREAM_WIDE: streams on the wide build even when the stream build holds
  bool stream_no_order = false; // $CEP_STREAM_NO_ORDER
  bool no_wm_fold = false;      // $CEP_NO_WM_FOLD: the watermark as its own pass
  bool host_trace = false;      // $CEP_HOST_TRACE: allocations and push phases on stderr
  int poison_byte = 0xFF;       // $CEP_POISON_BYTE
  uint64_t poison = 0;          // $CEP_POISON=mask: new device buffers filled with 0xFF (session.cpp DBuf)
};
Tuning tuning_from_env();
// the drain threshold the JIT kernels are compiled with ($CEP_WALK_FLUSH, default 24)
uint32_t tuning_walk_flush();

struct NfaArgs;
struct StencilArgs;
struct KeyState;

hipError_t launch_nfa(int F, const NfaArgs& a, uint64_t nslots, uint32_t code_len, hipStream_t st);
uint64_t ring_size(int F, uint64_t n_slots, uint32_t rcap);  // double-buffered run queues
uint64_t walkq_size(uint64_t n_slots, uint32_t wcap, uint32_t plog);  // deferred-walk queues + put logs
hipError_t launch_collect_retry(const KeyState* ks, uint64_t n, uint32_t* cap_list, uint32_t* conf_list,
                                uint32_t* counts, hipStream_t st);
hipError_t launch_compact(const KeyState* ks, uint64_t n_keys, uint64_t* bsum_m, uint64_t* bsum_p,
                          uint64_t* totals, hipStream_t st);
uint64_t scatter_heavy_bytes(uint64_t n_keys);
// exclusive scan, symbol.hip: `tmp` holds scan_u32_scratch(n) u32 words
uint64_t scan_u32_scratch(uint64_t n);
hipError_t scan_u32(const uint32_t* in, uint32_t* out, uint64_t n, uint32_t* tmp, hipStream_t st);
hipError_t symbol_keys(const uint8_t* bytes, const uint64_t* rec_off, const uint32_t* span, const int32_t* status,
                       uint64_t n, uint64_t max_symbols, uint32_t* key, uint64_t* n_symbols, uint32_t* err,
                       hipStream_t st);
hipError_t launch_scatter(const KeyState* ks, uint64_t n_keys, const uint64_t* bsum_m, const uint64_t* bsum_p,
                          const uint32_t* out, uint32_t* m_key, uint32_t* m_emit, uint64_t* m_off,
                          uint32_t* p_seq, uint16_t* p_stage, const uint64_t* totals, void* heavy_scratch,
                          hipStream_t st);
hipError_t launch_digest(uint64_t n, uint32_t arity, const uint16_t* names, const uint32_t* m_key,
                         const uint32_t* m_emit, const uint64_t* m_off, const uint32_t* p_seq,
                         const uint16_t* p_stage, unsigned long long* out, hipStream_t st);
hipError_t launch_wave_keys(const uint64_t* key_off, uint64_t n_keys, uint64_t n_events, uint32_t* wave_key,
                            uint32_t* zero, uint32_t n_zero, hipStream_t st);
uint64_t stencil_waves(uint64_t n_events);
hipError_t launch_stencil(int m, const StencilArgs& a, bool range, int ncol, hipStream_t st);
uint64_t stencil_tiles(uint64_t n_events);
hipError_t launch_decode_stock_json(const uint8_t* bytes, const uint64_t* rec_off, uint64_t n, int col_width,
                                    void* price, void* volume, int32_t* status, uint32_t* name_span,
                                    hipStream_t st);
hipError_t launch_max(const int64_t* ts, uint64_t n, unsigned long long* out, hipStream_t st);
struct Node;
hipError_t launch_live_floor(const Node* nodes, uint64_t n_nodes, uint64_t n_keys, uint32_t* floor, hipStream_t st);
std::vector<char> jit_code_object(const std::string& src, double* compile_s, bool touch = false);
// the wide build of a generated kernel (6 Dewey pairs; the source as generated is the narrow
// build): capacity re-runs and streaming sessions run it
inline std::string jit_wide_source(const std::string& src) { return "#define CEP_DEWEY_PAIRS 6\n" + src; }
// the stream build (streaming sessions): 3-pair versions in registers at the narrow build's 3
// waves per SIMD, in the wide build's memory layout (a stream's records and pointers outlive the
// launch); the put log (a stream cannot re-run a key: walk conflicts resolved in place); a key
// whose versions outgrow 3 pairs stops before that event for the wide build to continue
// (CEP_STREAM_STOP, nfa_lane.h stop_event)
// the stream build's register pairs, memory-layout pairs and put log: 3, 6, 1 (measurement
// builds, tuning.cpp: $CEP_STREAM_PAIRS, $CEP_STREAM_LAYOUT, $CEP_STREAM_PUTLOG=0 - the last
// two inexact for streams, for timing what they cost)
void tuning_stream_build(int* pairs, int* layout, int* plog);
inline std::string jit_stream_source(const std::string& src) {
  int pairs = 3, layout = 6, plog = 1;
  tuning_stream_build(&pairs, &layout, &plog);
  return "#define CEP_DEWEY_PAIRS " + std::to_string(pairs) + "\n#define CEP_LAYOUT_PAIRS " + std::to_string(layout) +
         "\n#define CEP_PUT_LOG " + std::to_string(plog) + "\n#define CEP_STREAM_STOP 1\n#define CEP_WALK_IN_PLACE 0\n"
         "#define CEP_PERSIST_LANES 0\n#define CEP_WAVES_EU 3\n" + src;
}
struct Cols;
size_t partition_scratch_bytes(uint64_t n, uint64_t n_keys);
hipError_t partition(const uint32_t* key, uint64_t n, uint64_t n_keys, int nf, Cols in, Cols out, uint32_t wide_mask,
                     const int64_t* ts_in, int64_t* ts_out, uint64_t* key_off, uint64_t* cnt, uint32_t* perm,
                     uint32_t* sorted_keys, uint32_t* idx, void* scratch, size_t scratch_bytes, unsigned* bad,
                     hipStream_t st, int rounds = 16);
// keys 0..n-1 ordered by est descending (16-bit sort keys, partition.hip est_key16) -> order;
// est_sorted: the sorted keys (inverted), key16: n words (tmp: scratch grown as needed)
hipError_t sort_keys_by_work(const uint32_t* est, uint32_t* est_sorted, uint32_t* key16, uint32_t* order,
                             uint64_t n, void*& tmp, size_t& tmp_bytes, hipStream_t st);
hipError_t sort_keys_scratch(uint64_t n, void*& tmp, size_t& tmp_bytes);
std::string jit_cache_key(const std::string& src);
hipError_t gather_keys(uint64_t n_sel, const uint32_t* sel, const uint64_t* src_off, const uint64_t* dst_off,
                       int nf, const uint32_t* col_bytes, const void* const* src_cols, void* const* dst_cols,
                       const int64_t* src_ts, int64_t* dst_ts, hipStream_t st);

}  // namespace cep
