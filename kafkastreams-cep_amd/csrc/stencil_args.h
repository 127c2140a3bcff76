// stencil_args.h — kernel arguments of the strict-contiguity stencil (stencil.hip).  Kept out
// of kernel_args.h, which is embedded into every JIT compile (and its cache key).
#pragma once
#include "kernel_args.h"

namespace cep {

struct RangeStage {  // conjunction of lo <= col_c <= hi for c in {0, 1}
  int64_t lo[2], hi[2];
};

struct StencilArgs {
  uint64_t n_keys, n_events;
  const uint64_t* key_off;
  const uint32_t* wave_key;  // key holding the first event of each wave's span (kStWave events)
  const int32_t* col[2];     // range fast path: up to two int columns
  RangeStage rs[8];
  // generic path (interpreted predicates)
  const DevQuery* q;
  const uint32_t* code;
  Cols cols;
  const int64_t* ts;
  uint16_t prog[kMaxStencil];
  uint16_t stage_name[kMaxStencil];    // walk order: stage name of pair t (t = 0 is the final event)
  bool aligned;              // col[] 16-B aligned: vector loads
  uint64_t n_chunk;          // stencil_mask: kStWave-event chunks (one a wave)
  // pass 1 -> pass 3
  // per 64-event word w (pass 1): {match bits lo, hi (bit i: a match ends at event 64 w + i), the
  // key holding event 64 w (bit 31: a key starts inside the word after its first event), event
  // 64 w's sequence number within that key}
  uint4* words;
  uint32_t* group_cnt;       // matches per stencil_emit block's span (pass 1, atomics; zeroed per batch)
  // output
  uint32_t* m_key;
  uint32_t* p_seq;           // [n_matches * m]
  uint64_t* total;           // number of matches (written by the last tile of stencil_emit)
  uint64_t* total_host;      // the same, into the session's pinned host copy (no D2H copy per batch)
  uint64_t out_cap;          // matches that fit the output arrays
  uint32_t* overflow;
};

}  // namespace cep
