// kernel_args.h — launch-argument structs shared by the HIP kernels and the host session.
#pragma once
#include <stdint.h>

#include "cep_layout.h"

namespace cep {

struct Cols {
  const void* p[kMaxFields];
};

// A global pool handed out in per-lane chunks (one atomic per chunk).
struct Pool {
  uint32_t* top;
  uint32_t cap;
  uint32_t chunk;
};

struct NfaArgs {
  const DevQuery* q;
  const uint32_t* code;
  uint64_t n_keys;
  const uint64_t* key_off;
  Cols cols;
  const int64_t* ts;
  void* rings;               // Rec<F>[n_slots * rcap]
  uint32_t rcap;
  const uint32_t* key_list;  // retry pass: slot i runs key key_list[i]; null = all keys
  uint32_t n_list;
  Node* nodes;
  Pred* preds;
  uint32_t* out;             // output chunks (kOutChunkWords words each)
  Pool node_pool, pred_pool, out_pool;
  KeyState* ks;
  uint32_t* n_capacity_err;  // keys that hit CEP_KEY_CAPACITY
};

struct RangeStage {  // conjunction of lo <= col_c <= hi for c in {0, 1}
  int64_t lo[2], hi[2];
};

struct StencilArgs {
  uint64_t n_keys, n_events;
  const uint64_t* key_off;
  const uint32_t* tile_key;  // first key of each tile
  const int32_t* col[2];     // range fast path: up to two int columns
  RangeStage rs[8];
  // generic path (interpreted predicates)
  const DevQuery* q;
  const uint32_t* code;
  Cols cols;
  const int64_t* ts;
  uint16_t prog[8];
  uint16_t stage_name[8];    // walk order: stage name of pair t (t = 0 is the final event)
  // output
  uint32_t* tile_counter;
  unsigned long long* status;  // per tile: [63:62] flag (1 aggregate, 2 inclusive), [61:0] value
  uint32_t* m_key;
  uint32_t* p_seq;           // [n_matches * m]
  uint64_t* total;           // number of matches (written by the last tile)
  unsigned long long* digest;
  uint64_t out_cap;          // matches that fit the output arrays
  uint32_t* overflow;
};

}  // namespace cep
