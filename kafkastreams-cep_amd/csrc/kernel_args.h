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
  void* walks;               // deferred-walk queues, wcap per slot, then plog put-log entries (nfa_lane.h)
  uint32_t wcap;
  uint32_t plog;             // put-log entries per slot: room for every put one event can log
                             // (2 * rcap + 4) twice over, at least kPutLogMin (session.cpp)
  uint32_t defer;            // 1: queue buffer walks and drain them wave-wide; 0: walk in place
  // Jobs: a job is (query qi of the launch, key), id qi * n_keys + key.  Without a job list, job
  // index i is query i % n_q on the key of rank i / n_q, rank -> key through `order` (lane
  // order; null = identity).  A retry pass lists its jobs explicitly.  (Streaming sessions,
  // job_next null: wave W runs query W % n_q on ranks (W / n_q) * 64 + lane.)
  const uint32_t* jobs;      // retry pass: job index i is job jobs[i]; null = the mapping above
  uint64_t n_jobs;           // job indices of the launch (persistent lanes)
  const uint32_t* order;     // key of each rank (longest-first lane order), null = identity
  uint32_t* job_next;        // persistent lanes (nfa_lane.h run_jobs): next job index to claim;
                             // null: one job per lane (streaming sessions)
  uint64_t spread;           // W > 0: an underfilled single-query launch of W waves, wave w's lane l
                             // running rank l * W + w (session.cpp run_nfa); 0: rank w * 64 + l
                             // (odd lanes take their row of ranks in reverse)
  uint32_t spread_iso;       // no spread: the K = spread_iso heaviest ranks run alone, one per wave
                             // (waves 0..K-1, lane 0), the other ranks 64 per wave in rank order
                             // from wave K (a stream's lane order, n_q 1)
  uint32_t n_q;              // queries of the launch (a kernel group, compile.cpp plan_groups)
  const int64_t* kc;         // their literal table, n_q x NKC (group kernels)
  Node* nodes;
  Pred* preds;               // the predecessor pool (a node's second and later pointers)
  Pred* preds0;              // a node's first pointer, one slot per node index
  uint32_t* out;             // output chunks (kOutChunkWords words each)
  Pool node_pool, pred_pool, out_pool;
  KeyState* ks;
  KeyCarry* carry;           // streaming: per-key state in/out (null: every key starts fresh)
  uint32_t widen;            // streaming: this launch continues the listed jobs the stream build
                             // stopped (KE_WIDEN) from their carried event, output appended
  uint32_t* est;             // cep_nfa_est: per-key work estimate (longest-first lane order)
  uint32_t est_blend;        // streams: blend the estimate with the key's running one (KeyCarry.west)
  uint64_t* bhits;           // cep_nfa_bits: bit p = the begin predicate (null folds) is true or
                             // throws at CSR position p (quiet lanes jump to the next set bit)
  uint64_t n_events;         // CSR positions of the batch (bits kernel)
  uint32_t* n_capacity_err;  // jobs to re-run (KE_RETRY / KE_CONFLICT)
  uint32_t* full;            // bit 0: a run queue overflowed this launch (the next batch starts
                             // with a bigger one, session.cpp)
  // watermark folded into the bitmap pass (session.cpp): cep_nfa_bits writes each block's
  // largest event time (of `ts`) to wm_blocks[block] (n_wm_blocks of them); cep_nfa_est's first
  // blocks reduce them into *wmax (order-preserving unsigned map, one atomicMax per block)
  int64_t* wm_blocks;
  uint64_t n_wm_blocks;
  unsigned long long* wmax;
  unsigned long long* prof;  // measurement builds ($CEP_PROF): the time split of nfa_lane.h, 16 counters
};

}  // namespace cep
