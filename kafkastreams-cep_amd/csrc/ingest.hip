// ingest.hip — the step before the matcher: StockEvent JSON records -> event columns.
//
// Replaces the demo's value deserializer StockEventSerDe.JsonSerDeserializer.deserialize
// (test:demo/StockEventSerDe.java:58-72): json-simple 1.1.1's JSONParser (pom.xml:99-104; not in
// /root/reference, restated here from its published lexer/parser) parses the record, then
//   new StockEvent((String) o.get("name"), (Long) o.get("price"), (Long) o.get("volume"))
// (test:demo/StockEvent.java:4-14).  Every record gets the outcome the Java call would have:
// the columns, or the exception that would escape deserialize() as a status code (CEP_JSON_*).
//
// Layout: the batch is Kafka-style record values back to back in HBM (bytes) with u64 record
// offsets rec_off[n+1].  One thread per record, two passes.  Pass 1 (decode_stock_json_kernel,
// 24 VGPRs): a 256-record block stages its byte span into LDS with coalesced 16-byte loads
// (a block whose span exceeds the tile reads HBM) and every lane runs the serializer-layout fast
// path; records it cannot take are marked pending.  Pass 2 (decode_stock_json_general) runs
// the full state machine on the pending records only.  HBM-bound: bytes + 8 B offset read once, the columns
// and status written once.
//
// json-simple semantics reproduced (the parts a StockEvent record can reach):
//  * lexer (Yylex): whitespace [ \t\n\r\f]; INT -?[0-9]+ -> Long.valueOf (overflow throws
//    NumberFormatException); DOUBLE INT(\.[0-9]+)?([eE][-+]?[0-9]+)? -> Double; longest match, so
//    "1." lexes INT then fails on '.'; true/false/null; strings with \" \\ \/ \b \f \n \r \t
//    \uXXXX escapes and raw bytes otherwise; any other byte outside a string -> ParseException;
//    an unknown escape -> the scanner's java.lang.Error; a string cut off by the end of input is
//    end of input.
//  * parser (JSONParser.parse): commas and colons are skipped wherever they are legal tokens of
//    the current container state, duplicate keys keep the last value (HashMap.put), one value
//    then end of input.
//  * deserialize: the top value must be a JSONObject (null -> NullPointerException on get);
//    casts and unboxing in argument order: name (String or null), price (Long, unboxed), volume.
#include <hip/hip_runtime.h>
#include <stdint.h>


#include "json_parser.h"

namespace cep {



constexpr int kIngestBlock = 256;
constexpr uint32_t kIngestLds = 16384;  // bytes of record text staged per block (avg record <= 64 B)
static_assert(kIngestLds % (16 * kIngestBlock) == 0, "the staging loads: whole 16-B chunks per thread");
constexpr int32_t kPending = -1;          // pass 1 left the record to the general state machine

template <typename T>
__device__ __forceinline__ void store_cols(void* price, void* volume, uint64_t r, int64_t p, int64_t v) {
  ((T*)price)[r] = (T)p;
  ((T*)volume)[r] = (T)v;
}

__device__ __forceinline__ void write_outcome(const json::Parser& P, uint64_t r, int col_width, void* price,
                                              void* volume, int32_t* status, uint32_t* name_span) {
  int64_t pv, vv;
  const int32_t st = json::outcome(P, col_width, &pv, &vv);
  if (col_width == 4) store_cols<int32_t>(price, volume, r, pv, vv);
  else store_cols<int64_t>(price, volume, r, pv, vv);
  status[r] = st;
  if (name_span) json::name_span(P, st, &name_span[2 * r], &name_span[2 * r + 1]);
}

// Pass 1: each 256-record block staged in LDS, the serializer-layout fast path per lane.
__global__ void __launch_bounds__(kIngestBlock) decode_stock_json_kernel(
    const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ rec_off, uint64_t n, int col_width,
    void* __restrict__ price, void* __restrict__ volume, int32_t* __restrict__ status,
    uint32_t* __restrict__ name_span) {
  __shared__ uint4 tile[kIngestLds / 16];
  const uint64_t r0 = (uint64_t)blockIdx.x * kIngestBlock;
  const uint64_t r1 = r0 + kIngestBlock < n ? r0 + kIngestBlock : n;
  const uint64_t A = rec_off[r0], B = rec_off[r1];
  // aligned 16-byte chunks g0..g1 cover the block's span [A, B); a chunk that holds at least one
  // byte of the span never leaves its pages
  const uint64_t skew = (uintptr_t)bytes & 15;
  const uint64_t g0 = (A + skew) >> 4, g1 = (B + skew + 15) >> 4;
  const bool staged = (g1 - g0) * 16 <= kIngestLds;
  if (staged) {
    const uint4* src = (const uint4*)((uintptr_t)bytes - skew);
    // every chunk load of the thread in flight before its LDS stores (a load-store loop waited
    // for each load in turn)
    constexpr int kIt = kIngestLds / 16 / kIngestBlock;
    uint4 v[kIt];
#pragma unroll
    for (int i = 0; i < kIt; i++) {
      const uint64_t c = g0 + threadIdx.x + (uint64_t)i * kIngestBlock;
      v[i] = c < g1 ? src[c] : uint4{0u, 0u, 0u, 0u};
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < kIt; i++) {
      const uint64_t c = g0 + threadIdx.x + (uint64_t)i * kIngestBlock;
      if (c < g1) tile[c - g0] = v[i];
    }
    __syncthreads();
  }
  const uint64_t r = r0 + threadIdx.x;
  if (r >= n) return;
  const uint64_t a = rec_off[r], b = rec_off[r + 1];
  json::Parser P;
  const uint32_t len = (uint32_t)(b - a);
  bool fast;
  if (staged) {
    // LDS: 32-bit byte offset into the tile, words read with ds_read (no flat pointer into LDS)
    const uint32_t o = (uint32_t)(a + skew - (g0 << 4));
    const uint32_t* tw = (const uint32_t*)tile;
    const uint32_t w0 = o >> 2;
    fast = json::parse_fast_any(P, [tw, w0](uint32_t j) { return tw[w0 + j]; }, o & 3, len);
  } else {
    const uint32_t* words = (const uint32_t*)((uintptr_t)(bytes + a) & ~(uintptr_t)3);
    fast = json::parse_fast_any(P, [words](uint32_t j) { return words[j]; }, (uint32_t)((uintptr_t)(bytes + a) & 3), len);
  }
  if (!fast) {
    status[r] = kPending;
    return;
  }
  write_outcome(P, r, col_width, price, volume, status, name_span);
}

// Pass 2: the records pass 1 could not take, through the general state machine (from HBM).
__global__ void __launch_bounds__(kIngestBlock) decode_stock_json_general(
    const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ rec_off, uint64_t n, int col_width,
    void* __restrict__ price, void* __restrict__ volume, int32_t* __restrict__ status,
    uint32_t* __restrict__ name_span) {
  // 4 records per thread: the status scan is the whole pass when nothing is pending
  const uint64_t r4 = ((uint64_t)blockIdx.x * kIngestBlock + threadIdx.x) * 4;
  int32_t st4[4];
#pragma unroll
  for (int k = 0; k < 4; k++) st4[k] = r4 + k < n ? status[r4 + k] : 0;
  for (int k = 0; k < 4; k++) {
    if (st4[k] != kPending) continue;
    const uint64_t r = r4 + k;
    const uint64_t a = rec_off[r], b = rec_off[r + 1];
    const uint32_t* words = (const uint32_t*)((uintptr_t)(bytes + a) & ~(uintptr_t)3);
    json::Parser P;
    json::parse_words(P, [words](uint32_t j) { return words[j]; }, (uint32_t)((uintptr_t)(bytes + a) & 3),
                      (uint32_t)(b - a));
    write_outcome(P, r, col_width, price, volume, status, name_span);
  }
}

hipError_t launch_decode_stock_json(const uint8_t* bytes, const uint64_t* rec_off, uint64_t n, int col_width,
                                    void* price, void* volume, int32_t* status, uint32_t* name_span,
                                    hipStream_t st) {
  if (n == 0) return hipSuccess;
  const dim3 grid((uint32_t)((n + kIngestBlock - 1) / kIngestBlock));
  hipLaunchKernelGGL(decode_stock_json_kernel, grid, dim3(kIngestBlock), 0, st, bytes, rec_off, n, col_width, price,
                     volume, status, name_span);
  const dim3 grid2((uint32_t)((n + 4 * kIngestBlock - 1) / (4 * kIngestBlock)));
  hipLaunchKernelGGL(decode_stock_json_general, grid2, dim3(kIngestBlock), 0, st, bytes, rec_off, n, col_width,
                     price, volume, status, name_span);
  return hipGetLastError();
}

}  // namespace cep
