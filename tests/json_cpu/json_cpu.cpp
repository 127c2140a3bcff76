// Host build of csrc/json_parser.h (TEST INFRASTRUCTURE): the exact per-record state machine the
// GPU decoder runs, driven record by record so `-m "not gpu"` tests check it against
// oracle/json_oracle.py.  Never linked into libcep.so.
#define __device__
#define __forceinline__ inline
#include "json_parser.h"

extern "C" void json_cpu_decode(const uint8_t* bytes, const uint64_t* rec_off, uint64_t n, int col_width,
                                int64_t* price, int64_t* volume, int32_t* status, uint32_t* span) {
  for (uint64_t r = 0; r < n; r++) {
    cep::json::Parser P;
    cep::json::parse_record(P, bytes + rec_off[r], (uint32_t)(rec_off[r + 1] - rec_off[r]));
    status[r] = cep::json::outcome(P, col_width, &price[r], &volume[r]);
    cep::json::name_span(P, status[r], &span[2 * r], &span[2 * r + 1]);
  }
}

// 1 if the record takes the fast path; its outcome and the general state machine's must agree
extern "C" int json_cpu_fast_agrees(const uint8_t* rec, uint32_t len, int* agrees) {
  const uint32_t* words = (const uint32_t*)((uintptr_t)rec & ~(uintptr_t)3);
  auto w = [words](uint32_t j) { return words[j]; };
  const uint32_t lead = (uint32_t)((uintptr_t)rec & 3);
  cep::json::Parser F, G;
  const int fast = cep::json::parse_fast_any(F, w, lead, len);
  cep::json::parse_words(G, w, lead, len);
  int64_t fp, fv, gp, gv;
  uint32_t fo, fl, go, gl;
  const int32_t fs = cep::json::outcome(F, 8, &fp, &fv), gs = cep::json::outcome(G, 8, &gp, &gv);
  cep::json::name_span(F, fs, &fo, &fl);
  cep::json::name_span(G, gs, &go, &gl);
  *agrees = !fast || (fs == gs && fp == gp && fv == gv && fo == go && fl == gl);
  return fast;
}
