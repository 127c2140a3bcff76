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
