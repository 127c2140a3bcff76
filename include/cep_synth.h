/* cep_synth.h — synthetic workload generators of the bench and the tests (libcep_synth.so).
 *
 * Test and bench infrastructure, NOT the matcher: libcep.so (include/cep.h) neither links
 * nor calls anything declared here.  The streams are kafkastreams-cep_amd/workloads.py's
 * (SURVEY §8d), bit for bit, generated in device memory.  Same conventions as cep.h: int
 * status (0 = ok), the message of the last failure from cep_synth_last_error(). */
#ifndef CEP_SYNTH_H_
#define CEP_SYNTH_H_
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CEP_SYNTH_OK 0
#define CEP_SYNTH_E_INVALID (-1)
#define CEP_SYNTH_E_HIP (-2)
#define CEP_SYNTH_E_NOMEM (-3)

const char* cep_synth_last_error(void);

/* kind 0 = "abc" (one int column v = h % 16), 1 = "stock" (int price random walk, int volume).
 * Fills device buffers: key_off [n_keys+1] (u64), cols[0..] (int32, n_events each).
 * cep_synth_count returns n_events for sizing. */
int cep_synth_count(int device, int kind, uint64_t seed, uint64_t n_keys, uint64_t key_base,
                    uint32_t mean_events, uint64_t* n_events);
/* Timestamps of a synthetic CSR stream in device memory: ts[i] = base + i (CSR position). */
int cep_synth_ts(int device, uint64_t n_events, int64_t base, int64_t* ts_dev);
int cep_synth_generate(int device, int kind, uint64_t seed, uint64_t n_keys, uint64_t key_base,
                       uint32_t mean_events, uint64_t* key_off_dev, int32_t* const* cols_dev);
/* The same stream in arrival order (round robin: ordered by (index within key, key)): the key
 * of every event in keys_dev [n_events], values in cols_dev. */
int cep_synth_generate_arrival(int device, int kind, uint64_t seed, uint64_t n_keys, uint64_t key_base,
                               uint32_t mean_events, uint32_t* keys_dev, int32_t* const* cols_dev);
/* StockEvent JSON values of n events as json-simple serializes them (StockEventSerDe.java:75-82),
 * {"name":"e<i+1>","price":P,"volume":V} (README.md:73-80): rec_off_dev[n+1] and *total (bytes)
 * are always written; the text goes to out_dev only when *total <= cap. */
int cep_synth_stock_json(int device, const int32_t* price_dev, const int32_t* volume_dev, uint64_t n,
                         uint8_t* out_dev, uint64_t cap, uint64_t* rec_off_dev, uint64_t* total);

#ifdef __cplusplus
}
#endif
#endif /* CEP_SYNTH_H_ */
