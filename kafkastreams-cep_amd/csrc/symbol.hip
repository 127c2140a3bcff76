// symbol.hip — [symbol] keying: the README query partitions its events by
// symbol (README.md:19-28, `[symbol]`: every event of a match has the same name), which this
// build runs as one NFA per key.  Given a batch of StockEvent JSON records decoded by
// cep_decode_stock_json (with name spans), every record gets the key id of its name: the index
// of that name among the batch's distinct names in order of first appearance.  The records
// then go to cep_push_batch as an arrival-order batch (key = symbol).
//
// Name identity is the Java String deserialize() builds (StockEventSerDe.java:63-66:
// new String(data, "UTF-8"), then json-simple's string scanner): the name's UTF-16 code units.
// A name is read as those units straight from the record bytes - ASCII, the JSON escapes
// (\" \\ \/ \b \f \n \r \t \uXXXX) and well-formed UTF-8 (1-4 bytes, no surrogates, no overlong
// forms) - so two spellings of one string ("a", "a") are one symbol.  A null name is a
// symbol of its own.  A name holding malformed UTF-8 (Java would substitute U+FFFD by rules this
// build does not restate) fails the call (CEP_E_INVALID): no guessed key.
//
// Passes (all HBM-bound, one thread per record):
//   sym_insert   decode + 64-bit hash of the units; open-addressing table (CAS on the hash word),
//                the slot's representative = the smallest record index (atomicMin)
//   sym_first    first[r] = 1 iff r is its slot's representative
//   scan         exclusive prefix sum of first[] (hand-written, three levels of 4096 per block)
//   sym_assign   key[r] = prefix[rep]; the record's units compared with the representative's
//                (a 64-bit hash collision between different names fails the call, never merges)
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "cep_internal.h"

namespace cep {

namespace {

constexpr uint32_t kSymNone = 0xFFFFFFFFu;
constexpr int kScanBlock = 256, kScanItems = 16, kScanTile = kScanBlock * kScanItems;

// UTF-16 code units of a JSON string's raw text (between the quotes), one at a time
struct NameUnits {
  const uint8_t* p;
  uint32_t n, i = 0;
  uint32_t low = 0;  // pending low surrogate of a 4-byte UTF-8 sequence
  __device__ NameUnits(const uint8_t* s, uint32_t len) : p(s), n(len) {}
  __device__ static int hex(uint8_t c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }
  // next unit (0..0xFFFF), -1 at the end, -2 on malformed input
  __device__ int next() {
    if (low) {
      const int u = (int)low;
      low = 0;
      return u;
    }
    if (i >= n) return -1;
    const uint8_t c = p[i];
    if (c == '\\') {
      if (i + 1 >= n) return -2;
      const uint8_t e = p[i + 1];
      i += 2;
      switch (e) {
        case '"': return '"';
        case '\\': return '\\';
        case '/': return '/';
        case 'b': return 8;
        case 'f': return 12;
        case 'n': return 10;
        case 'r': return 13;
        case 't': return 9;
        case 'u': {
          if (i + 4 > n) return -2;
          int v = 0;
          for (int k = 0; k < 4; k++) {
            const int h = hex(p[i + k]);
            if (h < 0) return -2;
            v = v * 16 + h;
          }
          i += 4;
          return v;
        }
        default: return -2;  // (the scanner throws on these: such records have a status)
      }
    }
    if (c < 0x80) {
      i++;
      return c;
    }
    // well-formed UTF-8 only
    int len = c >= 0xF0 && c <= 0xF4 ? 4 : c >= 0xE0 ? (c <= 0xEF ? 3 : 0) : c >= 0xC2 ? 2 : 0;
    if (!len || i + len > n) return -2;
    uint32_t cp = c & (len == 2 ? 0x1F : len == 3 ? 0x0F : 0x07);
    for (int k = 1; k < len; k++) {
      const uint8_t b = p[i + k];
      if ((b & 0xC0) != 0x80) return -2;
      cp = (cp << 6) | (b & 0x3F);
    }
    if ((len == 3 && (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF))) || (len == 4 && (cp < 0x10000 || cp > 0x10FFFF)))
      return -2;
    i += len;
    if (cp >= 0x10000) {
      cp -= 0x10000;
      low = 0xDC00 + (cp & 0x3FF);
      return (int)(0xD800 + (cp >> 10));
    }
    return (int)cp;
  }
};

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// hash of record r's name (0 is never returned: it marks an empty slot); *bad on malformed text
__device__ uint64_t name_hash(const uint8_t* bytes, const uint64_t* rec_off, const uint32_t* span, uint64_t r,
                              bool* bad) {
  const uint32_t len = span[2 * r + 1];
  uint64_t h = 0xCBF29CE484222325ull;
  if (len == 0xFFFFFFFFu) {
    h = 0x9E3779B97F4A7C15ull;  // null name
  } else {
    NameUnits it(bytes + rec_off[r] + span[2 * r], len & 0x7FFFFFFFu);
    for (;;) {
      const int u = it.next();
      if (u == -1) break;
      if (u == -2) {
        *bad = true;
        break;
      }
      h = (h ^ (uint64_t)(u + 1)) * 0x100000001B3ull;
    }
  }
  h = mix64(h);
  return h ? h : 1;
}

__global__ void __launch_bounds__(256) sym_insert(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ rec_off,
                                                  const uint32_t* __restrict__ span, const int32_t* __restrict__ status,
                                                  uint64_t n, unsigned long long* tab_hash, uint32_t* tab_rep,
                                                  uint64_t mask, uint32_t* slot_of, uint32_t* err) {
  const uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  if (status && status[r]) {  // deserialize() throws: the record never reaches the NFA
    slot_of[r] = kSymNone;
    return;
  }
  bool bad = false;
  const unsigned long long h = name_hash(bytes, rec_off, span, r, &bad);
  if (bad) {
    atomicOr(err, 1u);
    slot_of[r] = kSymNone;
    return;
  }
  uint64_t s = h & mask;
  for (uint64_t probe = 0; probe <= mask; probe++, s = (s + 1) & mask) {
    const unsigned long long cur = atomicCAS(&tab_hash[s], 0ull, h);
    if (cur == 0ull || cur == h) {
      atomicMin(&tab_rep[s], (uint32_t)r);
      slot_of[r] = (uint32_t)s;
      return;
    }
  }
  atomicOr(err, 2u);  // table full: more distinct names than max_symbols
  slot_of[r] = kSymNone;
}

__global__ void __launch_bounds__(256) sym_first(const uint32_t* __restrict__ slot_of, const uint32_t* __restrict__ tab_rep,
                                                 uint64_t n, uint32_t* first) {
  const uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  const uint32_t s = slot_of[r];
  first[r] = (s != kSymNone && tab_rep[s] == (uint32_t)r) ? 1u : 0u;
}

// ---- exclusive scan of u32 flags into u32 prefixes (n < 2^32), 4096 items per block
__global__ void __launch_bounds__(kScanBlock) scan_tiles(const uint32_t* __restrict__ in, uint64_t n, uint32_t* out,
                                                         uint32_t* tile_sum) {
  __shared__ uint32_t wsum[kScanBlock / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
  uint32_t v[kScanItems], t = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    v[k] = base + k < n ? in[base + k] : 0u;
    t += v[k];
  }
  // inclusive scan of the per-thread totals: within the wave, then across the 4 waves
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = t;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t pre = 0;
  for (uint32_t k = 0; k < w; k++) pre += wsum[k];
  uint32_t run = pre + x - t;  // exclusive prefix of this thread's first item
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    if (base + k < n) out[base + k] = run;
    run += v[k];
  }
  if (threadIdx.x == kScanBlock - 1) tile_sum[blockIdx.x] = pre + x;
}

__global__ void __launch_bounds__(kScanBlock) scan_add(uint32_t* out, uint64_t n, const uint32_t* __restrict__ tile_pre) {
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
  const uint32_t a = tile_pre[blockIdx.x];
#pragma unroll
  for (int k = 0; k < kScanItems; k++)
    if (base + k < n) out[base + k] += a;
}

__global__ void __launch_bounds__(256) sym_assign(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ rec_off,
                                                  const uint32_t* __restrict__ span, const uint32_t* __restrict__ slot_of,
                                                  const uint32_t* __restrict__ tab_rep, const uint32_t* __restrict__ prefix,
                                                  uint64_t n, uint32_t* key, uint32_t* err) {
  const uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  const uint32_t s = slot_of[r];
  if (s == kSymNone) {
    key[r] = kSymNone;
    return;
  }
  const uint32_t rep = tab_rep[s];
  key[r] = prefix[rep];
  if (rep == (uint32_t)r) return;
  // same hash: the same name, unit for unit, or the call fails
  const uint32_t la = span[2 * r + 1], lb = span[2 * rep + 1];
  if ((la == 0xFFFFFFFFu) != (lb == 0xFFFFFFFFu)) {
    atomicOr(err, 4u);
    return;
  }
  if (la == 0xFFFFFFFFu) return;
  NameUnits a(bytes + rec_off[r] + span[2 * r], la & 0x7FFFFFFFu);
  NameUnits b(bytes + rec_off[rep] + span[2 * rep], lb & 0x7FFFFFFFu);
  for (;;) {
    const int x = a.next(), y = b.next();
    if (x != y) {
      atomicOr(err, 4u);
      return;
    }
    if (x < 0) return;
  }
}

}  // namespace

// u32 words of scratch scan_u32 needs for n values: the tile sums and their scan, per level
uint64_t scan_u32_scratch(uint64_t n) {
  const uint64_t tiles = (n + kScanTile - 1) / kScanTile;
  return tiles <= 1 ? tiles * 2 : 2 * tiles + scan_u32_scratch(tiles);
}

// exclusive scan of n u32 (in -> out, n < 2^32 and the total too), recursing over the tile
// sums in `tmp` (scan_u32_scratch(n) words); shared with the partition (cep_internal.h)
hipError_t scan_u32(const uint32_t* in, uint32_t* out, uint64_t n, uint32_t* tmp, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const uint64_t tiles = (n + kScanTile - 1) / kScanTile;
  uint32_t *sums = tmp, *pre = tmp + tiles;
  hipLaunchKernelGGL(scan_tiles, dim3((uint32_t)tiles), dim3(kScanBlock), 0, st, in, n, out, sums);
  if (tiles > 1) {
    hipError_t e = scan_u32(sums, pre, tiles, tmp + 2 * tiles, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(scan_add, dim3((uint32_t)tiles), dim3(kScanBlock), 0, st, out, n, pre);
  }
  return hipGetLastError();
}

hipError_t symbol_keys(const uint8_t* bytes, const uint64_t* rec_off, const uint32_t* span, const int32_t* status,
                       uint64_t n, uint64_t max_symbols, uint32_t* key, uint64_t* n_symbols, uint32_t* err_out,
                       hipStream_t st) {
  *n_symbols = 0;
  *err_out = 0;
  if (n == 0) return hipSuccess;
  uint64_t cap = 1024;
  const uint64_t want = 2 * (max_symbols < n ? max_symbols : n);
  while (cap < want) cap <<= 1;
  // One plain device allocation carved into the call's arrays (no stream-ordered pool: every
  // device allocation of the library is hipMalloc, freed after the call's stream is drained;
  // DESIGN.md §7 "the arrival-order flake").  Layout: hash table (8 B), then u32 arrays.
  const uint64_t w_rep = cap, w_slot = n, w_first = n, w_prefix = n + 1, w_err = 1, w_stmp = scan_u32_scratch(n) + 1;
  const size_t block_bytes = 8 * cap + 4 * (w_rep + w_slot + w_first + w_prefix + w_err + w_stmp);
  void* block = nullptr;
  hipError_t e = hipMalloc(&block, block_bytes);
  if (e != hipSuccess) return e;
  unsigned long long* tab_hash = (unsigned long long*)block;
  uint32_t* tab_rep = (uint32_t*)(tab_hash + cap);
  uint32_t* slot_of = tab_rep + w_rep;
  uint32_t* first = slot_of + w_slot;
  uint32_t* prefix = first + w_first;
  uint32_t* err = prefix + w_prefix;
  uint32_t* stmp = err + w_err;
  auto ok = [&](hipError_t x) { if (e == hipSuccess) e = x; return e == hipSuccess; };
  if (ok(hipMemsetAsync(tab_hash, 0, 8 * cap, st)) && ok(hipMemsetAsync(tab_rep, 0xFF, 4 * cap, st)) &&
      ok(hipMemsetAsync(err, 0, 4, st))) {
    const dim3 g((uint32_t)((n + 255) / 256));
    hipLaunchKernelGGL(sym_insert, g, dim3(256), 0, st, bytes, rec_off, span, status, n, tab_hash, tab_rep, cap - 1,
                       slot_of, err);
    hipLaunchKernelGGL(sym_first, g, dim3(256), 0, st, slot_of, tab_rep, n, first);
    if (ok(scan_u32(first, prefix, n, stmp, st))) {
      hipLaunchKernelGGL(sym_assign, g, dim3(256), 0, st, bytes, rec_off, span, slot_of, tab_rep, prefix, n, key, err);
      uint32_t last[2] = {0, 0};
      if (ok(hipGetLastError()) && ok(hipMemcpyAsync(&last[0], prefix + n - 1, 4, hipMemcpyDeviceToHost, st)) &&
          ok(hipMemcpyAsync(&last[1], first + n - 1, 4, hipMemcpyDeviceToHost, st)) &&
          ok(hipMemcpyAsync(err_out, err, 4, hipMemcpyDeviceToHost, st)) && ok(hipStreamSynchronize(st)))
        *n_symbols = (uint64_t)last[0] + last[1];
    }
  }
  // the call's kernels are done before the block goes back (hipFree also waits for the device)
  (void)hipStreamSynchronize(st);
  (void)hipFree(block);
  return e;
}

}  // namespace cep
