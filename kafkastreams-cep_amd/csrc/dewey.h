// dewey.h — DeweyVersion as run-length encoded (value, count) pairs, plus pool allocation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cep_layout.h"
#include "kernel_args.h"

namespace cep {

// ------------------------------------------------------------------ DeweyVersion (RLE)
// nfa/DeweyVersion.java: addRun :51-56, addStage :84-86, isCompatible :62-82.
// Versions are canonical run-length encodings (adjacent pairs differ in value).  Every
// operation indexes the pair arrays with compile-time indices only (unrolled selects), so a
// Dewey held in a local stays in registers instead of scratch.
constexpr int P = kDeweyPairs;

// Each operation first copies its operands through an empty asm: the unrolled selects then
// pick between register values.  Selecting between loads instead lets LLVM fold them into
// one load through a computed address, which pins every Dewey it touches in scratch.
__device__ __forceinline__ Dewey dw_pin(const Dewey& d) {
  Dewey x;
  uint32_t n = d.n, len = d.len;
  asm("" : "+v"(n), "+v"(len));
  x.n = n;
  x.len = len;
#pragma unroll
  for (int k = 0; k < P; k++) {
    int32_t a = d.v[k];
    uint32_t b = d.c[k];
    asm("" : "+v"(a), "+v"(b));
    x.v[k] = a;
    x.c[k] = b;
  }
  return x;
}

// field-wise store (a struct copy from a local would be lowered through scratch)
__device__ __forceinline__ void dw_store(Dewey& dst, const Dewey& v) {
  const Dewey x = dw_pin(v);
  dst.n = x.n;
  dst.len = x.len;
#pragma unroll
  for (int k = 0; k < P; k++) {
    dst.v[k] = x.v[k];
    dst.c[k] = x.c[k];
  }
}

__device__ __forceinline__ void dw_init(Dewey& d, int32_t v) {
  d.n = 1;
  d.len = 1;
  d.v[0] = v;
  d.c[0] = 1;
#pragma unroll
  for (int k = 1; k < P; k++) {
    d.v[k] = 0;
    d.c[k] = 0;
  }
}

// the same version (canonical encodings: the same pairs in use)
__device__ __forceinline__ bool dw_equal(const Dewey& a0, const Dewey& b0) {
  const Dewey a = dw_pin(a0), b = dw_pin(b0);
  bool eq = a.n == b.n;
#pragma unroll
  for (int k = 0; k < P; k++)
    if ((uint32_t)k < a.n) eq = eq && a.v[k] == b.v[k] && a.c[k] == b.c[k];
  return eq;
}

__device__ __forceinline__ int32_t dw_last(const Dewey& d0) {
  const Dewey d = dw_pin(d0);
  int32_t r = d.v[0];
#pragma unroll
  for (int k = 1; k < P; k++)
    if ((uint32_t)k == d.n - 1) r = d.v[k];
  return r;
}

// last digit + 1; false when the RLE would need more than kDeweyPairs pairs
__device__ __forceinline__ bool dw_add_run(Dewey& d0) {
  Dewey d = dw_pin(d0);
  const uint32_t i = d.n - 1;
  uint32_t ci = 0;
  int32_t vi = 0, vprev = 0;
#pragma unroll
  for (int k = 0; k < P; k++) {
    if ((uint32_t)k == i) { ci = d.c[k]; vi = d.v[k]; }
    if ((uint32_t)k + 1 == i) vprev = d.v[k];
  }
  if (ci == 1) {
    const int32_t nv = vi + 1;
    const bool merge = i > 0 && vprev == nv;  // keep the encoding canonical
#pragma unroll
    for (int k = 0; k < P; k++) {
      if ((uint32_t)k == i) {
        d.v[k] = merge ? 0 : nv;
        d.c[k] = merge ? 0 : 1;
      }
      if (merge && (uint32_t)k + 1 == i) d.c[k] += 1;
    }
    if (merge) d.n--;
    d0 = d;
    return true;
  }
  if (d.n >= (uint32_t)P) return false;
#pragma unroll
  for (int k = 0; k < P; k++) {
    if ((uint32_t)k == i) d.c[k] = ci - 1;
    if ((uint32_t)k == i + 1) {
      d.v[k] = vi + 1;
      d.c[k] = 1;
    }
  }
  d.n++;
  d0 = d;
  return true;
}

// append digit 0
__device__ __forceinline__ bool dw_add_stage(Dewey& d0) {
  Dewey d = dw_pin(d0);
  const uint32_t i = d.n - 1;
  const int32_t vi = dw_last(d);
  if (vi == 0) {
#pragma unroll
    for (int k = 0; k < P; k++)
      if ((uint32_t)k == i) d.c[k] += 1;
    d.len++;
    d0 = d;
    return true;
  }
  if (d.n >= (uint32_t)P) return false;
#pragma unroll
  for (int k = 0; k < P; k++)
    if ((uint32_t)k == i + 1) {
      d.v[k] = 0;
      d.c[k] = 1;
    }
  d.n++;
  d.len++;
  d0 = d;
  return true;
}

// this.isCompatible(that)  (a = this, b = that)
__device__ __forceinline__ bool dw_compatible(const Dewey& a0, const Dewey& b0) {
  const Dewey a = dw_pin(a0), b = dw_pin(b0);
  if (a.len > b.len) {
    // b is a prefix of a: b's pairs but the last equal a's, b's last run is a prefix of a's run
    if (b.n > a.n) return false;
    bool ok = true;
#pragma unroll
    for (int k = 0; k < P; k++) {
      if ((uint32_t)k + 1 < b.n) ok = ok && a.v[k] == b.v[k] && a.c[k] == b.c[k];
      if ((uint32_t)k + 1 == b.n) ok = ok && a.v[k] == b.v[k] && a.c[k] >= b.c[k];
    }
    return ok;
  }
  if (a.len != b.len) return false;
  // equal length: all digits but the last equal, then a.last >= b.last.  Dropping the last
  // digit of a canonical RLE keeps it canonical: compare the shortened encodings exactly.
  const uint32_t an = a.n, bn = b.n;
  uint32_t alc = 0, blc = 0;
#pragma unroll
  for (int k = 0; k < P; k++) {
    if ((uint32_t)k + 1 == an) alc = a.c[k];
    if ((uint32_t)k + 1 == bn) blc = b.c[k];
  }
  const uint32_t an2 = alc == 1 ? an - 1 : an, bn2 = blc == 1 ? bn - 1 : bn;
  if (an2 != bn2) return false;
  bool ok = true;
#pragma unroll
  for (int k = 0; k < P; k++) {
    if ((uint32_t)k < an2) {
      const uint32_t ca = a.c[k] - ((uint32_t)k + 1 == an ? 1u : 0u);
      const uint32_t cb = b.c[k] - ((uint32_t)k + 1 == bn ? 1u : 0u);
      ok = ok && a.v[k] == b.v[k] && ca == cb;
    }
  }
  return ok && dw_last(a) >= dw_last(b);
}

// isCompatible (DeweyVersion.java:62-82) for versions of at most 2 RLE pairs, from plain
// values (a pointer's first Dewey quad is exactly this): the buffer walks' common case,
// a handful of compares instead of dw_compatible's unrolled 6-pair selects.  a = the walker,
// b = the pointer; canonical RLE (adjacent pairs differ in value).
__device__ __forceinline__ bool dw_compat2(uint32_t an, uint32_t alen, int32_t av0, uint32_t ac0, int32_t av1,
                                           uint32_t ac1, uint32_t bn, uint32_t blen, int32_t bv0, uint32_t bc0,
                                           int32_t bv1, uint32_t bc1) {
  if (alen > blen) {  // b is a prefix of a: b's last run fits in a's run at the same position
    if (bn > an) return false;
    if (bn == 0) return true;
    if (bn == 1) return av0 == bv0 && ac0 >= bc0;
    return av0 == bv0 && ac0 == bc0 && av1 == bv1 && ac1 >= bc1;
  }
  if (alen != blen) return false;
  // equal length: all digits but the last equal, then a.last >= b.last
  const uint32_t al = an == 2 ? ac1 - 1 : ac0 - 1, bl = bn == 2 ? bc1 - 1 : bc0 - 1;  // last run, shortened
  const uint32_t an2 = al == 0 ? an - 1 : an, bn2 = bl == 0 ? bn - 1 : bn;
  if (an2 != bn2) return false;
  bool ok = true;
  if (an2 >= 1) ok = av0 == bv0 && (an == 1 ? al : ac0) == (bn == 1 ? bl : bc0);
  if (an2 >= 2) ok = ok && av1 == bv1 && al == bl;
  const int32_t alast = an == 2 ? av1 : av0, blast = bn == 2 ? bv1 : bv0;
  return ok && alast >= blast;
}

// ------------------------------------------------------------------ pool allocation
__device__ __forceinline__ uint32_t pool_take(const Pool& p, uint32_t& cur, uint32_t& end) {
  if (cur == end) {
    const uint32_t b = atomicAdd(p.top, p.chunk);
    if (b >= p.cap || p.cap - b < p.chunk) return CEP_NONE;
    cur = b;
    end = b + p.chunk;
  }
  return cur++;
}

}  // namespace cep
