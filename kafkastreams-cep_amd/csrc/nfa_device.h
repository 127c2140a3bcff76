// nfa_device.h — device building blocks of the general NFA kernel: Dewey RLE versions,
// the predicate/aggregate bytecode interpreter (Java value semantics), pool allocation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cep_layout.h"
#include "kernel_args.h"

namespace cep {

// ------------------------------------------------------------------ DeweyVersion (RLE)
// nfa/DeweyVersion.java: addRun :51-56, addStage :84-86, isCompatible :62-82.
__device__ __forceinline__ void dw_init(Dewey& d, int32_t v) {
  d.n = 1;
  d.len = 1;
  d.v[0] = v;
  d.c[0] = 1;
}

// last digit + 1; false when the RLE needs more than kDeweyPairs pairs
__device__ __forceinline__ bool dw_add_run(Dewey& d) {
  uint32_t i = d.n - 1;
  if (d.c[i] == 1) {
    d.v[i] += 1;
    if (i > 0 && d.v[i - 1] == d.v[i]) {  // keep the encoding canonical
      d.c[i - 1] += 1;
      d.n--;
    }
    return true;
  }
  if (d.n >= (uint32_t)kDeweyPairs) return false;
  d.c[i] -= 1;
  d.v[i + 1] = d.v[i] + 1;
  d.c[i + 1] = 1;
  d.n++;
  return true;
}

// append digit 0
__device__ __forceinline__ bool dw_add_stage(Dewey& d) {
  uint32_t i = d.n - 1;
  if (d.v[i] == 0) {
    d.c[i] += 1;
    d.len++;
    return true;
  }
  if (d.n >= (uint32_t)kDeweyPairs) return false;
  d.v[d.n] = 0;
  d.c[d.n] = 1;
  d.n++;
  d.len++;
  return true;
}

// first L digits of a and b are equal
__device__ __forceinline__ bool dw_prefix_eq(const Dewey& a, const Dewey& b, uint32_t L) {
  uint32_t i = 0, j = 0, ra = a.c[0], rb = b.c[0];
  while (L > 0) {
    if (a.v[i] != b.v[j]) return false;
    uint32_t t = ra < rb ? ra : rb;
    if (t > L) t = L;
    L -= t;
    ra -= t;
    rb -= t;
    if (L == 0) break;
    if (ra == 0) { i++; ra = a.c[i]; }
    if (rb == 0) { j++; rb = b.c[j]; }
  }
  return true;
}

// this.isCompatible(that)
__device__ __forceinline__ bool dw_compatible(const Dewey& a, const Dewey& b) {
  if (a.len > b.len) return dw_prefix_eq(a, b, b.len);
  if (a.len == b.len) return dw_prefix_eq(a, b, a.len - 1) && a.v[a.n - 1] >= b.v[b.n - 1];
  return false;
}

// ------------------------------------------------------------------ bytecode interpreter
struct EvalIn {
  const Cols* cols;
  const uint8_t* ftype;
  const int64_t* ts;
  uint64_t pos;        // CSR position of the event
  const int64_t* W;    // fold registers of the run (predicates)
  uint32_t wnull;      // null bits of W
  int64_t curr;        // aggregator's current value
  bool curr_null;
};

__device__ __forceinline__ double as_f64(int64_t x) { return __longlong_as_double(x); }
__device__ __forceinline__ int64_t from_f64(double x) { return __double_as_longlong(x); }

__device__ __forceinline__ int64_t java_d2i(double d) {
  if (d != d) return 0;
  if (d >= 2147483647.0) return 2147483647;
  if (d <= -2147483648.0) return -2147483648LL;
  return (int64_t)(int32_t)d;
}
__device__ __forceinline__ int64_t java_d2l(double d) {
  if (d != d) return 0;
  if (d >= 9223372036854775807.0) return INT64_MAX;
  if (d <= -9223372036854775808.0) return INT64_MIN;
  return (int64_t)d;
}
__device__ __forceinline__ int64_t wrap32(int64_t x) { return (int64_t)(int32_t)(uint32_t)(uint64_t)x; }

// Evaluates the program at `pc`.  Returns the top value; *res_null tells whether it is a
// null box.  On a reference exception sets *err (KE_NPE / KE_ARITH) and returns 0.
__device__ int64_t interp(const uint32_t* __restrict__ code, uint32_t pc, const EvalIn& in,
                          bool* res_null, int* err) {
  int64_t st[kMaxStack];
  uint32_t nb = 0;  // null bit per stack slot
  int sp = 0;
  for (;;) {
    const uint32_t w = code[pc];
    const uint32_t arg = w >> 16;
    switch ((uint8_t)w) {
      case BC_END:
        *res_null = (nb >> (sp - 1)) & 1;
        return st[sp - 1];
      case BC_PUSH32:
        st[sp] = (int64_t)(int32_t)code[pc + 1];
        nb &= ~(1u << sp);
        sp++;
        pc += 2;
        continue;
      case BC_PUSH64:
        st[sp] = (int64_t)((uint64_t)code[pc + 1] | ((uint64_t)code[pc + 2] << 32));
        nb &= ~(1u << sp);
        sp++;
        pc += 3;
        continue;
      case BC_FIELD: {
        const uint8_t t = in.ftype[arg];
        int64_t v;
        if (t == 1) v = (int64_t)((const int32_t*)in.cols->p[arg])[in.pos];
        else v = ((const int64_t*)in.cols->p[arg])[in.pos];  // long and double (bits)
        st[sp] = v;
        nb &= ~(1u << sp);
        sp++;
        break;
      }
      case BC_TS:
        st[sp] = in.ts ? in.ts[in.pos] : (int64_t)in.pos;
        nb &= ~(1u << sp);
        sp++;
        break;
      case BC_SGET:
        st[sp] = in.W[arg];
        nb = (nb & ~(1u << sp)) | (((in.wnull >> arg) & 1u) << sp);
        sp++;
        break;
      case BC_SGETOR:
        if (!((in.wnull >> arg) & 1u)) st[sp - 1] = in.W[arg];
        nb &= ~(1u << (sp - 1));
        break;
      case BC_CURR:
        st[sp] = in.curr;
        nb = (nb & ~(1u << sp)) | ((in.curr_null ? 1u : 0u) << sp);
        sp++;
        break;
      case BC_UNBOX:
        if ((nb >> (sp - 1)) & 1u) { *err = KE_NPE; return 0; }
        break;
      case BC_ARITH: {
        const int64_t b = st[--sp];
        const int64_t a = st[sp - 1];
        const uint32_t op = arg & 15, t = arg >> 4;
        int64_t r;
        if (t == 3) {
          const double x = as_f64(a), y = as_f64(b);
          double z;
          switch (op) {
            case 0: z = __dadd_rn(x, y); break;
            case 1: z = __dsub_rn(x, y); break;
            case 2: z = __dmul_rn(x, y); break;
            case 3: z = __ddiv_rn(x, y); break;
            default: z = fmod(x, y); break;
          }
          r = from_f64(z);
        } else {
          const uint64_t ua = (uint64_t)a, ub = (uint64_t)b;
          switch (op) {
            case 0: r = (int64_t)(ua + ub); break;
            case 1: r = (int64_t)(ua - ub); break;
            case 2: r = (int64_t)(ua * ub); break;
            case 3:
              if (b == 0) { *err = KE_ARITH; return 0; }
              if (b == -1) r = (int64_t)(0 - ua);  // MIN / -1 wraps to MIN (JLS 15.17.2)
              else r = a / b;
              break;
            default:
              if (b == 0) { *err = KE_ARITH; return 0; }
              r = (b == -1) ? 0 : a % b;
              break;
          }
          if (t == 1) r = wrap32(r);
        }
        st[sp - 1] = r;
        break;
      }
      case BC_NEG: {
        const int64_t a = st[sp - 1];
        if (arg == 3) st[sp - 1] = from_f64(-as_f64(a));
        else if (arg == 1) st[sp - 1] = wrap32((int64_t)(0 - (uint64_t)a));
        else st[sp - 1] = (int64_t)(0 - (uint64_t)a);
        break;
      }
      case BC_CAST: {
        const uint32_t from = arg & 15, to = arg >> 4;
        const int64_t a = st[sp - 1];
        int64_t r = a;
        if (from == 3) {
          if (to == 1) r = java_d2i(as_f64(a));
          else if (to == 2) r = java_d2l(as_f64(a));
        } else if (to == 3) {
          r = from_f64((double)a);  // int/long -> double, round to nearest
        } else if (to == 1) {
          r = wrap32(a);
        }
        st[sp - 1] = r;
        break;
      }
      case BC_CMP: {
        const int64_t b = st[--sp];
        const int64_t a = st[sp - 1];
        const uint32_t op = arg & 15, t = arg >> 4;
        bool r;
        if (t == 3) {
          const double x = as_f64(a), y = as_f64(b);
          switch (op) {
            case 0: r = x < y; break;
            case 1: r = x <= y; break;
            case 2: r = x > y; break;
            case 3: r = x >= y; break;
            case 4: r = x == y; break;
            default: r = x != y; break;
          }
        } else {
          switch (op) {
            case 0: r = a < b; break;
            case 1: r = a <= b; break;
            case 2: r = a > b; break;
            case 3: r = a >= b; break;
            case 4: r = a == b; break;
            default: r = a != b; break;
          }
        }
        st[sp - 1] = r ? 1 : 0;
        break;
      }
      case BC_NOT:
        st[sp - 1] = st[sp - 1] ? 0 : 1;
        break;
      case BC_JF:
        if (st[sp - 1] == 0) { pc = arg; continue; }
        sp--;
        break;
      case BC_JT:
        if (st[sp - 1] != 0) { pc = arg; continue; }
        sp--;
        break;
      default:
        *err = KE_CAPACITY;
        return 0;
    }
    pc++;
  }
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
