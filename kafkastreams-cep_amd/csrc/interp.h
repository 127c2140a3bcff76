// interp.h — bytecode interpreter of the predicate/aggregate IR (AOT tier).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cep_layout.h"
#include "kernel_args.h"
#include "java.h"

namespace cep {

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

}  // namespace cep
