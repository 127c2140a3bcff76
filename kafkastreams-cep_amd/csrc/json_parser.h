// json_parser.h — json-simple 1.1.1's scanner + parser and StockEventSerDe's casts as a per-record
// byte state machine (see ingest.hip for the semantics and citations).  Plain C++ with
// __device__ markers: ingest.hip runs it one thread per record; tests/json_cpu.cpp compiles
// it for the host (test infrastructure) with the markers defined away.
#pragma once
#include <stdint.h>

#include "../../include/cep.h"

namespace cep {

namespace json {

enum Lex : uint8_t { L_WS, L_STR, L_ESC, L_UHEX, L_NEG, L_INT, L_DOT, L_FRAC, L_E, L_ESIGN, L_EXP, L_LIT };
enum Par : uint8_t { P_INIT, P_FIN, P_OBJ, P_KEY, P_ARR };
enum Kind : uint8_t { K_ABSENT, K_STRING, K_INT, K_DOUBLE, K_BOOL, K_NULL, K_OBJECT, K_ARRAY };
constexpr int kMaxDepth = 64;

// "name", "price", "volume" as little-endian byte packs (registers, no literal-table loads)
__device__ __forceinline__ uint32_t target_char(int t, int i) {
  const uint64_t k = t == 0 ? 0x656D616Eull : (t == 1 ? 0x6563697270ull : 0x656D756C6F76ull);
  return (uint32_t)(k >> (8 * i)) & 0xFF;
}
__device__ __forceinline__ int target_len(int t) { return t == 0 ? 4 : (t == 1 ? 5 : 6); }

__device__ __forceinline__ int hexval(uint8_t c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

struct Parser {
  // outcome
  int32_t status = 0;
  bool done = false;
  // lexer
  uint8_t lex = L_WS;
  uint8_t lit = 0, lit_pos = 0;  // literal id (0 true, 1 false, 2 null) and chars matched
  uint8_t uhex = 0;              // \u digits seen
  uint32_t ucode = 0;
  bool neg = false, ovf = false, frac_seen = false;
  uint64_t mag = 0;
  // string being lexed
  uint32_t s_start = 0;
  bool s_esc = false;
  uint8_t cand = 0, klen = 0;  // key matching against name/price/volume
  // parser
  uint8_t par = P_INIT;
  int depth = 0;
  uint64_t stack = 0;  // bit d-1 set: container at depth d is an object
  uint8_t top_kind = K_ABSENT;
  int8_t cur_key = -1;  // target id of the pending top-level key
  // the three fields (last value wins)
  uint8_t kind0 = K_ABSENT, kind1 = K_ABSENT, kind2 = K_ABSENT;  // name, price, volume
  int64_t val1 = 0, val2 = 0;
  uint32_t name_off = 0, name_len = 0;
  bool name_esc = false;

  __device__ __forceinline__ void fail(int32_t code) {
    status = code;
    done = true;
  }

  __device__ __forceinline__ bool key_pos() const { return par == P_OBJ && depth == 1; }

  __device__ __forceinline__ void str_char(uint32_t ch) {
    if (!cand) return;
#pragma unroll
    for (int t = 0; t < 3; t++)
      if ((cand >> t) & 1)
        if (klen >= target_len(t) || target_char(t, klen) != ch) cand &= ~(1u << t);
    klen++;
  }

  __device__ __forceinline__ void pop_container() {
    depth--;
    par = depth == 0 ? P_FIN : (((stack >> (depth - 1)) & 1) ? P_OBJ : P_ARR);
  }

  __device__ __forceinline__ void push_container(bool obj) {
    if (depth >= kMaxDepth) {
      fail(CEP_JSON_DEPTH);
      return;
    }
    if (obj) stack |= 1ull << depth;
    else stack &= ~(1ull << depth);
    depth++;
    par = obj ? P_OBJ : P_ARR;
  }

  // one parser token; tok is '{' '}' '[' ']' ',' ':' 'v' (value) or 0 (end of input)
  __device__ void token(uint8_t tok, uint8_t vkind, int64_t v, uint32_t so, uint32_t sl, bool sesc, int key) {
    switch (par) {
      case P_INIT:
        if (tok == 'v') { par = P_FIN; top_kind = vkind; }
        else if (tok == '{') { top_kind = K_OBJECT; push_container(true); }
        else if (tok == '[') { top_kind = K_ARRAY; push_container(false); }
        else fail(CEP_JSON_PARSE);
        return;
      case P_FIN:
        if (tok == 0) done = true;
        else fail(CEP_JSON_PARSE);
        return;
      case P_OBJ:
        if (tok == ',') return;
        if (tok == 'v' && vkind == K_STRING) { cur_key = depth == 1 ? key : -1; par = P_KEY; return; }
        if (tok == '}') { pop_container(); return; }
        fail(CEP_JSON_PARSE);
        return;
      case P_KEY:
        if (tok == ':') return;
        if (tok == 'v' || tok == '{' || tok == '[') {
          if (cur_key >= 0) {
            const uint8_t k = tok == 'v' ? vkind : (tok == '{' ? K_OBJECT : K_ARRAY);
            if (cur_key == 0) kind0 = k;
            else if (cur_key == 1) { kind1 = k; val1 = v; }
            else { kind2 = k; val2 = v; }
            if (cur_key == 0) { name_off = so; name_len = sl; name_esc = sesc; }
          }
          if (tok == 'v') par = P_OBJ;
          else push_container(tok == '{');
          return;
        }
        fail(CEP_JSON_PARSE);
        return;
      case P_ARR:
        if (tok == ',' || tok == 'v') return;
        if (tok == ']') { pop_container(); return; }
        if (tok == '{' || tok == '[') { push_container(tok == '{'); return; }
        fail(CEP_JSON_PARSE);
        return;
    }
  }

  // the number token that ended (INT or DOUBLE); false if it threw NumberFormatException
  __device__ __forceinline__ void end_number(bool is_double) {
    if (!is_double && ovf) { fail(CEP_JSON_NUMBER); return; }
    const int64_t v = is_double ? 0 : (neg ? (int64_t)(0ull - mag) : (int64_t)mag);
    token('v', is_double ? K_DOUBLE : K_INT, v, 0, 0, false, -1);
  }

  __device__ __forceinline__ void digit(uint8_t c) {
    const uint64_t lim = neg ? 0x8000000000000000ull : 0x7FFFFFFFFFFFFFFFull;
    const uint64_t d = c - '0';
    if (mag > (lim - d) / 10) ovf = true;
    else mag = mag * 10 + d;
  }

  // a byte outside any token
  __device__ void start(uint8_t c, uint32_t pos) {
    switch (c) {
      case ' ': case '\t': case '\n': case '\r': case '\f': return;
      case '{': case '}': case '[': case ']': case ',': case ':': token(c, 0, 0, 0, 0, false, -1); return;
      case '"':
        lex = L_STR; s_start = pos + 1; s_esc = false; klen = 0; cand = key_pos() ? 7 : 0;
        return;
      case 't': lex = L_LIT; lit = 0; lit_pos = 1; return;
      case 'f': lex = L_LIT; lit = 1; lit_pos = 1; return;
      case 'n': lex = L_LIT; lit = 2; lit_pos = 1; return;
      case '-': lex = L_NEG; neg = true; mag = 0; ovf = false; frac_seen = false; return;
      default:
        if (c >= '0' && c <= '9') { lex = L_INT; neg = false; mag = 0; ovf = false; frac_seen = false; digit(c); return; }
        fail(CEP_JSON_PARSE);  // ERROR_UNEXPECTED_CHAR
    }
  }

  __device__ void feed(uint8_t c, uint32_t pos) {
    switch (lex) {
      case L_WS: start(c, pos); return;
      case L_STR:
        if (c == '"') {
          lex = L_WS;
          int key = -1;
          if (cand) {
#pragma unroll
            for (int t = 0; t < 3; t++)
              if (((cand >> t) & 1) && klen == target_len(t)) key = t;
          }
          token('v', K_STRING, 0, s_start, pos - s_start, s_esc, key);
        } else if (c == '\\') {
          lex = L_ESC; s_esc = true;
        } else {
          str_char(c < 0x80 ? c : 0xFFFFu);
        }
        return;
      case L_ESC: {
        uint32_t ch;
        switch (c) {
          case '"': ch = '"'; break;
          case '\\': ch = '\\'; break;
          case '/': ch = '/'; break;
          case 'b': ch = '\b'; break;
          case 'f': ch = '\f'; break;
          case 'n': ch = '\n'; break;
          case 'r': ch = '\r'; break;
          case 't': ch = '\t'; break;
          case 'u': lex = L_UHEX; uhex = 0; ucode = 0; return;
          default: fail(CEP_JSON_LEX); return;
        }
        str_char(ch);
        lex = L_STR;
        return;
      }
      case L_UHEX: {
        const int h = hexval(c);
        if (h < 0) { fail(CEP_JSON_LEX); return; }
        ucode = ucode * 16 + (uint32_t)h;
        if (++uhex == 4) { str_char(ucode); lex = L_STR; }
        return;
      }
      case L_LIT: {
        const uint64_t s = lit == 0 ? 0x65757274ull : (lit == 1 ? 0x65736C6166ull : 0x6C6C756Eull);  // true false null
        if (((s >> (8 * lit_pos)) & 0xFF) != c) { fail(CEP_JSON_PARSE); return; }  // only "." matched at the start
        lit_pos++;
        if (((s >> (8 * lit_pos)) & 0xFF) == 0) {
          lex = L_WS;
          token('v', lit == 2 ? K_NULL : K_BOOL, 0, 0, 0, false, -1);
        }
        return;
      }
      case L_NEG:
        if (c >= '0' && c <= '9') { lex = L_INT; digit(c); return; }
        fail(CEP_JSON_PARSE);  // a lone '-'
        return;
      case L_INT:
        if (c >= '0' && c <= '9') { digit(c); return; }
        if (c == '.') { lex = L_DOT; return; }
        if (c == 'e' || c == 'E') { lex = L_E; return; }
        lex = L_WS;
        end_number(false);
        if (!done) start(c, pos);
        return;
      case L_DOT:  // "1." + non-digit: INT, then '.' is an unexpected char
        if (c >= '0' && c <= '9') { lex = L_FRAC; frac_seen = true; return; }
        end_number(false);
        if (!done) fail(CEP_JSON_PARSE);
        return;
      case L_FRAC:
        if (c >= '0' && c <= '9') return;
        if (c == 'e' || c == 'E') { lex = L_E; return; }
        lex = L_WS;
        end_number(true);
        if (!done) start(c, pos);
        return;
      case L_E:
        if (c >= '0' && c <= '9') { lex = L_EXP; return; }
        if (c == '+' || c == '-') { lex = L_ESIGN; return; }
        end_number(frac_seen);
        if (!done) fail(CEP_JSON_PARSE);  // 'e' re-lexed: unexpected char
        return;
      case L_ESIGN:
        if (c >= '0' && c <= '9') { lex = L_EXP; return; }
        end_number(frac_seen);
        if (!done) fail(CEP_JSON_PARSE);
        return;
      case L_EXP:
        if (c >= '0' && c <= '9') return;
        lex = L_WS;
        end_number(true);
        if (!done) start(c, pos);
        return;
    }
  }

  // end of the record: the EOF token, then deserialize()'s casts and unboxing
  __device__ void finish() {
    switch (lex) {
      case L_WS: case L_STR: break;  // a string cut off by the end of input is end of input
      case L_ESC: case L_UHEX: fail(CEP_JSON_LEX); return;
      case L_LIT: case L_NEG: fail(CEP_JSON_PARSE); return;
      case L_INT: case L_FRAC: case L_EXP: end_number(lex != L_INT); break;
      case L_DOT: end_number(false); if (!done) fail(CEP_JSON_PARSE); return;
      case L_E: case L_ESIGN: end_number(frac_seen); if (!done) fail(CEP_JSON_PARSE); return;
    }
    if (status) return;
    token(0, 0, 0, 0, 0, false, -1);
    if (status) return;
    if (top_kind == K_NULL) { status = CEP_JSON_NULL; return; }  // ((JSONObject) null).get
    if (top_kind != K_OBJECT) { status = CEP_JSON_CLASS_CAST; return; }
    if (kind0 != K_ABSENT && kind0 != K_NULL && kind0 != K_STRING) { status = CEP_JSON_CLASS_CAST; return; }
    for (int f = 1; f < 3; f++) {
      const uint8_t kf = f == 1 ? kind1 : kind2;
      if (kf == K_ABSENT || kf == K_NULL) { status = CEP_JSON_NULL; return; }
      if (kf != K_INT) { status = CEP_JSON_CLASS_CAST; return; }
    }
  }
};

// parse one record of len bytes whose first byte is byte `lead` (0..3) of word(0); word(j) returns
// the record's j-th aligned 32-bit word (an aligned word holding a byte of the record never
// leaves the record's pages)
template <typename Word>
__device__ __forceinline__ void parse_words(Parser& P, Word word, uint32_t lead, uint32_t len) {
  uint32_t i = 0;
  while (i < len && !P.done) {
    const uint32_t w = word((i + lead) >> 2);
    uint32_t k = (i + lead) & 3;
    for (; k < 4 && i < len && !P.done; k++, i++) P.feed((uint8_t)(w >> (8 * k)), i);
  }
  if (!P.done) P.finish();
}

// Fast paths for the two fixed layouts of StockEvent records, numbers of at most 18 digits and
// a name without '"' or '\\':
//   kLayoutSerializer {"volume":<int>,"price":<int>,"name":"<text>"}  what StockEventSerDe.serialize
//       writes (StockEventSerDe.java:75-82): json-simple's JSONObject is a HashMap, whose
//       iteration order for these three keys (default capacity 16) is bucket 0 volume, 6 price,
//       8 name
//   kLayoutReadme     {"name":"<text>","price":<int>,"volume":<int>}  the README's console records
//       (README.md:73-80)
// A straight scan every lane of a wave runs in step.  On success P holds exactly what the state
// machine would produce for that record; anything else returns false with P untouched and takes
// the general path.
constexpr int kLayoutSerializer = 0, kLayoutReadme = 1;

template <int kLayout, typename Word>
__device__ __forceinline__ bool parse_fast(Parser& P, Word word, uint32_t lead, uint32_t len) {
  if (len < 31) return false;
  uint32_t cj = 0xFFFFFFFFu, cw = 0;
  auto byte = [&](uint32_t i) -> uint32_t {
    const uint32_t p = i + lead, j = p >> 2;
    if (j != cj) { cj = j; cw = word(j); }
    return (cw >> (8 * (p & 3))) & 0xFF;
  };
  // bytes i..i+3 as one little-endian word (only called with i + 4 <= len: no read past the record)
  auto get4 = [&](uint32_t i) -> uint32_t {
    const uint32_t p = i + lead, j = p >> 2, sh = p & 3;
    const uint32_t lo = word(j);
    if (!sh) return lo;
    return (uint32_t)((((uint64_t)word(j + 1) << 32) | lo) >> (8 * sh));
  };
  auto lit = [&](uint32_t& i, uint64_t pack, int n) -> bool {  // n <= 8 bytes, little-endian pack
    bool ok = i + n <= len;
    int k = 0;
    for (; k + 4 <= n && ok; k += 4) ok = get4(i + k) == (uint32_t)(pack >> (8 * k));
    for (; k < n && ok; k++) ok = byte(i + k) == ((pack >> (8 * k)) & 0xFF);
    i += n;
    return ok;
  };
  auto num = [&](uint32_t& i, int64_t& v) -> bool {
    const bool neg = i < len && byte(i) == '-';
    i += neg;
    uint64_t m = 0;
    int nd = 0;
    while (i < len && nd <= 18) {
      const uint32_t c = byte(i);
      if (c - '0' > 9u) break;
      m = m * 10 + (c - '0');
      nd++;
      i++;
    }
    v = neg ? -(int64_t)m : (int64_t)m;
    return nd >= 1 && nd <= 18;
  };
  // the name's text from i to its closing quote: four bytes at a time (SWAR search for '"' or '\\')
  auto name = [&](uint32_t& i, uint32_t& n0, uint32_t& nl) -> bool {
    n0 = i;
    for (;;) {
      if (i + 4 <= len) {
        const uint32_t x = get4(i), q = x ^ 0x22222222u, e = x ^ 0x5C5C5C5Cu;
        const uint32_t m = ((q - 0x01010101u) & ~q & 0x80808080u) | ((e - 0x01010101u) & ~e & 0x80808080u);
        if (!m) { i += 4; continue; }
        i += (uint32_t)__builtin_ctz(m) >> 3;  // the lowest flagged byte is the first real match
      } else if (i >= len) {
        return false;
      }
      const uint32_t c = byte(i);
      if (c == '"') break;
      if (c == '\\') return false;
      i++;
    }
    nl = i - n0;
    i++;
    return true;
  };
  uint32_t i = 0, n0 = 0, nl = 0;
  int64_t pv, vv;
  if (kLayout == kLayoutSerializer) {
    if (!lit(i, 0x656D756C6F76227Bull, 8) || !lit(i, 0x3A22, 2) || !num(i, vv)) return false;  // {"volume":
    if (!lit(i, 0x226563697270222Cull, 8) || !lit(i, 0x3A, 1) || !num(i, pv)) return false;    // ,"price":
    if (!lit(i, 0x3A22656D616E222Cull, 8) || !lit(i, 0x22, 1) || !name(i, n0, nl)) return false;  // ,"name":"
  } else {
    if (!lit(i, 0x3A22656D616E227Bull, 8) || !lit(i, 0x22, 1) || !name(i, n0, nl)) return false;  // {"name":"
    if (!lit(i, 0x226563697270222Cull, 8) || !lit(i, 0x3A, 1) || !num(i, pv)) return false;    // ,"price":
    if (!lit(i, 0x656D756C6F76222Cull, 8) || !lit(i, 0x3A22, 2) || !num(i, vv)) return false;  // ,"volume":
  }
  if (i + 1 != len || byte(i) != '}') return false;
  P.kind0 = K_STRING; P.name_off = n0; P.name_len = nl; P.name_esc = false;
  P.kind1 = K_INT; P.val1 = pv; P.kind2 = K_INT; P.val2 = vv;
  P.status = 0; P.done = true;
  return true;
}

// either fixed layout (the serializer's first)
template <typename Word>
__device__ __forceinline__ bool parse_fast_any(Parser& P, Word word, uint32_t lead, uint32_t len) {
  return parse_fast<kLayoutSerializer>(P, word, lead, len) || parse_fast<kLayoutReadme>(P, word, lead, len);
}

// a record: the fast path, else the general state machine
template <typename Word>
__device__ __forceinline__ void parse_any(Parser& P, Word word, uint32_t lead, uint32_t len) {
  if (!parse_fast_any(P, word, lead, len)) parse_words(P, word, lead, len);
}

// the record at `base` in flat memory
__device__ __forceinline__ void parse_record(Parser& P, const uint8_t* base, uint32_t len) {
  const uint32_t* words = (const uint32_t*)((uintptr_t)base & ~(uintptr_t)3);
  parse_any(P, [words](uint32_t j) { return words[j]; }, (uint32_t)((uintptr_t)base & 3), len);
}

// the record's outcome for col_width-byte columns: status, and price/volume (0 on failure)
__device__ __forceinline__ int32_t outcome(const Parser& P, int col_width, int64_t* price, int64_t* volume) {
  int32_t st = P.status;
  int64_t pv = P.val1, vv = P.val2;
  if (st == 0 && col_width == 4 && (pv < INT32_MIN || pv > INT32_MAX || vv < INT32_MIN || vv > INT32_MAX))
    st = CEP_JSON_NARROW;
  if (st) pv = vv = 0;
  *price = pv;
  *volume = vv;
  return st;
}

// name span: offset and raw length of the name's text (bit 31: escapes), 0xFFFFFFFF if null/absent
__device__ __forceinline__ void name_span(const Parser& P, int32_t st, uint32_t* off, uint32_t* len) {
  const bool has = st == 0 && P.kind0 == K_STRING;
  *off = has ? P.name_off : 0;
  *len = has ? (P.name_len | (P.name_esc ? 0x80000000u : 0u)) : 0xFFFFFFFFu;
}

}  // namespace json

}  // namespace cep
