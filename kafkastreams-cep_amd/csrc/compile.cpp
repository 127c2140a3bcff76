// compile.cpp — query compiler: serialised Pattern chain -> stage table + predicate bytecode.
//
// Replaces StatesFactory.make (pattern/StatesFactory.java:41-127) and the lambda bodies of
// Matcher / Aggregator (pattern/Matcher.java, pattern/Aggregator.java), which arrive as the
// typed IR documented in include/cep.h.  Host-only code, linked into libcep.so.
#include <algorithm>
#include <functional>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "cep_internal.h"

namespace cep {

namespace {

struct Expr {
  uint8_t op = 0, t = 0, t2 = 0;
  int64_t i = 0;
  double d = 0;
  uint16_t idx = 0;
  std::unique_ptr<Expr> a, b;
  bool nullable() const { return op == 0x07 || op == 0x09; }
};
using ExprP = std::shared_ptr<Expr>;

struct In {
  const uint8_t* p;
  const uint8_t* e;
  template <class T> T get() {
    if (p + sizeof(T) > e) throw std::runtime_error("query IR truncated");
    T v;
    std::memcpy(&v, p, sizeof v);
    p += sizeof v;
    return v;
  }
  std::string str() {
    uint16_t n = get<uint16_t>();
    if (p + n > e) throw std::runtime_error("query IR truncated");
    std::string s((const char*)p, n);
    p += n;
    return s;
  }
};

std::unique_ptr<Expr> parse(In& in, int depth = 0) {
  if (depth > 256) throw std::runtime_error("query IR nested too deeply");
  auto x = std::make_unique<Expr>();
  x->op = in.get<uint8_t>();
  switch (x->op) {
    case 0x01: x->t = 1; x->i = in.get<int32_t>(); break;
    case 0x02: x->t = 2; x->i = in.get<int64_t>(); break;
    case 0x03: x->t = 3; x->d = in.get<double>(); break;
    case 0x04: x->t = 4; x->i = in.get<uint8_t>() ? 1 : 0; break;
    case 0x05: x->idx = in.get<uint16_t>(); break;
    case 0x06: x->t = 2; break;
    case 0x07: x->idx = in.get<uint16_t>(); break;
    case 0x08: x->idx = in.get<uint16_t>(); x->a = parse(in, depth + 1); break;
    case 0x09: break;
    case 0x10: case 0x11: case 0x12: case 0x13: case 0x14:
      x->t = in.get<uint8_t>(); x->a = parse(in, depth + 1); x->b = parse(in, depth + 1); break;
    case 0x15: x->t = in.get<uint8_t>(); x->a = parse(in, depth + 1); break;
    case 0x18: x->t2 = in.get<uint8_t>(); x->t = in.get<uint8_t>(); x->a = parse(in, depth + 1); break;
    case 0x20: case 0x21: case 0x22: case 0x23: case 0x24: case 0x25:
      x->t2 = in.get<uint8_t>(); x->t = 4; x->a = parse(in, depth + 1); x->b = parse(in, depth + 1); break;
    case 0x30: case 0x31: x->t = 4; x->a = parse(in, depth + 1); x->b = parse(in, depth + 1); break;
    case 0x32: x->t = 4; x->a = parse(in, depth + 1); break;
    default: throw std::runtime_error("unknown query IR opcode");
  }
  return x;
}

// ---- predicate composition at the Matcher level (Matcher.not/and/or, StatesFactory:87-107)
struct M {
  enum K { LEAF, TRUE_, NOT, AND, OR } k;
  const Expr* leaf = nullptr;
  std::shared_ptr<M> a, b;
};
using MP = std::shared_ptr<M>;
MP leaf(const Expr* e) { auto m = std::make_shared<M>(); m->k = M::LEAF; m->leaf = e; return m; }
MP mtrue() { auto m = std::make_shared<M>(); m->k = M::TRUE_; return m; }
MP mnot(MP x) { auto m = std::make_shared<M>(); m->k = M::NOT; m->a = x; return m; }
MP mand(MP x, MP y) { auto m = std::make_shared<M>(); m->k = M::AND; m->a = x; m->b = y; return m; }
MP mor(MP x, MP y) { auto m = std::make_shared<M>(); m->k = M::OR; m->a = x; m->b = y; return m; }

// ---- bytecode emission
struct Code {
  std::vector<uint32_t>& w;
  int depth = 0, maxDepth = 0;
  void push() { if (++depth > maxDepth) maxDepth = depth; }
  void pop(int n = 1) { depth -= n; }
  void op(uint8_t o, uint32_t arg = 0) { w.push_back(o | (arg << 16)); }

  void operand(const Expr* e) {  // value used by an operator: unbox a nullable one
    expr(e);
    if (e->nullable()) op(BC_UNBOX);
  }
  void expr(const Expr* e) {
    switch (e->op) {
      case 0x01: op(BC_PUSH32); w.push_back((uint32_t)(int32_t)e->i); push(); return;
      case 0x04: op(BC_PUSH32); w.push_back((uint32_t)e->i); push(); return;
      case 0x02: op(BC_PUSH64); w.push_back((uint32_t)(uint64_t)e->i); w.push_back((uint32_t)((uint64_t)e->i >> 32)); push(); return;
      case 0x03: {
        uint64_t bits;
        std::memcpy(&bits, &e->d, 8);
        op(BC_PUSH64); w.push_back((uint32_t)bits); w.push_back((uint32_t)(bits >> 32)); push();
        return;
      }
      case 0x05: op(BC_FIELD, e->idx); push(); return;
      case 0x06: op(BC_TS); push(); return;
      case 0x07: op(BC_SGET, e->idx); push(); return;
      case 0x08: expr(e->a.get()); op(BC_SGETOR, e->idx); return;  // default evaluated first (Java)
      case 0x09: op(BC_CURR); push(); return;
      case 0x10: case 0x11: case 0x12: case 0x13: case 0x14:
        operand(e->a.get()); operand(e->b.get());
        op(BC_ARITH, (uint32_t)(e->op - 0x10) | ((uint32_t)e->t << 4)); pop(); return;
      case 0x15: operand(e->a.get()); op(BC_NEG, e->t); return;
      case 0x18: operand(e->a.get()); op(BC_CAST, (uint32_t)e->t2 | ((uint32_t)e->t << 4)); return;
      case 0x20: case 0x21: case 0x22: case 0x23: case 0x24: case 0x25:
        operand(e->a.get()); operand(e->b.get());
        op(BC_CMP, (uint32_t)(e->op - 0x20) | ((uint32_t)e->t2 << 4)); pop(); return;
      case 0x30: case 0x31: {
        operand(e->a.get());
        size_t j = w.size();
        op(e->op == 0x30 ? BC_JF : BC_JT);
        pop();
        operand(e->b.get());
        w[j] |= (uint32_t)w.size() << 16;
        return;
      }
      case 0x32: operand(e->a.get()); op(BC_NOT); return;
    }
    throw std::runtime_error("bad expression");
  }
  void matcher(const M* m) {
    switch (m->k) {
      case M::TRUE_: op(BC_PUSH32); w.push_back(1); push(); return;
      case M::LEAF: operand(m->leaf); return;
      case M::NOT: matcher(m->a.get()); op(BC_NOT); return;
      case M::AND: case M::OR: {
        matcher(m->a.get());
        size_t j = w.size();
        op(m->k == M::AND ? BC_JF : BC_JT);
        pop();
        matcher(m->b.get());
        w[j] |= (uint32_t)w.size() << 16;
        return;
      }
    }
  }
};

struct PatternIR {
  uint16_t name;
  uint8_t card, strat;
  bool hasWindow;
  int64_t window;
  std::unique_ptr<Expr> pred;
  std::vector<std::pair<uint16_t, std::unique_ptr<Expr>>> aggs;
};

bool total(const Expr* e) {  // evaluation can never throw
  if (!e) return true;
  if (e->op == 0x07 || e->op == 0x09 || e->op == 0x08) return false;
  if ((e->op == 0x13 || e->op == 0x14) && e->t != 3) {
    if (!(e->b->op == 0x01 || e->b->op == 0x02) || e->b->i == 0) return false;
  }
  return total(e->a.get()) && total(e->b.get());
}

// Interval form of a predicate for the stencil fast path: a conjunction of comparisons of
// int fields with constants -> lo <= field <= hi per field.
struct Ranges {
  int field[2] = {-1, -1};
  int64_t lo[2] = {INT64_MIN, INT64_MIN}, hi[2] = {INT64_MAX, INT64_MAX};
  int n = 0;
  bool add(int f, int64_t l, int64_t h) {
    for (int i = 0; i < n; i++)
      if (field[i] == f) {
        lo[i] = std::max(lo[i], l);
        hi[i] = std::min(hi[i], h);
        return true;
      }
    if (n == 2) return false;
    field[n] = f;
    lo[n] = l;
    hi[n] = h;
    n++;
    return true;
  }
};

const Expr* int_field(const Expr* e, const std::vector<int>& ftypes) {
  if (e->op == 0x18 && e->t2 == 1 && e->t == 2) e = e->a.get();  // (long) int_field
  if (e->op == 0x05 && ftypes[e->idx] == 1) return e;
  return nullptr;
}

bool ranges_of(const Expr* e, const std::vector<int>& ftypes, Ranges& r) {
  if (e->op == 0x04) return e->i != 0;  // `true` adds nothing (false: not a range)
  if (e->op == 0x30) return ranges_of(e->a.get(), ftypes, r) && ranges_of(e->b.get(), ftypes, r);
  if (e->op < 0x20 || e->op > 0x24 || (e->t2 != 1 && e->t2 != 2)) return false;
  const Expr* f = int_field(e->a.get(), ftypes);
  const Expr* c = e->b.get();
  int op = e->op;
  if (!f) {  // const OP field  ->  field OP' const
    f = int_field(e->b.get(), ftypes);
    c = e->a.get();
    static const int flip[5] = {0x22, 0x23, 0x20, 0x21, 0x24};  // lt->gt, le->ge, gt->lt, ge->le
    op = flip[op - 0x20];
  }
  if (!f || !(c->op == 0x01 || c->op == 0x02)) return false;
  const int64_t k = c->i;
  switch (op) {
    case 0x20: return k != INT64_MIN && r.add(f->idx, INT64_MIN, k - 1);
    case 0x21: return r.add(f->idx, INT64_MIN, k);
    case 0x22: return k != INT64_MAX && r.add(f->idx, k + 1, INT64_MAX);
    case 0x23: return r.add(f->idx, k, INT64_MAX);
    default: return r.add(f->idx, k, k);
  }
}

enum { CARD_ONE = 0, CARD_OPTIONAL = 1, CARD_ZOM = 2, CARD_OOM = 3 };
enum { STRICT = 0, NEXT = 1, ANY = 2 };

}  // namespace

// StatesFactory.make/buildState over the parsed chain (pattern/StatesFactory.java:41-127)
struct Builder {
  cep_query* q;
  std::vector<PatternIR>& ps;
  std::vector<MP> edgePred;  // parallel to edges, filled by addEdge
  struct PendingEdge { int stage, edge; MP m; };
  std::vector<PendingEdge> pending;
  std::vector<std::pair<int, const std::vector<std::pair<uint16_t, std::unique_ptr<Expr>>>*>> stageAggs;
  std::vector<int64_t> window = std::vector<int64_t>(kMaxStages, -1);  // Stage.getWindowMs per stage

  int sk(uint16_t name, uint8_t type) {
    DevQuery& d = q->dev;
    for (uint32_t i = 0; i < d.n_sk; i++)
      if (d.sk_name[i] == name && d.sk_type[i] == type) return (int)i;
    if (d.n_sk >= (uint32_t)kMaxStageKeys) throw std::runtime_error("too many stage keys");
    d.sk_name[d.n_sk] = name;
    d.sk_type[d.n_sk] = type;
    return (int)d.n_sk++;
  }
  int newStage(uint16_t name, uint8_t type) {
    DevQuery& d = q->dev;
    if (d.n_stages >= (uint32_t)kMaxStages) throw std::runtime_error("too many stages (max 32)");
    int i = (int)d.n_stages++;
    DevStage& s = d.st[i];
    std::memset(&s, 0, sizeof s);
    s.sk = (uint8_t)sk(name, type);
    s.type = type;
    return i;
  }
  void addEdge(int st, uint8_t op, int target, MP m) {
    DevStage& s = q->dev.st[st];
    s.e[s.n_edges] = DevEdge{op, (uint8_t)(target < 0 ? 0xFF : target), kProgTrue};
    pending.push_back(PendingEdge{st, s.n_edges, m});
    s.n_edges++;
  }
  void setAggs(int st, const PatternIR& p) {
    DevStage& s = q->dev.st[st];
    if (p.aggs.size() > (size_t)kMaxAggs) throw std::runtime_error("too many folds in one pattern (max 8)");
    s.n_aggs = (uint8_t)p.aggs.size();
    stageAggs.push_back({st, &p.aggs});
  }

  int buildState(uint8_t type, const PatternIR& cur, int successorStage, const PatternIR* succ) {
    bool mandatory = cur.card == CARD_OOM;                                       // :70
    uint8_t currentType = mandatory ? (uint8_t)ST_NORMAL : type;                 // :72
    int st = newStage(cur.name, currentType);
    setAggs(st, cur);
    // window = this pattern's WITHIN, else the successor's, else -1 (StatesFactory.java:121-127)
    window[st] = cur.hasWindow ? cur.window : (succ && succ->hasWindow) ? succ->window : -1;
    if (!cur.pred) {  // new Stage.Edge(op, null, ...) -> IllegalArgumentException (Stage.java:159)
      q->info.compile_error = CEP_COMPILE_ILLEGAL_ARGUMENT;
      throw std::runtime_error("predicate cannot be null");
    }
    MP pred = leaf(cur.pred.get());
    uint8_t operation = cur.card == CARD_ONE ? (uint8_t)OP_BEGIN : (uint8_t)OP_TAKE;  // :80
    addEdge(st, operation, successorStage, pred);
    MP ignore;
    if (cur.strat == ANY) { ignore = mtrue(); addEdge(st, OP_IGNORE, -1, ignore); }      // :87-90
    if (cur.strat == NEXT) { ignore = mnot(pred); addEdge(st, OP_IGNORE, -1, ignore); }  // :93-96
    if (operation == OP_TAKE) {                                                          // :98-107
      if (!succ) {  // successorPattern.getPredicate() on null
        q->info.compile_error = CEP_COMPILE_NPE;
        throw std::runtime_error("a pattern cannot end with a Kleene/optional stage (NullPointerException)");
      }
      if (!succ->pred) {
        q->info.compile_error = CEP_COMPILE_ILLEGAL_ARGUMENT;
        throw std::runtime_error("predicate cannot be null");
      }
      MP s = leaf(succ->pred.get());
      MP proceed = cur.strat == STRICT ? mor(s, mnot(pred)) : mor(s, mand(mnot(pred), mnot(ignore)));
      addEdge(st, OP_PROCEED, successorStage, proceed);
    }
    if (mandatory) {                                                                     // :110-116
      int loop = st;
      int w = newStage(cur.name, type);
      addEdge(w, OP_BEGIN, loop, leaf(cur.pred.get()));
      setAggs(w, cur);
      window[w] = window[loop];
      st = w;
    }
    return st;
  }
};


// a compiled query's parse and stage build, kept for plan_groups
struct ParsedQuery {
  std::vector<PatternIR> ps;
  std::unique_ptr<Builder> b;
};

// ============================================================ JIT source generation
// Emits the per-query step policy compiled by hipRTC (jit.cpp): fields loaded once per
// event into registers, predicates and folds as straight-line Java-semantics code, and one
// function per stage implementing NFA.evaluate (nfa/NFA.java:162-250) with its edges,
// targets and aggregates as constants; PROCEED edges become direct calls.
namespace {

const char* ctype(int t) { return t == 1 ? "int32_t" : t == 2 ? "int64_t" : t == 3 ? "double" : "bool"; }

std::string lit(const Expr* e) {
  char b[64];
  switch (e->op) {
    case 0x01: std::snprintf(b, sizeof b, "((int32_t)%d)", (int)e->i); break;
    case 0x02: std::snprintf(b, sizeof b, "((int64_t)0x%llxull)", (unsigned long long)e->i); break;
    case 0x03: {
      uint64_t bits;
      std::memcpy(&bits, &e->d, 8);
      std::snprintf(b, sizeof b, "__longlong_as_double((long long)0x%llxull)", (unsigned long long)bits);
      break;
    }
    default: std::snprintf(b, sizeof b, "%s", e->i ? "true" : "false"); break;
  }
  return b;
}

// Literals of a query's predicates and folds, in generation order.  A group of queries that
// differ only in literal values (config 5's 64 stock-query variants) shares one kernel: every
// literal whose value differs across the group is read from a per-query constant table
// (K.c[i], loaded once per lane) instead of being compiled in.
struct LitCtx {
  bool param = false;                // literals may come from the table
  const std::vector<char>* inl = nullptr;  // param: literal i stays inline where inl[i] (null: none)
  std::vector<int64_t> values;       // every literal's bits (int, long, double bits, bool)
};

struct Gen {
  std::string s;
  int n = 0;
  LitCtx* L = nullptr;
  std::string fail;   // statement tail after `err = X;` (e.g. "return false;")
  int aggType = 0;    // state type of `curr` inside an aggregator
  // a matcher already evaluated without an exception on the same event and state (the
  // stage's edge-0 predicate, evaluated first by matchEdgesAndGet): its value is `knownName`
  const M* known = nullptr;
  std::string knownName;
  std::string t() { return "t" + std::to_string(n++); }
  void raise(const char* code, const std::string& cond) { s += "  if (" + cond + ") { err = " + code + "; " + fail + " }\n"; }

  // returns (value, null-flag or "")
  std::pair<std::string, std::string> expr(const Expr* e) {
    switch (e->op) {
      case 0x01: case 0x02: case 0x03: case 0x04: {
        const size_t i = L->values.size();
        int64_t bits = e->i;
        if (e->op == 0x03) std::memcpy(&bits, &e->d, 8);
        L->values.push_back(bits);
        if (!L->param || (L->inl && (*L->inl)[i])) return {lit(e), ""};
        const std::string k = "K.c[" + std::to_string(i) + "]";
        switch (e->op) {
          case 0x01: return {"((int32_t)" + k + ")", ""};
          case 0x02: return {"((int64_t)" + k + ")", ""};
          case 0x03: return {"__longlong_as_double(" + k + ")", ""};
          default: return {"(" + k + " != 0)", ""};
        }
      }
      case 0x05: return {"ev.f" + std::to_string(e->idx), ""};
      case 0x06: return {"ev.ts", ""};
      case 0x07: case 0x08: {
        const std::string si = std::to_string(e->idx);
        std::string dflt;
        if (e->op == 0x08) dflt = operand(e->a.get());  // the default argument is evaluated first
        const int st = stateType[e->idx];
        const std::string v = t();
        const std::string raw = st == 3 ? "__longlong_as_double(w.v[" + si + "])" : "(" + std::string(ctype(st)) + ")w.v[" + si + "]";
        const std::string nul = "((w.nm >> " + si + ") & 1u)";
        if (e->op == 0x08) {
          s += "  const " + std::string(ctype(st)) + " " + v + " = " + nul + " ? " + dflt + " : " + raw + ";\n";
          return {v, ""};
        }
        const std::string nf = t();
        s += "  const " + std::string(ctype(st)) + " " + v + " = " + raw + ";\n";
        s += "  const bool " + nf + " = " + nul + ";\n";
        return {v, nf};
      }
      case 0x09: return {"curr", "curr_null"};
      case 0x10: case 0x11: case 0x12: case 0x13: case 0x14: {
        const std::string a = operand(e->a.get()), b = operand(e->b.get());
        const std::string v = t();
        const int ty = e->t;
        std::string val;
        if (ty == 3) {
          static const char* fn[] = {"__dadd_rn", "__dsub_rn", "__dmul_rn", "__ddiv_rn", "fmod"};
          val = std::string(fn[e->op - 0x10]) + "(" + a + ", " + b + ")";
        } else {
          const std::string U = ty == 1 ? "uint32_t" : "uint64_t", T = ctype(ty);
          switch (e->op) {
            case 0x10: val = "(" + T + ")((" + U + ")" + a + " + (" + U + ")" + b + ")"; break;
            case 0x11: val = "(" + T + ")((" + U + ")" + a + " - (" + U + ")" + b + ")"; break;
            case 0x12: val = "(" + T + ")((" + U + ")" + a + " * (" + U + ")" + b + ")"; break;
            case 0x13:
              raise("KE_ARITH", b + " == 0");
              val = "(" + b + " == -1) ? (" + T + ")((" + U + ")0 - (" + U + ")" + a + ") : (" + T + ")(" + a + " / " + b + ")";
              break;
            default:
              raise("KE_ARITH", b + " == 0");
              val = "(" + b + " == -1) ? (" + T + ")0 : (" + T + ")(" + a + " % " + b + ")";
              break;
          }
        }
        s += "  const " + std::string(ctype(ty)) + " " + v + " = " + val + ";\n";
        return {v, ""};
      }
      case 0x15: {
        const std::string a = operand(e->a.get());
        const std::string v = t();
        std::string val = e->t == 3 ? "-" + a
                        : e->t == 1 ? "(int32_t)(0u - (uint32_t)" + a + ")"
                                    : "(int64_t)((uint64_t)0 - (uint64_t)" + a + ")";
        s += "  const " + std::string(ctype(e->t)) + " " + v + " = " + val + ";\n";
        return {v, ""};
      }
      case 0x18: {
        const std::string a = operand(e->a.get());
        const std::string v = t();
        const int f = e->t2, to = e->t;
        std::string val;
        if (f == to) val = a;
        else if (f == 3) val = to == 1 ? "(int32_t)java_d2i(" + a + ")" : "java_d2l(" + a + ")";
        else if (to == 3) val = "(double)" + a;
        else if (to == 1) val = "(int32_t)(uint32_t)(uint64_t)" + a;
        else val = "(int64_t)" + a;
        s += "  const " + std::string(ctype(to)) + " " + v + " = " + val + ";\n";
        return {v, ""};
      }
      case 0x20: case 0x21: case 0x22: case 0x23: case 0x24: case 0x25: {
        static const char* op[] = {"<", "<=", ">", ">=", "==", "!="};
        const std::string a = operand(e->a.get()), b = operand(e->b.get());
        const std::string v = t();
        s += "  const bool " + v + " = " + a + " " + op[e->op - 0x20] + " " + b + ";\n";
        return {v, ""};
      }
      case 0x30: case 0x31: {
        const std::string v = t();
        s += "  bool " + v + ";\n  {\n";
        const std::string a = operand(e->a.get());
        s += "  if (" + std::string(e->op == 0x30 ? "!" : "") + a + ") " + v + " = " + (e->op == 0x30 ? "false" : "true") + ";\n  else {\n";
        const std::string b = operand(e->b.get());
        s += "  " + v + " = " + b + ";\n  }\n  }\n";
        return {v, ""};
      }
      case 0x32: {
        const std::string a = operand(e->a.get());
        const std::string v = t();
        s += "  const bool " + v + " = !" + a + ";\n";
        return {v, ""};
      }
    }
    throw std::runtime_error("codegen: bad expression");
  }
  std::string operand(const Expr* e) {
    auto r = expr(e);
    if (!r.second.empty()) raise("KE_NPE", r.second);  // unboxing a null Integer/Long
    return r.first;
  }
  std::string matcher(const M* m) {
    if (known && m == known) return knownName;
    switch (m->k) {
      case M::TRUE_: return "true";
      case M::LEAF: return operand(m->leaf);
      case M::NOT: {
        const std::string a = matcher(m->a.get());
        const std::string v = t();
        s += "  const bool " + v + " = !" + a + ";\n";
        return v;
      }
      default: {
        const std::string v = t();
        s += "  bool " + v + ";\n  {\n";
        const std::string a = matcher(m->a.get());
        s += "  if (" + std::string(m->k == M::AND ? "!" : "") + a + ") " + v + " = " + (m->k == M::AND ? "false" : "true") + ";\n  else {\n";
        const std::string b = matcher(m->b.get());
        s += "  " + v + " = " + b + ";\n  }\n  }\n";
        return v;
      }
    }
  }
  std::vector<int> stateType;
};

void uses(const Expr* e, std::vector<bool>& fields, bool& ts) {
  if (!e) return;
  if (e->op == 0x05) fields[e->idx] = true;
  if (e->op == 0x06) ts = true;
  uses(e->a.get(), fields, ts);
  uses(e->b.get(), fields, ts);
}
void usesM(const M* m, std::vector<bool>& fields, bool& ts) {
  if (!m) return;
  if (m->k == M::LEAF) uses(m->leaf, fields, ts);
  usesM(m->a.get(), fields, ts);
  usesM(m->b.get(), fields, ts);
}

// ---- static fold nullness
// Which fold slots can be null when a queued record is stepped, per dispatch case (the stage a
// record's epsilon stage proceeds to).  The reference keys fold values by (state, run seq),
// `get` of an absent one is null (pattern/States.java:46-62), and a record's values come only
// from the steps that made it (NFA.evaluate, nfa/NFA.java:162-250): a consuming edge applies
// the stage's aggregates in order (:259-265; an arithmetic fold result is never null, `curr`
// or `state.get(x)` copies a nullness), a branch copies the current stage's non-null
// aggregates into an otherwise empty run (ValueStore.branch, pattern/ValueStore.java:92-97),
// the begin run starts empty (:74-81).  The step as generated (E<stage>) is run abstractly on a
// may-be-null bitmask over every combination of matched edges, through its PROCEED calls, to a
// fixpoint over the dispatch cases; a slot that is provably non-null in a case has its null
// bit masked off at that case's entry, so the compiler drops the unboxing checks (NPE paths)
// that read it and the exec-mask work around them.  Returns per stage the may-be-null mask of
// its dispatch case (-1: no queued record reaches it), or an empty vector when the search
// outgrew its budget (no masking).
static_assert(kMaxStates <= 32, "fold_nullness keeps a fold slot's null bit as 1u << slot");
static std::vector<int64_t> fold_nullness(const cep_query* q, const Builder& b) {
  const DevQuery& d = q->dev;
  const uint32_t all = d.n_states >= 32 ? ~0u : (1u << d.n_states) - 1u;
  std::vector<const std::vector<std::pair<uint16_t, std::unique_ptr<Expr>>>*> aggs(d.n_stages, nullptr);
  for (auto& sa : b.stageAggs) aggs[sa.first] = sa.second;
  std::vector<int64_t> mn(d.n_stages, -1);
  long budget = 2000000;
  auto fold = [&](int st, uint32_t m) {
    if (!aggs[st]) return m;
    for (auto& a : *aggs[st]) {
      const uint32_t bit = 1u << a.first;
      const Expr* e = a.second.get();
      if (e->op == 0x09) continue;  // `curr` itself: its own nullness
      if (e->op == 0x07) m = (m & ~bit) | (((m >> e->idx) & 1u) ? bit : 0u);  // state.get(x): x's
      else m &= ~bit;  // any operator unboxes its operands (NPE path) and yields a value
    }
    return m;
  };
  // outcomes of evaluate(cur) on w's mask `m`: (w's mask after, dispatch case of the record that
  // keeps the run's seq: -1 none, -2 a final match); branch records go straight into `mn`
  std::function<bool(int, uint32_t, int, std::vector<std::pair<uint32_t, int>>&)> eval =
      [&](int cur, uint32_t m, int top, std::vector<std::pair<uint32_t, int>>& out) -> bool {
    const DevStage& S = d.st[cur];
    for (uint32_t sub = 0; sub < (1u << S.n_edges); sub++) {
      if (--budget < 0) return false;
      bool T = false, B = false, I = false, P = false;
      int bt = -1, pt = -1;
      for (int e = 0; e < S.n_edges; e++) {
        if (!((sub >> e) & 1u)) continue;
        switch (S.e[e].op) {
          case OP_TAKE: T = true; break;
          case OP_BEGIN: B = true; bt = S.e[e].target; break;
          case OP_IGNORE: I = true; break;
          case OP_PROCEED: P = true; pt = S.e[e].target; break;
        }
      }
      const bool br = (P && T) || (I && T) || (I && B) || (I && P);
      int same = -1;
      const auto dispatch = [&](int st) { return d.st[st].type == ST_FINAL ? -2 : st; };
      if (!br) {
        if (T) same = cur;
        else if (B) same = dispatch(bt);
        else if (I) same = top;
      } else if (B) {
        same = dispatch(bt);
      }
      std::vector<std::pair<uint32_t, int>> inner;
      if (P) {
        if (d.st[pt].type == ST_FINAL) return false;  // (never built: PROCEED targets a pattern stage)
        if (!eval(pt, m, top, inner)) return false;
      } else {
        inner.push_back({m, -1});
      }
      for (auto& x : inner) {
        uint32_t mm = x.first;
        const int s2 = x.second != -1 ? x.second : same;
        if (br) {  // the branch record: the current stage's non-null aggregates, nothing else
          uint32_t bm = all;
          if (aggs[cur])
            for (auto& a : *aggs[cur]) bm &= ~(1u << a.first) | (mm & (1u << a.first));
          mn[cur] = (mn[cur] < 0 ? 0 : mn[cur]) | bm;
        }
        if (T || B) mm = fold(cur, mm);
        if (std::find(out.begin(), out.end(), std::make_pair(mm, s2)) == out.end()) out.push_back({mm, s2});
      }
    }
    return true;
  };
  auto run = [&](int st, uint32_t m, int top) {
    std::vector<std::pair<uint32_t, int>> out;
    if (!eval(st, m, top, out)) return false;
    for (auto& x : out)
      if (x.second >= 0) mn[x.second] = (mn[x.second] < 0 ? 0 : mn[x.second]) | x.first;
    return true;
  };
  // the begin run (a non-epsilon record: no dispatch case; its IGNORE re-adds itself, empty)
  if (!run((int)d.begin_stage, all, -3)) return {};
  for (bool changed = true; changed;) {
    changed = false;
    for (uint32_t s = 0; s < d.n_stages; s++) {
      if (mn[s] < 0) continue;
      const std::vector<int64_t> before = mn;
      if (!run((int)s, (uint32_t)mn[s], (int)s)) return {};
      if (mn != before) changed = true;
    }
  }
  return mn;
}

}  // namespace

static std::string generate_jit(const cep_query* q, const Builder& b, LitCtx& lits) {
  const DevQuery& d = q->dev;
  const int F = q->F;
  std::vector<int> stTypes(d.state_type, d.state_type + d.n_states);
  std::vector<bool> fields(d.n_fields, false);
  bool ts = q->windowed;  // semantic WITHIN compares event times
  for (auto& pe : b.pending) usesM(pe.m.get(), fields, ts);
  for (auto& sa : b.stageAggs)
    for (auto& a : *sa.second) uses(a.second.get(), fields, ts);
  std::string o;
  o += "// generated by libcep (compile.cpp generate_jit) — do not edit\n";
  // Dewey RLE pairs held in registers: the kernel as generated is the narrow build (3 pairs:
  // every run of the bench configs fits, SURVEY §8d sample); a job whose version would need
  // more reports KE_RETRY and is re-run by the wide build of the same source (6 pairs:
  // jit_wide_source), which also runs streaming sessions.
  int narrow = 3;
#ifdef CEP_MEASURE
  // tuning knobs of nfa_lane.h / cep_layout.h, measurement builds only (libcep_measure.so,
  // Makefile `measure`): $CEP_WALK_FLUSH, ..., $CEP_DEWEY_PAIRS.  (The drain threshold is
  // recorded with the group: session.cpp sizes streams' walk queues by the compiled value.)
  if (tuning_walk_flush() != 24) o += "#define CEP_WALK_FLUSH " + std::to_string(tuning_walk_flush()) + "\n";
  for (const char* knob : {"CEP_QUIET_CHUNK", "CEP_JOB_DRAIN", "CEP_PROF", "CEP_RING_LDS_SLOTS", "CEP_PARTIAL_DRAIN"})
    if (const char* v = std::getenv(knob))
      if (std::atoi(v) > 0) o += std::string("#define ") + knob + " " + std::to_string(std::atoi(v)) + "\n";
  if (const char* v = std::getenv("CEP_DEWEY_PAIRS"))
    if (std::atoi(v) > 0) narrow = std::atoi(v);
#endif
  o += "#ifndef CEP_DEWEY_PAIRS\n#define CEP_DEWEY_PAIRS " + std::to_string(narrow) + "\n";
  // the narrow build re-runs deferred-walk conflicts in the wide one instead of carrying the
  // put log (nfa_lane.h kPutLog)
  o += "#ifndef CEP_PUT_LOG\n#define CEP_PUT_LOG 0\n#endif\n";
  // ... and always defers its walks: the in-place path left out (nfa_lane.h CEP_WALK_IN_PLACE)
  o += "#ifndef CEP_WALK_IN_PLACE\n#define CEP_WALK_IN_PLACE 0\n#endif\n";
  // a single query's narrow build never runs persistent lanes (session.cpp: only kernel groups
  // and the re-runs, which take the wide build, do): its kernel holds run() alone, half the code
  if (!lits.param) o += "#ifndef CEP_PERSIST_LANES\n#define CEP_PERSIST_LANES 0\n#endif\n";
  // (3 waves per SIMD)
  o += "#define CEP_WAVES_EU 3\n#endif\n";
  // the wide build (6-pair Dewey versions: streams, re-runs) at 2 waves per SIMD: at 3 it
  // spills ~200 B of scratch and ran 20-25 % slower (profiles/r03)
  o += "#ifndef CEP_WAVES_EU\n#define CEP_WAVES_EU 2\n#endif\n";
  o += "#include <hip/hip_runtime.h>\n#include <stdint.h>\n#include \"cep_layout.h\"\n#include \"kernel_args.h\"\n";
  if (lits.param) o += "#define CEP_WALK_COMPAT2 1  // kernel group: the wider straight-line walk step\n";
  o += "#include \"dewey.h\"\n#include \"java.h\"\n#include \"nfa_lane.h\"\n\nnamespace cep {\nnamespace {\n\n";
  o += "constexpr int F = " + std::to_string(F) + ";\n";
  o += "struct Ev {\n";
  for (uint32_t f = 0; f < d.n_fields; f++)
    if (fields[f]) o += "  " + std::string(ctype(d.field_type[f])) + " f" + std::to_string(f) + ";\n";
  o += "  int64_t ts;\n};\n";
  o += "struct Fo {\n  int64_t v[F];\n  uint32_t nm;\n};\n";
  o += "struct Top {\n  uint32_t stage, event, ev_first, node, hsk;  // node hint of (hsk, event)\n};\n";
  o += "struct Out {\n  int produced;\n  int same;  // slot of the output record that keeps the run's sequence id\n};\n\n";
  // the begin predicate's own columns (the quiet scan loads only these)
  std::vector<bool> bfields(d.n_fields, false);
  bool bts = false;
  for (auto& pe : b.pending)
    if (pe.stage == (int)d.begin_stage && pe.edge == 0) usesM(pe.m.get(), bfields, bts);
  auto loader = [&](const char* name, const std::vector<bool>& use, bool uts) {
    o += std::string("__device__ __forceinline__ void ") + name + "(Ev& ev, const NfaArgs& A, uint64_t pos) {\n";
    for (uint32_t f = 0; f < d.n_fields; f++)
      if (fields[f])
        o += "  ev.f" + std::to_string(f) + " = " +
             (use[f] ? "((const " + std::string(ctype(d.field_type[f])) + "*)A.cols.p[" + std::to_string(f) + "])[pos]"
                     : std::string("0")) + ";\n";
    o += uts ? "  ev.ts = A.ts ? A.ts[pos] : (int64_t)pos;\n" : "  ev.ts = 0;\n";
    o += "}\n";
  };
  loader("ld_ev", fields, ts);
  loader("ld_bev", bfields, bts);
  // the begin predicate's columns for 4 consecutive positions p..p+3 (p % 4 == 0, all in the
  // batch, columns 16-B aligned: bev4_aligned): 16-B loads (cep_nfa_bits)
  o += "__device__ __forceinline__ bool bev4_aligned(const NfaArgs& A) {\n  return true";
  for (uint32_t f = 0; f < d.n_fields; f++)
    if (fields[f] && bfields[f] && d.field_type[f] != 0)
      o += " && ((uint64_t)A.cols.p[" + std::to_string(f) + "] & 15u) == 0";
  o += ";\n}\n";
  o += "__device__ __forceinline__ void ld_bev4(Ev* e, const NfaArgs& A, uint64_t p) {\n";
  for (uint32_t f = 0; f < d.n_fields; f++) {
    if (!fields[f]) continue;
    const std::string fs = "f" + std::to_string(f), col = "A.cols.p[" + std::to_string(f) + "]";
    if (!bfields[f]) {
      o += "  for (int j = 0; j < 4; j++) e[j]." + fs + " = 0;\n";
    } else if (d.field_type[f] == 1) {
      o += "  {\n    const int4 v = *reinterpret_cast<const int4*>((const int32_t*)" + col + " + p);\n";
      o += "    e[0]." + fs + " = v.x;\n    e[1]." + fs + " = v.y;\n    e[2]." + fs + " = v.z;\n    e[3]." + fs + " = v.w;\n  }\n";
    } else if (d.field_type[f] == 2 || d.field_type[f] == 3) {
      const std::string ct = ctype(d.field_type[f]), vt = d.field_type[f] == 2 ? "longlong2" : "double2";
      o += "  {\n    const " + vt + "* q = reinterpret_cast<const " + vt + "*>((const " + ct + "*)" + col + " + p);\n";
      o += "    const " + vt + " a = q[0], b = q[1];\n";
      o += "    e[0]." + fs + " = a.x;\n    e[1]." + fs + " = a.y;\n    e[2]." + fs + " = b.x;\n    e[3]." + fs + " = b.y;\n  }\n";
    } else {
      o += "  for (int j = 0; j < 4; j++) e[j]." + fs + " = ((const " + std::string(ctype(d.field_type[f])) + "*)" + col + ")[p + j];\n";
    }
  }
  o += bts ? "  for (int j = 0; j < 4; j++) e[j].ts = A.ts ? A.ts[p + j] : (int64_t)(p + j);\n"
           : "  for (int j = 0; j < 4; j++) e[j].ts = 0;\n";
  o += "}\n";
  o += "\n";
  // predicates, one per (stage, edge); folds one per (stage, aggregate)
  std::string pa;
  std::vector<std::vector<std::string>> predName(d.n_stages, std::vector<std::string>(3));
  // The later edges of a stage (IGNORE = !pred, PROCEED = succ || (!pred && !ignore)) embed the
  // edge-0 predicate itself; matchEdgesAndGet (NFA.java:267-273) evaluates edge 0 first, so
  // by then it returned without an exception and its value on the same event and state is m0:
  // those predicates take it as an argument instead of evaluating it again.
  std::vector<std::vector<bool>> predM0(d.n_stages, std::vector<bool>(3, false));
  std::vector<const M*> edge0(d.n_stages, nullptr);
  for (auto& pe : b.pending)
    if (pe.edge == 0 && pe.m->k != M::TRUE_) edge0[pe.stage] = pe.m.get();
  for (auto& pe : b.pending) {
    if (pe.m->k == M::TRUE_) { predName[pe.stage][pe.edge] = ""; continue; }
    Gen g;
    g.L = &lits;
    g.stateType = stTypes;
    g.fail = "return false;";
    const bool m0 = pe.edge > 0 && edge0[pe.stage] != nullptr;
    if (m0) {
      g.known = edge0[pe.stage];
      g.knownName = "m0";
    }
    const std::string v = g.matcher(pe.m.get());
    const std::string name = "P" + std::to_string(pe.stage) + "_" + std::to_string(pe.edge);
    predName[pe.stage][pe.edge] = name;
    predM0[pe.stage][pe.edge] = m0;
    pa += "__device__ __forceinline__ bool " + name + "(const Ev& ev, const Fo& w, int& err, const Kc& K" +
          (m0 ? ", bool m0" : "") + ") {\n" + g.s + "  (void)K;\n  return " + v + ";\n}\n";
  }
  std::vector<std::vector<std::string>> aggName(d.n_stages);
  for (auto& sa : b.stageAggs) {
    int k = 0;
    for (auto& a : *sa.second) {
      const int st = stTypes[a.first];
      Gen g;
      g.L = &lits;
      g.stateType = stTypes;
      g.fail = "return;";
      g.aggType = st;
      const std::string si = std::to_string(a.first);
      std::string head = "  const bool curr_null = (w.nm >> " + si + ") & 1u;\n";
      head += st == 3 ? "  const double curr = __longlong_as_double(w.v[" + si + "]);\n"
                      : "  const " + std::string(ctype(st)) + " curr = (" + ctype(st) + ")w.v[" + si + "];\n";
      auto r = g.expr(a.second.get());
      const std::string name = "A" + std::to_string(sa.first) + "_" + std::to_string(k++);
      aggName[sa.first].push_back(name);
      std::string store = st == 3 ? "__double_as_longlong(" + r.first + ")" : "(int64_t)" + r.first;
      std::string nul = r.second.empty() ? "0u" : "(" + r.second + " ? 1u : 0u)";
      pa += "__device__ __forceinline__ void " + name + "(const Ev& ev, Fo& w, int& err, const Kc& K) {\n" + head +
            g.s + "  (void)K;\n  w.v[" + si + "] = " + store + ";\n  w.nm = (w.nm & ~(1u << " + si + ")) | (" + nul +
            " << " + si + ");\n}\n";
    }
  }
  // the per-query constant table (parametric literals), then the predicates and folds
  const size_t nkc = lits.param ? lits.values.size() : 0;
  o += "constexpr int NKC = " + std::to_string(nkc) + ";  // literals per query in NfaArgs.kc\n";
  o += "struct Kc {\n  int64_t c[NKC > 0 ? NKC : 1];\n};\n";
  o += "__device__ __forceinline__ void ld_kc(Kc& K, const NfaArgs& A, uint32_t qi) {\n";
  o += "  for (int i = 0; i < NKC; i++) K.c[i] = A.kc[(uint64_t)qi * NKC + i];\n  (void)K; (void)A; (void)qi;\n}\n";
  o += pa;
  o += "\nstruct JitQ {\n  const NfaArgs& A;\n  Kc K;  // this lane's query constants (group kernels)\n";
  const DevStage& bs = d.st[d.begin_stage];
  const bool quiet = bs.n_edges == 1 && bs.e[0].op == OP_BEGIN;
  o += "  static constexpr bool quiet = " + std::string(quiet ? "true" : "false") + ";\n";
  o += "  static constexpr bool kBeginReg = quiet;\n";
  bool fold32 = true;  // every state a Java int: one word per fold slot in the run record
  for (uint32_t i = 0; i < d.n_states; i++) fold32 = fold32 && d.state_type[i] == 1;
  o += "  static constexpr bool kFold32 = " + std::string(fold32 ? "true" : "false") + ";\n";
  // run-queue slots in LDS per half ($CEP_RING_LDS caps it: measurement builds)
  std::string rl = "ring_lds_slots<RecLayout<F, kFold32>>()";
#ifdef CEP_MEASURE
  if (const char* v = std::getenv("CEP_RING_LDS")) rl = "(" + rl + " < " + std::to_string(std::atoi(v)) + " ? " + rl + " : " + std::to_string(std::atoi(v)) + ")";
#endif
  o += "  static constexpr uint32_t kRingLds = " + rl + ";\n";
  o += "  static constexpr uint32_t begin_stage = " + std::to_string(d.begin_stage) + ";\n";
  o += "  typedef Ev EvT;\n";
  o += "  __device__ explicit JitQ(const NfaArgs& a) : A(a) {}\n";
  o += "  __device__ __forceinline__ void set_query(uint32_t qi) { ld_kc(K, A, qi); }\n";
  o += "  __device__ __forceinline__ void load_ev(Ev& e, uint64_t pos) const { ld_ev(e, A, pos); }\n";
  o += "  __device__ __forceinline__ uint32_t stage_sk(uint32_t sw) const {\n    if (sw & kRecEps) return (sw >> 8) & 0xFF;\n    switch (sw & 0xFF) {\n";
  for (uint32_t s = 0; s < d.n_stages; s++) o += "      case " + std::to_string(s) + ": return " + std::to_string(d.st[s].sk) + ";\n";
  o += "    }\n    return 0;\n  }\n";
  if (q->windowed) {
    // semantic WITHIN: the window of a stage key (an epsilon stage keeps its source stage's
    // window), whether the key is BEGIN-typed (ComputationStage.isBeginState), event times
    o += "  static constexpr uint32_t FS = " + std::to_string(d.n_states) + ";  // fold slots FS, FS+1: the run's start time (lo, hi)\n";
    o += "  __device__ __forceinline__ int64_t sk_window(uint32_t sk) const {\n    switch (sk) {\n";
    for (uint32_t k = 0; k < d.n_sk; k++) {
      int64_t w = -1;
      for (uint32_t s = 0; s < d.n_stages; s++)
        if (d.st[s].sk == k) w = b.window[s];
      o += "      case " + std::to_string(k) + ": return (int64_t)" + std::to_string(w) + "ll;\n";
    }
    o += "    }\n    return -1;\n  }\n";
    uint32_t bmask = 0;
    for (uint32_t k = 0; k < d.n_sk; k++)
      if (d.sk_type[k] == ST_BEGIN) bmask |= 1u << k;
    o += "  __device__ __forceinline__ bool sk_begin(uint32_t sk) const { return (" + std::to_string(bmask) + "u >> sk) & 1u; }\n";
  }
  o += "  __device__ __forceinline__ uint16_t sk_name(uint32_t sk) const {\n    switch (sk) {\n";
  for (uint32_t k = 0; k < d.n_sk; k++) o += "      case " + std::to_string(k) + ": return " + std::to_string(d.sk_name[k]) + ";\n";
  o += "    }\n    return 0;\n  }\n";
  o += "  template <class LT>\n  __device__ __forceinline__ bool begin_pred(LT& L) {\n";
  const bool bpred = quiet && !predName[d.begin_stage][0].empty();
  if (bpred) {
    o += "    Fo w;\n    w.nm = (1u << F) - 1;\n    int err = 0;\n";
    o += "    const bool r = " + predName[d.begin_stage][0] + "(L.ev, w, err, K);\n    if (err) L.err = err;\n    return r;\n";
  } else {
    o += "    return true;\n";
  }
  o += "  }\n";
  // quiet scan: the chunk's loads issued together, then the predicate in event order (a
  // later event's result or exception is never used past the first hit)
  o += "  template <class LT>\n  __device__ __forceinline__ uint32_t begin_scan(LT& L, uint32_t j0, uint32_t lim) {\n";
  if (bpred) {
    o += "    Ev e[kQuietChunk];\n";
    o += "#pragma unroll\n    for (uint32_t i = 0; i < kQuietChunk; i++) ld_bev(e[i], A, L.base + (j0 + i < lim ? j0 + i : j0));\n";
    o += "#pragma unroll\n    for (uint32_t i = 0; i < kQuietChunk; i++) {\n      if (j0 + i >= lim) break;\n";
    o += "      Fo w;\n      w.nm = (1u << F) - 1;\n      int err = 0;\n";
    o += "      const bool r = " + predName[d.begin_stage][0] + "(e[i], w, err, K);\n";
    o += "      if (err) { L.err = err; return j0 + i; }\n      if (r) return j0 + i;\n    }\n    return lim;\n";
  } else {
    o += "    return j0;\n";
  }
  o += "  }\n";
  // stage functions in reverse creation order so that PROCEED targets are declared first:
  // targets always have a smaller stage index ($final = 0, built last -> first)
  for (uint32_t s = 0; s < d.n_stages; s++) {
    const DevStage& S = d.st[s];
    if (S.type == ST_FINAL) continue;
    const std::string SK = std::to_string(S.sk), SI = std::to_string(s);
    std::string f;
    f += "  template <class LT>\n  __device__ __forceinline__ void E" + SI +
         "(LT& L, const Top& top, const Dewey& ver, bool branching, uint32_t prev_sk, const Ev& ev, Fo& w, Out& o) {\n";
    f += "    int err = 0;\n";
    for (int e = 0; e < S.n_edges; e++) {  // matchEdgesAndGet: every predicate first, in order
      const std::string& pn = predName[s][e];
      f += "    const bool m" + std::to_string(e) + " = " +
           (pn.empty() ? std::string("true") : pn + "(ev, w, err, K" + (predM0[s][e] ? ", m0" : "") + ")") + ";\n";
      if (!pn.empty()) f += "    if (err) { L.err = err; return; }\n";
    }
    std::string hasT = "false", hasP = "false", hasI = "false", hasB = "false";
    for (int e = 0; e < S.n_edges; e++) {
      const std::string m = "m" + std::to_string(e);
      if (S.e[e].op == OP_TAKE) hasT = m;
      if (S.e[e].op == OP_PROCEED) hasP = m;
      if (S.e[e].op == OP_IGNORE) hasI = m;
      if (S.e[e].op == OP_BEGIN) hasB = m;
    }
    f += "    const bool br = (" + hasP + " && " + hasT + ") || (" + hasI + " && " + hasT + ") || (" + hasI + " && " + hasB +
         ") || (" + hasI + " && " + hasP + ");\n";
    f += "    bool consumed = false, ignored = false;\n    (void)consumed; (void)ignored;\n";
    // Not branching, at most one edge matched (isBranching holds for every pair of edges a stage
    // can have: {T,P} {I,T} {I,B} {I,P}): the consuming edge (TAKE: eps(cur -> cur); BEGIN:
    // eps(cur -> target)) and IGNORE (the record again) share one push_rec - the wave runs one
    // copy of it whichever edge each lane took.
    std::string cons = "false", consWord, procTarget;
    int procTI = -1;
    for (int e = 0; e < S.n_edges; e++) {
      const DevEdge& E = S.e[e];
      const std::string m = "m" + std::to_string(e);
      if (E.op == OP_TAKE) {
        cons = m;
        consWord = "kRecEps | (" + SK + "u << 8) | " + SI + "u";
      } else if (E.op == OP_BEGIN) {
        cons = m;
        consWord = "kRecEps | (" + SK + "u << 8) | " + std::to_string(E.target) + "u" +
                   (d.st[E.target].type == ST_FINAL ? " | kRecFinal" : "");
      } else if (E.op == OP_PROCEED) {
        procTI = (int)E.target;
      }
    }
    auto proceed = [&](const std::string& indent) {
      const DevStage& T = d.st[procTI];
      const std::string TI = std::to_string(procTI);
      std::string g;
      if (T.sk != S.sk) {  // one inlined copy of the target's code: addStage unless the run is branching
        g += indent + "Dewey v2 = ver;\n" + indent + "if (!branching && !dw_add_stage(v2)) { L.err = kDwFull; return; }\n";
        g += indent + "E" + TI + "(L, top, v2, branching, " + SK + ", ev, w, o);\n";
      } else {
        g += indent + "E" + TI + "(L, top, ver, branching, " + SK + ", ev, w, o);\n";
      }
      g += indent + "if (L.err) return;\n";
      return g;
    };
    f += "    if (!br) {\n";
    f += "      if (" + cons + " || " + hasI + ") {\n";
    f += "        uint32_t nd = top.node, sw = (top.stage & ~(kRecBranch | kRecFinal)) | (branching ? kRecBranch : 0u);\n";
    f += "        uint32_t e0 = top.event, ef = top.ev_first;\n";
    if (cons != "false") {
      f += "        if (" + cons + ") {\n";
      f += "          nd = L.put_link(" + SK + ", prev_sk, top.event, top.ev_first, ver, top.hsk, top.node);\n";
      f += "          if (L.err) return;\n";
      f += "          sw = " + consWord + ";\n          e0 = L.j;\n          ef = CEP_NONE;\n          consumed = true;\n        }\n";
    }
    f += "        const int r = L.push_rec(sw, e0, ef, ver, nd, !consumed);  // (!consumed: the record re-added as it is)\n";
    f += "        if (r < 0) return;\n        o.same = r;\n        o.produced++;\n      }\n";
    f += "    } else {\n";
    // branching: every matched edge in edge order, then the branch record
    for (int e = 0; e < S.n_edges; e++) {
      const DevEdge& E = S.e[e];
      const std::string m = "m" + std::to_string(e);
      if (E.op == OP_TAKE) {
        f += "      if (" + m + ") {\n";
        f += "        Dewey v2 = ver;\n        if (!dw_add_run(v2)) { L.err = kDwFull; return; }\n";
        f += "        L.put_link(" + SK + ", prev_sk, top.event, top.ev_first, v2, top.hsk, top.node);\n";
        f += "        if (L.err) return;\n        consumed = true;\n      }\n";
      } else if (E.op == OP_BEGIN) {
        f += "      if (" + m + ") {\n        const uint32_t nd = L.put_link(" + SK +
             ", prev_sk, top.event, top.ev_first, ver, top.hsk, top.node);\n        if (L.err) return;\n";
        f += "        const int r = L.push_rec(" + consWord + ", L.j, CEP_NONE, ver, nd);\n";
        f += "        if (r < 0) return;\n        o.same = r;\n        o.produced++;\n        consumed = true;\n      }\n";
      } else if (E.op == OP_IGNORE) {
        f += "      if (" + m + ") ignored = true;\n";
      }
    }
    f += "    }\n";
    // PROCEED (alone, or after the branching edges above): one inlined copy of the target
    if (procTI >= 0) f += "    if (" + hasP + ") {\n" + proceed("      ") + "    }\n";
    f += "    if (br) {\n";
    f += "      // the branch record (NFA.java:231-246)\n      if (prev_sk == kNoSk) { L.err = KE_NPE; return; }\n";
    f += "      Dewey v2 = ver;\n      if (!dw_add_run(v2)) { L.err = kDwFull; return; }\n";
    f += "      const int r = L.push_rec(kRecEps | kRecBranch | (prev_sk << 8) | " + SI +
         "u, ignored ? top.event : L.j, ignored ? top.ev_first : CEP_NONE, v2, ignored && prev_sk == top.hsk ? top.node : CEP_NONE);\n      if (r < 0) return;\n";
    f += "      uint32_t nm = (1u << F) - 1;\n      int64_t fv[F];\n      for (int s = 0; s < F; s++) fv[s] = 0;\n";
    for (int a = 0; a < S.n_aggs; a++) {
      const std::string si = std::to_string(S.agg_state[a]);
      f += "      if (!((w.nm >> " + si + ") & 1u)) { fv[" + si + "] = w.v[" + si + "]; nm &= ~(1u << " + si + "); }\n";
    }
    if (q->windowed) f += "      fv[FS] = w.v[FS];  // the branch keeps the run's start\n      fv[FS + 1] = w.v[FS + 1];\n";
    f += "      L.set_folds(r, fv, nm);\n      o.produced++;\n";
    f += "      L.walk_branch(prev_sk, top.event, top.ev_first, ver, prev_sk == top.hsk ? top.node : CEP_NONE);\n"
         "      if (L.err) return;\n    }\n";
    if (S.n_aggs) {
      f += "    if (consumed) {\n";
      for (auto& an : aggName[s]) f += "      " + an + "(ev, w, err, K);\n      if (err) { L.err = err; return; }\n";
      f += "    }\n";
    }
    f += "  }\n";
    o += f;
  }
  // step: dispatch on the record's stage (epsilon -> its PROCEED target, real -> begin stage)
  o += "  template <class LT>\n  __device__ __forceinline__ int step(LT& L, const Rec<F>& c) {\n";
  o += "    const Ev& ev = L.ev;\n    Fo w;\n";
  o += "    for (int s = 0; s < F; s++) w.v[s] = c.fold[s];\n    w.nm = c.nullmask;\n";
  if (q->windowed) {
    // semantic WITHIN (NFA.java:143-144 with the epsilon stage's window kept): a run whose start
    // is more than the window before this event is dropped (produced 0 -> removePattern); a
    // BEGIN-typed record restarts at this event (getFirstPatternTimestamp, NFA.java:347-349)
    o += "    {\n      const uint32_t csk = stage_sk(c.stage);\n";
    o += "      const bool cbeg = sk_begin(csk);\n";
    o += "      const int64_t start = cbeg ? ev.ts : (int64_t)(((uint64_t)(uint32_t)c.fold[FS + 1] << 32) | (uint32_t)c.fold[FS]);\n";
    o += "      if (!cbeg) {\n        const int64_t win = sk_window(csk);\n";
    o += "        if (win != -1 && ev.ts - start > win) return 0;\n      }\n";
    o += "      w.v[FS] = (int64_t)(uint32_t)(uint64_t)start;\n      w.v[FS + 1] = (int64_t)(uint32_t)((uint64_t)start >> 32);\n    }\n";
  }
  o += "    const Top top{c.stage, c.event, c.ev_first, c.node, (c.stage & kRecEps) ? ((c.stage >> 8) & 0xFFu) : kNoSk};\n    Out o{0, -1};\n";
  o += "    const bool brf = (c.stage & kRecBranch) != 0;\n";
  o += "    if (c.stage & kRecEps) {\n      const uint32_t esk = (c.stage >> 8) & 0xFF;\n      switch (c.stage & 0xFF) {\n";
  const std::vector<int64_t> nullable = fold_nullness(q, b);
  const uint32_t allStates = d.n_states >= 32 ? ~0u : (1u << d.n_states) - 1u;
  for (uint32_t s = 0; s < d.n_stages; s++) {
    if (d.st[s].type == ST_FINAL) continue;
    const std::string SI = std::to_string(s), SK = std::to_string(d.st[s].sk);
    // (one inlined copy of the stage's code per case: the version is addStage'd first when the
    // record's epsilon stage differs from its target and the run is not branching)
    o += "        case " + SI + ": {\n          Dewey v2 = c.ver;\n";
    if (!nullable.empty() && nullable[s] >= 0 && ((uint32_t)nullable[s] & allStates) != allStates)
      o += "          w.nm &= " + std::to_string((uint32_t)nullable[s] | ~allStates) +
           "u;  // static fold nullness: the other slots are never null here\n";
    o += "          if (esk != " + SK + "u && !brf && !dw_add_stage(v2)) { L.err = kDwFull; return -1; }\n";
    o += "          E" + SI + "(L, top, v2, brf, esk, ev, w, o);\n          break;\n        }\n";
  }
  o += "        default: L.err = KE_CAPACITY; return -1;\n      }\n    } else {\n";
  o += "      E" + std::to_string(d.begin_stage) + "(L, top, c.ver, brf, kNoSk, ev, w, o);\n    }\n";
  o += "    if (L.err) return -1;\n";
  o += "    if (o.same >= 0) L.set_folds(o.same, w.v, w.nm);\n";
  o += "    if (!(c.stage & kRecEps)) {  // begin state re-added with a new run (NFA.java:148-157)\n";
  o += "      Dewey v = c.ver;\n      if (o.produced > 0 && !dw_add_run(v)) { L.err = kDwFull; return -1; }\n";
  o += "      if (!L.readd_begin(c.stage & 0xFF, v)) return -1;\n";
  o += "      o.produced++;\n    }\n    return o.produced;\n  }\n};\n\n";
  // Occupancy: the narrow build at 3 waves per SIMD (<= 168 VGPRs; measured best: 2 waves
  // lose ~20 %, 4+ spill to scratch), the wide one at 2 (CEP_WAVES_EU above).
  // $CEP_JIT_WAVES overrides both in measurement builds (0: compiler's choice).
  std::string occ = " __attribute__((amdgpu_waves_per_eu(CEP_WAVES_EU)))";
#ifdef CEP_MEASURE
  if (const char* wv = std::getenv("CEP_JIT_WAVES")) {
    const int waves = std::atoi(wv);
    occ = waves > 0 ? " __attribute__((amdgpu_waves_per_eu(" + std::to_string(waves) + ")))" : "";
  }
#endif
  o += "}  // namespace\n\nextern \"C\" __global__ void __launch_bounds__(256)" + occ + " cep_nfa_jit(NfaArgs A) {\n";
  o += "  JitQ q(A);\n";
  o += "  __shared__ v4u ring_lds[JitQ::kRingLds > 0 ? 4 * 2 * JitQ::kRingLds * RecLayout<F, JitQ::kFold32>::kLdsQuads * 64 : 1];\n";
  o += "  run_key<F>(A, q, JitQ::kRingLds > 0 ? ring_lds : nullptr);\n}\n\n";
  if (bpred) {
    // Work estimate per key for the lane order (session.cpp): the run-steps the key would take
    // if every run lived to the end, sum over begin hits b of (n - b), plus the quiet scan.
    // One wave per key: the key's events are contiguous, so its loads coalesce.
    // The begin predicate with null folds is true or throws at CSR position p, for any query
    // of the launch (a group kernel: the union over its queries' constants; each lane still
    // evaluates its own predicate there)
    o += "__device__ __forceinline__ bool begin_hit_ev(const NfaArgs& A, const Ev& e) {\n";
    o += "  const uint32_t nq = (NKC > 0 && A.n_q > 1) ? A.n_q : 1;\n";
    o += "  for (uint32_t qi = 0; qi < nq; qi++) {\n    Kc K;\n    ld_kc(K, A, qi);\n    Fo f;\n";
    o += "    f.nm = (1u << F) - 1;\n    int err = 0;\n";
    o += "    if (" + predName[d.begin_stage][0] + "(e, f, err, K) || err) return true;\n  }\n  return false;\n}\n";
    o += "__device__ __forceinline__ bool begin_hit_at(const NfaArgs& A, uint64_t p) {\n";
    o += "  Ev e;\n  ld_bev(e, A, p);\n  return begin_hit_ev(A, e);\n}\n";
    // Work estimate per key for the lane order (session.cpp): the run-steps the key would take
    // if every run lived to the end, sum over begin hits b of (n - b), plus the quiet scan.
    // Read from the begin-hit bitmap (launched first): a lane per 64-event word, 1 bit per
    // event instead of the predicate's columns.  (A wave per key: 0.32 ms per streamed batch of
    // 1M keys, ~100 events each.)
    // G = est_lanes(...) lanes per key (cep_layout.h), 64 / G keys per wave; every lane stays for
    // the segmented reductions (a lane past the last key has no events)
    o += "extern \"C\" __global__ void __launch_bounds__(256) cep_nfa_est(NfaArgs A) {\n";
    o += "  const uint32_t G = est_lanes(A.n_events, A.n_keys);\n";
    o += "  const uint64_t k = ((uint64_t)blockIdx.x * 256 + threadIdx.x) / G;\n  const uint32_t lane = threadIdx.x & (G - 1);\n";
    o += "  const bool kin = k < A.n_keys;\n";
    o += "  const uint64_t base = kin ? A.key_off[k] : 0;\n  const uint32_t n = kin ? (uint32_t)(A.key_off[k + 1] - base) : 0u;\n";
    o += "  uint64_t w = 0;\n";
    o += "  const uint64_t p1 = base + n;\n";
    o += "  for (uint64_t wi = (base >> 6) + lane; n > 0 && wi <= ((p1 - 1) >> 6); wi += G) {\n";
    o += "    uint64_t bits = A.bhits[wi];\n    const uint64_t s = wi << 6;\n";
    o += "    if (s < base) bits &= ~0ull << (base - s);\n";
    o += "    if (p1 - s < 64) bits &= (1ull << (p1 - s)) - 1ull;\n";
    o += "    while (bits) {\n      const uint32_t b = (uint32_t)__builtin_ctzll(bits);\n      bits &= bits - 1ull;\n";
    o += "      w += n - (uint32_t)(s + b - base);\n    }\n  }\n";
    // (ordering by the span after the first begin hit instead, or by span then mean live
    // runs, was measured: cfg 3 31.5 -> 34.1 / 33.2 ms)
    o += "  for (int o = (int)G >> 1; o > 0; o >>= 1) w += __shfl_down(w, o, (int)G);\n";
    o += "  if (kin) {\n";
    o += "  w += n / kQuietChunk + 1;\n";
    o += "  if (A.carry && A.carry[k].live) w += (uint64_t)n * A.carry[k].count;  // a stream's carried runs\n";
    // a stream's order is kept steady across its batches (each launch lasts as long as its
    // heaviest wave: regrouping the keys every batch sums a different maximum each time): the
    // estimate is blended with the key's earlier ones, 7/8 of the running figure carried
    o += "  if (A.carry && A.est_blend) {\n    w += (uint64_t)A.carry[k].west - (A.carry[k].west >> 3);\n";
    o += "    w = w > 0xFFFFFFFFull ? 0xFFFFFFFFull : w;\n    if (lane == 0) A.carry[k].west = (uint32_t)w;\n  }\n";
    o += "  if (lane == 0) A.est[k] = w > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)w;\n  }\n";
    // the watermark's second level: the first (at most) 1024 blocks each reduce a strided
    // share of the bitmap blocks' maxima, one atomicMax per block (one per wave of a full
    // pass cost 10 ms on one word: DESIGN.md)
    o += "  if (A.wmax) {\n    const uint64_t R = gridDim.x < 1024 ? gridDim.x : 1024;\n";
    o += "    if (blockIdx.x < R && threadIdx.x < 64) {\n      int64_t m = INT64_MIN;\n";
    o += "      for (uint64_t i = blockIdx.x + R * (threadIdx.x & 63); i < A.n_wm_blocks; i += R * 64)\n";
    o += "        m = A.wm_blocks[i] > m ? A.wm_blocks[i] : m;\n";
    o += "      for (int o = 32; o > 0; o >>= 1) {\n        const int64_t y = __shfl_down(m, o, 64);\n";
    o += "        m = y > m ? y : m;\n      }\n";
    o += "      if (threadIdx.x == 0) atomicMax(A.wmax, (unsigned long long)m ^ 0x8000000000000000ull);\n";
    o += "    }\n  }\n}\n\n";
    // Begin-hit bitmap (NfaArgs.bhits).  A block owns 256 * kBitStrips positions as strips of
    // 1024: in a strip thread t holds positions 4t..4t+3 (16-B loads: 1 KiB a wave-instruction
    // for a 4-byte column), and a wave's 256 positions make 4 bitmap words - word q from the
    // ballots of lanes 16q..16q+15, bit 4i + j the j-th position of lane 16q + i (spread).
    // Quiet lanes (only the begin run) jump from set bit to set bit (nfa_lane.h run).  (One
    // position per thread and strip, 4-byte loads: 2.9 ms for 1e9 events with the watermark's
    // timestamps, 4.1 TB/s.)
    o += "__device__ __forceinline__ uint64_t bits_spread4(uint32_t x16) {\n  uint64_t x = x16;\n";
    o += "  x = (x | (x << 24)) & 0x000000FF000000FFull;\n  x = (x | (x << 12)) & 0x000F000F000F000Full;\n";
    o += "  x = (x | (x << 6)) & 0x0303030303030303ull;\n  x = (x | (x << 3)) & 0x1111111111111111ull;\n  return x;\n}\n";
    o += "extern \"C\" __global__ void __launch_bounds__(256) cep_nfa_bits(NfaArgs A) {\n";
    o += "  constexpr int S = " + std::to_string(kBitStrips / 4) + ";  // strips of 1024 positions\n";
    o += "  const uint64_t b0 = (uint64_t)blockIdx.x * (256 * " + std::to_string(kBitStrips) + ");\n";
    o += "  const uint64_t n = A.n_events;\n  const uint32_t lane = threadIdx.x & 63;\n";
    // the watermark's first level (session.cpp folds it here when the batch has timestamps): the
    // block's largest event time; its loads issued before the predicate's, both before the
    // bitmap stores (a store may alias them)
    o += "  const bool wmf = A.wm_blocks != nullptr;\n";
    o += "  const bool vec = bev4_aligned(A) && (!wmf || ((uint64_t)A.ts & 15u) == 0);\n";
    // (every strip's loads - timestamps and the predicate's columns - go out before any
    // predicate runs: 2.53 -> ~2.0 ms for 1e9 events with the watermark's timestamps in a
    // probe of this shape, profiles/micro/bits_probe.hip)
    o += "  int64_t t[S][4];\n  Ev e[S][4];\n#pragma unroll\n  for (int k = 0; k < S; k++) {\n";
    o += "    const uint64_t p = b0 + (uint64_t)k * 1024 + (uint64_t)threadIdx.x * 4;\n";
    o += "    if (wmf && vec && p + 4 <= n) {\n";
    o += "      const longlong2* q = reinterpret_cast<const longlong2*>(A.ts + p);\n";
    o += "      const longlong2 a = q[0], c = q[1];\n";
    o += "      t[k][0] = a.x;\n      t[k][1] = a.y;\n      t[k][2] = c.x;\n      t[k][3] = c.y;\n";
    o += "    } else {\n#pragma unroll\n      for (int j = 0; j < 4; j++) t[k][j] = wmf && p + j < n ? A.ts[p + j] : INT64_MIN;\n    }\n";
    o += "    if (vec && p + 4 <= n) {\n      ld_bev4(e[k], A, p);\n    } else {\n";
    o += "#pragma unroll\n      for (int j = 0; j < 4; j++) ld_bev(e[k][j], A, p + j < n ? p + j : 0);\n    }\n  }\n";
    o += "  int64_t m = INT64_MIN;\n#pragma unroll\n  for (int k = 0; k < S; k++)\n#pragma unroll\n";
    o += "    for (int j = 0; j < 4; j++) m = t[k][j] > m ? t[k][j] : m;\n";
    o += "#pragma unroll\n  for (int k = 0; k < S; k++) {\n    uint64_t B[4];\n";
    o += "    const uint64_t p = b0 + (uint64_t)k * 1024 + (uint64_t)threadIdx.x * 4;\n";
    o += "#pragma unroll\n    for (int j = 0; j < 4; j++) B[j] = __ballot(p + j < n && begin_hit_ev(A, e[k][j]));\n";
    o += "    uint64_t w = 0;  // lane q < 4: word q of the wave's 256 positions\n";
    o += "#pragma unroll\n    for (int q = 0; q < 4; q++) {\n      uint64_t x = 0;\n";
    o += "#pragma unroll\n      for (int j = 0; j < 4; j++) x |= bits_spread4((uint32_t)(B[j] >> (16 * q)) & 0xFFFFu) << j;\n";
    o += "      if (lane == (uint32_t)q) w = x;\n    }\n";
    o += "    const uint64_t ws = b0 + (uint64_t)k * 1024 + (uint64_t)(threadIdx.x >> 6) * 256 + (uint64_t)lane * 64;\n";
    o += "    if (lane < 4 && ws < n) A.bhits[ws >> 6] = w;\n  }\n";
    o += "  if (wmf) {\n";
    o += "    for (int o = 32; o > 0; o >>= 1) {\n      const int64_t y = __shfl_down(m, o, 64);\n      m = y > m ? y : m;\n    }\n";
    o += "    __shared__ int64_t wm[4];\n    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;\n    __syncthreads();\n";
    o += "    if (threadIdx.x == 0) {\n      int64_t x = wm[0];\n      for (int i = 1; i < 4; i++) x = wm[i] > x ? wm[i] : x;\n";
    o += "      A.wm_blocks[blockIdx.x] = x;\n    }\n  }\n}\n\n";
  }
  o += "}  // namespace cep\n";
  return o;
}

void compile_query(const uint8_t* ir, size_t n, cep_query* q) {
  In in{ir, ir + n};
  if (n < 8 || std::memcmp(ir, "CEPQ", 4) != 0) throw std::runtime_error("not a CEP query IR (magic)");
  in.p += 4;
  const uint32_t ver = in.get<uint32_t>();
  if (ver != 1 && ver != 2) throw std::runtime_error("unsupported query IR version");
  const uint32_t flags = ver == 2 ? in.get<uint32_t>() : 0u;  // v2: bit0 semantic WITHIN
  if (flags & ~1u) throw std::runtime_error("unknown query IR flags");
  q->semantic = (flags & 1u) != 0;
  DevQuery& d = q->dev;
  std::memset(&d, 0, sizeof d);
  uint16_t nf = in.get<uint16_t>();
  if (nf == 0 || nf > kMaxFields) throw std::runtime_error("1..16 event fields supported");
  for (int i = 0; i < nf; i++) {
    d.field_type[i] = in.get<uint8_t>();
    q->fieldNames.push_back(in.str());
  }
  d.n_fields = nf;
  uint16_t ns = in.get<uint16_t>();
  if (ns > kMaxStates) throw std::runtime_error("at most 8 fold states per query");
  for (int i = 0; i < ns; i++) {
    d.state_type[i] = in.get<uint8_t>();
    q->stateNames.push_back(in.str());
  }
  d.n_states = ns;
  uint16_t nn = in.get<uint16_t>();
  for (int i = 0; i < nn; i++) q->names.push_back(in.str());
  q->names.push_back("$final");
  uint16_t np = in.get<uint16_t>();
  if (np == 0) throw std::runtime_error("empty pattern");
  auto pq = std::make_shared<ParsedQuery>();  // kept for plan_groups
  std::vector<PatternIR>& ps = pq->ps;
  for (int i = 0; i < np; i++) {
    PatternIR p;
    p.name = in.get<uint16_t>();
    if (p.name >= nn) throw std::runtime_error("bad stage name index");
    p.card = in.get<uint8_t>();
    p.strat = in.get<uint8_t>();
    p.hasWindow = in.get<uint8_t>() != 0;
    p.window = in.get<int64_t>();
    if (in.get<uint8_t>()) p.pred = parse(in);
    uint16_t na = in.get<uint16_t>();
    for (int k = 0; k < na; k++) {
      uint16_t s = in.get<uint16_t>();
      if (s >= ns) throw std::runtime_error("bad fold state index");
      p.aggs.emplace_back(s, parse(in));
    }
    ps.push_back(std::move(p));
  }
  if (in.p != in.e) throw std::runtime_error("trailing bytes after query IR");
  q->info.n_patterns = np;
  q->info.n_names = (uint32_t)q->names.size();
  q->info.n_fields = nf;
  q->info.n_states = ns;

  pq->b.reset(new Builder{q, ps, {}, {}, {}});
  Builder& b = *pq->b;
  // $final (StatesFactory.java:46-47)
  int successor = b.newStage((uint16_t)nn, ST_FINAL);
  const PatternIR* successorPattern = nullptr;
  try {
    for (int i = np - 1; i >= 1; i--) {
      successor = b.buildState(ST_NORMAL, ps[i], successor, successorPattern);
      successorPattern = &ps[i];
    }
    d.begin_stage = (uint32_t)b.buildState(ST_BEGIN, ps[0], successor, successorPattern);
  } catch (std::runtime_error&) {
    if (q->info.compile_error) { q->info.n_stages = d.n_stages; return; }  // reference compile exception
    throw;
  }
  q->info.n_stages = d.n_stages;
  // semantic WITHIN: a run record carries its start time in two more fold slots; an epsilon
  // stage's window is its source stage's, found by stage key (stages sharing a key must agree)
  q->windowed = false;
  if (q->semantic) {
    for (uint32_t s = 0; s < d.n_stages; s++) q->windowed = q->windowed || b.window[s] >= 0;
    for (uint32_t s = 0; s < d.n_stages; s++)
      for (uint32_t t = 0; t < s; t++)
        if (d.st[s].sk == d.st[t].sk && b.window[s] != b.window[t])
          throw std::runtime_error("semantic WITHIN: stages with the same name and type carry different windows");
  }
  {
    const uint32_t slots = d.n_states + (q->windowed ? 2u : 0u);
    if (slots > 8) throw std::runtime_error("at most 6 fold states with semantic WITHIN");
    q->F = slots <= 2 ? 2 : slots <= 4 ? 4 : 8;
  }

  // bytecode: edge predicates, then folds
  q->code.clear();
  q->code.push_back(BC_END);  // offset 0 unused
  int maxDepth = 0;
  for (auto& pe : b.pending) {
    if (pe.m->k == M::TRUE_) continue;  // kProgTrue
    Code c{q->code};
    uint32_t off = (uint32_t)q->code.size();
    c.matcher(pe.m.get());
    c.op(BC_END);
    if (off >= kProgTrue) throw std::runtime_error("query bytecode too large");
    d.st[pe.stage].e[pe.edge].prog = (uint16_t)off;
    maxDepth = std::max(maxDepth, c.maxDepth);
  }
  for (auto& sa : b.stageAggs) {
    DevStage& s = d.st[sa.first];
    int k = 0;
    for (auto& agg : *sa.second) {
      Code c{q->code};
      uint32_t off = (uint32_t)q->code.size();
      c.expr(agg.second.get());  // a fold may return a null (e.g. `curr`)
      c.op(BC_END);
      if (off >= kProgTrue) throw std::runtime_error("query bytecode too large");
      s.agg_state[k] = agg.first;
      s.agg_prog[k] = (uint16_t)off;
      k++;
      maxDepth = std::max(maxDepth, c.maxDepth);
    }
  }
  if (maxDepth > kMaxStack) throw std::runtime_error("predicate expression too deep (stack > 16)");
  d.code_len = (uint32_t)q->code.size();

  // CEP_KIND_STENCIL gate: every pattern ONE + STRICT, predicates total
  // and state-free (so evaluating them everywhere cannot throw or differ), distinct names.
  // The stencil kernels are instantiated for 1..kMaxStencil stages (stencil.hip
  // launch_stencil); a longer strict chain runs on the NFA kernel.
  bool stencil = np <= kMaxStencil && !q->windowed;  // (semantic windows: runs expire on ts)
  std::vector<int> seen;
  for (auto& p : ps) {
    if (p.card != CARD_ONE || p.strat != STRICT || !total(p.pred.get())) stencil = false;
    // folds never influence a stencil match, but they run on every BEGIN and can throw
    // (a null `curr` unboxed, integer division): only total folds keep the stencil exact
    for (auto& a : p.aggs)
      if (!total(a.second.get())) stencil = false;
    for (int s : seen) if (s == p.name) stencil = false;
    seen.push_back(p.name);
  }
  if (stencil) {
    q->info.kind = CEP_KIND_STENCIL;
    q->info.arity = np;
    q->stencilProg.clear();
    // walk order: final event first -> stage names last..first
    for (int i = np - 1; i >= 0; i--) q->arityStage.push_back(ps[i].name);
    for (int i = 0; i < np; i++) {
      // predicate of pattern i = first edge of its stage (BEGIN edge)
      q->stencilProg.push_back(0);
    }
    // stages were built last -> first; stage index of pattern i: $final=0, p_{m-1}=1, ..., p0=m
    for (int i = 0; i < np; i++) q->stencilProg[i] = d.st[np - i].e[0].prog;
    // interval fast path: <= 8 stages, every predicate an int range over <= 2 shared columns
    std::vector<int> ftypes(d.field_type, d.field_type + nf);
    bool range = np <= 8;
    int cols[2] = {-1, -1}, ncols = 0;
    for (int i = 0; i < np && range; i++) {
      Ranges r;
      if (!ranges_of(ps[i].pred.get(), ftypes, r)) { range = false; break; }
      for (int c = 0; c < 2; c++) { q->rangeLo[i][c] = INT64_MIN; q->rangeHi[i][c] = INT64_MAX; }
      for (int x = 0; x < r.n; x++) {
        int slot = -1;
        for (int c = 0; c < ncols; c++) if (cols[c] == r.field[x]) slot = c;
        if (slot < 0) {
          if (ncols == 2) { range = false; break; }
          cols[ncols] = r.field[x];
          slot = ncols++;
        }
        q->rangeLo[i][slot] = r.lo[x];
        q->rangeHi[i][slot] = r.hi[x];
      }
    }
    q->stencilRange = range;
    q->nRangeCols = ncols == 0 ? 1 : ncols;
    q->rangeCols[0] = cols[0] < 0 ? 0 : cols[0];
    q->rangeCols[1] = cols[1] < 0 ? q->rangeCols[0] : cols[1];
  } else {
    q->info.kind = CEP_KIND_NFA;
    q->info.arity = 0;
  }
  LitCtx lits;
  q->jitSource = generate_jit(q, b, lits);
  q->parsed = pq;  // kept for kernel groups (plan_groups)
}

// Queries of a session that differ only in literal values share one kernel launch (a group):
// lanes = (key, query), every wave one query of 64 keys, the literals that differ read from a
// per-query table (NfaArgs.kc).  Groups keep first-appearance order; a query alone keeps its
// own literal-inlined kernel.
std::vector<GroupPlan> plan_groups(const std::vector<const cep_query*>& qs) {
  const size_t n = qs.size();
  std::vector<std::string> shape(n);
  std::vector<std::vector<int64_t>> vals(n);
  for (size_t i = 0; i < n; i++) {
    LitCtx L;
    L.param = true;
    shape[i] = generate_jit(qs[i], *qs[i]->parsed->b, L);
    vals[i] = L.values;
  }
  std::vector<GroupPlan> out;
  std::vector<char> done(n, 0);
  for (size_t i = 0; i < n; i++) {
    if (done[i]) continue;
    GroupPlan g;
    for (size_t j = i; j < n; j++)
      if (!done[j] && shape[j] == shape[i]) {
        g.members.push_back((int)j);
        done[j] = 1;
      }
    if (g.members.size() == 1) {
      g.source = qs[i]->jitSource;
    } else {
      std::vector<char> inl(vals[i].size(), 1);
      for (int m : g.members)
        for (size_t k = 0; k < inl.size(); k++) inl[k] = inl[k] && vals[m][k] == vals[i][k];
      LitCtx L;
      L.param = true;
      L.inl = &inl;
      g.source = generate_jit(qs[i], *qs[i]->parsed->b, L);
      g.nkc = (uint32_t)L.values.size();
      for (int m : g.members) g.table.insert(g.table.end(), vals[m].begin(), vals[m].end());
    }
    out.push_back(std::move(g));
  }
  return out;
}

}  // namespace cep
