// compile.cpp — query compiler: serialised Pattern chain -> stage table + predicate bytecode.
//
// Replaces StatesFactory.make (pattern/StatesFactory.java:41-127) and the lambda bodies of
// Matcher / Aggregator (pattern/Matcher.java, pattern/Aggregator.java), which arrive as the
// typed IR documented in include/cep.h.  Host-only code, linked into libcep.so.
#include <algorithm>
#include <climits>
#include <cstdio>
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
      st = w;
    }
    return st;
  }
};

void compile_query(const uint8_t* ir, size_t n, cep_query* q) {
  In in{ir, ir + n};
  if (n < 8 || std::memcmp(ir, "CEPQ", 4) != 0) throw std::runtime_error("not a CEP query IR (magic)");
  in.p += 4;
  if (in.get<uint32_t>() != 1) throw std::runtime_error("unsupported query IR version");
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
  std::vector<PatternIR> ps;
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

  Builder b{q, ps, {}, {}, {}};
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
  bool stencil = np <= 32;
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
}

}  // namespace cep
