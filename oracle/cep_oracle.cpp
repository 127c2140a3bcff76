// cep_oracle.cpp — TEST INFRASTRUCTURE ONLY (parity checker and CPU baseline).
//
// A literal C++ restatement of the reference's NFA hot path.  It keeps the reference's
// own data structures: a FIFO of ComputationStage objects, a hash map of buffer nodes
// keyed by (stage name, stage type, offset), ordered predecessor lists of
// (DeweyVersion object, key) pointers, int-vector Dewey versions, and a fold store keyed
// by (state name, run sequence).  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load it; the product path (libcep.so) never does.
//
// Parity is pinned by the reference's own known-answer tests:
// test:nfa/NFATest.java:41-245, test:nfa/DeweyVersionTest.java:8-44,
// test:nfa/buffer/SharedVersionedBufferTest.java:28-68, README.md:71-96
// (tests/golden/, tests/test_oracle_golden.py).
//
// Paths are relative to /root/reference/src/main/java/com/github/fhuz/kafka/streams/cep/.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <list>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace oracle {

// ------------------------------------------------------------------ Java exceptions
enum ErrCode { OK = 0, NPE = 1, ILLEGAL_STATE = 2, ARITHMETIC = 3, ILLEGAL_ARGUMENT = 4 };
struct JavaException {
  int code;
  std::string msg;
};
[[noreturn]] static void throwJ(int code, const char* m) { throw JavaException{code, m}; }

// ------------------------------------------------------------------ IR (independent parser)
enum { T_I32 = 1, T_I64 = 2, T_F64 = 3, T_BOOL = 4 };
struct Expr {
  uint8_t op = 0, t = 0, t2 = 0;
  int64_t i = 0;
  double d = 0;
  uint16_t idx = 0;
  std::unique_ptr<Expr> a, b;
};

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  template <class T> T get() {
    if (p + sizeof(T) > end) throw std::runtime_error("IR truncated");
    T v;
    std::memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  std::string str() {
    uint16_t n = get<uint16_t>();
    if (p + n > end) throw std::runtime_error("IR truncated");
    std::string s((const char*)p, n);
    p += n;
    return s;
  }
};

static std::unique_ptr<Expr> parseExpr(Reader& r) {
  auto e = std::make_unique<Expr>();
  e->op = r.get<uint8_t>();
  switch (e->op) {
    case 0x01: e->t = T_I32; e->i = r.get<int32_t>(); break;
    case 0x02: e->t = T_I64; e->i = r.get<int64_t>(); break;
    case 0x03: e->t = T_F64; e->d = r.get<double>(); break;
    case 0x04: e->t = T_BOOL; e->i = r.get<uint8_t>(); break;
    case 0x05: e->idx = r.get<uint16_t>(); break;
    case 0x06: e->t = T_I64; break;
    case 0x07: e->idx = r.get<uint16_t>(); break;
    case 0x08: e->idx = r.get<uint16_t>(); e->a = parseExpr(r); break;
    case 0x09: break;
    case 0x10: case 0x11: case 0x12: case 0x13: case 0x14:
      e->t = r.get<uint8_t>(); e->a = parseExpr(r); e->b = parseExpr(r); break;
    case 0x15: e->t = r.get<uint8_t>(); e->a = parseExpr(r); break;
    case 0x18: e->t2 = r.get<uint8_t>(); e->t = r.get<uint8_t>(); e->a = parseExpr(r); break;
    case 0x20: case 0x21: case 0x22: case 0x23: case 0x24: case 0x25:
      e->t2 = r.get<uint8_t>(); e->t = T_BOOL; e->a = parseExpr(r); e->b = parseExpr(r); break;
    case 0x30: case 0x31: e->t = T_BOOL; e->a = parseExpr(r); e->b = parseExpr(r); break;
    case 0x32: e->t = T_BOOL; e->a = parseExpr(r); break;
    default: throw std::runtime_error("bad IR opcode");
  }
  return e;
}

// boxed value: the reference stores java.lang.Integer / Long / Double objects
struct Val {
  int t = 0;  // 0 = null
  int64_t i = 0;
  double d = 0;
};

// ------------------------------------------------------------------ pattern/Pattern.java
enum Cardinality { ONE = 0, OPTIONAL = 1, ZERO_OR_MORE = 2, ONE_OR_MORE = 3 };
enum Strategy { STRICT = 0, NEXT = 1, ANY = 2 };

struct AggDef {
  uint16_t state;
  std::unique_ptr<Expr> fn;
};
struct PatternDef {
  uint16_t name;
  int cardinality, strategy;
  bool hasWindow;
  int64_t windowMs;
  std::unique_ptr<Expr> pred;  // null: no where()
  std::vector<AggDef> aggs;
};
struct QueryDef {
  bool semantic = false;  // build-only semantic WITHIN (epsilon stages keep their window)
  std::vector<int> fieldTypes;
  std::vector<int> stateTypes;
  std::vector<std::string> stateNames;
  std::vector<std::string> names;
  std::vector<PatternDef> patterns;  // p0 .. p_{m-1}
};

static QueryDef parseQuery(const uint8_t* ir, size_t n) {
  Reader r{ir, ir + n};
  if (n < 8 || std::memcmp(ir, "CEPQ", 4) != 0) throw std::runtime_error("bad IR magic");
  r.p += 4;
  const uint32_t ver = r.get<uint32_t>();
  if (ver != 1 && ver != 2) throw std::runtime_error("bad IR version");
  QueryDef q;
  q.semantic = ver == 2 && (r.get<uint32_t>() & 1u);  // v2 flags: bit0 semantic WITHIN
  uint16_t nf = r.get<uint16_t>();
  for (int i = 0; i < nf; i++) { q.fieldTypes.push_back(r.get<uint8_t>()); r.str(); }
  uint16_t ns = r.get<uint16_t>();
  for (int i = 0; i < ns; i++) { q.stateTypes.push_back(r.get<uint8_t>()); q.stateNames.push_back(r.str()); }
  uint16_t nn = r.get<uint16_t>();
  for (int i = 0; i < nn; i++) q.names.push_back(r.str());
  uint16_t np = r.get<uint16_t>();
  for (int i = 0; i < np; i++) {
    PatternDef p;
    p.name = r.get<uint16_t>();
    p.cardinality = r.get<uint8_t>();
    p.strategy = r.get<uint8_t>();
    p.hasWindow = r.get<uint8_t>() != 0;
    p.windowMs = r.get<int64_t>();
    if (r.get<uint8_t>()) p.pred = parseExpr(r);
    uint16_t na = r.get<uint16_t>();
    for (int k = 0; k < na; k++) {
      AggDef a;
      a.state = r.get<uint16_t>();
      a.fn = parseExpr(r);
      p.aggs.push_back(std::move(a));
    }
    q.patterns.push_back(std::move(p));
  }
  return q;
}

// ------------------------------------------------------------------ Matcher (pattern/Matcher.java)
struct EvalCtx;
struct Matcher {
  enum Kind { EXPR, TRUE_, NOT, AND, OR } kind;
  const Expr* expr = nullptr;
  std::shared_ptr<Matcher> a, b;
};
using MatcherP = std::shared_ptr<Matcher>;
static MatcherP mExpr(const Expr* e) { auto m = std::make_shared<Matcher>(); m->kind = Matcher::EXPR; m->expr = e; return m; }
static MatcherP mTrue() { auto m = std::make_shared<Matcher>(); m->kind = Matcher::TRUE_; return m; }
static MatcherP mNot(MatcherP x) { auto m = std::make_shared<Matcher>(); m->kind = Matcher::NOT; m->a = x; return m; }
static MatcherP mAnd(MatcherP x, MatcherP y) { auto m = std::make_shared<Matcher>(); m->kind = Matcher::AND; m->a = x; m->b = y; return m; }
static MatcherP mOr(MatcherP x, MatcherP y) { auto m = std::make_shared<Matcher>(); m->kind = Matcher::OR; m->a = x; m->b = y; return m; }

// ------------------------------------------------------------------ nfa/Stage.java, EdgeOperation.java
enum StateType { BEGIN = 0, NORMAL = 1, FINAL = 2 };
enum EdgeOp { OP_BEGIN = 0, OP_TAKE = 1, OP_PROCEED = 2, OP_IGNORE = 3 };

struct Stage;
using StageP = std::shared_ptr<Stage>;
struct Edge {
  EdgeOp op;
  MatcherP pred;
  Stage* target;  // real stages are owned by the query (StatesFactory output)
};
struct Stage {
  int name;  // interned stage name
  StateType type;
  int64_t windowMs = -1;                 // Stage.java:38
  const std::vector<AggDef>* aggregates = nullptr;  // null for epsilon stages (Stage.java:42-46)
  std::vector<Edge> edges;
  bool isBeginState() const { return type == BEGIN; }
  bool isFinalState() const { return type == FINAL; }
  bool equals(const Stage* o) const { return o && name == o->name && type == o->type; }  // :117-122
};

// Stage.newEpsilonState (Stage.java:42-46): name/type of `current`, single PROCEED(true) edge
// semantic: the build's semantic-WITHIN mode (IR v2 flag, not the reference): the epsilon stage
// also keeps `current`'s window, so ComputationStage.isOutOfWindow (:98-100) can fire
static StageP newEpsilonState(const Stage* current, Stage* target, bool semantic) {
  if (!current) throwJ(NPE, "newEpsilonState(null)");
  auto s = std::make_shared<Stage>();
  s->name = current->name;
  s->type = current->type;
  if (semantic) s->windowMs = current->windowMs;
  s->edges.push_back(Edge{OP_PROCEED, mTrue(), target});
  return s;
}

// pattern/StatesFactory.java:41-127
struct CompiledQuery {
  QueryDef def;
  std::vector<StageP> owned;     // all real stages (incl. ONE_OR_MORE loop stages)
  std::vector<Stage*> sequence;  // StatesFactory.make output: [$final, ..., begin]
  int finalName;
};

static int64_t windowOf(const PatternDef* cur, const PatternDef* succ) {  // :121-127
  if (cur->hasWindow) return cur->windowMs;
  if (succ && succ->hasWindow) return succ->windowMs;
  return -1;
}

static Stage* buildState(CompiledQuery& cq, StateType type, const PatternDef* cur, Stage* successorStage,
                         const PatternDef* successorPattern) {
  bool hasMandatoryState = cur->cardinality == ONE_OR_MORE;               // :70
  StateType currentType = hasMandatoryState ? NORMAL : type;              // :72
  auto stage = std::make_shared<Stage>();
  stage->name = cur->name;
  stage->type = currentType;
  int64_t w = windowOf(cur, successorPattern);
  stage->windowMs = w;
  stage->aggregates = &cur->aggs;
  if (!cur->pred) throwJ(ILLEGAL_ARGUMENT, "predicate cannot be null");  // Stage.java:159
  MatcherP predicate = mExpr(cur->pred.get());
  EdgeOp operation = cur->cardinality == ONE ? OP_BEGIN : OP_TAKE;     // :80
  stage->edges.push_back(Edge{operation, predicate, successorStage});
  MatcherP ignore;
  if (cur->strategy == ANY) {                                            // :87-90
    ignore = mTrue();
    stage->edges.push_back(Edge{OP_IGNORE, ignore, nullptr});
  }
  if (cur->strategy == NEXT) {                                           // :93-96
    ignore = mNot(predicate);
    stage->edges.push_back(Edge{OP_IGNORE, ignore, nullptr});
  }
  if (operation == OP_TAKE) {                                            // :98-107
    if (!successorPattern) throwJ(NPE, "successorPattern.getPredicate() on null");
    if (!successorPattern->pred) throwJ(ILLEGAL_ARGUMENT, "predicate cannot be null");
    MatcherP succ = mExpr(successorPattern->pred.get());
    MatcherP proceed = cur->strategy == STRICT ? mOr(succ, mNot(predicate))
                                               : mOr(succ, mAnd(mNot(predicate), mNot(ignore)));
    stage->edges.push_back(Edge{OP_PROCEED, proceed, successorStage});
  }
  cq.owned.push_back(stage);
  Stage* result = stage.get();
  if (hasMandatoryState) {                                               // :110-116
    Stage* loop = result;
    auto wrapper = std::make_shared<Stage>();
    wrapper->name = cur->name;
    wrapper->type = type;
    wrapper->edges.push_back(Edge{OP_BEGIN, mExpr(cur->pred.get()), loop});
    wrapper->windowMs = w;
    wrapper->aggregates = &cur->aggs;
    cq.owned.push_back(wrapper);
    result = wrapper.get();
  }
  return result;
}

static void make(CompiledQuery& cq) {  // :41-63
  auto& ps = cq.def.patterns;
  if (ps.empty()) throwJ(NPE, "Cannot make null pattern");
  auto fin = std::make_shared<Stage>();
  fin->name = cq.finalName;
  fin->type = FINAL;
  cq.owned.push_back(fin);
  Stage* successorStage = fin.get();
  cq.sequence.push_back(successorStage);
  const PatternDef* successorPattern = nullptr;
  for (int i = (int)ps.size() - 1; i >= 1; i--) {
    successorStage = buildState(cq, NORMAL, &ps[i], successorStage, successorPattern);
    cq.sequence.push_back(successorStage);
    successorPattern = &ps[i];
  }
  Stage* begin = buildState(cq, BEGIN, &ps[0], successorStage, successorPattern);
  cq.sequence.push_back(begin);
}

// ------------------------------------------------------------------ nfa/DeweyVersion.java
struct DeweyVersion {
  std::vector<int32_t> v;
  std::shared_ptr<DeweyVersion> addRun() const {  // :51-56
    auto n = std::make_shared<DeweyVersion>(*this);
    n->v.back() += 1;
    return n;
  }
  std::shared_ptr<DeweyVersion> addStage() const {  // :84-86
    auto n = std::make_shared<DeweyVersion>(*this);
    n->v.push_back(0);
    return n;
  }
  bool isCompatible(const DeweyVersion& that) const {  // :62-82
    if (v.size() > that.v.size()) {
      for (size_t i = 0; i < that.v.size(); i++)
        if (v[i] != that.v[i]) return false;
      return true;
    } else if (v.size() == that.v.size()) {
      size_t last = v.size() - 1;
      for (size_t i = 0; i < last; i++)
        if (v[i] != that.v[i]) return false;
      return v[last] >= that.v[last];
    }
    return false;
  }
  std::string str() const {
    std::string s;
    for (size_t i = 0; i < v.size(); i++) { if (i) s += "."; s += std::to_string(v[i]); }
    return s;
  }
  static std::shared_ptr<DeweyVersion> parse(const char* s) {
    auto d = std::make_shared<DeweyVersion>();
    const char* p = s;
    while (*p) { d->v.push_back((int32_t)std::strtol(p, (char**)&p, 10)); if (*p == '.') p++; }
    return d;
  }
};
using DeweyP = std::shared_ptr<DeweyVersion>;

// ------------------------------------------------------------------ nfa/buffer/impl/StackEventKey.java
struct StackEventKey {
  int name;
  StateType type;
  int64_t offset;  // Event identity within a key's stream (topic/partition implicit)
  bool operator==(const StackEventKey& o) const { return name == o.name && type == o.type && offset == o.offset; }
};
struct KeyHash {
  size_t operator()(const StackEventKey& k) const {
    return std::hash<int64_t>()(k.offset * 1000003 + k.name * 7 + (int)k.type);
  }
};

// nfa/buffer/impl/TimedKeyValue.java
struct Pointer {
  DeweyP version;
  bool hasKey;
  StackEventKey key;
};
struct TimedKeyValue {
  int64_t refs = 1;                                  // :35-37 (AtomicLong(1))
  std::unique_ptr<std::vector<Pointer>> predecessors;  // null until first addPredecessor
  int64_t decrementRefAndGet() { return refs == 0 ? 0 : --refs; }  // :58-60
  size_t npreds() const { return predecessors ? predecessors->size() : 0; }
  const Pointer* getPointerByVersion(const DeweyVersion& version) const {  // :83-92
    if (!predecessors) throwJ(NPE, "predecessors == null");
    for (auto& p : *predecessors)
      if (version.isCompatible(*p.version)) return &p;
    return nullptr;
  }
  void addPredecessor(DeweyP v, const StackEventKey* key) {  // :94-98
    if (!predecessors) predecessors = std::make_unique<std::vector<Pointer>>();
    predecessors->push_back(Pointer{v, key != nullptr, key ? *key : StackEventKey{}});
  }
  void removePredecessor(const Pointer& ptr) {  // :75-77, equality: key equals && version identity
    for (auto it = predecessors->begin(); it != predecessors->end(); ++it) {
      bool keyEq = it->hasKey == ptr.hasKey && (!ptr.hasKey || it->key == ptr.key);
      if (keyEq && it->version.get() == ptr.version.get()) { predecessors->erase(it); return; }
    }
  }
};
using TKVP = std::shared_ptr<TimedKeyValue>;

struct WalkEntry {
  int name;
  int64_t offset;
};

// nfa/buffer/impl/KVSharedVersionedBuffer.java over an unbounded in-memory store
struct Buffer {
  std::unordered_map<StackEventKey, TKVP, KeyHash> store;
  uint64_t maxNodes = 0, totalPuts = 0;

  TKVP get(const StackEventKey& k) {
    auto it = store.find(k);
    return it == store.end() ? nullptr : it->second;
  }
  void putStore(const StackEventKey& k, TKVP v) {
    store[k] = v;
    if (store.size() > maxNodes) maxNodes = store.size();
  }
  // put(currStage, currEvent, prevStage, prevEvent, version)  :80-97
  void put(const Stage* cur, int64_t currEvent, const Stage* prev, int64_t prevEvent, DeweyP version) {
    if (prevEvent < 0) throwJ(NPE, "prevEvent.topic on null event");
    StackEventKey prevKey{prev->name, prev->type, prevEvent};
    StackEventKey curKey{cur->name, cur->type, currEvent};
    TKVP sharedPrev = get(prevKey);
    if (!sharedPrev) throwJ(ILLEGAL_STATE, "Cannot find predecessor event");
    TKVP sharedCurr = get(curKey);
    if (!sharedCurr) sharedCurr = std::make_shared<TimedKeyValue>();
    sharedCurr->addPredecessor(version, &prevKey);
    putStore(curKey, sharedCurr);
    totalPuts++;
  }
  // put(stage, evt, version)  :117-128
  void put(const Stage* stage, int64_t evt, DeweyP version) {
    auto v = std::make_shared<TimedKeyValue>();
    v->addPredecessor(version, nullptr);
    putStore(StackEventKey{stage->name, stage->type, evt}, v);
    totalPuts++;
  }
  // branch  :99-110
  void branch(const Stage* stage, int64_t event, DeweyP version) {
    if (event < 0) throwJ(NPE, "event.topic on null event");
    Pointer pointer{version, true, StackEventKey{stage->name, stage->type, event}};
    const Pointer* pp = &pointer;
    Pointer cur = pointer;
    while (pp && pp->hasKey) {
      cur = *pp;
      TKVP val = get(cur.key);
      if (!val) throwJ(NPE, "branch: missing node");
      val->refs++;
      pp = val->getPointerByVersion(*cur.version);
    }
  }
  // peek  :143-171
  std::vector<WalkEntry> peek(const Stage* stage, int64_t event, DeweyP version, bool remove) {
    if (event < 0) throwJ(NPE, "event.topic on null event");
    std::vector<WalkEntry> seq;
    Pointer pointer{version, true, StackEventKey{stage->name, stage->type, event}};
    bool have = true;
    while (have && pointer.hasKey) {
      StackEventKey stateKey = pointer.key;
      TKVP stateValue = get(stateKey);
      if (!stateValue) throwJ(NPE, "peek: missing node");
      int64_t refsLeft = stateValue->decrementRefAndGet();
      if (remove && refsLeft == 0 && stateValue->npreds() <= 1) store.erase(stateKey);
      seq.push_back(WalkEntry{stateKey.name, stateKey.offset});
      const Pointer* next = stateValue->getPointerByVersion(*pointer.version);
      if (!next) { have = false; break; }
      Pointer nextCopy = *next;
      if (remove && refsLeft == 0) stateValue->removePredecessor(nextCopy);
      pointer = nextCopy;
    }
    return seq;
  }
};

// ------------------------------------------------------------------ nfa/ComputationStage.java
struct ComputationStage {
  StageP stageOwner;  // keeps epsilon stages alive
  Stage* stage;
  int64_t event = -1;  // -1 == null Event
  int64_t timestamp = -1;
  DeweyP version;
  int64_t sequence = 0;
  bool branching = false;
  bool isBeginState() const { return stage->isBeginState(); }                     // :105-107
  bool isForwarding() const { return stage->edges.size() == 1 && stage->edges[0].op == OP_PROCEED; }  // :113-116
  bool isForwardingToFinalState() const { return isForwarding() && stage->edges[0].target->isFinalState(); }
  bool isOutOfWindow(int64_t t) const { return stage->windowMs != -1 && (t - timestamp) > stage->windowMs; }
};
using CSP = std::shared_ptr<ComputationStage>;

static CSP makeCS(StageP owner, Stage* st, DeweyP v, int64_t event, int64_t ts, int64_t seq, bool br) {
  auto c = std::make_shared<ComputationStage>();
  c->stageOwner = owner;
  c->stage = st;
  c->version = v;
  c->event = event;
  c->timestamp = ts;
  c->sequence = seq;
  c->branching = br;
  return c;
}
// ComputationStage.setVersion rebuilds WITHOUT the branching flag (:76-84)
static CSP setVersion(const CSP& c, DeweyP v) { return makeCS(c->stageOwner, c->stage, v, c->event, c->timestamp, c->sequence, false); }

// ------------------------------------------------------------------ value semantics (Java)
struct EventView {
  const std::vector<int>* types;
  const void* const* cols;
  int64_t pos;
  int64_t ts;
};

static Val loadField(const EventView& ev, int idx) {
  Val v;
  int t = (*ev.types)[idx];
  v.t = t;
  if (t == T_I32) v.i = ((const int32_t*)ev.cols[idx])[ev.pos];
  else if (t == T_I64) v.i = ((const int64_t*)ev.cols[idx])[ev.pos];
  else v.d = ((const double*)ev.cols[idx])[ev.pos];
  return v;
}

struct FoldStore {  // one KeyValueStore per state name, keyed by run sequence (pattern/ValueStore.java)
  std::vector<std::unordered_map<int64_t, Val>> stores;
  Val get(int state, int64_t seq) const {
    auto& m = stores[state];
    auto it = m.find(seq);
    return it == m.end() ? Val{} : it->second;
  }
  void set(int state, int64_t seq, Val v) { stores[state][seq] = v; }
};

static int32_t wrap32(int64_t x) { return (int32_t)(uint32_t)(uint64_t)x; }

static Val unbox(Val v) {
  if (v.t == 0) throwJ(NPE, "unboxing null");
  return v;
}

struct Evaluator {
  const EventView* ev;
  const FoldStore* folds;  // null inside an Aggregator
  int64_t seq;
  Val curr;
  const std::vector<int>* stateTypes;

  Val eval(const Expr* e) {
    Val r;
    switch (e->op) {
      case 0x01: r.t = T_I32; r.i = e->i; return r;
      case 0x02: r.t = T_I64; r.i = e->i; return r;
      case 0x03: r.t = T_F64; r.d = e->d; return r;
      case 0x04: r.t = T_BOOL; r.i = e->i; return r;
      case 0x05: return loadField(*ev, e->idx);
      case 0x06: r.t = T_I64; r.i = ev->ts; return r;
      case 0x07:  // States.get -> ValueStore.get (nullable)
        if (!folds) throwJ(ILLEGAL_ARGUMENT, "no States inside an Aggregator");
        return folds->get(e->idx, seq);
      case 0x08: {  // States.getOrElse (:53-62); the default argument is evaluated first (Java)
        if (!folds) throwJ(ILLEGAL_ARGUMENT, "no States inside an Aggregator");
        Val d = eval(e->a.get());
        Val v = folds->get(e->idx, seq);
        return v.t ? v : d;
      }
      case 0x09: return curr;
      case 0x10: case 0x11: case 0x12: case 0x13: case 0x14: {
        Val a = unbox(eval(e->a.get()));
        Val b = unbox(eval(e->b.get()));
        r.t = e->t;
        if (e->t == T_F64) {
          switch (e->op) {
            case 0x10: r.d = a.d + b.d; break;
            case 0x11: r.d = a.d - b.d; break;
            case 0x12: r.d = a.d * b.d; break;
            case 0x13: r.d = a.d / b.d; break;
            default: r.d = std::fmod(a.d, b.d); break;
          }
          return r;
        }
        const bool i32 = e->t == T_I32;
        uint64_t ua = (uint64_t)a.i, ub = (uint64_t)b.i;
        switch (e->op) {
          case 0x10: r.i = i32 ? wrap32((int64_t)(ua + ub)) : (int64_t)(ua + ub); break;
          case 0x11: r.i = i32 ? wrap32((int64_t)(ua - ub)) : (int64_t)(ua - ub); break;
          case 0x12: r.i = i32 ? wrap32((int64_t)(ua * ub)) : (int64_t)(ua * ub); break;
          case 0x13:
            if (b.i == 0) throwJ(ARITHMETIC, "/ by zero");
            if (i32) r.i = (a.i == INT32_MIN && b.i == -1) ? INT32_MIN : (int32_t)a.i / (int32_t)b.i;
            else r.i = (a.i == INT64_MIN && b.i == -1) ? INT64_MIN : a.i / b.i;
            break;
          default:
            if (b.i == 0) throwJ(ARITHMETIC, "/ by zero");
            if (b.i == -1) r.i = 0;
            else r.i = i32 ? (int32_t)a.i % (int32_t)b.i : a.i % b.i;
            break;
        }
        return r;
      }
      case 0x15: {
        Val a = unbox(eval(e->a.get()));
        r.t = e->t;
        if (e->t == T_F64) r.d = -a.d;
        else if (e->t == T_I32) r.i = wrap32(-(int64_t)a.i);
        else r.i = (int64_t)(0 - (uint64_t)a.i);
        return r;
      }
      case 0x18: {  // casts: JLS 5.1.2 / 5.1.3
        Val a = unbox(eval(e->a.get()));
        r.t = e->t;
        int from = e->t2, to = e->t;
        if (from == T_F64) {
          double d = a.d;
          if (to == T_F64) { r.d = d; return r; }
          if (std::isnan(d)) { r.i = 0; return r; }
          if (to == T_I32) r.i = d >= 2147483647.0 ? INT32_MAX : d <= -2147483648.0 ? INT32_MIN : (int32_t)d;
          else r.i = d >= 9223372036854775807.0 ? INT64_MAX : d <= -9223372036854775808.0 ? INT64_MIN : (int64_t)d;
          return r;
        }
        if (to == T_F64) { r.d = (double)a.i; return r; }
        r.i = to == T_I32 ? wrap32(a.i) : a.i;
        return r;
      }
      case 0x20: case 0x21: case 0x22: case 0x23: case 0x24: case 0x25: {
        Val a = unbox(eval(e->a.get()));
        Val b = unbox(eval(e->b.get()));
        bool res;
        if (e->t2 == T_F64) {
          double x = a.d, y = b.d;
          switch (e->op) {
            case 0x20: res = x < y; break; case 0x21: res = x <= y; break;
            case 0x22: res = x > y; break; case 0x23: res = x >= y; break;
            case 0x24: res = x == y; break; default: res = x != y; break;
          }
        } else {
          int64_t x = a.i, y = b.i;
          switch (e->op) {
            case 0x20: res = x < y; break; case 0x21: res = x <= y; break;
            case 0x22: res = x > y; break; case 0x23: res = x >= y; break;
            case 0x24: res = x == y; break; default: res = x != y; break;
          }
        }
        r.t = T_BOOL;
        r.i = res;
        return r;
      }
      case 0x30: { r.t = T_BOOL; r.i = eval(e->a.get()).i && eval(e->b.get()).i; return r; }
      case 0x31: { r.t = T_BOOL; r.i = eval(e->a.get()).i || eval(e->b.get()).i; return r; }
      case 0x32: { r.t = T_BOOL; r.i = !eval(e->a.get()).i; return r; }
    }
    throwJ(ILLEGAL_ARGUMENT, "bad opcode");
  }
};

static bool matches(const Matcher* m, Evaluator& ev) {
  switch (m->kind) {
    case Matcher::TRUE_: return true;
    case Matcher::NOT: return !matches(m->a.get(), ev);
    case Matcher::AND: return matches(m->a.get(), ev) && matches(m->b.get(), ev);
    case Matcher::OR: return matches(m->a.get(), ev) || matches(m->b.get(), ev);
    default: return ev.eval(m->expr).i != 0;
  }
}

// ------------------------------------------------------------------ nfa/NFA.java
struct Match {
  int64_t emitPos;
  std::vector<WalkEntry> walk;
};

struct NFA {
  const CompiledQuery* q;
  Buffer buffer;
  FoldStore folds;
  std::deque<CSP> computationStages;
  int64_t runs = 1;  // NFA.java:56
  uint64_t runSteps = 0, maxLive = 0;

  explicit NFA(const CompiledQuery* cq) : q(cq) {  // initComputationStates :74-81
    folds.stores.resize(cq->def.stateNames.size());
    for (Stage* s : cq->sequence)
      if (s->isBeginState())
        computationStages.push_back(makeCS(nullptr, s, std::make_shared<DeweyVersion>(DeweyVersion{{1}}), -1, -1, 1, false));
  }

  // matchPattern(K, V, long) :94-109
  std::vector<Match> matchPattern(const EventView& ev) {
    size_t n = computationStages.size();
    if (n > maxLive) maxLive = n;
    std::vector<CSP> finalStates;
    while (n-- > 0) {
      CSP c = computationStages.front();
      computationStages.pop_front();
      runSteps++;
      std::vector<CSP> states = matchPatternCtx(ev, c);
      if (states.empty()) removePattern(c);
      else
        for (auto& s : states) if (s->isForwardingToFinalState()) finalStates.push_back(s);
      for (auto& s : states) if (!s->isForwardingToFinalState()) computationStages.push_back(s);
    }
    std::vector<Match> out;  // matchConstruction :111-115
    for (auto& c : finalStates) out.push_back(Match{ev.pos, buffer.peek(c->stage, c->event, c->version, true)});
    return out;
  }

  void removePattern(const CSP& c) { buffer.peek(c->stage, c->event, c->version, true); }  // :117-123

  // matchPattern(ComputationContext) :139-160
  std::vector<CSP> matchPatternCtx(const EventView& ev, const CSP& c) {
    std::vector<CSP> next;
    if (!c->isBeginState() && c->isOutOfWindow(ev.ts)) return next;
    next = evaluate(ev, c, c->stage, nullptr);
    if (c->isBeginState() && !c->isForwarding()) {
      DeweyP nv = next.empty() ? c->version : c->version->addRun();
      next.push_back(makeCS(c->stageOwner, c->stage, nv, -1, -1, ++runs, false));
    }
    return next;
  }

  // evaluate :162-250
  std::vector<CSP> evaluate(const EventView& ev, const CSP& cs, Stage* currentStage, Stage* previousStage) {
    const int64_t sequenceID = cs->sequence;
    const int64_t previousEvent = cs->event;
    const DeweyP version = cs->version;

    std::vector<const Edge*> matchedEdges;  // matchEdgesAndGet :267-273
    {
      Evaluator e{&ev, &folds, sequenceID, Val{}, &q->def.stateTypes};
      for (auto& edge : currentStage->edges)
        if (matches(edge.pred.get(), e)) matchedEdges.push_back(&edge);
    }
    std::vector<CSP> nextStages;
    bool has[4] = {false, false, false, false};
    for (auto* e : matchedEdges) has[e->op] = true;
    const bool isBranching = (has[OP_PROCEED] && has[OP_TAKE]) || (has[OP_IGNORE] && has[OP_TAKE]) ||
                             (has[OP_IGNORE] && has[OP_BEGIN]) || (has[OP_IGNORE] && has[OP_PROCEED]);  // :280-289
    const int64_t currentEvent = ev.pos;
    const int64_t startTime = cs->isBeginState() ? ev.ts : cs->timestamp;  // getFirstPatternTimestamp :347-349
    bool consumed = false, ignored = false;

    for (auto* e : matchedEdges) {
      StageP epsilonStage = newEpsilonState(currentStage, e->target, q->def.semantic);  // :179 (created for every edge)
      switch (e->op) {
        case OP_PROCEED: {
          CSP nextCS = cs;
          if (!e->target->equals(currentStage) && !cs->branching) nextCS = setVersion(cs, cs->version->addStage());
          auto sub = evaluate(ev, nextCS, e->target, currentStage);
          nextStages.insert(nextStages.end(), sub.begin(), sub.end());
          break;
        }
        case OP_TAKE:
          if (!isBranching) {
            StageP eps = newEpsilonState(currentStage, currentStage, q->def.semantic);
            nextStages.push_back(makeCS(eps, eps.get(), version, currentEvent, startTime, sequenceID, false));
            putToSharedBuffer(currentStage, previousStage, previousEvent, currentEvent, version);
          } else {
            putToSharedBuffer(currentStage, previousStage, previousEvent, currentEvent, version->addRun());
          }
          consumed = true;
          break;
        case OP_BEGIN:
          putToSharedBuffer(currentStage, previousStage, previousEvent, currentEvent, version);
          nextStages.push_back(makeCS(epsilonStage, epsilonStage.get(), version, currentEvent, startTime, sequenceID, false));
          consumed = true;
          break;
        case OP_IGNORE:
          if (!isBranching) nextStages.push_back(cs);
          ignored = true;
          break;
      }
    }
    if (isBranching) {
      int64_t newSequence = ++runs;
      int64_t latestMatchEvent = ignored ? previousEvent : currentEvent;
      StageP eps = newEpsilonState(previousStage, currentStage, q->def.semantic);
      nextStages.push_back(makeCS(eps, eps.get(), version->addRun(), latestMatchEvent, startTime, newSequence, true));
      if (!currentStage->aggregates) throwJ(NPE, "aggregates == null");
      for (auto& agg : *currentStage->aggregates) {  // ValueStore.branch :92-97
        Val o = folds.get(agg.state, sequenceID);
        if (o.t) folds.set(agg.state, newSequence, o);
      }
      buffer.branch(previousStage, previousEvent, version);
    }
    if (consumed) {  // evaluateAggregates :259-265
      if (!currentStage->aggregates) throwJ(NPE, "aggregates == null");
      for (auto& agg : *currentStage->aggregates) {
        Evaluator e{&ev, nullptr, sequenceID, folds.get(agg.state, sequenceID), &q->def.stateTypes};
        folds.set(agg.state, sequenceID, e.eval(agg.fn.get()));
      }
    }
    return nextStages;
  }

  void putToSharedBuffer(const Stage* cur, const Stage* prev, int64_t prevEvent, int64_t curEvent, DeweyP v) {
    if (prev) buffer.put(cur, curEvent, prev, prevEvent, v);
    else buffer.put(cur, curEvent, v);
  }
};

}  // namespace oracle

// ====================================================================== C API (tests only)
extern "C" {

typedef struct {
  uint64_t n_keys, n_matches, n_pairs;
  uint32_t* key;
  uint32_t* emit_pos;
  uint64_t* pair_off;
  uint32_t* pair_pos;
  uint16_t* pair_stage;
  int32_t* err_code;
  uint32_t* err_pos;
  // calibration statistics
  uint64_t run_steps;       // Σ records stepped
  uint64_t max_live_runs;   // max |queue| over keys and events
  uint64_t max_nodes_key;   // max live buffer nodes of one key
  uint64_t total_puts;      // Σ buffer puts
  uint64_t max_puts_key;
  double elapsed_s;
  int threads;
} oracle_result;

static thread_local char g_err[512];

const char* oracle_last_error(void) { return g_err; }

static std::shared_ptr<oracle::CompiledQuery> compileQuery(const uint8_t* ir, size_t n) {
  auto cq = std::make_shared<oracle::CompiledQuery>();
  cq->def = oracle::parseQuery(ir, n);
  cq->finalName = (int)cq->def.names.size();  // "$final" gets its own name id
  oracle::make(*cq);
  return cq;
}

// Compile only; returns 0, or the reference exception class on a compile-time throw.
int oracle_compile_check(const uint8_t* ir, size_t n) {
  try {
    compileQuery(ir, n);
    return 0;
  } catch (oracle::JavaException& e) {
    std::snprintf(g_err, sizeof g_err, "%s", e.msg.c_str());
    return e.code;
  } catch (std::exception& e) {
    std::snprintf(g_err, sizeof g_err, "%s", e.what());
    return -1;
  }
}

struct KeyOut {
  std::vector<oracle::Match> matches;
  int32_t err = 0;
  uint32_t errPos = 0;
  uint64_t runSteps = 0, maxLive = 0, maxNodes = 0, puts = 0;
};

// Runs one reference NFA per key over a CSR-by-key batch.  cols[f] points to n_events
// values of the IR's field type f; ts may be NULL (then ts = position).
int oracle_run(const uint8_t* ir, size_t ir_len, uint64_t n_keys, const uint64_t* key_off,
               const void* const* cols, const int64_t* ts, int n_threads, oracle_result** out) {
  std::shared_ptr<oracle::CompiledQuery> cq;
  try {
    cq = compileQuery(ir, ir_len);
  } catch (oracle::JavaException& e) {
    std::snprintf(g_err, sizeof g_err, "compile: %s", e.msg.c_str());
    return -(100 + e.code);
  } catch (std::exception& e) {
    std::snprintf(g_err, sizeof g_err, "compile: %s", e.what());
    return -1;
  }
  auto t0 = std::chrono::steady_clock::now();
  std::vector<KeyOut> keys(n_keys);
  if (n_threads <= 0) n_threads = (int)std::max(1u, std::thread::hardware_concurrency());
  std::atomic<uint64_t> next{0};
  auto worker = [&]() {
    for (;;) {
      uint64_t k = next.fetch_add(1);
      if (k >= n_keys) break;
      KeyOut& ko = keys[k];
      oracle::NFA nfa(cq.get());
      oracle::EventView ev{&cq->def.fieldTypes, cols, 0, 0};
      for (uint64_t p = key_off[k]; p < key_off[k + 1]; p++) {
        ev.pos = (int64_t)p;
        ev.ts = ts ? ts[p] : (int64_t)p;
        try {
          auto ms = nfa.matchPattern(ev);
          for (auto& m : ms) ko.matches.push_back(std::move(m));
        } catch (oracle::JavaException& e) {
          ko.err = e.code;
          ko.errPos = (uint32_t)p;
          break;
        }
      }
      ko.runSteps = nfa.runSteps;
      ko.maxLive = nfa.maxLive;
      ko.maxNodes = nfa.buffer.maxNodes;
      ko.puts = nfa.buffer.totalPuts;
    }
  };
  std::vector<std::thread> th;
  for (int i = 0; i < n_threads; i++) th.emplace_back(worker);
  for (auto& t : th) t.join();
  auto t1 = std::chrono::steady_clock::now();

  auto* r = (oracle_result*)std::calloc(1, sizeof(oracle_result));
  r->n_keys = n_keys;
  r->threads = n_threads;
  r->elapsed_s = std::chrono::duration<double>(t1 - t0).count();
  for (auto& k : keys) {
    r->n_matches += k.matches.size();
    for (auto& m : k.matches) r->n_pairs += m.walk.size();
    r->run_steps += k.runSteps;
    r->max_live_runs = std::max(r->max_live_runs, k.maxLive);
    r->max_nodes_key = std::max(r->max_nodes_key, k.maxNodes);
    r->total_puts += k.puts;
    r->max_puts_key = std::max(r->max_puts_key, k.puts);
  }
  r->key = (uint32_t*)std::malloc(sizeof(uint32_t) * (r->n_matches + 1));
  r->emit_pos = (uint32_t*)std::malloc(sizeof(uint32_t) * (r->n_matches + 1));
  r->pair_off = (uint64_t*)std::malloc(sizeof(uint64_t) * (r->n_matches + 1));
  r->pair_pos = (uint32_t*)std::malloc(sizeof(uint32_t) * (r->n_pairs + 1));
  r->pair_stage = (uint16_t*)std::malloc(sizeof(uint16_t) * (r->n_pairs + 1));
  r->err_code = (int32_t*)std::malloc(sizeof(int32_t) * (n_keys + 1));
  r->err_pos = (uint32_t*)std::malloc(sizeof(uint32_t) * (n_keys + 1));
  uint64_t mi = 0, pi = 0;
  r->pair_off[0] = 0;
  for (uint64_t k = 0; k < n_keys; k++) {
    r->err_code[k] = keys[k].err;
    r->err_pos[k] = keys[k].errPos;
    for (auto& m : keys[k].matches) {
      r->key[mi] = (uint32_t)k;
      r->emit_pos[mi] = (uint32_t)m.emitPos;
      for (auto& w : m.walk) {
        r->pair_pos[pi] = (uint32_t)w.offset;
        r->pair_stage[pi] = (uint16_t)w.name;
        pi++;
      }
      mi++;
      r->pair_off[mi] = pi;
    }
  }
  *out = r;
  return 0;
}

void oracle_free(oracle_result* r) {
  if (!r) return;
  std::free(r->key); std::free(r->emit_pos); std::free(r->pair_off); std::free(r->pair_pos);
  std::free(r->pair_stage); std::free(r->err_code); std::free(r->err_pos); std::free(r);
}

// ---- DeweyVersion KAT surface (test:nfa/DeweyVersionTest.java) ----
// ops: 'r' = addRun, 's' = addStage, applied left to right
int oracle_dewey_apply(const char* version, const char* ops, char* out, size_t outlen) {
  auto d = oracle::DeweyVersion::parse(version);
  for (const char* o = ops; *o; o++) d = (*o == 'r') ? d->addRun() : d->addStage();
  std::snprintf(out, outlen, "%s", d->str().c_str());
  return 0;
}
int oracle_dewey_compatible(const char* a, const char* b) {
  return oracle::DeweyVersion::parse(a)->isCompatible(*oracle::DeweyVersion::parse(b)) ? 1 : 0;
}

// ---- KVSharedVersionedBuffer KAT surface (test:nfa/buffer/SharedVersionedBufferTest.java) ----
struct oracle_buffer {
  oracle::Buffer b;
  std::vector<std::shared_ptr<oracle::Stage>> stages;
  oracle::Stage* stage(int name, int type) {
    for (auto& s : stages) if (s->name == name && s->type == type) return s.get();
    auto s = std::make_shared<oracle::Stage>();
    s->name = name;
    s->type = (oracle::StateType)type;
    stages.push_back(s);
    return s.get();
  }
};
oracle_buffer* oracle_buffer_new(void) { return new oracle_buffer(); }
void oracle_buffer_free(oracle_buffer* b) { delete b; }
int oracle_buffer_put_begin(oracle_buffer* b, int name, int type, int64_t off, const char* ver) {
  try { b->b.put(b->stage(name, type), off, oracle::DeweyVersion::parse(ver)); return 0; }
  catch (oracle::JavaException& e) { return e.code; }
}
int oracle_buffer_put(oracle_buffer* b, int name, int type, int64_t off, int pname, int ptype, int64_t poff, const char* ver) {
  try { b->b.put(b->stage(name, type), off, b->stage(pname, ptype), poff, oracle::DeweyVersion::parse(ver)); return 0; }
  catch (oracle::JavaException& e) { return e.code; }
}
// get/remove: writes up to cap (name, offset) pairs in walk order; returns count or -(code)
int oracle_buffer_peek(oracle_buffer* b, int name, int type, int64_t off, const char* ver, int remove,
                       int32_t* names, int64_t* offs, int cap) {
  try {
    auto w = b->b.peek(b->stage(name, type), off, oracle::DeweyVersion::parse(ver), remove != 0);
    int n = 0;
    for (auto& e : w) { if (n < cap) { names[n] = e.name; offs[n] = e.offset; } n++; }
    return n;
  } catch (oracle::JavaException& e) { return -e.code; }
}

}  // extern "C"
