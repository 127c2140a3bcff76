"""Typed predicate / aggregate IR and the tracer that lowers Python lambdas to it.

The reference's `Matcher.matches(K, V, long, States)` (pattern/Matcher.java:22) and
`Aggregator.aggregate(K, V, T)` (pattern/Aggregator.java:24) are opaque Java lambdas.
Here a lambda with the same argument list is *traced* once with proxy objects
(`v.price`, `ts`, `state.get("avg")`, `curr`) and becomes an expression tree that the
C-ABI library compiles into the matching kernel.

Value semantics follow Java exactly, because match sets must be bit-exact:
  * int (I32) / long (I64) arithmetic wraps; `/` and `%` truncate toward zero and raise
    ArithmeticException on a zero divisor (so `/` on integers is *Java* division, not
    Python true division);
  * binary numeric promotion int < long < double (JLS 5.6.2);
  * `state.get(name)` returns a nullable boxed value: using it in arithmetic or a
    comparison unboxes it and raises NullPointerException when it is null
    (pattern/States.java:46-48); `state.getOrElse(name, d)` never does (:53-62);
  * `&`, `|`, `~` are the short-circuit `Matcher.and/or/not` (pattern/Matcher.java:24-70);
    evaluation is left operand first.
"""
from __future__ import annotations

import struct

# ---- types -----------------------------------------------------------------------------
I32, I64, F64, BOOL = 1, 2, 3, 4
TYPE_NAMES = {I32: "int", I64: "long", F64: "double", BOOL: "boolean"}
_TYPE_ALIASES = {
    "int": I32, "i32": I32, "integer": I32, int: I32,
    "long": I64, "i64": I64,
    "double": F64, "f64": F64, float: F64,
    "bool": BOOL, "boolean": BOOL, bool: BOOL,
}


def as_type(t) -> int:
    if t in (I32, I64, F64, BOOL):
        return t
    if isinstance(t, str):
        t = t.lower()
    try:
        return _TYPE_ALIASES[t]
    except (KeyError, TypeError):
        raise TypeError(f"unknown value type {t!r} (use 'int', 'long' or 'double')")


def _promote(a: int, b: int) -> int:
    if BOOL in (a, b):
        raise TypeError("boolean operands are not numeric")
    return max(a, b)  # I32 < I64 < F64


# ---- opcodes (mirrored by include/cep.h CEP_OP_* and the oracle parser) ------------------
OP_CONST_I32, OP_CONST_I64, OP_CONST_F64, OP_CONST_BOOL = 0x01, 0x02, 0x03, 0x04
OP_FIELD, OP_TS, OP_STATE_GET, OP_STATE_GET_OR, OP_CURR = 0x05, 0x06, 0x07, 0x08, 0x09
OP_ADD, OP_SUB, OP_MUL, OP_DIV, OP_REM, OP_NEG = 0x10, 0x11, 0x12, 0x13, 0x14, 0x15
OP_CAST = 0x18
OP_LT, OP_LE, OP_GT, OP_GE, OP_EQ, OP_NE = 0x20, 0x21, 0x22, 0x23, 0x24, 0x25
OP_AND, OP_OR, OP_NOT = 0x30, 0x31, 0x32

_INT32_MIN, _INT32_MAX = -(1 << 31), (1 << 31) - 1
_INT64_MIN, _INT64_MAX = -(1 << 63), (1 << 63) - 1


class Expr:
    """A node of the typed IR. `type` is I32/I64/F64/BOOL; `nullable` marks a boxed value."""

    type: int = 0
    nullable: bool = False
    __hash__ = object.__hash__

    # -- numeric operators (Java semantics) --
    def _bin(self, other, op, swap=False):
        o = lift(other)
        a, b = (o, self) if swap else (self, o)
        return Arith(op, a, b)

    def __add__(self, o): return self._bin(o, OP_ADD)
    def __radd__(self, o): return self._bin(o, OP_ADD, True)
    def __sub__(self, o): return self._bin(o, OP_SUB)
    def __rsub__(self, o): return self._bin(o, OP_SUB, True)
    def __mul__(self, o): return self._bin(o, OP_MUL)
    def __rmul__(self, o): return self._bin(o, OP_MUL, True)
    def __truediv__(self, o): return self._bin(o, OP_DIV)
    def __rtruediv__(self, o): return self._bin(o, OP_DIV, True)
    __floordiv__ = __truediv__
    __rfloordiv__ = __rtruediv__
    def __mod__(self, o): return self._bin(o, OP_REM)
    def __rmod__(self, o): return self._bin(o, OP_REM, True)
    def __neg__(self): return Neg(self)
    def __pos__(self): return self

    # -- comparisons --
    def __lt__(self, o): return Cmp(OP_LT, self, lift(o))
    def __le__(self, o): return Cmp(OP_LE, self, lift(o))
    def __gt__(self, o): return Cmp(OP_GT, self, lift(o))
    def __ge__(self, o): return Cmp(OP_GE, self, lift(o))
    def __eq__(self, o): return Cmp(OP_EQ, self, lift(o))  # type: ignore[override]
    def __ne__(self, o): return Cmp(OP_NE, self, lift(o))  # type: ignore[override]

    # -- boolean (Matcher.and / or / not, short-circuit) --
    def __and__(self, o): return And(self, lift(o))
    def __rand__(self, o): return And(lift(o), self)
    def __or__(self, o): return Or(self, lift(o))
    def __ror__(self, o): return Or(lift(o), self)
    def __invert__(self): return Not(self)

    def __bool__(self):
        raise TypeError("a traced CEP expression has no Python truth value: use & | ~ "
                        "instead of and/or/not, and no if/else on event values")

    # -- Java casts --
    def as_int(self): return Cast(self, I32)
    def as_long(self): return Cast(self, I64)
    def as_double(self): return Cast(self, F64)

    def equals(self, other):
        """`value.equals(x)` of the reference's string tests (NFATest.java:46): code equality."""
        return self == other

    def children(self):
        return ()


def lift(x) -> Expr:
    if isinstance(x, Expr):
        return x
    if isinstance(x, bool):
        return Const(BOOL, x)
    if isinstance(x, int):
        if _INT32_MIN <= x <= _INT32_MAX:
            return Const(I32, x)
        if _INT64_MIN <= x <= _INT64_MAX:
            return Const(I64, x)
        raise OverflowError(f"integer literal {x} does not fit a Java long")
    if isinstance(x, float):
        return Const(F64, x)
    if isinstance(x, JLit):
        return Const(x.t, x.v)
    raise TypeError(f"cannot use {type(x).__name__} in a CEP expression")


class JLit:
    """Explicitly typed literal: `J.long(0)` is Java's `0L`."""

    def __init__(self, t, v):
        self.t, self.v = t, v


class J:
    @staticmethod
    def int(v): return JLit(I32, int(v))

    @staticmethod
    def long(v): return JLit(I64, int(v))

    @staticmethod
    def double(v): return JLit(F64, float(v))


class Const(Expr):
    def __init__(self, t, v):
        self.type = t
        if t == I32:
            v = int(v)
            if not _INT32_MIN <= v <= _INT32_MAX:
                raise OverflowError(v)
        elif t == I64:
            v = int(v)
            if not _INT64_MIN <= v <= _INT64_MAX:
                raise OverflowError(v)
        elif t == F64:
            v = float(v)
        else:
            v = bool(v)
        self.v = v


class Field(Expr):
    def __init__(self, idx, t, name):
        self.idx, self.type, self.name = idx, t, name


class Ts(Expr):
    type = I64


class StateGet(Expr):
    nullable = True

    def __init__(self, idx, t, name):
        self.idx, self.type, self.name = idx, t, name


class StateGetOr(Expr):
    def __init__(self, idx, t, name, default: Expr):
        if default.nullable or default.type != t:
            raise TypeError(f"getOrElse('{name}', ...) default must be a {TYPE_NAMES[t]} value "
                            f"(the reference would raise ClassCastException)")
        self.idx, self.type, self.name, self.default = idx, t, name, default

    def children(self):
        return (self.default,)


class Curr(Expr):
    nullable = True

    def __init__(self, t):
        self.type = t


def _widen(e: Expr, t: int) -> Expr:
    """Binary numeric promotion made explicit: evaluators never promote implicitly."""
    if e.type == t:
        return e
    if isinstance(e, Const):
        return Const(t, e.v)
    return Cast(e, t)


class Arith(Expr):
    def __init__(self, op, a: Expr, b: Expr):
        self.type = _promote(a.type, b.type)
        self.op, self.a, self.b = op, _widen(a, self.type), _widen(b, self.type)

    def children(self):
        return (self.a, self.b)


class Neg(Expr):
    def __init__(self, a: Expr):
        if a.type == BOOL:
            raise TypeError("cannot negate a boolean")
        self.a, self.type = a, a.type

    def children(self):
        return (self.a,)


class Cast(Expr):
    def __init__(self, a: Expr, t):
        if a.type == BOOL or t == BOOL:
            raise TypeError("no numeric<->boolean casts in Java")
        self.a, self.type = a, t

    def children(self):
        return (self.a,)


class Cmp(Expr):
    type = BOOL

    def __init__(self, op, a: Expr, b: Expr):
        if a.type == BOOL or b.type == BOOL:
            if not (a.type == BOOL and b.type == BOOL and op in (OP_EQ, OP_NE)):
                raise TypeError("ordered comparison of booleans")
            self.t = BOOL
        else:
            self.t = _promote(a.type, b.type)
            a, b = _widen(a, self.t), _widen(b, self.t)
        self.op, self.a, self.b = op, a, b

    def children(self):
        return (self.a, self.b)


class _Bool(Expr):
    type = BOOL


class And(_Bool):
    def __init__(self, a, b):
        _check_bool(a), _check_bool(b)
        self.a, self.b = a, b

    def children(self):
        return (self.a, self.b)


class Or(_Bool):
    def __init__(self, a, b):
        _check_bool(a), _check_bool(b)
        self.a, self.b = a, b

    def children(self):
        return (self.a, self.b)


class Not(_Bool):
    def __init__(self, a):
        _check_bool(a)
        self.a = a

    def children(self):
        return (self.a,)


def _check_bool(e: Expr):
    if e.type != BOOL:
        raise TypeError(f"expected a boolean expression, got {TYPE_NAMES.get(e.type, e.type)}")


TRUE = Const(BOOL, True)


# ---- tracing proxies ---------------------------------------------------------------------
class EventProxy:
    """The `value` argument of a traced lambda: attribute access yields typed field loads."""

    def __init__(self, schema):
        object.__setattr__(self, "_schema", schema)

    def __getattr__(self, name):
        s = object.__getattribute__(self, "_schema")
        return s.field_expr(name)

    def equals(self, other):
        # single-field string value, as in the reference's NFATest (value.equals("A"))
        s = object.__getattribute__(self, "_schema")
        return s.value_expr() == s.encode_literal(other)

    def __eq__(self, other):  # type: ignore[override]
        return self.equals(other)

    __hash__ = object.__hash__


class StatesProxy:
    """The `States` argument (pattern/States.java): `get` (nullable) and `getOrElse`."""

    def __init__(self, state_types: dict, state_index: dict):
        self._types, self._index = state_types, state_index

    def _lookup(self, name, t):
        if name not in self._index:
            raise KeyError(f"state '{name}' is read but never folded in this query; "
                           "declare it with .fold() (the reference would read null)")
        st = self._types[name]
        if t is not None and as_type(t) != st:
            raise TypeError(f"state '{name}' is a {TYPE_NAMES[st]}, read as {TYPE_NAMES[as_type(t)]}")
        return self._index[name], st

    def get(self, name, type=None):
        idx, t = self._lookup(name, type)
        return StateGet(idx, t, name)

    def getOrElse(self, name, default, type=None):
        idx, t = self._lookup(name, type)
        d = lift(default)
        if d.type != t and d.type in (I32, I64) and t in (I32, I64, F64) and isinstance(d, Const):
            d = Const(t, d.v)  # literal default retyped to the state's boxed type
        return StateGetOr(idx, t, name, d)

    get_or_else = getOrElse


class _KeyProxy:
    def __getattr__(self, name):
        raise TypeError("predicates on the record key are not supported by the columnar "
                        "engine (the key is implicit under key partitioning)")


def trace_matcher(fn, schema, state_types, state_index) -> Expr:
    if isinstance(fn, Expr):
        e = fn
    elif isinstance(fn, MatcherExpr):
        e = fn.lower(schema, state_types, state_index)
    else:
        e = lift(fn(_KeyProxy(), EventProxy(schema), Ts(), StatesProxy(state_types, state_index)))
    _check_bool(e)
    _check_no_curr(e)
    return e


def trace_aggregator(fn, schema, t) -> Expr:
    if isinstance(fn, Expr):
        e = fn
    else:
        e = lift(fn(_KeyProxy(), EventProxy(schema), Curr(t)))
    if e.type != t:
        if isinstance(e, Const) and e.type in (I32, I64) and t in (I32, I64, F64):
            e = Const(t, e.v)
        elif not e.nullable and e.type in (I32, I64, F64) and t in (I64, F64) and e.type < t:
            e = Cast(e, t)  # Java widening when the lambda returns a narrower primitive
        else:
            raise TypeError(f"fold returns {TYPE_NAMES.get(e.type)} but the state is "
                            f"{TYPE_NAMES[t]}")
    _check_no_state(e)
    return e


def _walk(e: Expr):
    yield e
    for c in e.children():
        yield from _walk(c)


def _check_no_curr(e):
    for n in _walk(e):
        if isinstance(n, Curr):
            raise TypeError("`curr` is only available inside fold()")


def _check_no_state(e):
    for n in _walk(e):
        if isinstance(n, (StateGet, StateGetOr)):
            raise TypeError("an Aggregator has no States argument (pattern/Aggregator.java:24)")


def reads_state(e: Expr) -> bool:
    return any(isinstance(n, (StateGet, StateGetOr)) for n in _walk(e))


def is_total(e: Expr) -> bool:
    """True when evaluating `e` can never raise (no nullable unboxing, no integer division)."""
    for n in _walk(e):
        if isinstance(n, (StateGet, Curr)):
            return False
        if isinstance(n, Arith) and n.op in (OP_DIV, OP_REM) and n.type in (I32, I64):
            if not (isinstance(n.b, Const) and n.b.v != 0):
                return False
    return True


# ---- Matcher combinators (pattern/Matcher.java:24-34) -------------------------------------
class MatcherExpr:
    """Deferred matcher composition so that lambdas and IR can be mixed, e.g.
    `Matcher.and_(lambda k, v, ts, s: v.volume > 1000, other)`."""

    def __init__(self, kind, *parts):
        self.kind, self.parts = kind, parts

    def lower(self, schema, st, si) -> Expr:
        ps = [trace_matcher(p, schema, st, si) for p in self.parts]
        if self.kind == "not":
            return Not(ps[0])
        if self.kind == "and":
            return And(ps[0], ps[1])
        return Or(ps[0], ps[1])


class Matcher:
    @staticmethod
    def not_(m): return MatcherExpr("not", m)

    @staticmethod
    def and_(a, b): return MatcherExpr("and", a, b)

    @staticmethod
    def or_(a, b): return MatcherExpr("or", a, b)


# ---- serialization -----------------------------------------------------------------------
def serialize(e: Expr, out: bytearray):
    """Prefix encoding consumed by libcep's compiler and the oracle (format: include/cep.h)."""
    if isinstance(e, Const):
        if e.type == I32:
            out += struct.pack("<Bi", OP_CONST_I32, e.v)
        elif e.type == I64:
            out += struct.pack("<Bq", OP_CONST_I64, e.v)
        elif e.type == F64:
            out += struct.pack("<Bd", OP_CONST_F64, e.v)
        else:
            out += struct.pack("<BB", OP_CONST_BOOL, 1 if e.v else 0)
    elif isinstance(e, Field):
        out += struct.pack("<BH", OP_FIELD, e.idx)
    elif isinstance(e, Ts):
        out += struct.pack("<B", OP_TS)
    elif isinstance(e, StateGet):
        out += struct.pack("<BH", OP_STATE_GET, e.idx)
    elif isinstance(e, StateGetOr):
        out += struct.pack("<BH", OP_STATE_GET_OR, e.idx)
        serialize(e.default, out)
    elif isinstance(e, Curr):
        out += struct.pack("<B", OP_CURR)
    elif isinstance(e, Arith):
        out += struct.pack("<BB", e.op, e.type)
        serialize(e.a, out)
        serialize(e.b, out)
    elif isinstance(e, Neg):
        out += struct.pack("<BB", OP_NEG, e.type)
        serialize(e.a, out)
    elif isinstance(e, Cast):
        out += struct.pack("<BBB", OP_CAST, e.a.type, e.type)
        serialize(e.a, out)
    elif isinstance(e, Cmp):
        out += struct.pack("<BB", e.op, e.t)
        serialize(e.a, out)
        serialize(e.b, out)
    elif isinstance(e, And):
        out += struct.pack("<B", OP_AND)
        serialize(e.a, out)
        serialize(e.b, out)
    elif isinstance(e, Or):
        out += struct.pack("<B", OP_OR)
        serialize(e.a, out)
        serialize(e.b, out)
    elif isinstance(e, Not):
        out += struct.pack("<B", OP_NOT)
        serialize(e.a, out)
    else:
        raise TypeError(f"cannot serialize {type(e).__name__}")


def to_str(e: Expr) -> str:
    """Readable form (debugging / error messages)."""
    ops = {OP_ADD: "+", OP_SUB: "-", OP_MUL: "*", OP_DIV: "/", OP_REM: "%", OP_LT: "<",
           OP_LE: "<=", OP_GT: ">", OP_GE: ">=", OP_EQ: "==", OP_NE: "!="}
    if isinstance(e, Const):
        return repr(e.v) + ("L" if e.type == I64 else "")
    if isinstance(e, Field):
        return f"v.{e.name}"
    if isinstance(e, Ts):
        return "ts"
    if isinstance(e, StateGet):
        return f"state.get({e.name!r})"
    if isinstance(e, StateGetOr):
        return f"state.getOrElse({e.name!r}, {to_str(e.default)})"
    if isinstance(e, Curr):
        return "curr"
    if isinstance(e, (Arith, Cmp)):
        return f"({to_str(e.a)} {ops[e.op]} {to_str(e.b)})"
    if isinstance(e, Neg):
        return f"-{to_str(e.a)}"
    if isinstance(e, Cast):
        return f"({TYPE_NAMES[e.type]}){to_str(e.a)}"
    if isinstance(e, And):
        return f"({to_str(e.a)} && {to_str(e.b)})"
    if isinstance(e, Or):
        return f"({to_str(e.a)} || {to_str(e.b)})"
    if isinstance(e, Not):
        return f"!{to_str(e.a)}"
    return "?"
