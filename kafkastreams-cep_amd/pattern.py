"""Query DSL — the reference's fluent API, same names and argument meaning.

  QueryBuilder.select([name])                       pattern/QueryBuilder.java:28-39
  SelectBuilder.optional/oneOrMore/zeroOrMore/
      skipTillNextMatch/skipTillAnyMatch/
      strictContiguity/where                        pattern/SelectBuilder.java:26-59
  PredicateBuilder.and_/fold/within/then/build      pattern/PredicateBuilder.java:34-55
  Pattern (chain via ancestor, level, name)         pattern/Pattern.java:25-211

`and` is a Python keyword, so `PredicateBuilder.and` is spelled `and_`.  Lambdas take the
reference's arguments — `where(lambda k, v, ts, state: ...)`,
`fold(name, lambda k, v, curr: ...)` — and are traced to the typed IR of `expr.py`.
`Pattern.to_ir()` serialises the chain for `cep_query_compile` (include/cep.h).
"""
from __future__ import annotations

import enum
import struct

from . import expr as X
from .schema import EventSchema


class Cardinality(enum.IntEnum):   # pattern/Pattern.java:27-42 (values are the IR codes)
    ONE = 0
    OPTIONAL = 1
    ZERO_OR_MORE = 2
    ONE_OR_MORE = 3


class SelectStrategy(enum.IntEnum):  # pattern/Pattern.java:44-57
    STRICT_CONTIGUITY = 0
    SKIP_TIL_NEXT_MATCH = 1
    SKIP_TIL_ANY_MATCH = 2


class TimeUnit(enum.Enum):  # java.util.concurrent.TimeUnit subset used by within()
    MILLISECONDS = 1
    SECONDS = 1000
    MINUTES = 60_000
    HOURS = 3_600_000
    DAYS = 86_400_000

    def toMillis(self, t: int) -> int:
        return int(t) * self.value


class Pattern:
    """One `select` of the chain (pattern/Pattern.java:59-211)."""

    def __init__(self, level: int = 0, name: str | None = None, ancestor: "Pattern | None" = None,
                 schema: EventSchema | None = None):
        self.level = level
        self.name = name
        self.ancestor = ancestor
        self.schema = schema if schema is not None else (ancestor.schema if ancestor else None)
        self.strategy = SelectStrategy.STRICT_CONTIGUITY   # Pattern.java:116
        self.cardinality = Cardinality.ONE                  # Pattern.java:75
        self.predicates: list = []                          # AND-ed in call order (:145-150)
        self.aggregates: list = []                          # (state, fn, type) in call order
        self.window_time: int | None = None
        self.window_unit: TimeUnit | None = None

    # Pattern.select(name) (Pattern.java:125-128)
    def select(self, name: str | None = None) -> "SelectBuilder":
        if name is not None:
            self.name = name
        return SelectBuilder(self)

    def getName(self) -> str:  # Pattern.java:160-162
        return self.name if self.name is not None else str(self.level)

    def getAncestor(self):
        return self.ancestor

    def __iter__(self):  # PatternIterator, last -> first (Pattern.java:189-210)
        p = self
        while p is not None:
            yield p
            p = p.ancestor

    def chain(self) -> list["Pattern"]:
        """Patterns first -> last."""
        return list(self)[::-1]

    # -- lowering -----------------------------------------------------------------------
    def _states(self):
        """Fold-state registry: name -> (index, type), in first-declaration order."""
        types: dict[str, int] = {}
        order: list[str] = []
        for p in self.chain():
            for name, fn, t in p.aggregates:
                if t is not None:
                    t = X.as_type(t)
                    if name in types and types[name] != t:
                        raise TypeError(f"state '{name}' folded as both {X.TYPE_NAMES[types[name]]} "
                                        f"and {X.TYPE_NAMES[t]} (ClassCastException in the reference)")
                    types[name] = t
                if name not in order:
                    order.append(name)
        for p in self.chain():  # infer undeclared types from the aggregator's own result
            for name, fn, t in p.aggregates:
                if name not in types:
                    types[name] = _infer_fold_type(fn, p.schema)
        return order, types

    def to_ir(self, semantic_within: bool = False) -> bytes:
        """The query as libcep IR.  semantic_within=False (parity mode, the default) keeps the
        reference's WITHIN exactly: it never prunes, because every non-begin run sits in an
        epsilon stage whose window is -1 (nfa/Stage.java:42-46, ComputationStage.java:98-100).
        semantic_within=True is the SASE semantics the README states (README.md:19-28,
        "WITHIN 1 hour"): an epsilon stage keeps the window of the stage it copies, so a run
        whose first event is more than the window older than the current event is dropped
        (NFA.java:143-144's check, then removePattern).  IR version 2 carries the flag."""
        chain = self.chain()
        schema = self.schema
        if schema is None:
            raise ValueError("QueryBuilder needs a schema (EventSchema) to lower lambdas")
        order, types = self._states()
        index = {n: i for i, n in enumerate(order)}
        names: list[str] = []
        for p in chain:
            if p.getName() not in names:
                names.append(p.getName())
        out = bytearray(b"CEPQ")
        if semantic_within:
            out += struct.pack("<II", 2, 1)  # version 2, flags bit0: semantic WITHIN
        else:
            out += struct.pack("<I", 1)
        out += struct.pack("<H", len(schema.names))
        for n, t in zip(schema.names, schema.types):
            out += struct.pack("<B", t) + _str(n)
        out += struct.pack("<H", len(order))
        for n in order:
            out += struct.pack("<B", types[n]) + _str(n)
        out += struct.pack("<H", len(names))
        for n in names:
            out += _str(n)
        out += struct.pack("<H", len(chain))
        for p in chain:
            out += struct.pack("<HBB", names.index(p.getName()), int(p.cardinality), int(p.strategy))
            if p.window_time is not None:
                out += struct.pack("<Bq", 1, p.window_unit.toMillis(p.window_time))
            else:
                out += struct.pack("<Bq", 0, -1)
            pred = None
            for m in p.predicates:
                e = X.trace_matcher(m, schema, types, index)
                pred = e if pred is None else X.And(pred, e)
            if pred is None:
                out += struct.pack("<B", 0)
            else:
                out += struct.pack("<B", 1)
                X.serialize(pred, out)
            out += struct.pack("<H", len(p.aggregates))
            for name, fn, _t in p.aggregates:
                e = X.trace_aggregator(fn, schema, types[name])
                out += struct.pack("<H", index[name])
                X.serialize(e, out)
        return bytes(out)

    def describe(self) -> str:
        lines = []
        order, types = self._states()
        index = {n: i for i, n in enumerate(order)}
        for p in self.chain():
            preds = [X.to_str(X.trace_matcher(m, p.schema, types, index)) for m in p.predicates]
            lines.append(f"{p.getName()}: {p.cardinality.name} {p.strategy.name} where "
                         f"{' && '.join(preds) or '<none>'}"
                         + (f" within {p.window_unit.toMillis(p.window_time)}ms" if p.window_time else ""))
        return "\n".join(lines)


def _infer_fold_type(fn, schema):
    for t in (X.I32, X.I64, X.F64):
        try:
            e = X.trace_aggregator(fn, schema, t)
        except TypeError:
            continue
        if e.type == t:
            return t
    raise TypeError("cannot infer the fold state type; pass type='int'|'long'|'double'")


def _str(s: str) -> bytes:
    b = s.encode("utf-8")
    return struct.pack("<H", len(b)) + b


class QueryBuilder:
    """pattern/QueryBuilder.java:20-40.  `schema` plays the role of the generic `V`."""

    def __init__(self, schema: EventSchema | None = None):
        self.schema = schema

    def select(self, name: str | None = None) -> "SelectBuilder":
        return SelectBuilder(Pattern(0, name, None, self.schema))


class SelectBuilder:
    """pattern/SelectBuilder.java:19-61."""

    def __init__(self, pattern: Pattern):
        self.pattern = pattern

    def optional(self):
        self.pattern.cardinality = Cardinality.OPTIONAL
        return self

    def oneOrMore(self):
        self.pattern.cardinality = Cardinality.ONE_OR_MORE
        return self

    def zeroOrMore(self):
        self.pattern.cardinality = Cardinality.ZERO_OR_MORE
        return self

    def skipTillNextMatch(self):
        self.pattern.strategy = SelectStrategy.SKIP_TIL_NEXT_MATCH
        return self

    def skipTillAnyMatch(self):
        self.pattern.strategy = SelectStrategy.SKIP_TIL_ANY_MATCH
        return self

    def strictContiguity(self):
        self.pattern.strategy = SelectStrategy.STRICT_CONTIGUITY
        return self

    def where(self, predicate) -> "PredicateBuilder":
        if predicate is None:
            raise ValueError("predicate cannot be null")  # Stage.java:159
        self.pattern.predicates.append(predicate)
        return PredicateBuilder(self.pattern)


class PredicateBuilder:
    """pattern/PredicateBuilder.java:22-56."""

    def __init__(self, pattern: Pattern):
        self.pattern = pattern

    def and_(self, predicate) -> "PredicateBuilder":
        self.pattern.predicates.append(predicate)
        return self

    def fold(self, state: str, aggregator, type=None) -> "PredicateBuilder":
        self.pattern.aggregates.append((state, aggregator, type))
        return self

    def within(self, time: int, unit: TimeUnit) -> "PredicateBuilder":
        self.pattern.window_time, self.pattern.window_unit = int(time), unit
        return self

    def then(self) -> Pattern:
        p = self.pattern
        return Pattern(p.level + 1, None, p, p.schema)

    def build(self) -> Pattern:
        return self.pattern


# Pattern.then() returns a Pattern whose select() continues the chain (PredicateBuilder.java:49-51)
