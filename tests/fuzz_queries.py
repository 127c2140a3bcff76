"""Seeded random queries and streams for differential testing (GPU vs oracle).

Queries mix every cardinality and selection strategy, fold state reads (`get`, nullable,
and `getOrElse`), integer division (ArithmeticException) and short-circuit logic, so the
runs branch, share buffer nodes and hit the reference's exception paths.
"""
import random

import numpy as np

from kafkastreams_cep_amd import EventSchema, QueryBuilder
from kafkastreams_cep_amd.pattern import Cardinality, SelectStrategy

SCHEMA = lambda: EventSchema({"a": "int", "b": "int"})


def _atom(rng, states):
    f = rng.choice(["a", "b"])
    c = rng.randint(0, 9)
    kind = rng.random()
    if states and kind < 0.25:
        st = rng.choice(states)
        if rng.random() < 0.5:
            return lambda k, v, ts, s, f=f, st=st: getattr(v, f) > s.get(st)
        d = rng.randint(0, 9)
        return lambda k, v, ts, s, f=f, st=st, d=d: getattr(v, f) < s.getOrElse(st, d)
    if kind < 0.32:
        return lambda k, v, ts, s, f=f, c=c: (getattr(v, f) + 1) / (getattr(v, "b") - 3) > c - 5
    op = rng.choice(["<", ">", "<=", ">=", "==", "!="])
    return {"<": lambda k, v, ts, s, f=f, c=c: getattr(v, f) < c,
            ">": lambda k, v, ts, s, f=f, c=c: getattr(v, f) > c,
            "<=": lambda k, v, ts, s, f=f, c=c: getattr(v, f) <= c,
            ">=": lambda k, v, ts, s, f=f, c=c: getattr(v, f) >= c,
            "==": lambda k, v, ts, s, f=f, c=c: getattr(v, f) == c,
            "!=": lambda k, v, ts, s, f=f, c=c: getattr(v, f) != c}[op]


def _pred(rng, states):
    a = _atom(rng, states)
    r = rng.random()
    if r < 0.2:
        b = _atom(rng, states)
        return lambda k, v, ts, s: a(k, v, ts, s) & b(k, v, ts, s)
    if r < 0.35:
        b = _atom(rng, states)
        return lambda k, v, ts, s: a(k, v, ts, s) | b(k, v, ts, s)
    if r < 0.45:
        return lambda k, v, ts, s: ~a(k, v, ts, s)
    return a


def random_query(seed: int, allow_any: bool = True):
    rng = random.Random(seed)
    S = SCHEMA()
    m = rng.randint(1, 4)
    states = []
    qb = QueryBuilder(S)
    p = None
    for i in range(m):
        sb = (qb.select(rng.choice([None, "x", "y", f"s{i}"])) if i == 0 else p.select(rng.choice([None, f"s{i}", "x"])))
        last = i == m - 1
        card = Cardinality.ONE if last or rng.random() < 0.45 else rng.choice(
            [Cardinality.OPTIONAL, Cardinality.ZERO_OR_MORE, Cardinality.ONE_OR_MORE])
        strat = rng.choice([SelectStrategy.STRICT_CONTIGUITY, SelectStrategy.SKIP_TIL_NEXT_MATCH]
                           + ([SelectStrategy.SKIP_TIL_ANY_MATCH] if allow_any else []))
        if card == Cardinality.OPTIONAL:
            sb = sb.optional()
        elif card == Cardinality.ZERO_OR_MORE:
            sb = sb.zeroOrMore()
        elif card == Cardinality.ONE_OR_MORE:
            sb = sb.oneOrMore()
        if strat == SelectStrategy.SKIP_TIL_NEXT_MATCH:
            sb = sb.skipTillNextMatch()
        elif strat == SelectStrategy.SKIP_TIL_ANY_MATCH:
            sb = sb.skipTillAnyMatch()
        pb = sb.where(_pred(rng, states))
        if rng.random() < 0.5:
            st = rng.choice(["u", "w"])
            kind = rng.randint(0, 2)
            if kind == 0:
                pb = pb.fold(st, lambda k, v, c: v.a, type="int")
            elif kind == 1:
                pb = pb.fold(st, lambda k, v, c: c + v.b, type="int")  # NPE on a null curr
            else:
                pb = pb.fold(st, lambda k, v, c: v.a * 2 - v.b, type="int")
            if st not in states:
                states.append(st)
        if rng.random() < 0.3:
            pb = pb.within(rng.randint(1, 5), __import__("kafkastreams_cep_amd").TimeUnit.MILLISECONDS)
        p = pb.build() if last else pb.then()
    return p


def random_stream(seed: int, n_keys: int, max_len: int):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, max_len + 1, size=n_keys)
    off = np.zeros(n_keys + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    n = int(off[-1])
    a = rng.integers(0, 10, size=n).astype(np.int32)
    b = rng.integers(0, 10, size=n).astype(np.int32)
    return off, [a, b]
