"""Reference queries and synthetic workload definitions (BASELINE.json configs 1-5).

Queries are the reference's own (README.md:33-49, test:nfa/NFATest.java:41-245,
test:demo/CEPStockKStreamsDemo.java:37-53) written with this package's DSL, plus the
synthetic configs of SURVEY §8d.

Synthetic streams are generated directly in key-partitioned (CSR) form: key k holds n_k
events (mean M, spread ±⌊√M⌋, like a uniform key hash would give), and every event value
is a counter-based SplitMix64 hash of (seed, key, index-in-key), so any subset of keys can
be regenerated independently (the CPU-baseline sample) and the GPU generator
(csrc/synth_gen.hip) reproduces this module bit for bit.  Event id = CSR position.
"""
from __future__ import annotations

import dataclasses

import numpy as np

from .expr import J
from .pattern import QueryBuilder, TimeUnit
from .schema import EventSchema

M64 = (1 << 64) - 1


# ------------------------------------------------------------------------------ queries
def stock_query(variant: str = "readme", schema: EventSchema | None = None,
                begin_volume: int = 1000, dip_num: int = 80):
    """SEQ(Stock+ a[], Stock b) — README.md:33-49 ("readme": oneOrMore, int casts),
    NFATest.java:215-231 ("test": zeroOrMore, getOrElse), demo ("demo": long fields).
    `begin_volume` / `dip_num` parameterise config 5's 64 query variants
    (a[1].volume > begin_volume, b.volume < dip_num% of a[a.LEN].volume)."""
    if schema is None:
        schema = EventSchema({"price": "long", "volume": "long"}) if variant == "demo" else \
            EventSchema({"price": "int", "volume": "int"})
    dip = dip_num / 100.0
    q = QueryBuilder(schema).select()
    p = q.where(lambda k, v, ts, s: v.volume > begin_volume).fold("avg", lambda k, v, c: v.price).then()
    sb = p.select()
    sb = sb.oneOrMore() if variant == "readme" else sb.zeroOrMore()
    p = (sb.skipTillNextMatch()
         .where(lambda k, v, ts, s: v.price > s.get("avg"))
         .fold("avg", lambda k, v, c: (c + v.price) / 2)
         .fold("volume", lambda k, v, c: v.volume)
         .then())
    if variant == "readme":
        pred = lambda k, v, ts, s: v.volume < dip * s.get("volume")
    elif variant == "demo":
        pred = lambda k, v, ts, s: v.volume < dip * s.getOrElse("volume", J.long(0))
    else:
        pred = lambda k, v, ts, s: v.volume < dip * s.getOrElse("volume", 0)
    return p.select().skipTillNextMatch().where(pred).within(1, TimeUnit.HOURS).build()


def strict_abc_query(schema: EventSchema | None = None):
    """Config 2: SEQ(A, B, C) strict contiguity, A: v<4, B: 4<=v<8, C: v>=8."""
    schema = schema or EventSchema({"v": "int"})
    return (QueryBuilder(schema)
            .select("A").where(lambda k, v, ts, s: v.v < 4).then()
            .select("B").where(lambda k, v, ts, s: (v.v >= 4) & (v.v < 8)).then()
            .select("C").where(lambda k, v, ts, s: v.v >= 8).build())


def any_kleene_query(schema: EventSchema | None = None, carry_volume: bool = False):
    """Config 4: skip_till_any Kleene+ with folds and a tight WITHIN (run-explosion stress).

    As written the query throws NullPointerException in the reference on
    about half of the keys: a branched run copies only the current stage's aggregates
    (NFA.java:243, ValueStore.java:92-97), so S2's `state.get("volume")` reads null on every
    run branched at S1.  `carry_volume=True` is the stress workload SURVEY §8d intends ("no
    Appendix-C exception path fires"): S1 also folds `volume` (keeping its value), so a
    branch at S1 copies it, and S2 reads it with `getOrElse("volume", 0)` (a run branched at
    S2, which has no aggregates, carries no folds at all).  No key throws; runs accumulate at
    S1/S2 and orphan buffer nodes grow.  Oracle, keys 0, 500, ...: 0 of 2000 keys
    throw, up to 23 live runs and 1003 buffer nodes per key, 1566 matches.  The literal query
    stays the parity case."""
    schema = schema or EventSchema({"price": "int", "volume": "int"})
    s1 = (QueryBuilder(schema)
          .select("S0").where(lambda k, v, ts, s: v.volume > 1000)
          .fold("avg", lambda k, v, c: v.price).fold("volume", lambda k, v, c: v.volume).then()
          .select("S1").oneOrMore().skipTillAnyMatch()
          .where(lambda k, v, ts, s: v.price > s.get("avg"))
          .fold("avg", lambda k, v, c: (c + v.price) / 2).fold("sum", lambda k, v, c: v.price, type="int"))
    if carry_volume:
        s1 = s1.fold("volume", lambda k, v, c: c)
    s2 = s1.then().select("S2").skipTillAnyMatch()
    if carry_volume:
        s2 = s2.where(lambda k, v, ts, s: v.volume * 5 < 4 * s.getOrElse("volume", 0))
    else:
        s2 = s2.where(lambda k, v, ts, s: v.volume * 5 < 4 * s.get("volume"))
    return s2.within(10, TimeUnit.MILLISECONDS).build()


def multi_queries(n: int = 64):
    """Config 5: 64 stock-query variants over one shared stream."""
    return [stock_query("readme", begin_volume=1000 + 10 * (q % 8), dip_num=60 + 5 * (q // 8)) for q in range(n)]


# ------------------------------------------------------------------------------ generator
def splitmix64(x: np.ndarray) -> np.ndarray:
    """SplitMix64 finaliser over uint64 arrays (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _h(seed: int, key: np.ndarray, j: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = np.uint64(seed) ^ (key.astype(np.uint64) * np.uint64(0xD1B54A32D192ED03)) ^ \
            (j.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15))
    return splitmix64(splitmix64(x))


@dataclasses.dataclass
class SynthConfig:
    """One synthetic stream: `kind` is "stock" (price/volume random walk) or "abc" (v%16)."""
    name: str
    kind: str
    n_keys: int
    mean_events: int
    seed: int
    key_base: int = 0  # global id of key 0 (shards of one stream use disjoint key ranges)

    @property
    def spread(self) -> int:
        return int(np.floor(np.sqrt(self.mean_events)))


CONFIGS = {
    2: SynthConfig("cfg2_strict_abc", "abc", 10_000, 10_000, 0xCE90000 + 2),
    3: SynthConfig("cfg3_stock", "stock", 1_000_000, 1_000, 0xCE90000 + 3),
    4: SynthConfig("cfg4_any_kleene", "stock", 1_000_000, 1_000, 0xCE90000 + 3),  # same stream as cfg 3
    5: SynthConfig("cfg5_multi_query", "stock", 1_000_000, 1_000, 0xCE90000 + 3),
}


def key_counts(cfg: SynthConfig, keys: np.ndarray | None = None) -> np.ndarray:
    keys = np.arange(cfg.n_keys, dtype=np.uint64) if keys is None else np.asarray(keys, np.uint64)
    gk = keys + np.uint64(cfg.key_base)
    j = np.full(gk.shape, 0xFFFFFFFF, dtype=np.uint64)
    h = _h(cfg.seed, gk, j)
    s = cfg.spread
    return (cfg.mean_events - s + (h % np.uint64(2 * s + 1)).astype(np.int64)).astype(np.int64)


def key_offsets(cfg: SynthConfig) -> np.ndarray:
    """CSR offsets u64[n_keys + 1] of the whole stream (no event values)."""
    off = np.zeros(cfg.n_keys + 1, np.uint64)
    np.cumsum(key_counts(cfg), out=off[1:])
    return off


def generate(cfg: SynthConfig, keys: np.ndarray | None = None):
    """Host (numpy) generator for `keys` (default: all).  Returns (key_off u64, columns)."""
    keys = np.arange(cfg.n_keys, dtype=np.int64) if keys is None else np.asarray(keys, np.int64)
    counts = key_counts(cfg, keys)
    key_off = np.zeros(len(keys) + 1, dtype=np.uint64)
    np.cumsum(counts, out=key_off[1:])
    n = int(key_off[-1])
    kid = np.repeat(np.arange(len(keys)), counts)
    j = np.arange(n, dtype=np.int64) - np.repeat(key_off[:-1].astype(np.int64), counts)
    gk = (keys[kid] + cfg.key_base).astype(np.uint64)
    h = _h(cfg.seed, gk, j.astype(np.uint64))
    if cfg.kind == "abc":
        return key_off, [(h % np.uint64(16)).astype(np.int32)]
    # stock: price = max(1, price + step), step in {-2..2}, from base 100 + key % 100
    step = (h % np.uint64(5)).astype(np.int64) - 2
    base = (100 + (gk % np.uint64(100))).astype(np.int64)
    price = np.empty(n, dtype=np.int64)
    for i in range(len(keys)):  # clamped walk: p_j = S_j + max(0, max_{i<=j}(1 - S_i))
        a, b = int(key_off[i]), int(key_off[i + 1])
        if a == b:
            continue
        S = base[a] + np.cumsum(step[a:b])
        price[a:b] = S + np.maximum(0, np.maximum.accumulate(1 - S))
    u = ((h >> np.uint64(8)) % np.uint64(500)).astype(np.int64)
    r = (h >> np.uint64(20)).astype(np.uint64)
    vol = np.where(u == 0, 1001 + (r % np.uint64(100)).astype(np.int64),
                   np.where(u == 1, (r % np.uint64(700)).astype(np.int64),
                            900 + (r % np.uint64(101)).astype(np.int64)))
    return key_off, [price.astype(np.int32), vol.astype(np.int32)]


def generate_arrival(cfg: SynthConfig, keys: np.ndarray | None = None):
    """The same stream in arrival order (round robin: by index within key, then key), as
    csrc/partition.hip produces it.  Returns (key of each event u32, columns)."""
    key_off, cols = generate(cfg, keys)
    counts = np.diff(key_off.astype(np.int64))
    kid = np.repeat(np.arange(len(counts), dtype=np.int64), counts)
    j = np.arange(int(key_off[-1]), dtype=np.int64) - np.repeat(key_off[:-1].astype(np.int64), counts)
    order = np.lexsort((kid, j))
    return kid[order].astype(np.uint32), [c[order] for c in cols]


# ------------------------------------------------------------------------------ digest
def _mix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def match_digest(key, emit_seq, pair_off, pair_seq, pair_stage) -> int:
    """Order-independent checksum of a match set, identical to the kernels' (cep_match_digest):
    Σ_m h_m, h_m = mix(... mix(mix(C ^ key<<32 ^ emit) ^ (stage_0<<32 | seq_0)) ...)."""
    key = np.asarray(key, np.uint64)
    n = len(key)
    if n == 0:
        return 0
    off = np.asarray(pair_off, np.int64)
    lens = off[1:] - off[:-1]
    seq = np.asarray(pair_seq, np.uint64)
    st = np.asarray(pair_stage, np.uint64)
    with np.errstate(over="ignore"):
        h = _mix64(np.uint64(0x9E3779B97F4A7C15) ^ (key << np.uint64(32)) ^ np.asarray(emit_seq, np.uint64))
        for i in range(int(lens.max()) if n else 0):
            sel = lens > i
            idx = off[:-1][sel] + i
            h[sel] = _mix64(h[sel] ^ ((st[idx] << np.uint64(32)) | seq[idx]))
        return int(h.sum(dtype=np.uint64))
