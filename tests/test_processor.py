"""CEPProcessor (kafkastreams_cep_amd/processor.py) against the reference's processor behaviour.

* README.md:73-96: the demo's eight records give exactly the four JSON lines the README
  prints, after the demo's own rendering (test:demo/CEPStockKStreamsDemo.java:60-71: stage
  lists reversed to oldest-first, stages in json-simple HashMap order);
* a many-key interleaved stream forwards the same Sequences in the same order as one
  reference NFA per key run record by record (the oracle), whatever the batch size;
* null values are skipped (CEPProcessor.java:157);
* a key that throws raises that exception after every match of an earlier record was
  forwarded and none of a later one, and the processor stays failed.

The CPU tests run the processor's host logic over an oracle-backed stand-in for the device
session (tests/proc_fake.py); the `gpu` tests run the same cases through libcep.so.
"""
import base64
import json

import numpy as np
import pytest

import oracle
from kafkastreams_cep_amd import QueryBuilder
from kafkastreams_cep_amd import native as N
from kafkastreams_cep_amd import processor as P
from kafkastreams_cep_amd import workloads as W
from proc_fake import OracleStreamSession

README_EVENTS = [("e1", 100, 1010), ("e2", 120, 990), ("e3", 120, 1005), ("e4", 121, 999),
                 ("e5", 120, 999), ("e6", 125, 750), ("e7", 120, 950), ("e8", 120, 700)]  # README.md:73-80
README_LINES = ['{"0":["e1"],"1":["e2","e3","e4","e5"],"2":["e6"]}',  # README.md:93-96
                '{"0":["e3"],"1":["e4"],"2":["e6"]}',
                '{"0":["e1"],"1":["e2","e3","e4","e5","e6","e7"],"2":["e8"]}',
                '{"0":["e3"],"1":["e4","e6"],"2":["e8"]}']
T0 = 1_600_000_000_000


def _java_hash(s: str) -> int:
    h = 0
    for ch in s:
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h


def demo_json(seq: P.Sequence) -> str:
    """The demo's `matches` processor (CEPStockKStreamsDemo.java:60-71): a JSONObject (a
    HashMap of capacity 16: entries in bucket order) of stage -> names, oldest first."""
    items = list(seq.as_map().items())
    items.sort(key=lambda kv: ((_java_hash(kv[0]) ^ (_java_hash(kv[0]) >> 16)) & 15))
    return "{" + ",".join(f'"{k}":' + json.dumps([e.value["name"] for e in reversed(v)], separators=(",", ":"))
                          for k, v in items) + "}"


def _factory(gpu):
    return None if gpu else OracleStreamSession


def run_records(pattern, records, batch_size, gpu, punctuate_every=0):
    """Plays (key, value, timestamp) records into a processor; -> (context, processor)."""
    ctx = P.RecordContext("StockEvents", 0)
    proc = P.CEPProcessor(pattern, batch_size=batch_size, max_keys=1024, session_factory=_factory(gpu))
    proc.init(ctx)
    for i, (k, v, ts) in enumerate(records):
        ctx.send(k, v, ts)
        if punctuate_every and (i + 1) % punctuate_every == 0:
            proc.punctuate(ts)
    proc.close()
    return ctx, proc


def _readme_records(key="AAPL"):
    return [(key, {"name": n, "price": p, "volume": v}, T0 + i) for i, (n, p, v) in enumerate(README_EVENTS)]


def forwarded_view(ctx):
    """Forwarded Sequences as [[(stage, [offsets in list order])...] in map order]."""
    out = []
    for k, seq in ctx.forwarded:
        assert k is None  # context.forward(null, seq), CEPProcessor.java:161
        out.append([(st, [e.offset for e in evs]) for st, evs in seq.as_map().items()])
    return out


def expected_view(pattern, records):
    """One reference NFA per key over the whole stream (the oracle), matches in the order the
    reference forwards them: by arrival of the completing record, emission order within it."""
    ir = pattern.to_ir()
    names = N.Query(ir).stage_names
    keys = {}
    kid = np.array([keys.setdefault(k, len(keys)) for k, _, _ in records], np.int64)
    by_key = np.argsort(kid, kind="stable")
    counts = np.bincount(kid, minlength=len(keys))
    off = np.zeros(len(keys) + 1, np.uint64)
    np.cumsum(counts, out=off[1:])
    S = pattern.schema
    cols = [np.array([r[1][n] for r in records], np.int32)[by_key] for n in S.names]
    ts = np.array([r[2] for r in records], np.int64)[by_key]
    r = oracle.run(ir, off, cols, ts)
    emit = by_key[r["emit_pos"].astype(np.int64)]
    out = []
    for m in np.argsort(emit, kind="stable").tolist():
        a, b = int(r["pair_off"][m]), int(r["pair_off"][m + 1])
        seq = {}
        for st, pos in zip(r["pair_stage"][a:b].tolist(), r["pair_pos"][a:b].tolist()):
            seq.setdefault(names[st], []).append(int(by_key[pos]))
        out.append(list(seq.items()))
    err = [(int(by_key[int(r["err_pos"][j])]), int(r["err_code"][j])) for j in range(len(keys)) if r["err_code"][j]]
    return out, emit, err


def random_records(seed, n_keys=24, n=600):
    rng = np.random.default_rng(seed)
    price = {k: 100 + k % 7 for k in range(n_keys)}
    recs = []
    for i in range(n):
        k = int(rng.integers(n_keys))
        price[k] += int(rng.integers(-2, 3))
        u = rng.random()
        vol = int(rng.integers(1001, 1100)) if u < 0.15 else (int(rng.integers(300, 700)) if u < 0.35 else
                                                             int(rng.integers(900, 1000)))
        recs.append((f"k{k}", {"name": f"e{i}", "price": price[k], "volume": vol}, T0 + i))
    return recs


def arith_query():
    """The README query with a trap in the first stage: `v.volume > 1000 && v.price / v.price
    == 1` throws ArithmeticException on a begin candidate with price 0."""
    S = W.stock_query("readme").schema
    return (QueryBuilder(S).select()
            .where(lambda k, v, ts, s: (v.volume > 1000) & (v.price / v.price == 1))
            .fold("avg", lambda k, v, c: v.price).then()
            .select().oneOrMore().skipTillNextMatch()
            .where(lambda k, v, ts, s: v.price > s.get("avg"))
            .fold("avg", lambda k, v, c: (c + v.price) / 2).fold("volume", lambda k, v, c: v.volume).then()
            .select().skipTillNextMatch().where(lambda k, v, ts, s: v.volume < 0.8 * s.get("volume"))
            .within(1, W.TimeUnit.HOURS).build())


# ---- host logic (CPU) --------------------------------------------------------------------
def test_event_and_sequence_semantics():
    a = P.Event("k", 1, 10, "t", 0, 5)
    assert a == P.Event("other", 2, 99, "t", 0, 5) and hash(a) == hash(P.Event(None, None, 0, "t", 0, 5))
    assert a != P.Event("k", 1, 10, "t", 1, 5)
    assert a.compare_to(P.Event("k", 1, 0, "t", 0, 6)) == -1  # same partition: offsets
    assert a.compare_to(P.Event("k", 1, 0, "u", 0, 1)) == 1   # across partitions: timestamps
    s1 = P.Sequence().add("0", a).add("1", P.Event("k", 1, 11, "t", 0, 6)).add("1", P.Event("k", 1, 12, "t", 0, 7))
    s2 = P.Sequence().add("1", P.Event("k", 1, 12, "t", 0, 7)).add("1", P.Event("k", 1, 11, "t", 0, 6)).add("0", a)
    assert s1 == s2 and s1.size() == 3 and [e.offset for e in s1.get("1")] == [6, 7]
    assert s1 != P.Sequence().add("0", a)
    assert P.Sequence().add("0", a) == s1  # one-directional, as Sequence.java:59-73


@pytest.mark.parametrize("batch", [1, 3, 8, 1000])
def test_readme_demo_cpu(batch):
    ctx, _ = run_records(W.stock_query("readme"), _readme_records(), batch, gpu=False)
    assert [demo_json(s) for _, s in ctx.forwarded] == README_LINES


def test_null_values_skipped_cpu():
    recs = _readme_records()
    with_nulls = []
    for r in recs:
        with_nulls += [r, ("AAPL", None, r[2])]
    ctx = P.RecordContext()
    proc = P.CEPProcessor(W.stock_query("readme"), batch_size=2, session_factory=OracleStreamSession)
    proc.init(ctx)
    for k, v, ts in with_nulls:
        ctx.send(k, v, ts)
    proc.close()
    assert [demo_json(s) for _, s in ctx.forwarded] == README_LINES


@pytest.mark.parametrize("batch,punct", [(1, 0), (7, 0), (64, 5), (10_000, 0)])
def test_interleaved_keys_forward_order_cpu(batch, punct):
    recs = random_records(11, n_keys=12, n=300)
    exp, _, err = expected_view(W.stock_query("readme"), recs)
    assert not err and len(exp) > 5
    ctx, _ = run_records(W.stock_query("readme"), recs, batch, gpu=False, punctuate_every=punct)
    assert forwarded_view(ctx) == exp


def _arith_records():
    recs = random_records(5, n_keys=6, n=200)
    bad = 120
    k = recs[bad][0]
    recs[bad] = (k, {"name": "bad", "price": 0, "volume": 1500}, recs[bad][2])
    return recs, bad


def _check_error_run(gpu, batch):
    q = arith_query()
    recs, bad = _arith_records()
    exp, emit, err = expected_view(q, recs)
    assert err == [(bad, 3)]
    n_before = int(np.sum(emit < bad))
    assert 0 < n_before < len(exp)  # matches both before and after the failing record
    ctx = P.RecordContext("StockEvents", 0)
    proc = P.CEPProcessor(q, batch_size=batch, max_keys=64, session_factory=_factory(gpu))
    proc.init(ctx)
    with pytest.raises(P.ArithmeticException) as ei:
        for k, v, ts in recs:
            ctx.send(k, v, ts)
        proc.close()
    assert ei.value.event.offset == bad and ei.value.key == recs[bad][0]
    assert forwarded_view(ctx) == exp[:n_before]
    with pytest.raises(P.ArithmeticException):
        proc.process("k0", {"name": "x", "price": 1, "volume": 1})
    proc.close()


@pytest.mark.parametrize("batch", [1, 16, 1000])
def test_key_exception_after_earlier_matches_cpu(batch):
    _check_error_run(False, batch)


def _check_restart_from_store(gpu, batch, commit_every, crash_at):
    """in_memory=False: the processor commits its state to the `_cep_nfa` store on punctuate;
    after a crash a new processor (same stores) restores it in init(), the records since the
    last commit are replayed (Kafka's at-least-once delivery), and the Sequences forwarded
    after the restart complete exactly the uninterrupted run's (CEPProcessor.java:117-134,
    159-160)."""
    recs = random_records(13, n_keys=40 if gpu else 8, n=1500 if gpu else 240)
    q = W.stock_query("readme")
    exp, emit, err = expected_view(q, recs)
    assert not err and len(exp) > 5
    stores = {}
    ctx = P.RecordContext("StockEvents", 3, stores=stores)
    proc = P.CEPProcessor(q, batch_size=batch, max_keys=256, session_factory=_factory(gpu))
    proc.init(ctx)
    committed, n_fwd_at_commit = 0, 0
    for i, (k, v, ts) in enumerate(recs[:crash_at]):
        ctx.send(k, v, ts, offset=i)
        if (i + 1) % commit_every == 0:
            proc.punctuate(ts)
            committed, n_fwd_at_commit = i + 1, len(ctx.forwarded)
    assert P.NFA_STATES_STORE in stores and ("StockEvents", 3) in stores[P.NFA_STATES_STORE]
    before = forwarded_view(ctx)[:n_fwd_at_commit]
    # crash: the processor and its device session are gone (nothing after the commit survives)
    if hasattr(proc.session, "close"):
        proc.session.close()
    ctx2 = P.RecordContext("StockEvents", 3, stores=stores)
    proc2 = P.CEPProcessor(q, batch_size=batch, max_keys=256, session_factory=_factory(gpu))
    proc2.init(ctx2)
    for i, (k, v, ts) in enumerate(recs[committed:], start=committed):
        ctx2.send(k, v, ts, offset=i)
    proc2.close()
    assert before + forwarded_view(ctx2) == exp


@pytest.mark.parametrize("batch,commit_every,crash_at", [(4, 50, 130), (64, 37, 200), (1, 100, 100)])
def test_restart_from_store_cpu(batch, commit_every, crash_at):
    _check_restart_from_store(False, batch, commit_every, crash_at)


def test_in_memory_writes_no_store():
    stores = {}
    ctx = P.RecordContext("t", 0, stores=stores)
    proc = P.CEPProcessor(W.stock_query("readme"), in_memory=True, batch_size=4, session_factory=OracleStreamSession)
    proc.init(ctx)
    for k, v, ts in _readme_records():
        ctx.send(k, v, ts)
    proc.close()
    assert stores == {}


# ---- through libcep on the GPU -----------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("batch,commit_every,crash_at", [(16, 200, 700), (1000, 500, 1200)])
def test_restart_from_store_gpu(batch, commit_every, crash_at):
    _check_restart_from_store(True, batch, commit_every, crash_at)


@pytest.mark.gpu
def test_retained_records_bounded_gpu():
    """1e6 records over 500 keys through the strict SEQ(A, B, C) query (runs die within three
    records, their nodes are deleted by removePattern / match extraction): the records the
    processor holds stay bounded (cep_live_floor), and the forwarded matches equal the
    oracle's.  Bound: a key's live nodes span its last two records; plus one batch."""
    rng = np.random.default_rng(3)
    n, n_keys, batch = 1_000_000, 500, 20_000
    keys = rng.integers(0, n_keys, size=n)
    vals = rng.integers(0, 16, size=n).astype(np.int32)
    q = W.strict_abc_query()
    ctx = P.RecordContext("t", 0)
    proc = P.CEPProcessor(q, batch_size=batch, max_keys=n_keys)
    proc.init(ctx)
    most = 0
    n_fwd = 0
    for i in range(n):
        ctx.send(int(keys[i]), {"v": int(vals[i])}, T0 + i)
        if (i + 1) % batch == 0:
            most = max(most, proc.retained_records())
            n_fwd += len(ctx.forwarded)
            ctx.forwarded.clear()
    proc.close()
    n_fwd += len(ctx.forwarded)
    assert most <= 3 * n_keys, most
    off = np.zeros(n_keys + 1, np.uint64)
    np.cumsum(np.bincount(keys, minlength=n_keys), out=off[1:])
    r = oracle.run(q.to_ir(), off, [vals[np.argsort(keys, kind="stable")]])
    assert n_fwd == r["n_matches"] > 1000


@pytest.mark.gpu
def test_live_floor_stock_query_gpu():
    """cep_live_floor on the README query: every key's floor is at most the first record of a
    live run's chain; records before a key's first begin event (volume > 1000) are dropped."""
    recs = random_records(17, n_keys=30, n=3000)
    ctx = P.RecordContext("StockEvents", 0)
    proc = P.CEPProcessor(W.stock_query("readme"), batch_size=500, max_keys=64)
    proc.init(ctx)
    for k, v, ts in recs:
        ctx.send(k, v, ts)
    proc.flush()
    assert proc.retained_records() < len(recs)
    exp, _, _ = expected_view(W.stock_query("readme"), recs)
    assert forwarded_view(ctx) == exp
    proc.close()
@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 3, 1000])
def test_readme_demo_gpu(batch):
    ctx, _ = run_records(W.stock_query("readme"), _readme_records(), batch, gpu=True)
    assert [demo_json(s) for _, s in ctx.forwarded] == README_LINES


@pytest.mark.gpu
@pytest.mark.parametrize("batch,punct", [(5, 0), (97, 0), (4096, 250)])
def test_interleaved_keys_forward_order_gpu(batch, punct):
    recs = random_records(11, n_keys=200, n=3000)
    exp, _, err = expected_view(W.stock_query("readme"), recs)
    assert not err and len(exp) > 20
    ctx, _ = run_records(W.stock_query("readme"), recs, batch, gpu=True, punctuate_every=punct)
    assert forwarded_view(ctx) == exp


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 16, 1000])
def test_key_exception_after_earlier_matches_gpu(batch):
    _check_error_run(True, batch)


@pytest.mark.gpu
def test_semantic_within_processor_gpu():
    """semantic_within=True enforces the README query's WITHIN 1 hour on the record times.  1 ms
    apart: the README's 4 matches.  15 minutes apart: the run begun at e1 (0 min) has expired
    by e8 (105 min), so its second match goes; the run begun at e3 (30 min) still completes at
    e8.  40 minutes apart: every run expires before its dip.  The default processor (the
    reference's WITHIN, never pruning) gives the 4 matches whatever the spacing."""
    recs = _readme_records()
    r = README_LINES
    for semantic, gap, want in [(True, 1, r), (True, 15 * 60_000, [r[0], r[1], r[3]]), (True, 40 * 60_000, []),
                                (False, 40 * 60_000, r)]:
        ctx = P.RecordContext("StockEvents", 0)
        proc = P.CEPProcessor(W.stock_query("readme"), batch_size=3, max_keys=16, semantic_within=semantic)
        proc.init(ctx)
        for i, (k, v, _) in enumerate(recs):
            ctx.send(k, v, T0 + i * gap)
        proc.close()
        assert [demo_json(s) for _, s in ctx.forwarded] == want, (semantic, gap)


def test_checkpoint_is_plain_data():
    """The checkpoint's host half is versioned JSON (no pickle): values go through the
    value serde; a value the default JSON serde cannot encode asks for a serde of its own."""
    import json
    stores = {}
    ctx = P.RecordContext("StockEvents", 0, stores=stores)
    proc = P.CEPProcessor(W.stock_query("readme"), batch_size=4, session_factory=OracleStreamSession)
    proc.init(ctx)
    for k, v, ts in _readme_records():
        ctx.send(k, v, ts)
    proc.punctuate(0)
    blob = stores[P.NFA_STATES_STORE][("StockEvents", 0)]
    assert blob[:8] == b"CEPPROC2"
    n = int.from_bytes(blob[8:16], "little")
    host = json.loads(blob[16 + n:].decode())
    assert host["version"] == 3 and len(host["keys"]) == len(host["events"]) == len(host["base"])
    proc2 = P.CEPProcessor(W.stock_query("readme"), batch_size=4, session_factory=OracleStreamSession)
    proc2.init(P.RecordContext("StockEvents", 0, stores=stores))
    assert [[(e.offset, e.value) for e in evs] for evs in proc2._events] == \
        [[(e.offset, e.value) for e in evs] for evs in proc._events]
    with pytest.raises(ValueError):
        proc2.restore(b"CEPPROC1" + blob[8:])

    class Obj:
        def __init__(self, name, price, volume):
            self.name, self.price, self.volume = name, price, volume

    #  an attribute-style value the default serde cannot encode fails at its first
    # record, not at the next commit; in memory it needs no serde at all
    proc3 = P.CEPProcessor(W.stock_query("readme"), batch_size=4, session_factory=OracleStreamSession)
    ctx3 = P.RecordContext("StockEvents", 0, stores={})
    proc3.init(ctx3)
    with pytest.raises(TypeError):
        ctx3.send("k", Obj("e1", 100, 1010), 0)
    proc4 = P.CEPProcessor(W.stock_query("readme"), in_memory=True, batch_size=3, session_factory=OracleStreamSession)
    ctx4 = P.RecordContext("StockEvents", 0)
    proc4.init(ctx4)
    for k, v, ts in _readme_records():
        ctx4.send(k, Obj(**v), ts)
    proc4.close()
    ref_ctx, _ = run_records(W.stock_query("readme"), _readme_records(), 3, gpu=False)
    assert forwarded_view(ctx4) == forwarded_view(ref_ctx) and len(ctx4.forwarded) == 4


class _Obj:
    def __init__(self, name, price, volume):
        self.name, self.price, self.volume = name, price, volume

    def __eq__(self, o):
        return isinstance(o, _Obj) and vars(self) == vars(o)


class _ObjSerde:
    """a user value serde for attribute-style values"""

    @staticmethod
    def serialize(o):
        return json.dumps([o.name, o.price, o.volume]).encode()

    @staticmethod
    def deserialize(b):
        return _Obj(*json.loads(b.decode()))


def test_json_serde_keeps_types():
    """ the default checkpoint serde gives back what it was given: tuple keys, dicts
    with non-string keys, bytes, non-finite floats, numpy scalars."""
    for x in [("AAPL", 3), {"a": (1, 2), 5: [None, True]}, {"__cep__": 1}, b"\x00\xff", float("inf"),
              np.int32(7), np.float64(2.5), [("x",), {}], "s", 12, None]:
        y = P.JsonSerde.deserialize(P.JsonSerde.serialize(x))
        assert y == x and type(y) is type(x), (x, y)
    assert np.isnan(P.JsonSerde.deserialize(P.JsonSerde.serialize(float("nan"))))
    with pytest.raises(TypeError):
        P.JsonSerde.serialize({1, 2})


def test_checkpoint_version2_reads_plain_json():
    """ host-half version 3 is the tagged JsonSerde encoding; a version-2 blob (plain
    JSON values) still restores, and a value dict holding a "__cep__" key comes back as data."""
    import json
    stores = {}
    ctx = P.RecordContext("StockEvents", 0, stores=stores)
    proc = P.CEPProcessor(W.stock_query("readme"), batch_size=4, session_factory=OracleStreamSession)
    proc.init(ctx)
    recs = _readme_records()
    for k, v, ts in recs[:3]:
        ctx.send(k, dict(v, tag={"__cep__": "x"}), ts)
    proc.punctuate(0)
    blob = stores[P.NFA_STATES_STORE][("StockEvents", 0)]
    n = int.from_bytes(blob[8:16], "little")
    host = json.loads(blob[16 + n:].decode())
    assert host["version"] == 3
    # rewrite the host half as version 2 wrote it: values as plain JSON
    host["version"] = 2
    host["events"] = [[[ts, t, pa, off, base64.b64encode(json.dumps(P.JsonSerde.deserialize(base64.b64decode(v))).encode()).decode()]
                       for ts, t, pa, off, v in evs] for evs in host["events"]]
    host["keys"] = [base64.b64encode(json.dumps(P.JsonSerde.deserialize(base64.b64decode(k))).encode()).decode()
                    for k in host["keys"]]
    old = blob[:16 + n] + json.dumps(host).encode()
    proc2 = P.CEPProcessor(W.stock_query("readme"), batch_size=4, session_factory=OracleStreamSession)
    proc2.init(P.RecordContext("StockEvents", 0, stores={}))
    proc2.restore(old)
    assert [[e.value for e in evs] for evs in proc2._events] == [[e.value for e in evs] for evs in proc._events]
    assert proc2._events[0][0].value["tag"] == {"__cep__": "x"}
    host["version"] = 1
    with pytest.raises(ValueError):
        proc2.restore(blob[:16 + n] + json.dumps(host).encode())


@pytest.mark.parametrize("user_serde", [False, True])
def test_restart_tuple_keys_and_object_values(user_serde):
    """ a persistent processor over tuple keys - and, with a user value serde,
    attribute-style values - restores from its checkpoint and forwards what an uninterrupted
    one forwards (the same Sequences, the same key and value objects)."""
    recs = random_records(13, n_keys=8, n=240)
    recs = [((k, int(k[1:])), (_Obj(**v) if user_serde else dict(v, extra={1: (2, 3)})), ts) for k, v, ts in recs]
    q = W.stock_query("readme")
    kw = dict(batch_size=16, max_keys=64, session_factory=OracleStreamSession,
              value_serde=_ObjSerde if user_serde else None)
    ref_ctx = P.RecordContext("StockEvents", 1)
    ref = P.CEPProcessor(q, **kw)
    ref.init(ref_ctx)
    for i, (k, v, ts) in enumerate(recs):
        ref_ctx.send(k, v, ts, offset=i)
    ref.close()
    stores = {}
    ctx = P.RecordContext("StockEvents", 1, stores=stores)
    proc = P.CEPProcessor(q, **kw)
    proc.init(ctx)
    n_at_commit = 0
    for i, (k, v, ts) in enumerate(recs[:150]):
        ctx.send(k, v, ts, offset=i)
        if i == 119:
            proc.punctuate(ts)
            n_at_commit = len(ctx.forwarded)
    # crash after record 149; the restored processor gets records 120.. again
    ctx2 = P.RecordContext("StockEvents", 1, stores=stores)
    proc2 = P.CEPProcessor(q, **kw)
    proc2.init(ctx2)
    assert all(isinstance(k, tuple) for k in proc2._keys)
    for i, (k, v, ts) in enumerate(recs[120:], start=120):
        ctx2.send(k, v, ts, offset=i)
    proc2.close()

    def view(c):
        return [[(st, [(e.key, e.offset, e.value) for e in evs]) for st, evs in sq.as_map().items()]
                for _, sq in c.forwarded]

    want = view(ref_ctx)
    assert len(want) > 5
    assert view(ctx)[:n_at_commit] + view(ctx2) == want
