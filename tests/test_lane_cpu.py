"""The GPU lane logic (csrc/nfa_lane.h + the query's generated step), built for the host by
tests/lane_cpu.py, against the oracle: reference KATs, the stock configs at small size and
random fuzz queries, with walks deferred (the kernel's default) and in place (the retry
path).  No GPU: this pins the per-event logic and the deferred-walk machinery on CPU; the
GPU parity tests (test_gpu_parity.py) run the same code on the device."""
import os

import numpy as np
import pytest

import lane_cpu
import oracle
from fuzz_queries import random_query, random_stream
from ref_queries import STOCK_KATS, STRING_KATS, build_case, kats
from kafkastreams_cep_amd import native as N
from kafkastreams_cep_amd import workloads as W

KAT_CASES = [n for n in kats() if n in STRING_KATS or n in STOCK_KATS]


@pytest.mark.parametrize("defer", [True, False])
@pytest.mark.parametrize("name", KAT_CASES)
def test_lane_kats(name, defer):
    q, off, cols = build_case(name, kats()[name])
    ir = q.to_ir()
    lane_cpu.assert_same(lane_cpu.run(ir, off, cols, defer=defer), oracle.run(ir, off, cols), off)


@pytest.mark.parametrize("variant", ["readme", "test"])
def test_lane_stock_small(variant):
    cfg = W.SynthConfig("t", "stock", 200, 600, 0xCE90000 + 3)
    off, cols = W.generate(cfg)
    ir = W.stock_query(variant).to_ir()
    r = oracle.run(ir, off, cols, threads=8)
    assert r["n_matches"] > 20
    g = lane_cpu.run(ir, off, cols)
    assert g["bits_used"]
    lane_cpu.assert_same(g, r, off)
    lane_cpu.assert_same(lane_cpu.run(ir, off, cols, bits=False), r, off)  # the chunked quiet scan


def test_lane_any_kleene_small():
    cfg = W.SynthConfig("t", "stock", 100, 300, 0xCE90000 + 4)
    off, cols = W.generate(cfg)
    ir = W.any_kleene_query().to_ir()
    lane_cpu.assert_same(lane_cpu.run(ir, off, cols), oracle.run(ir, off, cols, threads=8), off)


@pytest.mark.parametrize("query", ["readme", "cfg4s"])
def test_lane_narrow_dewey_build(query):
    """The narrow build (3 Dewey pairs in registers, the kernel libcep runs first): on the
    bench streams no version outgrows it and every key equals the oracle; on the reference's
    KATs the keys whose versions need more pairs report KE_RETRY internally (here, after the
    driver's same-build re-runs, capacity) and every other key is exact."""
    cfg = W.CONFIGS[3]
    off, cols = W.generate(cfg, np.arange(0, 1_000_000, 5000))
    q = W.stock_query("readme") if query == "readme" else W.any_kleene_query(carry_volume=True)
    ir = q.to_ir()
    lane_cpu.assert_same(lane_cpu.run(ir, off, cols, narrow=True), oracle.run(ir, off, cols, threads=8), off)


def test_lane_narrow_build_overflow_is_capacity():
    over = 0
    for name in KAT_CASES:
        q, off, cols = build_case(name, kats()[name])
        ir = q.to_ir()
        g, r = lane_cpu.run(ir, off, cols, narrow=True), oracle.run(ir, off, cols)
        bad = g["err_code"] == 16
        over += int(bad.sum())
        np.testing.assert_array_equal(g["err_code"][~bad], r["err_code"][~bad])
    assert over > 0  # (some KAT needs more than 3 pairs: the retry path is exercised on the GPU)


@pytest.mark.parametrize("case", ["nfa_skip_till_any", "fuzz8", "fuzz96", "fuzz80"])
def test_lane_stream_widen(case):
    """Streams run the stream build (3-pair versions): a key whose versions outgrow them stops
    before that event, undone (nfa_lane.h stop_event), and the wide build continues it over
    the same state - per key the same matches and errors as the whole stream in one pass."""
    import stream_split as SS
    if case.startswith("fuzz"):
        seed = int(case[4:])
        q = random_query(seed)
        off, cols = random_stream(seed, 60, 14)
    else:
        q, off, cols = build_case(case, kats()[case])
    ir = q.to_ir()
    r = oracle.run(ir, off, cols)
    outs = [lane_cpu.run(ir, ko, cs, rcap=16384, streaming=True, reset=(b == 0))
            for b, (ko, cs) in enumerate(SS.split(off, cols, 3, seed=7))]
    assert sum(o["widened"] for o in outs) > 0
    np.testing.assert_array_equal(outs[-1]["err_code"], r["err_code"])
    assert SS.merge(outs) == SS.oracle_per_key(r, off)


@pytest.mark.parametrize("seed", list(range(3, 160, 16)) + [21, 80, 393, 571])
def test_lane_stream_forced_stops(seed, monkeypatch):
    """Stops forced at pseudo-random records mid-event (CEP_TEST_WIDEN: after earlier records'
    puts, pushes, twin writes and walks), on fuzz queries including the exact-conflict seeds:
    the undo plus the wide build's continuation equal the oracle."""
    import stream_split as SS
    monkeypatch.setenv("CEP_LANE_DEFINES", "CEP_TEST_WIDEN=5")
    q = random_query(seed)
    ir = q.to_ir()
    if oracle.compile_check(ir):
        pytest.skip("reference compile-time exception")
    off, cols = random_stream(seed, 60, 14)
    r = oracle.run(ir, off, cols)
    outs = [lane_cpu.run(ir, ko, cs, rcap=16384, streaming=True, reset=(b == 0))
            for b, (ko, cs) in enumerate(SS.split(off, cols, 3, seed=seed))]
    assert sum(o["widened"] for o in outs) > 0
    np.testing.assert_array_equal(outs[-1]["err_code"], r["err_code"])
    assert SS.merge(outs) == SS.oracle_per_key(r, off)


def test_lane_stream_forced_stops_stock(monkeypatch):
    """The same on the README and config-4 stress queries (twin slots, LDS ring slots)."""
    import stream_split as SS
    monkeypatch.setenv("CEP_LANE_DEFINES", "CEP_TEST_WIDEN=11")
    cfg = W.SynthConfig("t", "stock", 60, 500, 0xCE90000 + 3)
    off, cols = W.generate(cfg)
    for q in (W.stock_query("readme"), W.any_kleene_query(carry_volume=True)):
        ir = q.to_ir()
        r = oracle.run(ir, off, cols, threads=8)
        outs = [lane_cpu.run(ir, ko, cs, streaming=True, reset=(b == 0))
                for b, (ko, cs) in enumerate(SS.split(off, cols, 4, seed=4))]
        assert sum(o["widened"] for o in outs) > 0
        np.testing.assert_array_equal(outs[-1]["err_code"], r["err_code"])
        assert SS.merge(outs) == SS.oracle_per_key(r, off)


@pytest.mark.parametrize("streaming", [False, True])
def test_lane_spread(streaming, monkeypatch):
    """An underfilled launch spread over W waves (session.cpp run_nfa, NfaArgs.spread): wave w's
    lane l runs rank l * W + w, odd lanes reversed; the grid's waves past W (its last block)
    stay idle - a key run by two lanes would corrupt its stream."""
    import stream_split as SS
    monkeypatch.setenv("CEP_LANE_SPREAD", "4")  # 4 waves x 64 lanes >= 200 keys
    monkeypatch.setenv("CEP_LANE_NO_PERSIST", "1")  # (per batch: one lane per key, as session.cpp)
    cfg = W.SynthConfig("t", "stock", 200, 300, 0xCE90000 + 3)
    off, cols = W.generate(cfg)
    ir = W.stock_query("readme").to_ir()
    r = oracle.run(ir, off, cols, threads=8)
    if not streaming:
        lane_cpu.assert_same(lane_cpu.run(ir, off, cols), r, off)
        return
    outs = [lane_cpu.run(ir, ko, cs, streaming=True, reset=(b == 0))
            for b, (ko, cs) in enumerate(SS.split(off, cols, 3, seed=3))]
    np.testing.assert_array_equal(outs[-1]["err_code"], r["err_code"])
    assert SS.merge(outs) == SS.oracle_per_key(r, off)


def test_lane_stream_isolated_keys(monkeypatch):
    """A stream's launch with its first keys alone in their waves and the rest 64 per wave from
    there (session.cpp $CEP_STREAM_ISO, NfaArgs.spread_iso without spread), in emulated waves."""
    import stream_split as SS
    monkeypatch.setenv("CEP_LANE_STREAM_ISO", "7")
    monkeypatch.setenv("CEP_LANE_WAVES", "1")
    cfg = W.SynthConfig("t", "stock", 150, 400, 0xCE90000 + 3)
    off, cols = W.generate(cfg)
    ir = W.stock_query("readme").to_ir()
    r = oracle.run(ir, off, cols, threads=8)
    outs = [lane_cpu.run(ir, ko, cs, streaming=True, reset=(b == 0))
            for b, (ko, cs) in enumerate(SS.split(off, cols, 3, seed=5))]
    np.testing.assert_array_equal(outs[-1]["err_code"], r["err_code"])
    assert SS.merge(outs) == SS.oracle_per_key(r, off)


def test_lane_capacity_retry():
    """rcap 2: most keys overflow the run queue and are re-run with walks in place."""
    cfg = W.SynthConfig("t", "stock", 100, 400, 0xCE90000 + 3)
    off, cols = W.generate(cfg)
    ir = W.stock_query("test").to_ir()
    g = lane_cpu.run(ir, off, cols, rcap=2)
    assert g["retried"] > 0
    lane_cpu.assert_same(g, oracle.run(ir, off, cols, threads=8), off)


def test_lane_one_lane_per_key_small_pools(monkeypatch):
    """session.cpp's launch for a single query: one lane per key (no job claiming), node and
    pointer pools far below the batch's need, so most keys re-run on persistent lanes."""
    monkeypatch.setenv("CEP_LANE_NO_PERSIST", "1")
    monkeypatch.setenv("CEP_LANE_POOL", "3000")
    cfg = W.SynthConfig("t", "abc", 300, 400, 0xCE90000 + 2)
    off, cols = W.generate(cfg)
    ir = W.strict_abc_query().to_ir()
    g = lane_cpu.run(ir, off, cols)
    assert g["retried"] > 0
    lane_cpu.assert_same(g, oracle.run(ir, off, cols, threads=8), off)


@pytest.mark.parametrize("seed", range(0, 160, 8))
def test_lane_fuzz(seed):
    q = random_query(seed)
    ir = q.to_ir()
    if oracle.compile_check(ir):
        pytest.skip("reference compile-time exception")
    off, cols = random_stream(seed, 60, 14)
    r = oracle.run(ir, off, cols)
    lane_cpu.assert_same(lane_cpu.run(ir, off, cols), r, off)
    lane_cpu.assert_same(lane_cpu.run(ir, off, cols, defer=False), r, off)


@pytest.mark.parametrize("seed", [21, 80, 393, 571])
def test_lane_exact_conflicts(seed):
    """Fuzz streams where a deferred walk deletes a node that a later put found live (the
    reference's "Cannot find predecessor event"): resolved in the same launch through the put
    log (nfa_lane.h header), no re-run, and equal to the oracle - per batch and streaming."""
    import stream_split as SS
    q = random_query(seed)
    ir = q.to_ir()
    off, cols = random_stream(seed, 60, 14)
    r = oracle.run(ir, off, cols)
    g = lane_cpu.run(ir, off, cols)
    assert g["stats"]["exact_conflicts"] > 0 and g["retried"] == 0
    lane_cpu.assert_same(g, r, off)
    outs = []
    for i, (ko, cs) in enumerate(SS.split(off, cols, 3, seed=seed)):
        m = lane_cpu.run(ir, ko, cs, rcap=16384, streaming=True, reset=i == 0)
        outs.append(m)
    assert SS.merge(outs) == SS.oracle_per_key(r, off)
    np.testing.assert_array_equal(outs[-1]["err_code"], r["err_code"])


@pytest.mark.parametrize("query,n_batches", [("readme", 3), ("test", 4), ("any_kleene", 3), ("strict", 5)])
def test_lane_streaming_batches(query, n_batches):
    """A streaming session fed the stream in consecutive pieces per key produces, per key, the
    same matches (global sequence numbers) and errors as the whole stream in one pass."""
    import stream_split as SS
    cfg = W.SynthConfig("t", "abc" if query == "strict" else "stock", 60, 500, 0xCE90000 + 3)
    off, cols = W.generate(cfg)
    q = {"readme": lambda: W.stock_query("readme"), "test": lambda: W.stock_query("test"),
         "any_kleene": W.any_kleene_query, "strict": W.strict_abc_query}[query]()
    ir = q.to_ir()
    r = oracle.run(ir, off, cols, threads=8)
    batches = SS.split(off, cols, n_batches, seed=n_batches)
    outs = [lane_cpu.run(ir, ko, cs, streaming=True, reset=(b == 0)) for b, (ko, cs) in enumerate(batches)]
    assert SS.merge(outs) == SS.oracle_per_key(r, off)
    last = outs[-1]
    np.testing.assert_array_equal(last["err_code"], r["err_code"])
    bad = r["err_code"] != 0
    np.testing.assert_array_equal(last["err_seq"][bad].astype(np.uint64),
                                  r["err_pos"][bad].astype(np.uint64) - np.asarray(off, np.uint64)[:-1][bad])


@pytest.mark.parametrize("seed", range(3, 160, 16))
def test_lane_streaming_fuzz(seed):
    import stream_split as SS
    q = random_query(seed)
    ir = q.to_ir()
    if oracle.compile_check(ir):
        pytest.skip("reference compile-time exception")
    off, cols = random_stream(seed, 60, 14)
    r = oracle.run(ir, off, cols)
    batches = SS.split(off, cols, 3, seed=seed)
    # a stream cannot re-run a key that outgrows its run queue: size it like the retries would
    outs = [lane_cpu.run(ir, ko, cs, rcap=16384, streaming=True, reset=(b == 0)) for b, (ko, cs) in enumerate(batches)]
    np.testing.assert_array_equal(outs[-1]["err_code"], r["err_code"])
    assert SS.merge(outs) == SS.oracle_per_key(r, off)


def test_lane_query_group():
    """Config 5's 64 stock-query variants as one kernel group (literals from the per-query
    table, wave W = query W % 64 on 64 keys) against the oracle, query by query; plus a group
    that hits the capacity retry."""
    cfg = W.SynthConfig("t", "stock", 70, 500, 0xCE90000 + 5)
    off, cols = W.generate(cfg)
    irs = [p.to_ir() for p in W.multi_queries(64)]
    res = lane_cpu.run_group(irs, off, cols)
    assert all(r["n_group"] == 64 for r in res)
    for ir, g in zip(irs, res):
        lane_cpu.assert_same(g, oracle.run(ir, off, cols), off)
    small = lane_cpu.run_group(irs[56:64], off, cols, rcap=2)
    for ir, g in zip(irs[56:64], small):
        lane_cpu.assert_same(g, oracle.run(ir, off, cols), off)


@pytest.mark.parametrize("seed", list(range(0, 160, 16)) + [21, 80, 393, 571])
def test_lane_partial_drains(seed, monkeypatch):
    """Partial drains (nfa_lane.h flush(may_stop)) forced at every flush, with a 4-walk flush
    threshold: walks stay queued across flushes and events, in order, and the put log keeps
    the entries they can still conflict with (seeds 21-571: exact conflicts) - fuzz queries
    per batch and as a stream."""
    import stream_split as SS
    monkeypatch.setenv("CEP_LANE_DEFINES", "CEP_PARTIAL_DRAIN=2 CEP_WALK_FLUSH=4")
    q = random_query(seed)
    ir = q.to_ir()
    if oracle.compile_check(ir):
        pytest.skip("reference compile-time exception")
    off, cols = random_stream(seed, 60, 14)
    r = oracle.run(ir, off, cols)
    g = lane_cpu.run(ir, off, cols)
    lane_cpu.assert_same(g, r, off)
    if seed in (21, 80, 393, 571):  # resolved through the log, no re-run
        assert g["stats"]["exact_conflicts"] > 0 and g["retried"] == 0
    batches = SS.split(off, cols, 3, seed=seed)
    outs = [lane_cpu.run(ir, ko, cs, rcap=16384, streaming=True, reset=(b == 0)) for b, (ko, cs) in enumerate(batches)]
    np.testing.assert_array_equal(outs[-1]["err_code"], r["err_code"])
    assert SS.merge(outs) == SS.oracle_per_key(r, off)


def test_lane_partial_drains_group(monkeypatch):
    """The same on a kernel group (persistent lanes, config 5's heaviest variants) and the
    config-4 stress query."""
    monkeypatch.setenv("CEP_LANE_DEFINES", "CEP_PARTIAL_DRAIN=2 CEP_WALK_FLUSH=4")
    cfg = W.SynthConfig("t", "stock", 40, 400, 0xCE90000 + 7)
    off, cols = W.generate(cfg)
    irs = [p.to_ir() for p in W.multi_queries(64)[52:64]]
    for ir, g in zip(irs, lane_cpu.run_group(irs, off, cols)):
        lane_cpu.assert_same(g, oracle.run(ir, off, cols), off)
    ir = W.any_kleene_query(carry_volume=True).to_ir()
    lane_cpu.assert_same(lane_cpu.run(ir, off, cols), oracle.run(ir, off, cols), off)


def test_dewey_short_compat_matches_general():
    """dewey.h dw_compat2 (the buffer walks' 2-pair fast path) equals dw_compatible on every
    pair of canonical versions of at most 2 RLE pairs over small digits."""
    import subprocess
    import tempfile
    here = os.path.dirname(os.path.abspath(__file__))
    exe = os.path.join(tempfile.mkdtemp(), "dewey_check")
    subprocess.check_call([lane_cpu.CLANG, "-x", "c++", "-std=c++17", "-O1", "-w", f"-I{os.path.join(here, 'lane_cpu')}",
                           f"-I{lane_cpu.CSRC}", os.path.join(here, "lane_cpu", "dewey_check.cpp"), "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout
    assert out.strip().endswith("bad 0") and "checked 14400" in out


def test_lane_partial_drain_conflict_runs_earlier_walks(monkeypatch):
    """a partial drain that finds a conflict keeps draining every walk queued
    before the put that throws (their matches and exceptions come first in the reference).
    Seed 21 with a 32-walk flush threshold lost such walks before the fix."""
    monkeypatch.setenv("CEP_LANE_DEFINES", "CEP_PARTIAL_DRAIN=2 CEP_WALK_FLUSH=32")
    q = random_query(21)
    ir = q.to_ir()
    off, cols = random_stream(21, 60, 14)
    g = lane_cpu.run(ir, off, cols)
    assert g["stats"]["exact_conflicts"] > 0
    lane_cpu.assert_same(g, oracle.run(ir, off, cols), off)


@pytest.mark.parametrize("persist", [True, False])
@pytest.mark.parametrize("case", ["stock", "any_kleene", "group", "fuzz", "stream"])
def test_lane_whole_waves(case, persist, monkeypatch):
    """The same lane code run as whole 64-lane waves (tests/lane_cpu/wave_emu.h: every lane a
    fiber, each cross-lane operation a rendezvous of the wave's live lanes), so the wave-wide
    drains, partial drains and job claiming see their real neighbours: equal to the oracle.
    persist False: one lane per key as libcep launches single queries and streams."""
    import stream_split as SS
    monkeypatch.setenv("CEP_LANE_WAVES", "1")
    if not persist:
        monkeypatch.setenv("CEP_LANE_NO_PERSIST", "1")
    if case == "group":
        cfg = W.SynthConfig("t", "stock", 40, 300, 0xCE90000 + 8)
        off, cols = W.generate(cfg)
        irs = [p.to_ir() for p in W.multi_queries(64)[48:64]]
        for ir, g in zip(irs, lane_cpu.run_group(irs, off, cols)):
            lane_cpu.assert_same(g, oracle.run(ir, off, cols), off)
        return
    if case == "fuzz":
        for seed in (5, 21, 80, 393):
            ir = random_query(seed).to_ir()
            if oracle.compile_check(ir):
                continue
            off, cols = random_stream(seed, 60, 14)
            lane_cpu.assert_same(lane_cpu.run(ir, off, cols), oracle.run(ir, off, cols), off)
        return
    cfg = W.SynthConfig("t", "stock", 130, 400, 0xCE90000 + 3)
    off, cols = W.generate(cfg)
    ir = (W.any_kleene_query() if case == "any_kleene" else W.stock_query("readme")).to_ir()
    r = oracle.run(ir, off, cols, threads=8)
    if case == "stream":
        batches = SS.split(off, cols, 3, seed=3)
        outs = [lane_cpu.run(ir, ko, cs, streaming=True, reset=(b == 0)) for b, (ko, cs) in enumerate(batches)]
        assert SS.merge(outs) == SS.oracle_per_key(r, off)
        return
    lane_cpu.assert_same(lane_cpu.run(ir, off, cols), r, off)
    lane_cpu.assert_same(lane_cpu.run(ir, off, cols, narrow=True), r, off)


@pytest.mark.parametrize("seed", [3, 21, 80, 393, 571])
def test_lane_whole_wave_conflicts_and_partial_drains(seed, monkeypatch):
    """Whole 64-lane waves, one lane per key, under forced partial drains and a small drain
    threshold, on fuzz streams whose deferred walks conflict with later puts: per batch and as
    a stream (wide build, put log)."""
    import stream_split as SS
    monkeypatch.setenv("CEP_LANE_WAVES", "1")
    monkeypatch.setenv("CEP_LANE_NO_PERSIST", "1")
    monkeypatch.setenv("CEP_LANE_DEFINES", "CEP_PARTIAL_DRAIN=2 CEP_WALK_FLUSH=4")
    ir = random_query(seed).to_ir()
    if oracle.compile_check(ir):
        pytest.skip("reference compile-time exception")
    off, cols = random_stream(seed, 60, 14)
    r = oracle.run(ir, off, cols)
    lane_cpu.assert_same(lane_cpu.run(ir, off, cols), r, off)
    g = lane_cpu.run(ir, off, cols, narrow=True)  # (keys whose versions outgrow 3 pairs: capacity here)
    ok = g["err_code"] != 16
    np.testing.assert_array_equal(g["err_code"][ok], r["err_code"][ok])
    batches = SS.split(off, cols, 3, seed=seed)
    outs = [lane_cpu.run(ir, ko, cs, rcap=16384, streaming=True, reset=(b == 0)) for b, (ko, cs) in enumerate(batches)]
    np.testing.assert_array_equal(outs[-1]["err_code"], r["err_code"])
    assert SS.merge(outs) == SS.oracle_per_key(r, off)


def test_lane_whole_wave_small_queue_retry(monkeypatch):
    """Whole waves whose records overflow a 2-record run queue: the key is re-run (KE_RETRY),
    exact."""
    monkeypatch.setenv("CEP_LANE_WAVES", "1")
    monkeypatch.setenv("CEP_LANE_NO_PERSIST", "1")
    cfg = W.SynthConfig("t", "stock", 100, 400, 0xCE90000 + 3)
    off, cols = W.generate(cfg)
    ir = W.stock_query("test").to_ir()
    g = lane_cpu.run(ir, off, cols, rcap=2)
    assert g["retried"] > 0
    lane_cpu.assert_same(g, oracle.run(ir, off, cols, threads=8), off)


def _nullness_queries():
    """fuzz queries whose generated step masks fold null bits (compile.cpp fold_nullness), plus
    hand-made ones: skip_till_any branching with folds on both stages, getOrElse reads, and a
    PROCEED chain of optional / zeroOrMore stages carrying folds"""
    from kafkastreams_cep_amd import EventSchema, QueryBuilder
    qs = []
    for seed in range(0, 400):
        q = random_query(seed)
        ir = q.to_ir()
        if oracle.compile_check(ir):
            continue
        if "static fold nullness" in N.Query(ir).jit_source:
            qs.append((f"fuzz{seed}", ir, seed))
        if len(qs) >= 10:
            break
    S = EventSchema({"a": "int", "b": "int"})
    qb = QueryBuilder(S)
    any2 = (qb.select("x").where(lambda k, v, ts, s: v.a > 2).fold("u", lambda k, v, c: v.a, type="int").then()
            .select("y").oneOrMore().skipTillAnyMatch().where(lambda k, v, ts, s: v.b > s.get("u"))
            .fold("u", lambda k, v, c: c + v.b, type="int").fold("w", lambda k, v, c: v.a * 2 - v.b, type="int").then()
            .select("z").skipTillAnyMatch().where(lambda k, v, ts, s: v.a < s.getOrElse("w", 5)).build())
    chain = (QueryBuilder(S).select("p").where(lambda k, v, ts, s: v.a >= 5).fold("u", lambda k, v, c: v.a, type="int")
             .then().select("q").optional().skipTillNextMatch().where(lambda k, v, ts, s: v.b < s.getOrElse("u", 3))
             .fold("w", lambda k, v, c: c + v.a, type="int").then()
             .select("r").zeroOrMore().skipTillNextMatch().where(lambda k, v, ts, s: v.a > s.get("u"))
             .fold("u", lambda k, v, c: c + v.b, type="int").then()
             .select("t").where(lambda k, v, ts, s: v.b != s.getOrElse("w", 1)).build())
    qs += [("any_two_stage_folds", any2.to_ir(), 7), ("proceed_chain", chain.to_ir(), 11)]
    return qs


@pytest.mark.parametrize("name,ir,seed", _nullness_queries())
def test_lane_static_fold_nullness_is_exact(name, ir, seed):
    """ the static fold nullness masks (`w.nm &= ...` at each dispatch case) change
    nothing: the generated step with and without them gives the same matches and the same
    exceptions on the same streams, both equal to the oracle."""
    src = N.Query(ir).jit_source
    masked = [ln for ln in src.splitlines() if "static fold nullness" in ln]
    if not masked and name.startswith("fuzz"):
        pytest.skip("no mask generated")
    plain = "\n".join(ln for ln in src.splitlines() if "static fold nullness" not in ln) + "\n"
    off, cols = random_stream(seed, 80, 16)
    r = oracle.run(ir, off, cols)
    a = lane_cpu.run(ir, off, cols)
    b = _run_source(ir, plain, off, cols)
    lane_cpu.assert_same(a, r, off)
    lane_cpu.assert_same(b, r, off)


def _run_source(ir, source, off, cols):
    """lane_cpu.run on an explicit kernel source (a single query: the group path of run() with a
    one-member plan)"""
    g = {"source": source, "members": [0], "literals": np.zeros((1, 0), np.int64)}
    m = lane_cpu.run(ir, off, cols, _group=g)
    key_off = np.asarray(off, np.uint64)
    m["emit_pos"] = (key_off[m["key"].astype(np.int64) % (len(key_off) - 1)] + m["emit_seq"]).astype(np.uint64)
    pk = np.repeat(m["key"].astype(np.int64) % (len(key_off) - 1), np.diff(m["pair_off"].astype(np.int64)))
    m["pair_pos"] = (key_off[pk] + m["pair_seq"]).astype(np.uint64)
    return m


@pytest.mark.parametrize("case", ["readme", "cfg4s", "kats"] + [f"fuzz{s}" for s in range(24)])
def test_lane_fused_walks(case, monkeypatch):
    """Fused branch + extraction walks (nfa_lane.h CEP_WALK_FUSE: on in kernel groups, forced
    on here for single queries) give the oracle's matches and errors; on the stock streams the
    fused build walks fewer branch hops than the unfused one (the walk-hop counters of the CPU
    lane build) with every extraction hop still walked."""
    if case in ("readme", "cfg4s"):
        off, cols = W.generate(W.CONFIGS[3], np.arange(0, 1_000_000, 7919))
        q = W.stock_query("readme") if case == "readme" else W.any_kleene_query(carry_volume=True)
        cases = [(q.to_ir(), off, cols)]
    elif case == "kats":
        cases = []
        for n in KAT_CASES:
            q, off, cols = build_case(n, kats()[n])
            cases.append((q.to_ir(), off, cols))
    else:
        seed = int(case[4:])
        off, cols = random_stream(seed, 60, 14)
        cases = [(random_query(seed).to_ir(), off, cols)]
    for ir, off, cols in cases:
        monkeypatch.setenv("CEP_LANE_DEFINES", "CEP_WALK_FUSE=0")
        plain = lane_cpu.run(ir, off, cols)
        monkeypatch.setenv("CEP_LANE_DEFINES", "CEP_WALK_FUSE=1")
        fused = lane_cpu.run(ir, off, cols)
        lane_cpu.assert_same(fused, oracle.run(ir, off, cols), off)
        assert fused["stats"]["hops_emit"] == plain["stats"]["hops_emit"]
        assert fused["stats"]["hops_branch"] <= plain["stats"]["hops_branch"]
        if case == "readme":
            assert fused["stats"]["hops_branch"] < plain["stats"]["hops_branch"]
