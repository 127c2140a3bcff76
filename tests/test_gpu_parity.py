"""GPU parity: libcep.so's HIP kernels vs the CPU oracle and the reference's own KATs.

Bit-exact on every array: match keys, emission events, walk pairs (stage, event) in
reference order, per-key exception class and position, and the device checksum.
"""
import json
import os

import numpy as np
import pytest

import oracle
from fuzz_queries import random_query, random_stream
from gpu_helpers import assert_parity, gpu_run, session_result
from ref_queries import STOCK_KATS, STRING_KATS, build_case, kats, sequences
from kafkastreams_cep_amd import native as N
from kafkastreams_cep_amd import workloads as W

pytestmark = pytest.mark.gpu
TIERS = [N.CEP_TIER_JIT, N.CEP_TIER_INTERP]

NFA_CASES = [n for n in kats() if n in STRING_KATS or n in STOCK_KATS]


@pytest.mark.parametrize("tier", TIERS)
@pytest.mark.parametrize("force_nfa", [False, True])
@pytest.mark.parametrize("name", NFA_CASES)
def test_reference_kats_on_gpu(name, force_nfa, tier):
    case = kats()[name]
    q, off, cols = build_case(name, case)
    ir = q.to_ir()
    g = gpu_run(ir, off, cols, force_nfa=force_nfa, tier=tier)
    assert int(g["err_code"][0]) == 0
    if "expected_count" in case:
        assert g["n_matches"] == case["expected_count"]
    else:
        names = N.Query(ir).stage_names
        g["pair_seq_or_pos"] = g["pair_pos"]
        exp = [{k: sorted(v) for k, v in e.items()} for e in case["expected"]]
        assert sequences(g, names) == exp
    assert_parity(g, oracle.run(ir, off, cols), off)


def test_strict_kat_uses_stencil():
    q, off, cols = build_case("nfa_strict_one_run", kats()["nfa_strict_one_run"])
    assert gpu_run(q.to_ir(), off, cols)["kind"] == N.CEP_KIND_STENCIL


@pytest.mark.parametrize("tier", TIERS)
@pytest.mark.parametrize("force_nfa", [False, True])
def test_cfg2_strict_abc_small(force_nfa, tier):
    cfg = W.SynthConfig("t", "abc", 300, 400, 0xCE90000 + 2)
    off, cols = W.generate(cfg)
    ir = W.strict_abc_query().to_ir()
    assert_parity(gpu_run(ir, off, cols, force_nfa=force_nfa, tier=tier), oracle.run(ir, off, cols, threads=8), off)


@pytest.mark.parametrize("n", [8, 9, 12])
def test_long_strict_chain(n):
    """a strict ONE-only chain of more than 8 stages compiles for the NFA kernel
    (the stencil is instantiated for at most 8) and matches the oracle."""
    from test_native_abi import strict_chain
    rng = np.random.default_rng(n)
    off = np.array([0, 3000, 3000, 7000], np.uint64)
    v = (np.arange(7000) % 4).astype(np.int32)  # long runs of the chain's own pattern
    v[rng.integers(0, 7000, size=300)] = rng.integers(0, 4, size=300)
    ir = strict_chain(n).to_ir()
    r = oracle.run(ir, off, [v])
    assert r["n_matches"] > 100
    assert_parity(gpu_run(ir, off, [v]), r, off)


def test_stencil_many_short_keys():
    """More key starts than a 4096-event tile holds keys: the LDS boundary table path."""
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 6, size=20000)
    off = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    v = rng.integers(0, 16, size=int(off[-1])).astype(np.int32)
    ir = W.strict_abc_query().to_ir()
    assert_parity(gpu_run(ir, off, [v]), oracle.run(ir, off, [v], threads=8), off)


def range_chain(n):
    """SEQ(S0..S{n-1}) all ONE + strict, S_i: i%4 <= v <= i%4 (the stencil's range fast path)."""
    from kafkastreams_cep_amd import EventSchema, QueryBuilder
    b = QueryBuilder(EventSchema({"v": "int"}))
    for i in range(n):
        sel = b.select(f"S{i}").where(lambda k, v, ts, s, i=i: (v.v >= i % 4) & (v.v <= i % 4))
        b = sel.then() if i < n - 1 else sel
    return b.build()


def _boundary_stream(seed):
    rng = np.random.default_rng(seed)
    lens = ([4096, 4095, 1, 4097, 8, 7, 9, 0, 0, 4088, 3, 70000, 0, 5] + rng.integers(0, 4, 3000).tolist()
            + [3 * 4096 - 1, 2, 6, 4096] + rng.integers(0, 70, 300).tolist() + [0, 0])
    off = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    n = int(off[-1])
    v = (np.arange(n) % 4).astype(np.int32)  # long runs of the chains' own pattern
    v[rng.integers(0, n, size=n // 50)] = rng.integers(0, 4, size=n // 50)
    return off, v


@pytest.mark.parametrize("m", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("chain", ["range", "generic"])
def test_stencil_key_boundaries(m, chain):
    """Key starts at and around stencil_mask's 4096-event wave boundaries and among the 8
    events before one, empty keys (also last), a key spanning more than 16 waves (wave_keys'
    block path) and more than 64 keys starting in one wave (the key-offset chunk loop)."""
    from test_native_abi import strict_chain
    off, v = _boundary_stream(m)
    ir = (range_chain(m) if chain == "range" else strict_chain(m)).to_ir()
    assert N.Query(ir).kind == N.CEP_KIND_STENCIL
    r = oracle.run(ir, off, [v], threads=8)
    assert r["n_matches"] > 1000
    assert_parity(gpu_run(ir, off, [v]), r, off)


def test_stencil_empty_batch_after_matches():
    """an empty batch on a session whose previous stencil batch matched reports no
    matches and checksum 0 (not the previous batch's pinned count)."""
    q = N.Query(W.strict_abc_query().to_ir())
    s = N.Session(q)
    off, cols = W.generate(W.SynthConfig("t", "abc", 100, 300, 0xCE90000 + 2))
    s.push(off, cols)
    assert s.digest(0)[0] > 0
    s.push(np.zeros(101, np.uint64), [np.zeros(0, np.int32)])
    assert s.digest(0) == (0, 0)
    assert s.matches(0)["n_matches"] == 0
    s.push(off, cols)  # and the session still works
    assert_parity(session_result(s, 0, off, q.kind), oracle.run(q.ir, off, cols), off)


def test_stencil_pipelined_pushes():
    """Stencil pushes return without a host sync: batches queued back to back, then the last
    batch's results, and the device time of every batch (cep_timing_totals)."""
    q = N.Query(W.strict_abc_query().to_ir())
    s = N.Session(q)
    batches = [W.generate(W.SynthConfig("t", "abc", 200 + 50 * i, 300, 0xCE90000 + 20 + i)) for i in range(20)]
    s.timing_totals(0, reset=True)
    for off, cols in batches:
        s.push(off, cols)
    ms, aux, n = s.timing_totals(0)
    assert n == 20 and ms > 0 and aux == 0  # (the stencil's key-index pass is not timed)
    off, cols = batches[-1]
    assert_parity(session_result(s, 0, off, q.kind), oracle.run(q.ir, off, cols), off)
    s.timing_totals(0, reset=True)
    assert s.timing_totals(0)[2] == 0


@pytest.mark.parametrize("tier", TIERS)
@pytest.mark.parametrize("variant", ["readme", "test", "demo"])
def test_cfg3_stock_small(variant, tier):
    cfg = W.SynthConfig("t", "stock", 1500, 1000, 0xCE90000 + 3)
    off, cols = W.generate(cfg, np.arange(0, 1_000_000, 667)[:1500])
    if variant == "demo":
        cols = [c.astype(np.int64) for c in cols]
    ir = W.stock_query(variant).to_ir()
    r = oracle.run(ir, off, cols, threads=8)
    assert r["n_matches"] > 100
    assert_parity(gpu_run(ir, off, cols, tier=tier), r, off)


def test_cfg3_medium_bit_exact():
    """Config 3 at 50k keys (every 20th key of the BASELINE stream, 50M events): every match,
    event id, emission order and exception bit-exact against the oracle - a launch the size of
    an 8-GPU shard's third, so the spread lane mapping (session.cpp, underfilled launches) and
    the narrow build's re-runs run at scale."""
    cfg = W.CONFIGS[3]
    off, cols = W.generate(cfg, np.arange(0, 1_000_000, 20))
    ir = W.stock_query("readme").to_ir()
    r = oracle.run(ir, off, cols, threads=16)
    assert r["n_matches"] > 30000
    assert_parity(gpu_run(ir, off, cols), r, off)


@pytest.mark.parametrize("query", ["readme", "cfg4s", "cfg4"])
def test_full_size_digest_matches_oracle(query):
    """ The benched configurations at their full size against the oracle,
    not a key sample: config 3's 1e9 events over 1M keys (generated in HBM, the same bits as
    workloads.generate) on the README query and on config 4's query, stress variant and as
    written (NPE on about half of the keys) - match count, checksum over every (key, emission,
    pairs) and the keys with an exception.  The README checksum is the bench line's
    `a81bb860df5becf5`."""
    cfg = W.CONFIGS[3]
    stream = N.synth_stream("stock", cfg.seed, cfg.n_keys, cfg.mean_events)
    q = W.stock_query("readme") if query == "readme" else W.any_kleene_query(carry_volume=(query == "cfg4s"))
    ir = q.to_ir()
    s = N.Session(N.Query(ir))
    s.push_device(stream)
    got = s.digest(0) + (int(np.count_nonzero(s.key_errors(0)[0])),)
    s.close()
    off, cols = stream.download()
    del stream
    r = oracle.run(ir, off, cols, threads=16)
    emit = r["emit_pos"].astype(np.uint64) - off[r["key"].astype(np.int64)]
    pk = np.repeat(r["key"].astype(np.int64), np.diff(r["pair_off"].astype(np.int64)))
    pseq = r["pair_pos"].astype(np.uint64) - off[pk]
    want = (r["n_matches"], W.match_digest(r["key"], emit, r["pair_off"], pseq, r["pair_stage"]),
            int(np.count_nonzero(r["err_code"])))
    assert got == want
    if query == "readme":
        assert f"{got[1]:016x}" == "a81bb860df5becf5"


def test_shard_rank2_bit_exact():
    """ The slowest world-8 shard of the headline stream at its full size:
    the ~125k keys Kafka's partitioner gives rank 2 (murmur2(key) % 8), ~125M events - the
    underfilled launch the projected scaling times (every wave resident, the heaviest keys
    spread over the wave slots) - every match and exception equal to the oracle's."""
    from kafkastreams_cep_amd import shard as SH
    cfg = W.CONFIGS[3]
    keys = np.nonzero(SH.partition_of(np.arange(cfg.n_keys, dtype=np.uint32), 8) == 2)[0]
    assert 120_000 < len(keys) < 130_000
    off, cols = W.generate(cfg, keys)
    ir = W.stock_query("readme").to_ir()
    r = oracle.run(ir, off, cols, threads=16)
    assert r["n_matches"] > 50_000
    assert_parity(gpu_run(ir, off, cols), r, off)


def test_cfg3_streaming_medium_bit_exact():
    """ The streaming path the processor runs, at scale against the oracle
    instead of the GPU's own per-batch checksum: config 3 at 20k keys (every 50th key of the
    BASELINE stream, 20M events) cut into 10 consecutive batches per key at random points - every
    key's matches (global sequence numbers, emission order, stage names) and exceptions equal
    the oracle's single pass (the stream build, its carried run queues and pools, the lane
    order blended across batches)."""
    import stream_split as SS
    cfg = W.CONFIGS[3]
    off, cols = W.generate(cfg, np.arange(0, 1_000_000, 50))
    ir = W.stock_query("readme").to_ir()
    r = oracle.run(ir, off, cols, threads=16)
    assert r["n_matches"] > 10000
    s = N.Session(N.Query(ir), streaming=True)
    outs = []
    for ko, cs in SS.split(off, cols, 10, seed=10):
        s.push(ko, cs)
        m = s.matches(0)
        m["err_code"], m["err_seq"] = s.key_errors(0)
        outs.append(m)
    assert SS.merge(outs) == SS.oracle_per_key(r, off)
    np.testing.assert_array_equal(outs[-1]["err_code"], r["err_code"])


def test_cfg4_stress_medium_bit_exact():
    """Config 4's stress variant at 20k keys (20M events, ~200 buffer nodes per key)."""
    cfg = W.CONFIGS[3]
    off, cols = W.generate(cfg, np.arange(0, 1_000_000, 50))
    ir = W.any_kleene_query(carry_volume=True).to_ir()
    r = oracle.run(ir, off, cols, threads=16)
    assert r["n_matches"] > 10000 and int(np.count_nonzero(r["err_code"])) == 0
    assert_parity(gpu_run(ir, off, cols), r, off)


def test_cfg5_medium_bit_exact():
    """Config 5's 64-variant kernel group on 2000 keys of the BASELINE stream (2M events x 64
    queries): every query bit-exact against the oracle."""
    cfg = W.CONFIGS[3]
    off, cols = W.generate(cfg, np.arange(0, 1_000_000, 500))
    qs = [N.Query(p.to_ir()) for p in W.multi_queries(64)]
    s = N.Session(qs)
    s.push(off, cols)
    total, want = 0, []
    for i, q in enumerate(qs):
        r = oracle.run(q.ir, off, cols, threads=16)
        total += r["n_matches"]
        want.append(r)
        assert_parity(session_result(s, i, off), r, off)
    assert total > 50000
    s.push(off, cols)  # a second batch of the same session (pools sized from the first)
    for i, r in enumerate(want):
        assert_parity(session_result(s, i, off), r, off)


def test_cfg5_20k_keys_digest():
    """ Config 5's kernel group at ten times the medium test's keys: 20k keys
    of the BASELINE stream (every 50th, 20M events) x 64 queries in one launch per batch - per
    query the match count, the checksum over every (key, emission, pairs) and the keys with an
    exception equal the oracle's."""
    cfg = W.CONFIGS[3]
    off, cols = W.generate(cfg, np.arange(0, 1_000_000, 50))
    qs = [N.Query(p.to_ir()) for p in W.multi_queries(64)]
    s = N.Session(qs)
    s.push(off, cols)
    total = 0
    for i, q in enumerate(qs):
        r = oracle.run(q.ir, off, cols, threads=16)
        emit = r["emit_pos"].astype(np.uint64) - off[r["key"].astype(np.int64)]
        pk = np.repeat(r["key"].astype(np.int64), np.diff(r["pair_off"].astype(np.int64)))
        pseq = r["pair_pos"].astype(np.uint64) - off[pk]
        want = (r["n_matches"], W.match_digest(r["key"], emit, r["pair_off"], pseq, r["pair_stage"]),
                int(np.count_nonzero(r["err_code"])))
        assert s.digest(i) + (int(np.count_nonzero(s.key_errors(i)[0])),) == want, i
        total += r["n_matches"]
    assert total > 300_000


@pytest.mark.parametrize("tier", TIERS)
def test_cfg4_any_kleene_small(tier):
    cfg = W.SynthConfig("t", "stock", 400, 300, 0xCE90000 + 4)
    off, cols = W.generate(cfg)
    ir = W.any_kleene_query().to_ir()
    assert_parity(gpu_run(ir, off, cols, tier=tier), oracle.run(ir, off, cols, threads=8), off)


@pytest.mark.parametrize("tier", TIERS)
def test_cfg4_stress_variant_small(tier):
    """Config 4's benched stress variant (S1 carries volume, S2 reads it with getOrElse): no
    key throws, runs accumulate, bit-exact against the oracle on 500 keys
    of the cfg-3 stream."""
    cfg = W.CONFIGS[3]
    keys = np.arange(0, 1_000_000, 2000)[:500]
    off, cols = W.generate(cfg, keys)
    ir = W.any_kleene_query(carry_volume=True).to_ir()
    r = oracle.run(ir, off, cols, threads=8)
    assert r["n_matches"] > 100 and int(np.count_nonzero(r["err_code"])) == 0
    assert_parity(gpu_run(ir, off, cols, tier=tier), r, off)


@pytest.mark.parametrize("groups", [True, False])
def test_cfg5_multi_query_session(groups):
    """Config 5: all 64 stock-query variants in one session.  With kernel groups they run as
    ONE launch (lanes = (query, key), literals from the per-query table); without, one launch
    each.  Every query's matches, event ids, emission order, errors and checksum equal the
    oracle's (the old test ran 8 queries and compared counts only)."""
    cfg = W.SynthConfig("t", "stock", 300, 600, 0xCE90000 + 5)
    off, cols = W.generate(cfg)
    qs = [N.Query(p.to_ir()) for p in W.multi_queries(64)]
    s = N.Session(qs, groups=groups)
    s.push(off, cols)
    assert s.timing(0)[2] >= 1
    total = 0
    for i, q in enumerate(qs):
        r = oracle.run(q.ir, off, cols, threads=8)
        total += r["n_matches"]
        assert_parity(session_result(s, i, off), r, off)
    assert total > 10000


def test_heavy_key_output():
    """Config 5's heaviest (query, key) job: stream key 39664 under variant q63 emits 1474
    matches / 615005 event ids (a 400x-the-mean key).  Its output chain is scattered by a
    whole wave (scatter_heavy); alone and beside light keys, persistent lanes or not."""
    cfg = W.SynthConfig("t", "stock", 1_000_000, 1000, W.CONFIGS[3].seed)
    off, cols = W.generate(cfg, np.array([5, 39664, 7, 11]))
    ir = W.multi_queries(64)[63].to_ir()
    r = oracle.run(ir, off, cols)
    assert r["n_pairs"] > 600_000
    assert_parity(gpu_run(ir, off, cols), r, off)
    qs = [N.Query(p.to_ir()) for p in W.multi_queries(64)[60:]]  # a group: persistent lanes
    s = N.Session(qs)
    s.push(off, cols)
    assert_parity(session_result(s, 3, off), r, off)


def test_cfg5_group_capacity_retry():
    """A kernel group whose jobs overflow a 2-record run queue and tiny pools: the jobs that
    hit a limit are collected on the device and re-run; every query still equals the oracle."""
    cfg = W.SynthConfig("t", "stock", 200, 500, 0xCE90000 + 5)
    off, cols = W.generate(cfg)
    qs = [N.Query(p.to_ir()) for p in W.multi_queries(64)[48:]]
    s = N.Session(qs, max_runs=2, pool_factor=0.0005)
    s.push(off, cols)
    for i, q in enumerate(qs):
        assert_parity(session_result(s, i, off), oracle.run(q.ir, off, cols, threads=8), off)
    s.push(off, cols)  # pools sized from the first batch's use: same results
    for i, q in enumerate(qs):
        assert_parity(session_result(s, i, off), oracle.run(q.ir, off, cols, threads=8), off)


def test_mixed_session_groups():
    """Queries of different shapes in one session: stock variants share a group, the
    any-Kleene query and the zeroOrMore variant run alone, the strict query on the stencil."""
    cfg = W.SynthConfig("t", "stock", 250, 400, 0xCE90000 + 3)
    off, cols = W.generate(cfg)
    ps = [W.stock_query("readme", begin_volume=1000), W.any_kleene_query(), W.stock_query("readme", begin_volume=1005),
          W.stock_query("test"), W.stock_query("readme", dip_num=90)]
    qs = [N.Query(p.to_ir()) for p in ps]
    assert [g["members"] for g in N.group_plans(qs)] == [[0, 2, 4], [1], [3]]
    s = N.Session(qs)
    s.push(off, cols)
    for i, q in enumerate(qs):
        assert_parity(session_result(s, i, off), oracle.run(q.ir, off, cols, threads=8), off)


FUZZ_SEEDS = range(0, 160)
FUZZ_JIT_SEEDS = range(0, 160, 2)  # every JIT query is its own compiled kernel (cached by build())


@pytest.mark.parametrize("tier,seed", [(N.CEP_TIER_INTERP, s) for s in FUZZ_SEEDS] +
                         [(N.CEP_TIER_JIT, s) for s in FUZZ_JIT_SEEDS])
def test_fuzz_queries_vs_oracle(seed, tier):
    q = random_query(seed)
    ir = q.to_ir()
    if oracle.compile_check(ir):
        pytest.skip("reference compile-time exception")
    off, cols = random_stream(seed, 60, 14)
    assert_parity(gpu_run(ir, off, cols, tier=tier), oracle.run(ir, off, cols), off)


def test_edge_cases_empty_and_single():
    ir = W.stock_query("readme").to_ir()
    # no keys at all
    off = np.zeros(1, np.uint64)
    g = gpu_run(ir, off, [np.zeros(0, np.int32), np.zeros(0, np.int32)])
    assert g["n_matches"] == 0
    # keys with 0 and 1 events around a full README key
    case = kats()["stock_readme"]
    ev = np.array(case["events"], np.int32)
    off = np.array([0, 0, 1, 1, 9, 9], np.uint64)
    price = np.concatenate([[100], ev[:, 0]]).astype(np.int32)
    vol = np.concatenate([[1500], ev[:, 1]]).astype(np.int32)
    g = gpu_run(ir, off, [price, vol])
    assert_parity(g, oracle.run(ir, off, [price, vol]), off)
    assert g["n_matches"] == 4 and set(g["key"].tolist()) == {3}


def test_error_parity_npe_illegal_state():
    """zeroOrMore stock variant with state.get (no getOrElse): a dip before any take makes
    the PROCEED walk miss its predecessor (H2, IllegalStateException); README variant on a
    stream starting with a dip reads a null fold (NullPointerException)."""
    S = W.stock_query("test").schema
    from kafkastreams_cep_amd import QueryBuilder
    q = (QueryBuilder(S).select().where(lambda k, v, ts, s: v.volume > 1000).fold("avg", lambda k, v, c: v.price).then()
         .select().zeroOrMore().skipTillNextMatch().where(lambda k, v, ts, s: v.price > s.get("avg"))
         .fold("avg", lambda k, v, c: (c + v.price) / 2).fold("volume", lambda k, v, c: v.volume).then()
         .select().skipTillNextMatch().where(lambda k, v, ts, s: v.volume < 0.8 * s.getOrElse("volume", 5000)).build())
    ir = q.to_ir()
    price = np.array([100, 90, 95, 120, 80], np.int32)
    vol = np.array([1500, 900, 100, 900, 100], np.int32)
    off = np.array([0, 5], np.uint64)
    r = oracle.run(ir, off, [price, vol])
    assert r["err_code"][0] in (1, 2)
    assert_parity(gpu_run(ir, off, [price, vol]), r, off)


def test_synth_generator_matches_numpy():
    for kind, cfg in (("stock", W.SynthConfig("t", "stock", 300, 200, 99, key_base=12345)),
                      ("abc", W.SynthConfig("t", "abc", 50, 1000, 7))):
        d = N.synth_stream(kind, cfg.seed, cfg.n_keys, cfg.mean_events, cfg.key_base)
        off_g, cols_g = d.download()
        off_h, cols_h = W.generate(cfg)
        np.testing.assert_array_equal(off_g, off_h)
        for a, b in zip(cols_g, cols_h):
            np.testing.assert_array_equal(a, b)


def test_device_resident_batch_and_digest():
    cfg = W.SynthConfig("t", "stock", 2000, 500, 0xCE90000 + 3)
    d = N.synth_stream("stock", cfg.seed, cfg.n_keys, cfg.mean_events)
    q = N.Query(W.stock_query("readme").to_ir())
    s = N.Session(q)
    s.push_device(d)
    n, dig = s.digest(0)
    off, cols = d.download()
    r = oracle.run(q.ir, off, cols, threads=8)
    g = gpu_run(q.ir, off, cols)
    assert n == r["n_matches"] and (n, dig) == g["digest"]


def test_device_shard_gather():
    """A rank's shard of a device stream (Kafka partitioner + cep_gather_keys) equals the host
    split (shard.gather_host), timestamps included, and matches like the oracle on it."""
    from kafkastreams_cep_amd import shard as SH
    cfg = W.SynthConfig("t", "stock", 500, 300, 0xCE90000 + 3)
    d = N.synth_stream("stock", cfg.seed, cfg.n_keys, cfg.mean_events)
    ts = N.synth_ts(d.n_events, 1000)
    off, cols = d.download()
    for world, rank in ((2, 0), (2, 1), (8, 5)):
        keys, loff = SH.shard_layout(off, world, rank)
        sh, sts = N.shard_stream(d, keys, loff, ts)
        o2, c2 = sh.download()
        np.testing.assert_array_equal(o2, loff)
        for a, b in zip(c2, SH.gather_host(off, cols, keys, loff)):
            np.testing.assert_array_equal(a, b)
        t2 = sts.download(np.int64, sh.n_events)
        np.testing.assert_array_equal(t2, SH.gather_host(off, [1000 + np.arange(d.n_events)], keys, loff)[0])
        ir = W.stock_query("readme").to_ir()
        s = N.Session(N.Query(ir))
        s.push_device(sh, sts.ptr)
        assert s.watermark() == int(t2.max())
        assert_parity(session_result(s, 0, o2), oracle.run(ir, o2, c2), o2)


def test_watermark():
    q = N.Query(W.stock_query("readme").to_ir())
    s = N.Session(q)
    off = np.array([0, 3], np.uint64)
    s.push(off, [np.array([1, 2, 3], np.int32), np.array([1, 2, 3], np.int32)], ts=np.array([5, 9, 7]))
    assert s.watermark() == 9
    # the max kernel's 16-byte path, its odd tail and a lone event; the maximum first, inside, last
    rng = np.random.default_rng(11)
    for n in (1, 2, 5, 1001, (1 << 20) + 3):
        for where in (0, n // 2, n - 1):
            ts = rng.integers(-(1 << 40), 1 << 40, n)
            ts[where] = (1 << 41) + n
            off = np.array([0, n], np.uint64)
            s.push(off, [np.zeros(n, np.int32), np.zeros(n, np.int32)], ts=ts)
            assert s.watermark() == (1 << 41) + n
    # an 8-byte-aligned device pointer (the scalar path)
    d = N.synth_stream("stock", 5, 40, 30)
    t = N.synth_ts(d.n_events + 1, -7)
    s2 = N.Session(q)
    s2.push_device(d, t.ptr + 8)
    assert s2.watermark() == -7 + d.n_events


def test_watermark_folded():
    """> 64 keys: the watermark comes from the bitmap pass's block maxima reduced by the
    estimate pass (session.cpp wm_fold), not from its own pass; the maximum in the first,
    a middle and the last event, batch sizes around the bitmap block (4096 events), unaligned
    device timestamps."""
    q = N.Query(W.stock_query("readme").to_ir())
    s = N.Session(q)
    rng = np.random.default_rng(12)
    for nk, mean in ((65, 3), (100, 41), (1000, 40), (3000, 700)):
        d = N.synth_stream("stock", 7, nk, mean)
        off, cols = d.download()
        n = d.n_events
        for where in (0, n // 2, n - 1):
            ts = rng.integers(-(1 << 40), 1 << 40, n)
            ts[where] = (1 << 41) + n
            s.push(off, cols, ts=ts)
            assert s.watermark() == (1 << 41) + n, (nk, n, where)
    d = N.synth_stream("stock", 5, 400, 30)
    t = N.synth_ts(d.n_events + 1, -7)
    s.push_device(d, t.ptr + 8)
    assert s.watermark() == -7 + d.n_events


def test_cfg2_full_size_checksum():
    """Config 2 at its BASELINE size (1e8 events over 1e4 keys, generated in HBM): the
    stencil's match count and checksum equal the oracle's on the same stream."""
    cfg = W.CONFIGS[2]
    d = N.synth_stream("abc", cfg.seed, cfg.n_keys, cfg.mean_events)
    q = N.Query(W.strict_abc_query().to_ir())
    assert q.kind == N.CEP_KIND_STENCIL
    s = N.Session(q)
    s.push_device(d)
    n, dig = s.digest(0)
    off, cols = d.download()
    r = oracle.run(q.ir, off, cols, threads=16)
    emit_seq = r["emit_pos"].astype(np.uint64) - off[r["key"].astype(np.int64)]
    pk = np.repeat(r["key"].astype(np.int64), np.diff(r["pair_off"].astype(np.int64)))
    pseq = r["pair_pos"].astype(np.uint64) - off[pk]
    assert n == r["n_matches"] > 3_000_000
    assert dig == W.match_digest(r["key"], emit_seq, r["pair_off"], pseq, r["pair_stage"])
    # size-independent property: every match is 3 consecutive events of one key, A B C
    m = s.matches(0)
    seq = m["pair_seq"].reshape(-1, 3).astype(np.int64)
    assert np.all(seq[:, 0] == seq[:, 1] + 1) and np.all(seq[:, 1] == seq[:, 2] + 1)
    v = cols[0]
    base = off[m["key"].astype(np.int64)].astype(np.int64)
    assert np.all(v[base + seq[:, 2]] < 4) and np.all((v[base + seq[:, 1]] >= 4) & (v[base + seq[:, 1]] < 8))
    assert np.all(v[base + seq[:, 0]] >= 8)


@pytest.mark.parametrize("tier", TIERS)
def test_capacity_retry_small_queue(tier):
    """A 2-record run queue overflows on most keys; they are re-run with 8x, 64x, 512x
    the queue and the result is still exact."""
    cfg = W.SynthConfig("t", "stock", 300, 600, 0xCE90000 + 3)
    off, cols = W.generate(cfg)
    ir = W.stock_query("readme").to_ir()
    q = N.Query(ir)
    s = N.Session(q, max_runs=2, tier=tier)
    r = oracle.run(ir, off, cols, threads=8)
    assert r["max_live_runs"] > 2
    assert_parity(gpu_run(ir, off, cols, session=s), r, off)


def test_pool_growth_tiny_pools():
    """Node/predecessor/output pools sized far below need: keys that run out are retried
    with grown pools (indices of the kept prefix stay valid)."""
    cfg = W.SynthConfig("t", "stock", 500, 800, 0xCE90000 + 3)
    off, cols = W.generate(cfg)
    ir = W.stock_query("readme").to_ir()
    s = N.Session(N.Query(ir), pool_factor=0.001)
    assert_parity(gpu_run(ir, off, cols, session=s), oracle.run(ir, off, cols, threads=8), off)


@pytest.mark.parametrize("tier", TIERS)
@pytest.mark.parametrize("query,n_batches", [("readme", 3), ("test", 5), ("any_kleene", 3), ("strict", 4)])
def test_streaming_session_batches(query, n_batches, tier):
    """cep_opts.streaming: the stream cut into consecutive batches per key gives, per key, the
    oracle's single-pass matches (global sequence numbers) and exceptions."""
    import stream_split as SS
    kind = "abc" if query == "strict" else "stock"
    cfg = W.SynthConfig("t", kind, 400, 700, 0xCE90000 + 3)
    off, cols = W.generate(cfg)
    q = {"readme": lambda: W.stock_query("readme"), "test": lambda: W.stock_query("test"),
         "any_kleene": W.any_kleene_query, "strict": W.strict_abc_query}[query]()
    ir = q.to_ir()
    r = oracle.run(ir, off, cols, threads=8)
    s = N.Session(N.Query(ir), streaming=True, tier=tier, max_runs=64)
    outs = []
    for ko, cs in SS.split(off, cols, n_batches, seed=n_batches):
        s.push(ko, cs)
        m = s.matches(0)
        m["err_code"], m["err_seq"] = s.key_errors(0)
        outs.append(m)
    assert SS.merge(outs) == SS.oracle_per_key(r, off)
    np.testing.assert_array_equal(outs[-1]["err_code"], r["err_code"])


@pytest.mark.parametrize("case", ["nfa_skip_till_any", "fuzz8", "fuzz80", "fuzz96"])
def test_streaming_widen_continuation(case):
    """Streams run the stream build (3-pair Dewey versions); a key whose versions outgrow it
    stops before that event and the wide build continues it in the same batch (nfa_lane.h
    stop_event, session.cpp run_nfa): these queries need 4+ pairs on their streams, and the
    merged matches and exceptions equal the oracle's single pass."""
    import stream_split as SS
    from fuzz_queries import random_query, random_stream
    from ref_queries import build_case, kats
    if case.startswith("fuzz"):
        seed = int(case[4:])
        q = random_query(seed)
        off, cols = random_stream(seed, 60, 14)
    else:
        q, off, cols = build_case(case, kats()[case])
    ir = q.to_ir()
    r = oracle.run(ir, off, cols)
    s = N.Session(N.Query(ir), streaming=True, max_runs=16384)
    outs, widened = [], 0
    for ko, cs in SS.split(off, cols, 3, seed=7):
        s.push(ko, cs)
        widened += s.stats(0)["retried_jobs"]
        m = s.matches(0)
        m["err_code"], m["err_seq"] = s.key_errors(0)
        outs.append(m)
    assert widened > 0
    assert SS.merge(outs) == SS.oracle_per_key(r, off)
    np.testing.assert_array_equal(outs[-1]["err_code"], r["err_code"])


@pytest.mark.parametrize("query", ["readme", "any_kleene"])
def test_streaming_snapshot_restore(query):
    """cep_session_snapshot / cep_session_restore: after every batch the stream's state moves
    to a brand-new session through a snapshot blob; the merged matches and exceptions equal
    the oracle's single pass (and the uninterrupted streaming session's)."""
    import stream_split as SS
    cfg = W.SynthConfig("t", "stock", 300, 700, 0xCE90000 + 4)
    off, cols = W.generate(cfg)
    q = W.stock_query("readme") if query == "readme" else W.any_kleene_query()
    ir = q.to_ir()
    r = oracle.run(ir, off, cols, threads=8)
    s = N.Session(N.Query(ir), streaming=True, max_runs=64)
    outs = []
    for ko, cs in SS.split(off, cols, 4, seed=7):
        s.push(ko, cs)
        m = s.matches(0)
        m["err_code"], m["err_seq"] = s.key_errors(0)
        outs.append(m)
        blob = s.snapshot()
        s.close()
        s = N.Session(N.Query(ir), streaming=True, max_runs=64)
        s.restore(blob)
    assert SS.merge(outs) == SS.oracle_per_key(r, off)
    np.testing.assert_array_equal(outs[-1]["err_code"], r["err_code"])


def test_streaming_reset_restarts_every_key():
    """cep_session_reset: a streaming session that has run batches and is reset matches a
    fresh session pushed the same batches (allocations reused, every key from the initial
    state)."""
    import stream_split as SS
    cfg = W.SynthConfig("t", "stock", 300, 600, 0xCE90000 + 5)
    off, cols = W.generate(cfg)
    ir = W.stock_query("readme").to_ir()
    r = oracle.run(ir, off, cols, threads=8)
    s = N.Session(N.Query(ir), streaming=True)
    parts = SS.split(off, cols, 3, seed=3)
    for ko, cs in parts[:2]:
        s.push(ko, cs)
    s.reset()
    outs = []
    for ko, cs in parts:
        s.push(ko, cs)
        outs.append(s.matches(0))
    assert SS.merge(outs) == SS.oracle_per_key(r, off)
    assert s.watermark() == np.iinfo(np.int64).min


def test_streaming_device_slices_checksum():
    """bench.py's streaming figure: the stream cut per key into consecutive device slices
    (native.gather_ranges) and pushed through one streaming session gives, summed over the
    batches, the per-batch session's match count and checksum of the whole stream."""
    import bench
    cfg = W.CONFIGS[3]
    stream = N.synth_stream("stock", cfg.seed, 3000, 1000)
    q = N.Query(W.stock_query("readme").to_ir())
    whole = N.Session(q)
    whole.push_device(stream)
    want = whole.digest(0)
    s = N.Session(q, streaming=True)
    n, dig = 0, 0
    for p in bench.slice_stream(stream, 7):
        s.push_device(p)
        m, d = s.digest(0)
        n, dig = n + m, (dig + d) % (1 << 64)
    assert want[0] > 100 and (n, dig) == want


def test_snapshot_rejects_mismatch():
    ir = W.stock_query("readme").to_ir()
    s = N.Session(N.Query(ir), streaming=True)
    s.push(np.array([0, 2], np.uint64), [np.array([1, 2], np.int32), np.array([1, 2], np.int32)])
    blob = s.snapshot()
    other = N.Session(N.Query(W.any_kleene_query().to_ir()), streaming=True)
    with pytest.raises(N.CepError):
        other.restore(blob)  # a different query
    opts = N.Session(N.Query(ir), streaming=True, max_runs=64)
    with pytest.raises(N.CepError):
        opts.restore(blob)  # other ring geometry
    with pytest.raises(N.CepError):
        N.Session(N.Query(ir), streaming=True).restore(blob[:40])  # truncated
    with pytest.raises(N.CepError):
        N.Session(N.Query(ir)).snapshot()  # not a streaming session
    fresh = N.Session(N.Query(ir), streaming=True)
    fresh.restore(blob)
    assert fresh.snapshot() == blob


def test_streaming_rejects_other_key_space():
    s = N.Session(N.Query(W.stock_query("readme").to_ir()), streaming=True)
    s.push(np.array([0, 2], np.uint64), [np.array([1, 2], np.int32), np.array([1, 2], np.int32)])
    with pytest.raises(N.CepError):
        s.push(np.array([0, 1, 2], np.uint64), [np.array([1, 2], np.int32), np.array([1, 2], np.int32)])


@pytest.mark.parametrize("query", ["readme", "strict"])
def test_arrival_order_batch(query):
    """An arrival-order batch (key id per event) is partitioned on the GPU (stable per key) and
    matches exactly like the same stream handed over key-partitioned."""
    kind = "abc" if query == "strict" else "stock"
    cfg = W.SynthConfig("t", kind, 700, 400, 0xCE90000 + 3)
    off, cols = W.generate(cfg)
    keys, acols = W.generate_arrival(cfg)
    ir = (W.strict_abc_query() if query == "strict" else W.stock_query("readme")).to_ir()
    s = N.Session(N.Query(ir))
    s.push_arrival(keys, acols, cfg.n_keys)
    ko, arrival, ms = s.layout()
    np.testing.assert_array_equal(ko, off)
    for a, c in zip(acols, cols):  # each CSR position holds its arrival event
        np.testing.assert_array_equal(a[arrival], c)
    assert ms > 0
    g = s.matches(0)
    code, seq = s.key_errors(0)
    g["err_code"], g["err_seq"] = code, seq
    g["digest"] = s.digest(0)
    g["emit_pos"] = (off[g["key"].astype(np.int64)] + g["emit_seq"]).astype(np.uint64)
    pk = np.repeat(g["key"].astype(np.int64), np.diff(g["pair_off"].astype(np.int64)))
    g["pair_pos"] = (off[pk] + g["pair_seq"]).astype(np.uint64)
    assert_parity(g, oracle.run(ir, off, cols, threads=8), off)


@pytest.mark.parametrize("shape", ["round_robin", "sorted", "one_key", "random", "runs", "tiny"])
def test_partition_shapes(shape):
    """The onesweep partition (partition.hip: one count pass, a tile look-back per pass) against
    numpy's stable argsort, on key orders that take every path of its counting and ranking: keys
    arriving round-robin over 300k keys (3 passes of 7 bits; a wave's high digits all equal),
    sorted (every wave's digits equal), a single key, random, long runs of one key, and a
    batch smaller than one wave."""
    rng = np.random.default_rng(11)
    n_keys = {"round_robin": 300_000, "sorted": 70_000, "one_key": 5_000, "random": 1 << 20, "runs": 4_096,
              "tiny": 300}[shape]
    n = {"tiny": 37}.get(shape, 6_000_000)
    if shape == "round_robin":
        keys = (np.arange(n, dtype=np.int64) % n_keys).astype(np.uint32)
    elif shape == "sorted":
        keys = np.sort(rng.integers(0, n_keys, n)).astype(np.uint32)
    elif shape == "one_key":
        keys = np.full(n, n_keys - 1, np.uint32)
    elif shape == "runs":
        keys = np.repeat(rng.integers(0, n_keys, n // 1000 + 1), 1000)[:n].astype(np.uint32)
    else:
        keys = rng.integers(0, n_keys, n).astype(np.uint32)
    vals = rng.integers(0, 16, n).astype(np.int32)
    s = N.Session(N.Query(W.strict_abc_query().to_ir()))
    s.push_arrival(keys, [vals], n_keys)
    ko, arrival, _ = s.layout()
    want = np.zeros(n_keys + 1, np.uint64)
    np.cumsum(np.bincount(keys, minlength=n_keys), out=want[1:])
    np.testing.assert_array_equal(ko, want)
    np.testing.assert_array_equal(arrival, np.argsort(keys, kind="stable"))


@pytest.mark.parametrize("query", ["readme", "strict"])
def test_repeated_batch_allocates_nothing(query):
    """ A session pushed a batch of the shape it has already seen reuses
    every device buffer - pools, run queues, the bitmap, the lane order's scratch, the
    partition's - so a push makes no allocation (an allocation inside a push's timed interval
    would count its host time, hipFree synchronises, as kernel time), key-partitioned and in
    arrival order; and the repeated pushes give the same matches."""
    kind = "abc" if query == "strict" else "stock"
    cfg = W.SynthConfig("t", kind, 3000, 400, 0xCE90000 + 3)
    off, cols = W.generate(cfg)
    keys, acols = W.generate_arrival(cfg)
    ir = (W.strict_abc_query() if query == "strict" else W.stock_query("readme")).to_ir()
    s = N.Session(N.Query(ir))
    s.push(off, cols)
    first = s.digest(0)
    assert s.stats(0)["allocs"] > 0
    seen = []  # (push kind, stats, digest): the whole history in a failure's message

    def check(kind):
        seen.append((kind, s.stats(0), s.digest(0)))
        if seen[-1][1]["allocs"] or seen[-1][2] != first:
            diag = {}
            if kind == "arrival":  # was the partition right?
                ko, perm, _ = s.layout()
                diag["key_off_equal"] = bool(np.array_equal(ko, off))
                if perm is not None:
                    pk = keys[perm.astype(np.int64)]
                    diag["perm_keys_sorted"] = bool(np.all(np.diff(pk.astype(np.int64)) >= 0))
                    diag["perm_stable"] = bool(np.all((np.diff(perm.astype(np.int64)) > 0) | (np.diff(pk.astype(np.int64)) > 0)))
            pytest.fail(json.dumps({"pushes": seen, "diag": diag}))
    for _ in range(3):
        s.push(off, cols)
        check("csr")
    s.push_arrival(keys, acols, cfg.n_keys)
    seen.append(("arrival first", s.stats(0), s.digest(0)))
    for _ in range(6):
        s.push_arrival(keys, acols, cfg.n_keys)
        check("arrival")


@pytest.mark.gpu
def test_sessions_interleaved_on_their_streams():
    """ The conditions of the round-5 arrival-order flake, all at once: two
    sessions on their own non-blocking streams - one taking arrival-order pushes (partition +
    NFA), one stencil pushes that return without a host sync and are not read back between
    pushes - interleaved with JSON decode + `[symbol]` keys on the default stream and a third
    session's key-partitioned pushes.  Every result stays exactly what the same push gives alone."""
    cfg = W.SynthConfig("t", "stock", 3000, 400, 0xCE90000 + 3)
    off, cols = W.generate(cfg)
    keys, acols = W.generate_arrival(cfg)
    scfg = W.SynthConfig("t", "abc", 2000, 2000, 0xCE90000 + 2)
    soff, scols = W.generate(scfg)
    a = N.Session(N.Query(W.stock_query("readme").to_ir()))
    b = N.Session(N.Query(W.strict_abc_query().to_ir()))
    c = N.Session(N.Query(W.stock_query("readme").to_ir()))
    a.push(off, cols)
    want_a = a.digest(0)
    b.push(soff, scols)
    want_b = b.digest(0)
    c.push(off, cols)
    jcfg = W.SynthConfig("t", "stock", 300, 60, W.CONFIGS[3].seed)
    jk, jc = W.generate_arrival(jcfg)
    recs = [b'{"volume":%d,"price":%d,"name":"SYM%d"}' % (int(v), int(p), int(k)) for k, p, v in zip(jk, jc[0], jc[1])]
    jb = N.StockJsonBatch.from_records(recs)
    seen = []
    for i in range(8):
        a.push_arrival(keys, acols, cfg.n_keys)
        b.push(soff, scols)  # (no read-back: its kernels may still run during what follows)
        d = N.decode_stock_json(jb, 4)
        sk, n_sym = N.symbol_keys(jb, d)
        c.push(off, cols)
        b.push(soff, scols)
        got_a = a.digest(0)
        got_c = c.digest(0)
        ok_sym = n_sym == jcfg.n_keys and np.array_equal(sk.download(np.uint32, len(recs)), jk.astype(np.uint32))
        seen.append((i, got_a == want_a, got_c == want_a, ok_sym, a.stats(0)["allocs"]))
        if i % 2:
            seen[-1] += (b.digest(0) == want_b,)
    assert all(all(x for x in s[1:4]) and (s[4] == 0 or s[0] == 0) and (len(s) < 6 or s[5]) for s in seen), seen
    assert b.digest(0) == want_b


def test_arrival_generator_matches_numpy():
    cfg = W.SynthConfig("t", "stock", 300, 200, 77, key_base=5)
    st = N.synth_arrival_stream("stock", cfg.seed, cfg.n_keys, cfg.mean_events, cfg.key_base)
    keys, cols = st.download()
    k2, c2 = W.generate_arrival(cfg)
    np.testing.assert_array_equal(keys, k2)
    for a, b in zip(cols, c2):
        np.testing.assert_array_equal(a, b)


def test_arrival_rejects_bad_key():
    s = N.Session(N.Query(W.stock_query("readme").to_ir()))
    with pytest.raises(N.CepError):
        s.push_arrival(np.array([0, 5], np.uint32), [np.array([1, 2], np.int32), np.array([1, 2], np.int32)], 2)


def test_lane_balance_figure():
    """cep_lane_balance: the longest-first lane order packs waves of similar work (closer to
    1.0 than key-index order); both are >= 1 by construction."""
    cfg = W.SynthConfig("t", "stock", 20000, 300, 0xCE90000 + 3)
    off, cols = W.generate(cfg)
    s = N.Session(N.Query(W.stock_query("readme").to_ir()))
    s.push(off, cols)
    ordered, identity = s.lane_balance(0)
    assert 1.0 <= ordered <= identity
    s2 = N.Session(N.Query(W.strict_abc_query().to_ir()))  # stencil: no lane order
    s2.push(*W.generate(W.SynthConfig("t", "abc", 100, 100, 1)))
    with pytest.raises(N.CepError):
        s2.lane_balance(0)
