"""Semantic WITHIN: the window the README query states (README.md:19-28,
"WITHIN 1 hour") actually prunes runs.  The reference's own WITHIN never fires — every
non-begin run sits in an epsilon stage whose window is -1 (nfa/Stage.java:42-46,
ComputationStage.java:98-100) — so this mode is a build option (IR v2 flag,
`Pattern.to_ir(semantic_within=True)`), never the parity mode.  Its definition: an epsilon
stage keeps the window of the stage it copies; NFA.java:143-144's check then drops a non-begin
run whose start (getFirstPatternTimestamp, :347-349) is more than the window before the
current event, and removePattern collects it (:101-103).

Parity anchor: the oracle's semantic mode (oracle/cep_oracle.cpp newEpsilonState with
`semantic`), itself the reference restatement with that one line changed; it is not pinned by
a reference fixture (the reference has no such mode): "parity unpinned" beyond the oracle.
CPU tests run the generated kernel code through tests/lane_cpu; GPU tests through libcep.
"""
import numpy as np
import pytest

import lane_cpu
import oracle
from kafkastreams_cep_amd import native as N
from kafkastreams_cep_amd import workloads as W

QUERIES = {"readme": lambda: W.stock_query("readme"), "test": lambda: W.stock_query("test"),
           "any_kleene": W.any_kleene_query}


def stream(n_keys=300, mean=400, gap=60_000, seed=1):
    """cfg-3 style stock stream; event times with random gaps (mean `gap` ms) so a 1 h window
    spans ~3.6e6 / gap events"""
    cfg = W.SynthConfig("t", "stock", n_keys, mean, W.CONFIGS[3].seed)
    off, cols = W.generate(cfg)
    rng = np.random.default_rng(seed)
    ts = np.cumsum(rng.integers(0, 2 * gap, int(off[-1]))).astype(np.int64) + 1_600_000_000_000
    return off, cols, ts


def ts_for(query, ts):
    # cfg 4's window is 10 ms: event times 1 ms apart on average there
    return ts // 60_000 if query == "any_kleene" else ts


@pytest.mark.parametrize("query", list(QUERIES))
def test_lane_semantic_vs_oracle(query):
    off, cols, ts = stream()
    t = ts_for(query, ts)
    ir = QUERIES[query]().to_ir(semantic_within=True)
    r = oracle.run(ir, off, cols, ts=t, threads=8)
    lane_cpu.assert_same(lane_cpu.run(ir, off, cols, ts=t), r, off)
    lane_cpu.assert_same(lane_cpu.run(ir, off, cols, ts=t, defer=False), r, off)


def test_lane_semantic_streaming():
    """A run's start time crosses batch boundaries (it is carried in the run record)."""
    import stream_split as SS
    off, cols, ts = stream(n_keys=200, mean=500)
    ir = W.stock_query("readme").to_ir(semantic_within=True)
    r = oracle.run(ir, off, cols, ts=ts, threads=8)
    outs = []
    for i, (ko, cs) in enumerate(SS.split(off, list(cols) + [ts], 4, seed=4)):
        m = lane_cpu.run(ir, ko, cs[:-1], ts=cs[-1], streaming=True, reset=(i == 0), rcap=64)
        outs.append(m)
    assert SS.merge(outs) == SS.oracle_per_key(r, off)


def test_semantic_prunes_and_parity_mode_does_not():
    """The window decides: with wide gaps runs expire (fewer matches than parity mode); with
    event times 1 ms apart a 1 h window never expires and the semantic result equals parity."""
    off, cols, ts = stream()
    q = W.stock_query("readme")
    par = oracle.run(q.to_ir(), off, cols, ts=ts, threads=8)
    sem = oracle.run(q.to_ir(semantic_within=True), off, cols, ts=ts, threads=8)
    assert sem["n_matches"] < par["n_matches"]
    dense = np.arange(int(off[-1]), dtype=np.int64)
    sem2 = oracle.run(q.to_ir(semantic_within=True), off, cols, ts=dense, threads=8)
    par2 = oracle.run(q.to_ir(), off, cols, ts=dense, threads=8)
    for k in ("n_matches", "n_pairs"):
        assert sem2[k] == par2[k]
    np.testing.assert_array_equal(sem2["pair_pos"], par2["pair_pos"])


def test_semantic_ir_compiles_and_gates():
    """IR v2 compiles on the host (no GPU); a windowed strict chain leaves the stencil path;
    the parity-mode IR is unchanged (v1)."""
    strict = W.strict_abc_query()
    assert N.Query(strict.to_ir()).kind == N.CEP_KIND_STENCIL
    assert N.Query(strict.to_ir(semantic_within=True)).kind == N.CEP_KIND_STENCIL  # no window: same
    q = W.stock_query("readme")
    assert q.to_ir()[4:8] == b"\x01\x00\x00\x00"
    src = N.Query(q.to_ir(semantic_within=True)).jit_source
    assert "sk_window" in src and "FS + 1" in src
    assert "sk_window" not in N.Query(q.to_ir()).jit_source


# ------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("query", list(QUERIES))
def test_gpu_semantic_vs_oracle(query):
    from gpu_helpers import assert_parity, gpu_run
    off, cols, ts = stream(n_keys=2000, mean=500)
    t = ts_for(query, ts)
    ir = QUERIES[query]().to_ir(semantic_within=True)
    r = oracle.run(ir, off, cols, ts=t, threads=8)
    assert_parity(gpu_run(ir, off, cols, ts=t), r, off)


@pytest.mark.gpu
def test_gpu_semantic_group_of_variants():
    """Config 5's variants in semantic mode: one kernel group, every query exact."""
    from gpu_helpers import assert_parity, session_result
    off, cols, ts = stream(n_keys=400, mean=500)
    qs = [p.to_ir(semantic_within=True) for p in W.multi_queries(16)]
    s = N.Session([N.Query(ir) for ir in qs])
    s.push(off, cols, ts)
    assert s.stats(0)["group_queries"] == 16
    for i, ir in enumerate(qs):
        assert_parity(session_result(s, i, off), oracle.run(ir, off, cols, ts=ts, threads=8), off)


@pytest.mark.gpu
def test_gpu_semantic_streaming():
    """A streaming session carries each run's start across batches."""
    import stream_split as SS
    off, cols, ts = stream(n_keys=300, mean=600)
    ir = W.stock_query("readme").to_ir(semantic_within=True)
    r = oracle.run(ir, off, cols, ts=ts, threads=8)
    s = N.Session(N.Query(ir), streaming=True, max_runs=64)
    outs = []
    for ko, cs in SS.split(off, list(cols) + [ts], 4, seed=4):
        s.push(ko, cs[:-1], cs[-1])
        m = s.matches(0)
        m["err_code"], m["err_seq"] = s.key_errors(0)
        outs.append(m)
    assert SS.merge(outs) == SS.oracle_per_key(r, off)


@pytest.mark.gpu
def test_gpu_semantic_needs_jit_tier():
    ir = W.stock_query("readme").to_ir(semantic_within=True)
    with pytest.raises(N.CepError):
        N.Session(N.Query(ir), tier=N.CEP_TIER_INTERP)
