"""The GPU lane logic (csrc/nfa_lane.h + the query's generated step), built for the host by
tests/lane_cpu.py, against the oracle: reference KATs, the stock configs at small size and
random fuzz queries, with walks deferred (the kernel's default) and in place (the retry
path).  No GPU: this pins the per-event logic and the deferred-walk machinery on CPU; the
GPU parity tests (test_gpu_parity.py) run the same code on the device."""
import numpy as np
import pytest

import lane_cpu
import oracle
from fuzz_queries import random_query, random_stream
from ref_queries import STOCK_KATS, STRING_KATS, build_case, kats
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
    lane_cpu.assert_same(lane_cpu.run(ir, off, cols), r, off)


def test_lane_any_kleene_small():
    cfg = W.SynthConfig("t", "stock", 100, 300, 0xCE90000 + 4)
    off, cols = W.generate(cfg)
    ir = W.any_kleene_query().to_ir()
    lane_cpu.assert_same(lane_cpu.run(ir, off, cols), oracle.run(ir, off, cols, threads=8), off)


def test_lane_capacity_retry():
    """rcap 2: most keys overflow the run queue and are re-run with walks in place."""
    cfg = W.SynthConfig("t", "stock", 100, 400, 0xCE90000 + 3)
    off, cols = W.generate(cfg)
    ir = W.stock_query("test").to_ir()
    g = lane_cpu.run(ir, off, cols, rcap=2)
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
