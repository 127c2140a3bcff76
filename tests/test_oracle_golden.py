"""The CPU oracle (oracle/cep_oracle.cpp) against the reference's own known-answer tests.

Pins the oracle before it is trusted as the parity checker.
"""
import numpy as np
import pytest

import oracle
from ref_queries import STOCK_KATS, STRING_KATS, build_case, kats, sequences

NFA_CASES = [n for n in kats() if n in STRING_KATS or n in STOCK_KATS]


def _names(q):
    chain = q.chain()
    names = []
    for p in chain:
        if p.getName() not in names:
            names.append(p.getName())
    return names + ["$final"]


@pytest.mark.parametrize("name", NFA_CASES)
def test_oracle_nfa_kats(name):
    case = kats()[name]
    q, off, cols = build_case(name, case)
    r = oracle.run(q.to_ir(), off, cols)
    assert int(r["err_code"][0]) == 0
    if "expected_count" in case:
        assert r["n_matches"] == case["expected_count"]
        return
    r["pair_seq_or_pos"] = r["pair_pos"]
    got = sequences(r, _names(q))
    exp = [{k: sorted(v) for k, v in e.items()} for e in case["expected"]]
    assert got == exp  # exact content and forward order


def test_oracle_readme_walk_order():
    """README.md:93-96 lists events oldest-first after the demo reverses walk order
    (test:demo/CEPStockKStreamsDemo.java:65-67): the walk is final stage first, newest first."""
    case = kats()["stock_readme"]
    q, off, cols = build_case("stock_readme", case)
    r = oracle.run(q.to_ir(), off, cols)
    a, b = int(r["pair_off"][0]), int(r["pair_off"][1])
    assert r["pair_pos"][a:b].tolist() == [5, 4, 3, 2, 1, 0]
    assert r["emit_pos"].tolist() == [5, 5, 7, 7]


def test_oracle_dewey_kats():
    case = kats()["dewey"]
    for v, ops, exp in case["apply"]:
        assert oracle.dewey(v, ops) == exp
    for a, b, exp in case["compatible"]:
        assert oracle.dewey_compatible(a, b) == exp


@pytest.mark.parametrize("name", ["buffer_one_run", "buffer_branching_run"])
def test_oracle_buffer_kats(name):
    case = kats()[name]
    sid = {"first": (0, 0), "second": (1, 1), "latest": (2, 2)}  # name id, StateType
    b = oracle.Buffer()
    for cur, off, prev, poff, ver in case["puts"]:
        if prev is None:
            assert b.put_begin(*sid[cur], off, ver) == 0
        else:
            assert b.put(*sid[cur], off, *sid[prev], poff, ver) == 0
    for (stage, off, ver), exp in case["gets"]:
        walk = b.peek(*sid[stage], off, ver, remove=False)
        assert len(walk) == exp["size"]
        for st, (nid, _) in sid.items():
            assert sum(1 for n, _ in walk if n == nid) == exp[st]
