"""Shared helpers for the GPU parity tests: run a query through libcep and the oracle on
the same CSR batch and compare everything bit for bit."""
import numpy as np

import oracle
from kafkastreams_cep_amd import native as N
from kafkastreams_cep_amd import workloads as W


def gpu_run(ir, key_off, cols, force_nfa=False, ts=None, session=None, tier=N.CEP_TIER_JIT, query=0, push=True):
    q = N.Query(ir)
    s = session or N.Session(q, force_nfa=force_nfa, tier=tier)
    if push:
        s.push(key_off, cols, ts)
    return session_result(s, query, key_off, q.kind)


def session_result(s, query, key_off, kind=None):
    """The last batch's matches and key errors of one query of session `s`, as gpu_run."""
    m = s.matches(query)
    code, seq = s.key_errors(query)
    m["err_code"], m["err_seq"] = code, seq
    m["digest"] = s.digest(query)
    m["kind"] = kind
    off = np.asarray(key_off, np.uint64)
    m["emit_pos"] = (off[m["key"].astype(np.int64)] + m["emit_seq"]).astype(np.uint64)
    pair_key = np.repeat(m["key"].astype(np.int64), np.diff(m["pair_off"].astype(np.int64)))
    m["pair_pos"] = (off[pair_key] + m["pair_seq"]).astype(np.uint64)
    return m


def assert_parity(g, r, key_off):
    """GPU result `g` equals oracle result `r` exactly (matches, order, errors)."""
    assert g["n_matches"] == r["n_matches"], (g["n_matches"], r["n_matches"])
    assert g["n_pairs"] == r["n_pairs"]
    np.testing.assert_array_equal(g["key"], r["key"])
    np.testing.assert_array_equal(g["emit_pos"], r["emit_pos"].astype(np.uint64))
    np.testing.assert_array_equal(g["pair_off"], r["pair_off"])
    np.testing.assert_array_equal(g["pair_pos"], r["pair_pos"].astype(np.uint64))
    np.testing.assert_array_equal(g["pair_stage"], r["pair_stage"])
    np.testing.assert_array_equal(g["err_code"], r["err_code"])
    off = np.asarray(key_off, np.uint64)
    bad = r["err_code"] != 0
    np.testing.assert_array_equal(g["err_seq"][bad].astype(np.uint64) + off[:-1][bad],
                                  r["err_pos"][bad].astype(np.uint64))
    # the device checksum equals the host checksum of the oracle's matches
    emit_seq = r["emit_pos"].astype(np.uint64) - off[r["key"].astype(np.int64)]
    pk = np.repeat(r["key"].astype(np.int64), np.diff(r["pair_off"].astype(np.int64)))
    pseq = r["pair_pos"].astype(np.uint64) - off[pk]
    d = W.match_digest(r["key"], emit_seq, r["pair_off"], pseq, r["pair_stage"])
    assert g["digest"] == (r["n_matches"], d)
