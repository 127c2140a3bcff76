"""[symbol] keying (README.md:19-28): StockEvent JSON records -> one key per
distinct name, in order of first appearance (cep_symbol_keys, csrc/symbol.hip), then the
arrival-order batch keyed by symbol through the matcher.

Oracle: oracle/json_oracle.py's json-simple restatement gives each record's name as Java
would hold it; names are compared as UTF-16 code units (Java String.equals).  The reference
has no symbol-keying code of its own (its processor runs every key of a partition in one NFA,
SURVEY H13), so the key numbering is this build's definition: parity unpinned beyond the
oracle restatement."""
import numpy as np
import pytest

import json_oracle as JO
import oracle
from kafkastreams_cep_amd import native as N
from kafkastreams_cep_amd import workloads as W


def oracle_symbol_keys(records):
    """key per record (None where deserialize() throws) in order of first appearance"""
    ids, out = {}, []
    for rec in records:
        st = JO.deserialize(rec, 4)[0]
        if st:
            out.append(None)
            continue
        name = JO._parse(rec).get("name")
        ident = None if name is None else str(name).encode("utf-16-le", "surrogatepass")
        out.append(ids.setdefault(ident, len(ids)))
    return out, len(ids)


# the same symbols spelled differently must collapse; different ones must not
NAMES = [b"AAPL", b"A\\u0041PL", b"MSFT", b"M\\/SFT", b"M/SFT", "Zürich".encode(), b"Z\\u00fcrich",
         "\U0001F600x".encode(), b"\\ud83d\\ude00x", b"tab\\tx", b"tab\tx", b"", b"\\\"q\\\""]


def records_with(names, n, seed):
    rng = np.random.default_rng(seed)
    recs = []
    for i in range(n):
        c = rng.integers(0, len(names) + 3)
        p, v = int(rng.integers(1, 200)), int(rng.integers(0, 1100))
        if c < len(names):
            recs.append(b'{"name":"%s","price":%d,"volume":%d}' % (names[c], p, v))
        elif c == len(names):
            recs.append(b'{"name":null,"price":%d,"volume":%d}' % (p, v))  # a null name
        elif c == len(names) + 1:
            recs.append(b'{"name":"AAPL","price":"x","volume":1}')  # ClassCastException
        else:
            recs.append(b'{"volume":%d,"price":%d,"name":"AAPL"}' % (v, p))  # serializer's key order
    return recs


def test_oracle_symbol_identity():
    keys, n = oracle_symbol_keys([b'{"name":"%s","price":1,"volume":1}' % s for s in NAMES])
    # AAPL = AAPL; M\/SFT = M/SFT; Zürich both ways; the emoji raw and as a surrogate pair;
    # a raw tab and \t
    assert keys == [0, 0, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 7] and n == 8


@pytest.mark.gpu
def test_gpu_symbol_keys_vs_oracle():
    recs = records_with(NAMES, 20000, 7)
    want, n_sym = oracle_symbol_keys(recs)
    b = N.StockJsonBatch.from_records(recs)
    d = N.decode_stock_json(b, 4)
    keys, n = N.symbol_keys(b, d)
    got = keys.download(np.uint32, len(recs))
    assert n == n_sym
    np.testing.assert_array_equal(got, np.array([0xFFFFFFFF if k is None else k for k in want], np.uint32))


@pytest.mark.gpu
def test_gpu_symbol_keys_many_symbols_and_small_table():
    recs = [b'{"name":"S%d","price":1,"volume":2}' % (i * 7919 % 5000) for i in range(60000)]
    want, n_sym = oracle_symbol_keys(recs)
    b = N.StockJsonBatch.from_records(recs)
    d = N.decode_stock_json(b, 4)
    keys, n = N.symbol_keys(b, d)
    assert n == n_sym == 5000
    np.testing.assert_array_equal(keys.download(np.uint32, len(recs)), np.array(want, np.uint32))
    with pytest.raises(N.CepError):  # more names than the table holds
        N.symbol_keys(b, d, max_symbols=100)
    # between n_sym/2 and n_sym the table (>= 2 x max_symbols slots) does not fill,
    # but the limit still fails the call
    for m in (2600, 4000, 4999):
        with pytest.raises(N.CepError):
            N.symbol_keys(b, d, max_symbols=m)
    assert N.symbol_keys(b, d, max_symbols=5000)[1] == 5000


@pytest.mark.gpu
def test_gpu_symbol_keys_malformed_utf8_fails():
    recs = [b'{"name":"ok","price":1,"volume":2}', b'{"name":"bad\xff","price":1,"volume":2}']
    b = N.StockJsonBatch.from_records(recs)
    d = N.decode_stock_json(b, 4)
    if d.download()["status"][1] != 0:
        pytest.skip("decoder rejected the record itself")
    with pytest.raises(N.CepError):
        N.symbol_keys(b, d)


@pytest.mark.gpu
def test_gpu_json_symbol_keyed_matching():
    """JSON records of a cfg-3 stream (symbol = "SYM<k>", arrival order round robin) -> decode ->
    symbol keys -> arrival-order batch -> the README query per symbol == the oracle on the same
    events grouped by symbol (keys numbered by first appearance)."""
    cfg = W.SynthConfig("t", "stock", 300, 200, W.CONFIGS[3].seed)
    akeys, acols = W.generate_arrival(cfg)
    recs = [b'{"volume":%d,"price":%d,"name":"SYM%d"}' % (int(v), int(p), int(k))
            for k, p, v in zip(akeys, acols[0], acols[1])]
    b = N.StockJsonBatch.from_records(recs)
    d = N.decode_stock_json(b, 4)
    keys, n_sym = N.symbol_keys(b, d)
    assert n_sym == cfg.n_keys
    got_keys = keys.download(np.uint32, len(recs))
    # first appearance in round-robin arrival order = key order
    np.testing.assert_array_equal(got_keys, akeys.astype(np.uint32))
    ir = W.stock_query("readme").to_ir()
    s = N.Session(N.Query(ir))
    st = N.ArrivalStream(n_sym, len(recs), keys, [d.price, d.volume])
    s.push_arrival_device(st)
    m = s.matches(0)
    off, cols = W.generate(cfg)
    r = oracle.run(ir, off, cols, threads=8)
    assert m["n_matches"] == r["n_matches"] > 0
    emit = r["emit_pos"].astype(np.uint64) - off[r["key"].astype(np.int64)]
    np.testing.assert_array_equal(m["key"], r["key"])
    np.testing.assert_array_equal(m["emit_seq"], emit)
    np.testing.assert_array_equal(m["pair_stage"], r["pair_stage"])
