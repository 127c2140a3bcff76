"""CPU checks of the JSON ingest oracle (oracle/json_oracle.py): the README demo records decode
to the README's values (README.md:73-80, the one reference fixture) and are the console
producer's layout; the serializer's own layout (StockEventSerDe.java:75-82, json-simple's HashMap
order) decodes to the same values; the hand-written json-simple cases give their outcomes."""
import json_cases as JC
import pytest

import json_oracle as J


def test_readme_records_decode():
    for rec, price, vol in JC.README:
        st, p, v, span = J.deserialize(rec)
        assert (st, p, v) == (J.OK, price, vol)
        off, ln, esc = span
        name = rec[off:off + ln]
        assert J.readme_record(name.decode(), p, v) == rec and not esc
        ser = J.serialize(name.decode(), p, v)  # what StockEventSerDe.serialize writes
        assert ser.startswith(b'{"volume":') and J.deserialize(ser)[:3] == (J.OK, price, vol)


@pytest.mark.parametrize("rec,code", JC.CASES)
def test_case_outcomes(rec, code):
    assert J.deserialize(rec)[0] == code, rec


def test_narrow_for_int32_columns():
    assert J.deserialize(b'{"price":3000000000,"volume":2}', 4)[0] == J.NARROW
    assert J.deserialize(b'{"price":-2147483648,"volume":2147483647}', 4)[:3] == (J.OK, -(1 << 31), (1 << 31) - 1)


def test_deep_nesting_parses_in_reference():
    # json-simple has no depth limit; the GPU decoder stops at 64 (CEP_JSON_DEPTH, documented)
    assert J.deserialize(JC.deep(100))[0] == J.OK


def test_fuzz_covers_every_outcome():
    seen = {J.deserialize(r)[0] for r in JC.fuzz(1, 4000)}
    assert {J.OK, J.PARSE, J.CLASS_CAST, J.NULL} <= seen


# ---- the GPU decoder's state machine, compiled for the host (tests/json_cpu.py) ----

import json_cpu  # noqa: E402
import numpy as np  # noqa: E402


def _same(records, col_width=8):
    got = json_cpu.decode(records, col_width)
    exp = json_cpu.oracle_arrays([J.deserialize(r, col_width) for r in records])
    for g, e, what in zip(got, exp, ("status", "price", "volume", "name_span")):
        bad = np.nonzero((g != e).reshape(len(records), -1).any(axis=1))[0]
        assert len(bad) == 0, (what, [(records[i], g[i], e[i]) for i in bad[:5]])


def test_lane_parser_cases():
    _same([c for c, _ in JC.CASES] + [r for r, _, _ in JC.README])
    _same([c for c, _ in JC.CASES], col_width=4)


def test_lane_parser_fuzz():
    _same(JC.fuzz(7, 20000))


def test_lane_parser_depth_limit():
    st = json_cpu.decode([JC.deep(63), JC.deep(64)])[0]
    assert st.tolist() == [J.OK, J.DEPTH]  # 64 levels incl. the record object; deeper is CEP_JSON_DEPTH (documented)


def test_fast_path_taken_for_serializer_records_and_exact():
    canon = [J.serialize("e%d" % i, p, v) for i, (p, v) in enumerate(
        [(1, 2), (-5, 0), (123456789012345678, -999999999999999999), (120, 1010)])] + [r for r, _, _ in JC.README]
    assert all(json_cpu.fast_path(r) == (True, True) for r in canon)
    # 19-digit numbers, escapes, other layouts: general path
    canon += [J.readme_record("e%d" % i, p, v) for i, (p, v) in enumerate([(1, 2), (-5, 0)])]
    assert all(json_cpu.fast_path(r) == (True, True) for r in canon)
    for r in (J.serialize("e", 1234567890123456789, 1), b'{"name":"a\\"b","price":1,"volume":2}',
              b'{"price":1,"volume":2,"name":"a"}', b'{"name":"a","price":1,"volume":2} ',
              b'{"volume":2,"price":1,"name":"a"} ', b'{"volume":2,"price":1,"name":"a\\u0041"}'):
        assert json_cpu.fast_path(r)[0] is False
    for r in [c for c, _ in JC.CASES] + JC.fuzz(5, 5000):
        assert json_cpu.fast_path(r)[1], r


def test_fast_path_name_lengths():
    for n in range(0, 24):
        for name in ("x" * n, "é" * (n // 2), "a" * n + '\\"', "\t" * n):
            r = b'{"name":"%s","price":%d,"volume":%d}' % (name.encode(), n, -n)
            fast, agree = json_cpu.fast_path(r)
            assert agree, r
            assert fast == ("\\" not in name), r
