"""GPU parity of the JSON ingest (csrc/ingest.hip, cep_decode_stock_json) against
oracle/json_oracle.py: the README demo records (README.md:73-80), the hand-written json-simple
cases, seeded fuzz, the LDS-staged and HBM paths, unaligned spans, and at bench size the
serialize -> decode round trip; then README JSON -> decoder -> NFA end to end."""
import ctypes as C

import numpy as np
import pytest

import json_cases as JC
import json_cpu
import json_oracle as J
import oracle
from kafkastreams_cep_amd import native as N
from kafkastreams_cep_amd import workloads as W

pytestmark = pytest.mark.gpu


def gpu_decode(records, col_width=8):
    out = N.decode_stock_json(N.StockJsonBatch.from_records(records), col_width).download()
    return out["status"], out["price"].astype(np.int64), out["volume"].astype(np.int64), out["name_span"]


def assert_oracle(records, col_width=8):
    got = gpu_decode(records, col_width)
    exp = json_cpu.oracle_arrays([J.deserialize(r, col_width) for r in records])
    for g, e, what in zip(got, exp, ("status", "price", "volume", "name_span")):
        bad = np.nonzero((g != e).reshape(len(records), -1).any(axis=1))[0]
        assert len(bad) == 0, (what, [(records[i], g[i], e[i]) for i in bad[:5]])


def test_readme_records():
    recs = [r for r, _, _ in JC.README]
    for w in (8, 4):
        st, p, v, span = gpu_decode(recs, w)
        assert st.tolist() == [0] * 8
        assert p.tolist() == [x for _, x, _ in JC.README] and v.tolist() == [x for _, _, x in JC.README]
        assert [recs[i][span[i, 0]:span[i, 0] + span[i, 1]] for i in range(8)] == [b"e%d" % (i + 1) for i in range(8)]


@pytest.mark.parametrize("col_width", [8, 4])
def test_cases_vs_oracle(col_width):
    assert_oracle([c for c, _ in JC.CASES] * 3, col_width)


def test_fuzz_vs_oracle():
    assert_oracle(JC.fuzz(11, 50000))


def test_depth_limit():
    st = gpu_decode([JC.deep(63), JC.deep(64), JC.deep(200)])[0]
    assert st.tolist() == [J.OK, J.DEPTH, J.DEPTH]


def test_hbm_path_long_records():
    # 256-record blocks whose span exceeds the 24 KiB LDS tile parse straight from HBM
    pad = [b" " * (i % 300) for i in range(3000)]
    recs = [b'{"name":"e%d",%s"price":%d,"volume":%d}' % (i, pad[i], i * 7 - 500, i) for i in range(3000)]
    recs[1000] = b'{"x":"' + b"y" * 100000 + b'","price":1,"volume":2}'  # one huge record
    assert_oracle(recs)


def test_empty_batch_and_empty_records():
    assert gpu_decode([])[0].tolist() == []
    assert_oracle([b""] * 300 + [b"{}"] + [b""] * 300)


class _Skewed:
    def __init__(self, buf, skew):
        self.ptr = buf.ptr + skew


def test_unaligned_spans():
    recs = JC.fuzz(3, 3000)
    for skew in (1, 3, 7, 13):
        off = np.zeros(len(recs) + 1, np.uint64)
        off[1:] = np.cumsum([len(r) for r in recs])
        off += 5  # the batch starts 5 bytes into the buffer, the buffer `skew` bytes into the allocation
        blob = np.frombuffer(b"#####" + b"".join(recs), np.uint8)
        d = N.DeviceBuffer(blob.nbytes + 64)
        host = np.zeros(blob.nbytes + 64, np.uint8)
        host[skew:skew + blob.nbytes] = blob
        d.upload(host)
        o = N.DeviceBuffer(off.nbytes)
        o.upload(off)
        b = N.StockJsonBatch(len(recs), blob.nbytes, _Skewed(d, skew), o)
        out = N.decode_stock_json(b).download()
        exp = json_cpu.oracle_arrays([J.deserialize(r) for r in recs])
        assert np.array_equal(out["status"], exp[0]) and np.array_equal(out["price"], exp[1])
        assert np.array_equal(out["volume"], exp[2]) and np.array_equal(out["name_span"], exp[3])


def test_synth_records_are_json_simple_serialization():
    price = np.array([100, 120, 120, 121, 120, 125, 120, 120, -7, 0], np.int32)
    vol = np.array([1010, 990, 1005, 999, 999, 750, 950, 700, 2147483647, -2147483648], np.int32)
    pb, vb = N.DeviceBuffer(price.nbytes), N.DeviceBuffer(vol.nbytes)
    pb.upload(price)
    vb.upload(vol)
    data, off = N.StockJsonBatch.synth(pb, vb, len(price)).download()
    recs = [data[int(off[i]):int(off[i + 1])] for i in range(len(price))]
    # what StockEventSerDe.serialize writes (json-simple's HashMap key order), byte for byte;
    # the README's console records (README.md:73-80) carry the same values in another order
    assert recs == [J.serialize("e%d" % (i + 1), int(price[i]), int(vol[i])) for i in range(len(price))]
    assert [J.deserialize(r)[:3] for r in recs[:8]] == [J.deserialize(r)[:3] for r, _, _ in JC.README]


def test_round_trip_at_bench_size():
    s = N.synth_stream("stock", 0xCE90003, 20000, 1000)  # ~2e7 events
    b = N.StockJsonBatch.synth(s.cols[0], s.cols[1], s.n_events)
    out = N.decode_stock_json(b, 4, name_spans=False)
    st = out.status.download(np.int32, s.n_events)
    assert int(np.count_nonzero(st)) == 0
    _, cols = s.download()
    assert np.array_equal(out.price.download(np.int32, s.n_events), cols[0])
    assert np.array_equal(out.volume.download(np.int32, s.n_events), cols[1])


def test_readme_json_to_matches():
    """README.md:64-96 end to end: the 8 JSON records -> GPU decode -> NFA -> the README's 4 matches."""
    recs = [r for r, _, _ in JC.README]
    dec = N.decode_stock_json(N.StockJsonBatch.from_records(recs), 4, name_spans=False)
    assert dec.status.download(np.int32, 8).tolist() == [0] * 8
    off = np.array([0, 8], np.uint64)
    ob = N.DeviceBuffer(off.nbytes)
    ob.upload(off)
    ir = W.stock_query("readme").to_ir()
    s = N.Session(N.Query(ir), device=0)
    s.push_device(N.DeviceStream(1, 8, ob, [dec.price, dec.volume]))
    m = s.matches(0)
    r = oracle.run(ir, off, [np.array([x for _, x, _ in JC.README], np.int32),
                             np.array([x for _, _, x in JC.README], np.int32)])
    assert m["n_matches"] == r["n_matches"] == 4
    assert np.array_equal(m["pair_seq"], r["pair_pos"]) and np.array_equal(m["pair_stage"], r["pair_stage"])
