"""Multi-rank path on the CPU: bench.py's key sharding of ONE global stream (Kafka's
DefaultPartitioner over the key ids, kafkastreams-cep_amd/shard.py: the real split function
the bench uses) and its gloo/RCCL reductions (all-gather of counts, wrapping checksum sum over
global key ids, min watermark), with the oracle standing in for the per-GPU matcher (no GPU
here; tests/test_gpu_parity.py checks the device gather against shard.gather_host).
The union of the shards must equal one rank running all keys."""
import os
import socket
import sys
import tempfile

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K, MEAN = 300, 300


def _global_stream():
    import cepamd  # noqa: F401
    from kafkastreams_cep_amd import workloads as W

    cfg = W.SynthConfig("t", "stock", K, MEAN, W.CONFIGS[3].seed)
    return W.generate(cfg)


def _digest(r, off, key_ids):
    """the oracle result's checksum with global key ids (bench.global_digest's definition)"""
    from kafkastreams_cep_amd import workloads as W

    k = r["key"].astype(np.int64)
    emit = r["emit_pos"].astype(np.uint64) - off[k]
    pk = np.repeat(k, np.diff(r["pair_off"].astype(np.int64)))
    pseq = r["pair_pos"].astype(np.uint64) - off[pk]
    return W.match_digest(key_ids[k], emit, r["pair_off"], pseq, r["pair_stage"])


def _shard_result(rank, world):
    import cepamd  # noqa: F401
    import oracle
    from kafkastreams_cep_amd import shard as SH
    from kafkastreams_cep_amd import workloads as W

    off, cols = _global_stream()
    keys, loff = SH.shard_layout(off, world, rank)
    lcols = SH.gather_host(off, cols, keys, loff)
    r = oracle.run(W.stock_query("readme").to_ir(), loff, lcols, threads=2)
    return int(loff[-1]), r["n_matches"], _digest(r, loff, keys.astype(np.int64)), keys


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import bench

    dist = bench.Dist(backend="gloo")
    n_ev, n_m, dig, keys = _shard_result(rank, world)
    per = dist.gather([n_ev, n_m, len(keys)])
    total = dist.sum_u64(dig)
    wm = dist.min_i64(1000 + rank)
    dist.barrier()
    if rank == 0:
        np.save(out, np.array([per[:, 0].sum(), per[:, 1].sum(), total >> 32, total & 0xFFFFFFFF, wm,
                               per[:, 2].sum()], np.int64))
    dist.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_kafka_partitioner_is_a_partition():
    sys.path[:0] = [ROOT]
    import cepamd  # noqa: F401
    from kafkastreams_cep_amd import shard as SH

    keys = np.arange(100_000, dtype=np.uint32)
    for n in (1, 2, 4, 8):
        p = SH.partition_of(keys, n)
        assert p.min() >= 0 and p.max() < n
        counts = np.bincount(p, minlength=n)
        assert counts.min() > 0.9 * len(keys) / n  # murmur2 spreads the keys evenly
    # Kafka's murmur2 restated a second way (scalar Java int arithmetic) for a few keys
    def murmur2_scalar(key):
        data = key.to_bytes(4, "big")
        m, h = 0x5BD1E995, (0x9747B28C ^ 4) & 0xFFFFFFFF
        k = data[0] | data[1] << 8 | data[2] << 16 | data[3] << 24
        k = (k * m) & 0xFFFFFFFF
        k ^= k >> 24
        k = (k * m) & 0xFFFFFFFF
        h = (h * m) & 0xFFFFFFFF
        h ^= k
        h ^= h >> 13
        h = (h * m) & 0xFFFFFFFF
        h ^= h >> 15
        return h
    for key in (0, 1, 2, 255, 256, 65535, 123456789, 2**31 - 1, 2**32 - 1):
        assert int(SH.murmur2_int_keys([key])[0]) == murmur2_scalar(key)


def _murmur2_bytes(data: bytes) -> int:
    """Kafka's Utils.murmur2 over any byte array (clients/.../common/utils/Utils.java), as a
    signed Java int: 4-byte little-endian blocks, then the 1-3 tail bytes, then the final mix."""
    m = 0x5BD1E995
    h = (0x9747B28C ^ len(data)) & 0xFFFFFFFF
    for i in range(len(data) // 4):
        k = data[4 * i] | data[4 * i + 1] << 8 | data[4 * i + 2] << 16 | data[4 * i + 3] << 24
        k = (k * m) & 0xFFFFFFFF
        k ^= k >> 24
        k = (k * m) & 0xFFFFFFFF
        h = ((h * m) & 0xFFFFFFFF) ^ k
    rem, b = len(data) % 4, len(data) & ~3
    if rem == 3:
        h ^= data[b + 2] << 16
    if rem >= 2:
        h ^= data[b + 1] << 8
    if rem >= 1:
        h = ((h ^ data[b]) * m) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * m) & 0xFFFFFFFF
    h ^= h >> 15
    return h - (1 << 32) if h >= 1 << 31 else h


def test_murmur2_pinned_by_kafka_vectors():
    """(murmur2 was parity unpinned) The partitioner's hash against the test
    vectors Kafka publishes for Utils.murmur2 (kafka-clients UtilsTest.testMurmur2; Kafka is a
    dependency of the reference, not part of /root/reference): the general byte-array form
    reproduces all six, and the partitioner's 4-byte key path (shard.murmur2_int_keys, the
    big-endian serialization of each u32 key id) equals it on every key of a sample."""
    sys.path[:0] = [ROOT]
    import cepamd  # noqa: F401
    from kafkastreams_cep_amd import shard as SH

    kafka = {b"21": -973932308, b"foobar": -790332482, b"a-little-bit-long-string": -985981536,
             b"a-little-bit-longer-string": -1486304829,
             b"lkjh234lh9fiuh90y23oiuhsafujhadof229phr9h19h89h8": -58897971, b"abc": 479470107}
    for data, want in kafka.items():
        assert _murmur2_bytes(data) == want, data
    keys = np.concatenate([np.arange(5000, dtype=np.uint32),
                           np.random.default_rng(5).integers(0, 2**32, 5000, dtype=np.uint64).astype(np.uint32)])
    got = SH.murmur2_int_keys(keys).astype(np.int64)
    want = np.array([_murmur2_bytes(int(k).to_bytes(4, "big")) & 0xFFFFFFFF for k in keys], np.int64)
    np.testing.assert_array_equal(got, want)


def test_two_rank_sharding_matches_single_rank():
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.npy")
        mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
        got = np.load(out)
    import cepamd  # noqa: F401
    import oracle
    from kafkastreams_cep_amd import workloads as W

    shards = [_shard_result(r, 2) for r in range(2)]
    off, cols = _global_stream()
    whole = oracle.run(W.stock_query("readme").to_ir(), off, cols, threads=2)
    whole_digest = _digest(whole, off, np.arange(K, dtype=np.int64))
    # every key in exactly one shard, every event in its key's shard
    assert sorted(np.concatenate([s[3] for s in shards]).tolist()) == list(range(K))
    assert got[5] == K and got[0] == sum(s[0] for s in shards) == int(off[-1])
    # the union of the shards' matches is the single rank's: counts and global-key checksum
    assert got[1] == sum(s[1] for s in shards) == whole["n_matches"] > 0
    assert (int(got[2]) << 32 | int(got[3])) == sum(s[2] for s in shards) % (1 << 64) == whole_digest
    assert got[4] == 1000
    n0 = int(np.isin(whole["key"], shards[0][3]).sum())
    assert (n0, whole["n_matches"] - n0) == (shards[0][1], shards[1][1])
