"""Key sharding across GPUs: one global key-partitioned stream, each rank owns
the keys whose partition is its rank, with no state shared between ranks.

The partition function is Kafka's DefaultPartitioner for a keyed record, which decides the
Kafka partition - hence the stream task and the reference's CEPProcessor/NFA instance
(CEPProcessor.java:117-134) - a key belongs to:

    partition(key) = toPositive(murmur2(serialize(key))) % n_partitions

with the key id serialized as kafka-clients' IntegerSerializer does (4 bytes, big-endian).
murmur2 and toPositive are kafka-clients' org.apache.kafka.common.utils.Utils (0.10.0.0-cp1,
the version /pom.xml:55-65 pins; not vendored in /root/reference, restated here from its
published algorithm).  Parity of this function with Kafka itself is unpinned (no Kafka jar
here); what the tests pin is that the shards partition the keys and their union of matches
equals one rank running every key.

`shard_layout` computes a rank's key list and local CSR offsets on the host; the events are
then gathered on the device (cep_gather_keys, native.gather_keys) or, in CPU tests, by
`gather_host`.
"""
from __future__ import annotations

import numpy as np

_M = np.uint32(0x5BD1E995)
_SEED = np.uint32(0x9747B28C)


def murmur2_int_keys(keys) -> np.ndarray:
    """Kafka Utils.murmur2 over the 4-byte big-endian serialization of each u32 key (array)."""
    k = np.asarray(keys, np.uint32)
    with np.errstate(over="ignore"):
        # the 4 bytes b0..b3 (big-endian) read little-endian = the byte-swapped key
        k = ((k & 0xFF) << 24) | ((k & 0xFF00) << 8) | ((k >> 8) & 0xFF00) | (k >> 24)
        k = k.astype(np.uint32)
        h = np.full(k.shape, _SEED ^ np.uint32(4), np.uint32)  # seed ^ length
        k = k * _M
        k ^= k >> np.uint32(24)
        k = k * _M
        h = h * _M
        h ^= k
        h ^= h >> np.uint32(13)
        h = h * _M
        h ^= h >> np.uint32(15)
    return h.astype(np.uint32)


def partition_of(keys, n_parts: int) -> np.ndarray:
    """toPositive(murmur2(key)) % n_parts (Kafka DefaultPartitioner for a keyed record)."""
    return ((murmur2_int_keys(keys) & np.uint32(0x7FFFFFFF)) % np.uint32(n_parts)).astype(np.int64)


def shard_layout(key_off, n_parts: int, part: int, key_ids=None):
    """Rank `part`'s shard of a CSR stream: (keys: global key indices it owns, ascending,
    local_off: u64 CSR offsets of those keys' events in the shard)."""
    key_off = np.asarray(key_off, np.uint64)
    nk = len(key_off) - 1
    ids = np.arange(nk, dtype=np.uint32) if key_ids is None else np.asarray(key_ids, np.uint32)
    keys = np.nonzero(partition_of(ids, n_parts) == part)[0].astype(np.uint32)
    counts = (key_off[1:] - key_off[:-1])[keys]
    local_off = np.zeros(len(keys) + 1, np.uint64)
    np.cumsum(counts, out=local_off[1:])
    return keys, local_off


def gather_host(key_off, cols, keys, local_off):
    """The shard's columns (host numpy; the device does this with cep_gather_keys)."""
    key_off = np.asarray(key_off, np.uint64)
    if len(keys) == 0:
        return [c[:0] for c in cols]
    idx = np.concatenate([np.arange(int(key_off[k]), int(key_off[k + 1])) for k in keys])
    return [np.asarray(c)[idx] for c in cols]
