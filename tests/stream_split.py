"""Streaming sessions (cep_opts.streaming): cut one CSR stream into consecutive batches per
key, and compare the concatenated per-key output of the batches with a single-pass result."""
import numpy as np


def split(key_off, cols, n_batches, seed):
    """Cuts every key's events at random points into n_batches consecutive segments; returns
    [(key_off_b, cols_b)] (each batch a CSR over all keys, empty segments allowed)."""
    rng = np.random.default_rng(seed)
    off = np.asarray(key_off, np.int64)
    cnt = np.diff(off)
    cuts = np.sort(rng.integers(0, cnt[:, None] + 1, size=(len(cnt), n_batches - 1)), axis=1)
    bounds = np.concatenate([np.zeros((len(cnt), 1), np.int64), cuts, cnt[:, None]], axis=1)
    out = []
    for b in range(n_batches):
        lo, hi = off[:-1] + bounds[:, b], off[:-1] + bounds[:, b + 1]
        ko = np.zeros(len(cnt) + 1, np.uint64)
        np.cumsum(hi - lo, out=ko[1:])
        idx = np.concatenate([np.arange(a, z) for a, z in zip(lo, hi)]) if len(cnt) else np.zeros(0, np.int64)
        out.append((ko, [c[idx.astype(np.int64)] for c in cols]))
    return out


def per_key(key, emit_seq, pair_off, pair_seq, pair_stage):
    """{key: [(emit_seq, ((stage, seq), ...)), ...]} in output order"""
    res = {}
    for i, k in enumerate(np.asarray(key).tolist()):
        a, z = int(pair_off[i]), int(pair_off[i + 1])
        pairs = tuple(zip(np.asarray(pair_stage[a:z]).tolist(), np.asarray(pair_seq[a:z]).tolist()))
        res.setdefault(k, []).append((int(emit_seq[i]), pairs))
    return res


def oracle_per_key(r, key_off):
    off = np.asarray(key_off, np.uint64)
    key = r["key"].astype(np.int64)
    emit = r["emit_pos"].astype(np.uint64) - off[key]
    pk = np.repeat(key, np.diff(r["pair_off"].astype(np.int64)))
    pseq = r["pair_pos"].astype(np.uint64) - off[pk]
    return per_key(key, emit, r["pair_off"], pseq, r["pair_stage"])


def merge(batch_results):
    """concatenates per-key outputs of consecutive batches (results carry global sequence numbers)"""
    res = {}
    for m in batch_results:
        for k, v in per_key(m["key"], m["emit_seq"], m["pair_off"], m["pair_seq"], m["pair_stage"]).items():
            res.setdefault(k, []).extend(v)
    return res
