"""An oracle-backed stand-in for a streaming libcep session - TEST INFRASTRUCTURE ONLY.

Lets the CPU tests drive `CEPProcessor`'s host logic (buffering, key ids, Sequence
reconstruction, forward order, error raising) without a GPU: every push re-runs the oracle
over each key's whole history (one reference NFA per key is deterministic) and returns the
matches whose completing record arrived in this push, with per-key sequence numbers, as the
streaming session does (include/cep.h cep_poll_matches / cep_key_errors).
"""
import numpy as np

import oracle
from kafkastreams_cep_amd import native as N


class OracleStreamSession:
    def __init__(self, ir: bytes):
        self.ir = ir
        self.stage_names = N.Query(ir).stage_names
        self.hist: dict[int, tuple[list, list]] = {}  # key -> (per-column lists, ts list)
        self.pushes = 0
        self._m = None
        self._err = None

    def push_arrival(self, keys, cols, n_keys, ts):
        self.pushes += 1
        keys = np.asarray(keys, np.int64)
        before = {}
        for i, k in enumerate(keys.tolist()):
            h = self.hist.setdefault(k, ([[] for _ in cols], []))
            before.setdefault(k, len(h[1]))
            for c, col in zip(h[0], cols):
                c.append(col[i])
            h[1].append(int(ts[i]))
        touched = sorted(before)
        lens = [len(self.hist[k][1]) for k in touched]
        off = np.zeros(len(touched) + 1, np.uint64)
        np.cumsum(lens, out=off[1:])
        ccols = [np.concatenate([np.asarray(self.hist[k][0][f], dtype=np.asarray(cols[f]).dtype)
                                 for k in touched]) for f in range(len(cols))]
        cts = np.concatenate([np.asarray(self.hist[k][1], np.int64) for k in touched])
        r = oracle.run(self.ir, off, ccols, cts)
        key, emit, poff, pseq, pst = [], [], [0], [], []
        for m in range(int(r["n_matches"])):
            j = int(r["key"][m])
            k = touched[j]
            e = int(r["emit_pos"][m]) - int(off[j])
            if e < before[k]:
                continue
            a, b = int(r["pair_off"][m]), int(r["pair_off"][m + 1])
            key.append(k)
            emit.append(e)
            pseq += [int(p) - int(off[j]) for p in r["pair_pos"][a:b]]
            pst += r["pair_stage"][a:b].tolist()
            poff.append(len(pseq))
        self._m = {"n_matches": len(key), "n_pairs": len(pseq), "key": np.asarray(key, np.uint32),
                   "emit_seq": np.asarray(emit, np.uint32), "pair_off": np.asarray(poff, np.uint64),
                   "pair_seq": np.asarray(pseq, np.uint32), "pair_stage": np.asarray(pst, np.uint16)}
        code = np.zeros(n_keys, np.int32)
        seq = np.zeros(n_keys, np.uint32)
        for j, k in enumerate(touched):
            if r["err_code"][j]:
                code[k] = r["err_code"][j]
                seq[k] = int(r["err_pos"][j]) - int(off[j])
        self._err = (code, seq)

    def snapshot(self) -> bytes:
        import pickle  # (this fake's own state)
        return pickle.dumps(self.hist)

    def restore(self, blob: bytes) -> None:
        import pickle
        self.hist = pickle.loads(blob)

    def matches(self, query=0):
        return self._m

    def key_errors(self, query=0, n_keys=None):
        return self._err

    def close(self):
        pass
