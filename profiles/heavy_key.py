"""The heaviest (query, key) job of config 5 alone: cfg-3 stream key 39664 under variant q63
(615k emitted event ids in the reference, 400x the mean key).  A batch of that one key (or
`--copies` lanes of it) prices the per-lane sequential path - events, branch walks, match walks
- that bounds config 5's step.  Also times the oracle on the same key (one thread).
    python profiles/heavy_key.py [--key K] [--query Q] [--copies C]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import cepamd  # noqa: E402,F401
from kafkastreams_cep_amd import native as N  # noqa: E402
from kafkastreams_cep_amd import workloads as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--key", type=int, default=39664)
    ap.add_argument("--query", type=int, default=63)
    ap.add_argument("--copies", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--oracle", action="store_true")
    ap.add_argument("--streaming", action="store_true", help="streaming session: walks in place, a lane per key")
    args = ap.parse_args()
    cfg = W.SynthConfig("t", "stock", 1_000_000, 1000, W.CONFIGS[3].seed)
    off, cols = W.generate(cfg, np.full(args.copies, args.key))
    ir = W.multi_queries(64)[args.query].to_ir()
    ks = []
    s = None
    for _ in range(args.steps + 1):
        # a streaming session continues its keys: a fresh one per step; a per-batch session is
        # reused (its pools sized from the warm-up batch, as in a steady stream of batches)
        if s is None or args.streaming:
            s = N.Session(N.Query(ir), streaming=args.streaming, max_runs=64 if args.streaming else 0)
        s.push(off, cols)
        ks.append(s.timing(0)[0])
    ks = ks[1:]
    m = s.matches(0)
    res = {"key": args.key, "query": args.query, "copies": args.copies, "events_per_key": int(off[1]),
           "kernel_ms": min(ks), "matches": m["n_matches"], "pairs": m["n_pairs"], "stats": s.stats(0)}
    if args.oracle:
        import oracle
        o1, c1 = W.generate(cfg, np.array([args.key]))
        t = time.perf_counter()
        r = oracle.run(ir, o1, c1, threads=1)
        res["oracle_s"] = time.perf_counter() - t
        res["oracle_pairs"] = r["n_pairs"]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
