"""Underfilled launches (a rank's shard of the multi-GPU split): each world-`W` shard of the
cfg-3 stream timed with the keys spread over every wave slot ($CEP_SPREAD=1, the default) and
contiguous (CEP_SPREAD=0); the heaviest keys of the stream timed alone (the latency floor of
one key's chain of events).  One JSON line per measurement.
    python profiles/spread_probe.py [--world 8] [--steps 2]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cepamd  # noqa: E402,F401
from kafkastreams_cep_amd import native as N  # noqa: E402
from kafkastreams_cep_amd import shard as SH  # noqa: E402
from kafkastreams_cep_amd import workloads as W  # noqa: E402


def timed(s, st, steps):
    s.push_device(st)
    N.lib().cep_sync(s.h)
    t = []
    for _ in range(steps):
        t0 = time.perf_counter()
        s.push_device(st)
        N.lib().cep_sync(s.h)
        t.append(1e3 * (time.perf_counter() - t0))
    return min(t), s.stats(0)["main_ms"], s.digest(0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--heavy", default="694500,184250,969750,686750,798500")
    ap.add_argument("--ranks", default="")
    args = ap.parse_args()
    cfg = W.CONFIGS[3]
    stream = N.synth_stream("stock", cfg.seed, cfg.n_keys, cfg.mean_events)
    off = stream.key_off.download(np.uint64, stream.n_keys + 1)
    q = N.Query(W.stock_query("readme").to_ir())
    modes = os.environ.get("SPREAD_MODES", "0,1").split(",")
    sess = {}
    for sp in modes:  # (knobs are read when a session is made)
        os.environ["CEP_SPREAD"] = sp
        sess[sp] = N.Session(q)
    os.environ.pop("CEP_SPREAD", None)
    s = N.Session(q)
    ranks = [int(r) for r in args.ranks.split(",")] if args.ranks else range(args.world)
    for r in ranks:
        keys, loff = SH.shard_layout(off, args.world, r)
        sh, _ = N.shard_stream(stream, keys, loff)
        for sp in modes:
            wall, main_ms, dig = timed(sess[sp], sh, args.steps)
            print(json.dumps({"rank": r, "spread": sp, "keys": int(len(keys)), "wall_ms": wall, "main_ms": main_ms,
                              "digest": list(dig)}), flush=True)
        del sh
    for k in [int(x) for x in args.heavy.split(",") if x]:
        keys = np.array([k], np.int64)
        loff = np.array([0, int(off[k + 1] - off[k])], np.uint64)
        sh, _ = N.shard_stream(stream, keys, loff)
        wall, main_ms, dig = timed(s, sh, args.steps)
        print(json.dumps({"key": k, "alone": True, "events": int(loff[1]), "wall_ms": wall, "main_ms": main_ms,
                          "digest": list(dig)}), flush=True)
    wall, main_ms, dig = timed(s, stream, args.steps)
    print(json.dumps({"all_keys": stream.n_keys, "wall_ms": wall, "main_ms": main_ms, "digest": list(dig)}), flush=True)


if __name__ == "__main__":
    main()
