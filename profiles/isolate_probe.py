"""Underfilled launches with the heaviest ranks alone in their waves ($CEP_ISOLATE=K: waves
0..K-1 each run one of the K heaviest keys of the launch, the other keys spread over the
remaining waves).  Each world-`W` shard of the cfg-3 stream timed per K; the digests must not
change with K.  One JSON line per measurement.
    python profiles/isolate_probe.py [--world 8] [--iso 0,256,512,1024] [--steps 2]
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
    ap.add_argument("--iso", default="0,256,512,1024,2048")
    ap.add_argument("--ranks", default="")
    args = ap.parse_args()
    cfg = W.CONFIGS[3]
    stream = N.synth_stream("stock", cfg.seed, cfg.n_keys, cfg.mean_events)
    off = stream.key_off.download(np.uint64, stream.n_keys + 1)
    q = N.Query(W.stock_query("readme").to_ir())
    isos = [int(x) for x in args.iso.split(",")]
    sess = {}
    for k in isos:  # knobs are read when a session is made
        os.environ["CEP_ISOLATE"] = str(k)
        sess[k] = N.Session(q)
    os.environ.pop("CEP_ISOLATE", None)
    ranks = [int(r) for r in args.ranks.split(",")] if args.ranks else range(args.world)
    worst = {k: 0.0 for k in isos}
    for r in ranks:
        keys, loff = SH.shard_layout(off, args.world, r)
        sh, _ = N.shard_stream(stream, keys, loff)
        dig0 = None
        for k in isos:
            wall, main_ms, dig = timed(sess[k], sh, args.steps)
            dig0 = dig0 or list(dig)
            worst[k] = max(worst[k], main_ms)
            print(json.dumps({"rank": r, "isolate": k, "keys": int(len(keys)), "wall_ms": wall, "main_ms": main_ms,
                              "same_digest": list(dig) == dig0}), flush=True)
        del sh
    print(json.dumps({"slowest_shard_main_ms": worst}), flush=True)


if __name__ == "__main__":
    main()
