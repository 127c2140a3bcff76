"""The heaviest cfg-3 key (stream key 694500: 1021 events, ~3.4 live runs per event) alone, or a
world-8 shard, pushed `--steps` times: a small target for rocprofv3 PMC passes (instructions
and wave cycles of one lane's chain).
    python profiles/heavy_alone.py [--key 694500 | --shard 2] [--steps 3]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cepamd  # noqa: E402,F401
from kafkastreams_cep_amd import native as N  # noqa: E402
from kafkastreams_cep_amd import shard as SH  # noqa: E402
from kafkastreams_cep_amd import workloads as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--key", type=int, default=694500)
    ap.add_argument("--shard", type=int, default=-1)
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    cfg = W.CONFIGS[3]
    stream = N.synth_stream("stock", cfg.seed, cfg.n_keys, cfg.mean_events)
    off = stream.key_off.download(np.uint64, stream.n_keys + 1)
    if args.shard >= 0:
        keys, loff = SH.shard_layout(off, 8, args.shard)
    else:
        keys = np.array([args.key])
        loff = np.array([0, int(off[args.key + 1] - off[args.key])], np.uint64)
    sh, _ = N.shard_stream(stream, keys, loff)
    del stream
    s = N.Session(N.Query(W.stock_query("readme").to_ir()))
    for _ in range(args.steps):
        s.push_device(sh)
    N.lib().cep_sync(s.h)
    print(s.stats(0), s.digest(0), flush=True)


if __name__ == "__main__":
    main()
