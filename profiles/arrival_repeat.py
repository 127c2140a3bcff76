"""Repeated arrival-order pushes on one session (the VERDICT r4 e2e outlier): per push the
batch stats, whether the partition's key offsets equal the CSR ones, and the match digest.
    python profiles/arrival_repeat.py [--pushes 30] [--keys 3000] [--mean 400]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import cepamd  # noqa: E402,F401
from kafkastreams_cep_amd import native as N  # noqa: E402
from kafkastreams_cep_amd import workloads as W  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pushes", type=int, default=30)
ap.add_argument("--keys", type=int, default=3000)
ap.add_argument("--mean", type=int, default=400)
ap.add_argument("--csr-first", type=int, default=4)
args = ap.parse_args()
cfg = W.SynthConfig("t", "stock", args.keys, args.mean, 0xCE90000 + 3)
off, cols = W.generate(cfg)
keys, acols = W.generate_arrival(cfg)
s = N.Session(N.Query(W.stock_query("readme").to_ir()))
for i in range(args.csr_first):
    s.push(off, cols)
    print(json.dumps({"push": "csr", "i": i, "stats": s.stats(0), "digest": list(s.digest(0))}), flush=True)
for i in range(args.pushes):
    s.push_arrival(keys, acols, cfg.n_keys)
    st = s.stats(0)
    ko, _, pms = s.layout()
    print(json.dumps({"push": "arrival", "i": i, "stats": st, "layout_ok": bool(np.array_equal(ko, off)),
                      "partition_ms": pms, "digest": list(s.digest(0))}), flush=True)
