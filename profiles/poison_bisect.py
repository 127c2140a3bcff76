"""Which device buffer a first push reads before any kernel wrote it: one session per
allocation ordinal k with only that allocation poisoned ($CEP_POISON=1<<k, measurement build),
one push; compare the digest with the unpoisoned run (--bit -2).  (CEP_MEASURE=1.)
    python profiles/poison_bisect.py [--arrival] [--bit K]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cepamd  # noqa: E402,F401
from kafkastreams_cep_amd import native as N  # noqa: E402
from kafkastreams_cep_amd import workloads as W  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--arrival", action="store_true")
ap.add_argument("--bit", type=int, default=-2, help="only this ordinal (one process per bit); -1: all")
args = ap.parse_args()
cfg = W.SynthConfig("t", "stock", 3000, 400, 0xCE90000 + 3)
off, cols = W.generate(cfg)
keys, acols = W.generate_arrival(cfg)


def one(mask):
    os.environ["CEP_POISON"] = str(mask)
    s = N.Session(N.Query(W.stock_query("readme").to_ir()))
    if args.arrival:
        s.push_arrival(keys, acols, cfg.n_keys)
    else:
        s.push(off, cols)
    r = (s.digest(0), s.stats(0))
    s.close()
    return r


if args.bit == -2:
    print("ref", one(0), flush=True)
else:
    d, st = one(-1 if args.bit < 0 else 1 << args.bit)
    print("bit", args.bit, d, st, flush=True)
