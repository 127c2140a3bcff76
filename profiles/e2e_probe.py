"""Per-push breakdown of bench.py's end-to-end figure (arrival-order cfg-3 batches): wall time
of cep_push_batch, of the layout query, the partition / matching kernel times and the batch
stats (re-runs, pools).
    python profiles/e2e_probe.py [--keys N] [--steps K]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cepamd  # noqa: E402,F401
from kafkastreams_cep_amd import native as N  # noqa: E402
from kafkastreams_cep_amd import workloads as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=4)
    args = ap.parse_args()
    cfg = W.CONFIGS[3]
    st = N.synth_arrival_stream("stock", cfg.seed, args.keys, 1000, 0)
    s = N.Session(N.Query(W.stock_query("readme").to_ir()))
    for i in range(args.steps):
        t0 = time.perf_counter()
        s.push_arrival_device(st)
        t1 = time.perf_counter()
        off, perm, ms = N.C.c_void_p(), N.C.c_void_p(), N.C.c_double()
        N._check(N.lib().cep_batch_layout(s.h, N.CEP_MEM_DEVICE, N.C.byref(off), N.C.byref(perm), N.C.byref(ms)))
        t2 = time.perf_counter()
        print(json.dumps({"push": i, "push_s": t1 - t0, "layout_s": t2 - t1, "partition_ms": ms.value,
                          "timing": s.timing(0), "stats": s.stats(0)}), flush=True)


if __name__ == "__main__":
    main()
