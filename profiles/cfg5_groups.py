"""Config 5 (64 stock-query variants, one session) on the cfg-3 stream in HBM: the kernel
group (one launch, lanes = (query, key)) against one launch per query.  Prints per mode the
step time, the group's kernel ms, matches, pairs, key errors and re-run jobs.
    python profiles/cfg5_groups.py [--keys N] [--modes group,separate]
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
from kafkastreams_cep_amd import workloads as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=100_000)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--modes", default="group,separate")
    args = ap.parse_args()
    cfg = W.CONFIGS[3]
    stream = N.synth_stream("stock", cfg.seed, args.keys, cfg.mean_events)
    qs = [N.Query(p.to_ir()) for p in W.multi_queries(64)]
    for mode in args.modes.split(","):
        s = N.Session(qs, groups=(mode == "group"))
        s.push_device(stream)  # warm-up: pools sized from this batch's use
        t = []
        for _ in range(args.steps):
            t0 = time.perf_counter()
            s.push_device(stream)
            t.append(time.perf_counter() - t0)
        kms = [s.timing(i)[0] for i in range(len(qs))]
        n_m = n_p = errs = 0
        for i in range(len(qs)):
            m = N.Matches()
            N._check(N.lib().cep_poll_matches(s.h, i, N.CEP_MEM_DEVICE, N.C.byref(m)))
            n_m += m.n_matches
            n_p += m.n_pairs
            errs += int(np.count_nonzero(s.key_errors(i)[0]))
        res = {"mode": mode, "keys": args.keys, "events": stream.n_events, "step_s": min(t),
               "kernel_ms": kms[0] if mode == "group" else sum(kms), "launches": s.timing(0)[2],
               "matches": n_m, "pairs": n_p, "key_errors": errs, "stats0": s.stats(0), "stats63": s.stats(63)}
        print(json.dumps(res), flush=True)
        s.close()


if __name__ == "__main__":
    main()
