"""JIT-knob ablations of cep_nfa_jit on the README stock query (cfg 3): each variant's kernel
is compiled on the box (its knobs are part of the generated source) and timed on the heaviest
key alone (one lane: the latency floor of a key's chain), on a world-8 shard (underfilled
launch) and on the whole 1M-key stream.  One JSON line per (variant, workload).
    python profiles/knob_probe.py 'CEP_CHAIN_CACHE=3' 'CEP_RING_LDS_SLOTS=6,CEP_RESIDENT_WAVES=4' ...
(an empty argument = the default build)
"""
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

KNOBS = ("CEP_CHAIN_CACHE", "CEP_RING_LDS_SLOTS", "CEP_RESIDENT_WAVES", "CEP_WALK_FLUSH", "CEP_JIT_WAVES",
         "CEP_SPREAD", "CEP_QUIET_CHUNK")


def timed(s, st, steps=2):
    s.push_device(st)
    N.lib().cep_sync(s.h)
    t = []
    for _ in range(steps):
        t0 = time.perf_counter()
        s.push_device(st)
        N.lib().cep_sync(s.h)
        t.append(1e3 * (time.perf_counter() - t0))
    return {"wall_ms": min(t), "main_ms": s.stats(0)["main_ms"], "digest": list(s.digest(0)),
            "retried": s.stats(0)["retried_jobs"]}


def main():
    variants = sys.argv[1:] or [""]
    cfg = W.CONFIGS[3]
    stream = N.synth_stream("stock", cfg.seed, cfg.n_keys, cfg.mean_events)
    off = stream.key_off.download(np.uint64, stream.n_keys + 1)
    heavy = 694500
    hs, _ = N.shard_stream(stream, np.array([heavy]), np.array([0, int(off[heavy + 1] - off[heavy])], np.uint64))
    keys, loff = SH.shard_layout(off, 8, 2)
    sh, _ = N.shard_stream(stream, keys, loff)
    for v in variants:
        for k in KNOBS:
            os.environ.pop(k, None)
        kv = dict(x.split("=") for x in v.split(",") if x)
        os.environ.update(kv)
        t0 = time.perf_counter()
        q = N.Query(W.stock_query("readme").to_ir())
        s = N.Session(q)
        res = {"variant": kv, "compile_s": None}
        res["heavy_key"] = timed(s, hs)
        res["compile_s"] = time.perf_counter() - t0 - res["heavy_key"]["wall_ms"] * 3e-3
        res["shard_w8_r2"] = timed(s, sh)
        res["all_1m"] = timed(s, stream)
        s.close()
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
