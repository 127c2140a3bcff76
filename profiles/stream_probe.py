"""Where a streaming session's time goes (bench.py streaming figure: the cfg-3 stream as 10
consecutive batches per key).  Prints per batch: wall time of the push, the matching kernel,
the whole kernel sequence; then the same slices pushed to a per-batch session (every key from
the initial state each batch: not the stream's semantics, a timing reference for the per-batch
machinery - narrow build, deferred walks, slot-ordered run queues).
    python profiles/stream_probe.py [--slices 10] [--keys 1000000]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from kafkastreams_cep_amd import native as N  # noqa: E402
from kafkastreams_cep_amd import workloads as W  # noqa: E402


def run(s, parts, label):
    rows = []
    for p in parts:
        t0 = time.perf_counter()
        s.push_device(p)
        N.lib().cep_sync(s.h)
        st = s.stats(0)
        rows.append({"wall_ms": 1e3 * (time.perf_counter() - t0), "main_ms": st["main_ms"], "kernel_ms": st["kernel_ms"],
                     "retried": st["retried_jobs"]})
    tot = {k: sum(r[k] for r in rows) for k in ("wall_ms", "main_ms", "kernel_ms")}
    print(json.dumps({"label": label, "total": tot, "batches": rows}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slices", type=int, default=10)
    ap.add_argument("--keys", type=int, default=1_000_000)
    args = ap.parse_args()
    cfg = W.CONFIGS[3]
    stream = N.synth_stream("stock", cfg.seed, args.keys, cfg.mean_events)
    parts = bench.slice_stream(stream, args.slices)
    q = N.Query(W.stock_query("readme").to_ir())
    s = N.Session(q, streaming=True)
    for it in range(2):
        s.reset()
        run(s, parts, f"streaming pass {it}")
    s.close()
    s = N.Session(q)
    for it in range(2):
        run(s, parts, f"per-batch sessions pass {it}")


if __name__ == "__main__":
    main()
