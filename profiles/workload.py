"""One bench workload on its own, for rocprofv3 kernel traces / PMC passes and timing probes
(run on the GPU box from the repo root).  Each mode pushes its batches `--steps` times after
one warmup push and prints one JSON line per mode on stdout.

    python profiles/workload.py cfg3 [--keys N]        README stock query (bench headline)
    python profiles/workload.py cfg4s                   config 4 stress (carry_volume variant)
    python profiles/workload.py cfg4                    config 4 as written (the parity case)
    python profiles/workload.py cfg4sem                 config 4, semantic WITHIN
    python profiles/workload.py cfg5 [--keys 125000]    64 stock-query variants, one batch
    python profiles/workload.py stream [--slices 10]    cfg 3 as consecutive streaming batches
    python profiles/workload.py shards [--world 8]      each rank's shard of cfg 3 alone
    python profiles/workload.py arrival                 cfg 3 in arrival order (partition + NFA)

$CEP_PROF=1 (set before the query is compiled) makes libcep print the kernel's time split
(nfa_lane.h CEP_PROF) on stderr per launch.
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
from kafkastreams_cep_amd import shard as SH  # noqa: E402
from kafkastreams_cep_amd import workloads as W  # noqa: E402


def timed(sess, stream, steps, ts=None):
    sess.push_device(stream, ts.ptr if ts is not None else None)
    out = []
    for _ in range(steps):
        t0 = time.perf_counter()
        sess.push_device(stream, ts.ptr if ts is not None else None)
        N.lib().cep_sync(sess.h)
        st = sess.stats(0)
        out.append({"wall_ms": 1e3 * (time.perf_counter() - t0), "main_ms": st["main_ms"],
                    "kernel_ms": st["kernel_ms"], "retried": st["retried_jobs"]})
    return out


def figures(sess, n_keys):
    n_m, n_p, n_e = bench.match_figures(sess, 0, n_keys)
    st = sess.stats(0)
    return {"matches": n_m, "pairs": n_p, "key_errors": n_e, "nodes": st["nodes_used"], "preds": st["preds_used"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode")
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--slices", type=int, default=10)
    ap.add_argument("--world", type=int, default=8)
    args = ap.parse_args()
    cfg = W.CONFIGS[3]
    m = args.mode
    res = {"mode": m, "keys": args.keys}
    if m == "cfg5":
        stream = N.synth_stream("stock", cfg.seed, args.keys, cfg.mean_events)
        s = N.Session([N.Query(p.to_ir()) for p in W.multi_queries(64)])
        res["runs"] = timed(s, stream, args.steps)
        tot = [bench.match_figures(s, i, stream.n_keys) for i in range(64)]
        res.update(matches=sum(t[0] for t in tot), pairs=sum(t[1] for t in tot), key_errors=sum(t[2] for t in tot))
        print(json.dumps(res), flush=True)
        return
    if m == "arrival":  # the end-to-end figure's push: partition on the GPU, then the NFA
        st = N.synth_arrival_stream("stock", cfg.seed, args.keys, cfg.mean_events, 0, 0)
        s = N.Session(N.Query(W.stock_query("readme").to_ir()))
        s.push_arrival_device(st)
        runs = []
        for _ in range(args.steps):
            t0 = time.perf_counter()
            s.push_arrival_device(st)
            N.lib().cep_sync(s.h)
            runs.append({"wall_ms": 1e3 * (time.perf_counter() - t0), "partition_ms": bench._partition_ms(s),
                         "kernel_ms": s.stats(0)["kernel_ms"]})
        res.update(events=st.n_events, runs=runs, checksum=f"{s.digest(0)[1]:016x}")
        print(json.dumps(res), flush=True)
        return
    stream = N.synth_stream("stock", cfg.seed, args.keys, cfg.mean_events)
    res["events"] = stream.n_events
    if m in ("cfg3", "cfg4", "cfg4s", "cfg4sem"):
        p = {"cfg3": W.stock_query("readme"), "cfg4": W.any_kleene_query(),
             "cfg4s": W.any_kleene_query(carry_volume=True), "cfg4sem": W.any_kleene_query()}[m]
        ts = N.synth_ts(stream.n_events, bench.TS_BASE) if m in ("cfg3", "cfg4sem") else None
        s = N.Session(N.Query(p.to_ir(semantic_within=(m == "cfg4sem"))))
        res["runs"] = timed(s, stream, args.steps, ts)
        res.update(figures(s, stream.n_keys))
        res["checksum"] = f"{s.digest(0)[1]:016x}"
    elif m == "stream":
        res.update(bench.streaming_cfg3(0, stream, args.slices, args.steps, bench.Dist()))
    elif m == "shards":
        res.update(bench.projected_scaling(0, cfg, stream, args.world, args.steps, bench.Dist()))
    else:
        raise SystemExit(f"unknown mode {m}")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
