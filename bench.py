#!/usr/bin/env python3
"""bench.py — events/sec of the README stock Kleene+ query on 1/2/4/8 MI355X.

BASELINE.json metric: "events/sec (whole node) + matches/sec, stock Kleene+ query, 1M keys,
1/2/4/8 GPU".  One step = one pass of the matcher (libcep.so: cep_nfa_jit + compaction) over
one batch of 1M keys x ~1000 events per GPU (config 3's shape), inputs already
resident in HBM, every key starting from the NFA's initial state.  Keys are sharded across
ranks with no data-path collective (weak scaling: each rank owns its own 1M keys); RCCL only
all-gathers counts/checksums and reduces the watermark.

    python bench.py                      # N=1, defaults finish in a few minutes
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N

Prints ONE JSON line on rank 0 (contract in the task statement; fields documented in
DESIGN.md §7).  `roofline` prices cep_nfa_jit at SURVEY §8(d)'s algorithmic bytes (columns read
once + 4 B per emitted event id + 4 B per match) against 8 TB/s; `cpu_baseline` times the
oracle (oracle/cep_oracle.cpp, the literal restatement of the reference NFA) on a 1/8 key
sample on this host's cores.  `ingest` is the JSON decoder (csrc/ingest.hip) on the cfg-3
stream serialized as StockEvent records, with its own roofline and CPU baseline.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import cepamd  # noqa: E402,F401
from kafkastreams_cep_amd import native as N  # noqa: E402
from kafkastreams_cep_amd import workloads as W  # noqa: E402

METRIC = "events/sec (whole node) + matches/sec, stock Kleene+ query, 1M keys, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


class Dist:
    """torch.distributed when launched with WORLD_SIZE > 1: "nccl" (= RCCL over xGMI) on the
    GPUs, "gloo" on the CPU (tests/test_distributed.py)."""

    def __init__(self, backend=None):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.torch = None
        if self.world > 1:
            import torch
            import torch.distributed as dist

            self.backend = backend or "nccl"
            self.device = "cuda" if self.backend == "nccl" else "cpu"
            if self.device == "cuda":
                torch.cuda.set_device(self.local)
            dist.init_process_group(self.backend)
            self.torch, self.dist = torch, dist

    def barrier(self):
        if self.torch:
            self.dist.barrier()
            if self.device == "cuda":
                self.torch.cuda.synchronize()

    def gather(self, vals):
        """all-gather a small float64 vector from every rank -> [world, len]"""
        if not self.torch:
            return np.asarray([vals], dtype=np.float64)
        t = self.torch.tensor(vals, dtype=self.torch.float64, device=self.device)
        out = [self.torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return np.stack([o.cpu().numpy() for o in out])

    def sum_u64(self, v):
        """wrapping 64-bit sum over ranks (checksums), via an all-gather of two 32-bit halves"""
        if not self.torch:
            return v % (1 << 64)
        t = self.torch.tensor([v & 0xFFFFFFFF, v >> 32], dtype=self.torch.int64, device=self.device)
        out = [self.torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return sum(int(o[0]) + (int(o[1]) << 32) for o in out) % (1 << 64)

    def min_i64(self, v):
        if not self.torch:
            return v
        t = self.torch.tensor([v], dtype=self.torch.int64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
        return int(t.item())

    def close(self):
        if self.torch:
            self.dist.destroy_process_group()


def run_steps(sess, stream, steps, warmup, dist):
    for _ in range(warmup):
        sess.push_device(stream)
    kern, aux = [], []
    dist.barrier()
    N.lib().cep_sync(sess.h)
    t0 = time.perf_counter()
    for _ in range(steps):
        sess.push_device(stream)  # returns after the batch's kernels complete
        k, a, _ = sess.timing(0)
        kern.append(k)
        aux.append(a)
    N.lib().cep_sync(sess.h)
    dist.barrier()
    return time.perf_counter() - t0, float(np.mean(kern)), float(np.mean(aux))


def load_traffic(name):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            return json.load(f).get(name)
    except (OSError, ValueError):
        return None


def cpu_baseline(cfg, variant, threads, every):
    """Oracle on keys 0, every, 2*every, ... of the same stream (numpy generator = GPU
    generator bit for bit).  Also checks GPU == oracle on that sample (checksum)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the checker / CPU baseline only

    keys = np.arange(0, cfg.n_keys, every)
    off, cols = W.generate(cfg, keys)
    ir = W.stock_query(variant).to_ir()
    r = oracle.run(ir, off, cols, threads=threads)
    n_ev = int(off[-1])
    # parity spot check on the sample: device checksum vs host checksum of the oracle output
    emit = r["emit_pos"].astype(np.uint64) - off[r["key"].astype(np.int64)]
    pk = np.repeat(r["key"].astype(np.int64), np.diff(r["pair_off"].astype(np.int64)))
    pseq = r["pair_pos"].astype(np.uint64) - off[pk]
    want = (r["n_matches"], W.match_digest(r["key"], emit, r["pair_off"], pseq, r["pair_stage"]))
    s = N.Session(N.Query(ir), device=0)
    s.push(off, cols)
    got = s.digest(0)
    s.close()
    return {"value": n_ev / r["elapsed_s"], "unit": "events/s", "cores": r["threads"], "kind": "port",
            "sample": f"{len(keys)} of {cfg.n_keys} keys (every {every}th), {n_ev} events, "
                      f"{r['n_matches']} matches, {r['elapsed_s']:.2f} s on {r['threads']} threads",
            "matches_per_s": r["n_matches"] / r["elapsed_s"],
            "parity_on_sample": bool(got == want)}


def secondary_strict(device, steps, warmup, dist):
    """Config 2: strict SEQ(A,B,C), 1e8 events over 1e4 keys, the three stencil passes."""
    cfg = W.CONFIGS[2]
    stream = N.synth_stream("abc", cfg.seed, cfg.n_keys, cfg.mean_events, 0, device)
    q = N.Query(W.strict_abc_query().to_ir())
    s = N.Session(q, device=device)
    el, kms, _ = run_steps(s, stream, steps, warmup, dist)
    n_m, _ = s.digest(0)
    n_ev = stream.n_events
    alg = 4.0 * n_ev + 16.0 * n_m  # one int column + (key + 3 event ids) per match
    res = {"workload": "cfg2: strict SEQ(A,B,C) v<4 | 4<=v<8 | v>=8, 1e4 keys x 1e4 events",
           "value": n_ev * steps / el, "unit": "events/s", "matches_per_step": n_m,
           "ms_per_step": 1e3 * el / steps,
           "roofline": {"bound": "hbm", "achieved": alg / (kms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": alg / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                        "traffic": load_traffic("stencil"), "kernel": "stencil_mask+stencil_emit",
                        "kernel_ms": kms, "algorithmic_bytes": alg}}
    s.close()
    return res


def other_configs(device, steps, warmup, dist, keys):
    """BASELINE configs 4 and 5 on the cfg-3 stream at `keys` keys x ~1000 events on one GPU
    (parity-tested at reduced size in tests/test_gpu_parity.py): cfg 4 = skip_till_any Kleene+
    with folds and a 10 ms window, cfg 5 = 64 stock-query variants in one session, which
    reads the stream once per query launch.  Reported as stream events/s and, for cfg 5,
    query-events/s (stream events x queries)."""
    cfg = W.CONFIGS[3]
    stream = N.synth_stream("stock", cfg.seed, keys, 1000, 0, device)
    out = {}
    for name, queries in (("cfg4", [W.any_kleene_query()]), ("cfg5", W.multi_queries(64))):
        qs = [N.Query(p.to_ir()) for p in queries]
        s = N.Session(qs, device=device)
        el, _, _ = run_steps(s, stream, steps, warmup, dist)
        kms = [s.timing(i)[0] for i in range(len(qs))]
        n_m = sum(s.digest(i)[0] for i in range(len(qs)))
        s.close()
        ev_s = stream.n_events * steps / el
        out[name] = {"workload": ("cfg4: skip_till_any Kleene+ with folds avg/sum, within 10 ms" if name == "cfg4"
                                  else "cfg5: 64 stock-query variants, one session") +
                     f", {keys} keys x ~1000 events ({stream.n_events} events) on 1 GPU",
                     "value": ev_s, "unit": "events/s", "ms_per_step": 1e3 * el / steps,
                     "queries": len(qs), "query_events_per_s": ev_s * len(qs),
                     "kernel_ms_sum": float(sum(kms)), "matches_per_step": int(n_m)}
    return out


def end_to_end(args, device, dist):
    """SURVEY §8(d)'s secondary figure: the same cfg-3 workload handed over in arrival order
    (a key id per event, round-robin interleaved), so each step includes the device partition
    (stable radix sort by key + column gather, csrc/partition.hip) before the NFA."""
    cfg = W.CONFIGS[3]
    st = N.synth_arrival_stream("stock", cfg.seed, args.keys, args.mean, dist.rank * args.keys, device)
    q = N.Query(W.stock_query(args.variant).to_ir())
    s = N.Session(q, device=device)
    for _ in range(max(1, args.warmup)):
        s.push_arrival_device(st)
    part, kern = [], []
    dist.barrier()
    N.lib().cep_sync(s.h)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        s.push_arrival_device(st)
        part.append(_partition_ms(s))
        kern.append(s.timing(0)[0])
    N.lib().cep_sync(s.h)
    el = time.perf_counter() - t0
    n_m, _ = s.digest(0)
    s.close()
    return {"workload": "cfg3 stock query, arrival-order batches (partition on the GPU + NFA)",
            "value": st.n_events * args.steps / el, "unit": "events/s", "ms_per_step": 1e3 * el / args.steps,
            "partition_ms": float(np.mean(part)), "nfa_kernel_ms": float(np.mean(kern)),
            "matches_per_step": n_m}


def ingest(device, steps, keys, cpu_sample):
    """the step before the matcher.  The cfg-3 stream at `keys` keys x ~1000
    events as StockEvent JSON record values back to back in HBM (json-simple's serialization,
    StockEventSerDe.java:75-82), decoded by cep_decode_stock_json (csrc/ingest.hip) into the int32
    price/volume columns the matcher reads.  Timed with HIP events on the launch stream;
    algorithmic bytes = record text + 8 B offset read + 4+4+4 B (price, volume, status) written
    per record.  CPU baseline: oracle/json_oracle.py (the json-simple restatement, 1 thread) on
    the first `cpu_sample` records."""
    import ctypes as C

    hip = C.CDLL("libamdhip64.so")
    cfg = W.CONFIGS[3]
    stream = N.synth_stream("stock", cfg.seed, keys, 1000, 0, device)
    batch = N.StockJsonBatch.synth(stream.cols[0], stream.cols[1], stream.n_events, device)
    n = stream.n_events
    out = N.DecodedStock(n, 4, device, name_spans=False)
    # HIP events on the stream the kernel is launched on (the null stream)
    e0, e1 = C.c_void_p(), C.c_void_p()
    assert hip.hipSetDevice(device) == 0 and hip.hipEventCreate(C.byref(e0)) == 0
    assert hip.hipEventCreate(C.byref(e1)) == 0
    N.decode_stock_json(batch, 4, out, None)
    assert hip.hipDeviceSynchronize() == 0
    hip.hipEventRecord(e0, None)
    for _ in range(steps):
        N.decode_stock_json(batch, 4, out, None)
    hip.hipEventRecord(e1, None)
    assert hip.hipEventSynchronize(e1) == 0
    f = C.c_float()
    assert hip.hipEventElapsedTime(C.byref(f), e0, e1) == 0
    hip.hipEventDestroy(e0)
    hip.hipEventDestroy(e1)
    ms = f.value / steps
    bad = int(np.count_nonzero(out.status.download(np.int32, n)))
    alg = batch.nbytes + 8 * (n + 1) + 12 * n
    achieved = alg / (ms * 1e-3) / 1e9
    res = {"workload": f"StockEvent JSON -> int32 columns, cfg3 stream {keys} keys x ~1000 events ({n} records, "
                       f"{batch.nbytes} bytes)", "value": n / (ms * 1e-3), "unit": "records/s",
           "ms_per_step": ms, "bytes_per_s": batch.nbytes / (ms * 1e-3), "failed_records": bad,
           "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": load_traffic("decode_stock_json_kernel"),
                        "kernel": "decode_stock_json_kernel (+ decode_stock_json_general over pending records)",
                        "algorithmic_bytes": alg}}
    if cpu_sample:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import json_oracle

        data, off = batch.download()
        m = min(cpu_sample, n)
        t0 = time.perf_counter()
        exp = json_oracle.decode_batch(data[:int(off[m])], off[:m + 1], 4)
        el = time.perf_counter() - t0
        _, cols = stream.download()
        ok = all(e[0] == 0 for e in exp) and [e[1] for e in exp] == cols[0][:m].tolist()
        res["cpu_baseline"] = {"value": m / el, "unit": "records/s", "cores": 1, "kind": "port",
                               "sample": f"first {m} records, {el:.2f} s, 1 thread (oracle/json_oracle.py)",
                               "parity_on_sample": bool(ok)}
    return res


def _partition_ms(s):
    off, perm, ms = N.C.c_void_p(), N.C.c_void_p(), N.C.c_double()
    N._check(N.lib().cep_batch_layout(s.h, N.CEP_MEM_DEVICE, N.C.byref(off), N.C.byref(perm), N.C.byref(ms)))
    return ms.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--keys", type=int, default=1_000_000, help="keys per GPU")
    ap.add_argument("--mean", type=int, default=1000, help="mean events per key")
    ap.add_argument("--variant", default="readme", choices=["readme", "test"])
    ap.add_argument("--cpu-threads", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--cpu-every", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the arrival-order end-to-end figure")
    ap.add_argument("--no-other", action="store_true", help="skip the cfg 4 / cfg 5 figures")
    ap.add_argument("--no-ingest", action="store_true", help="skip the JSON ingest figure")
    ap.add_argument("--other-keys", type=int, default=100_000, help="keys of the cfg 4 / cfg 5 figures")
    args = ap.parse_args()

    dist = Dist()
    if dist.world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={dist.world}", file=sys.stderr)
    device = dist.local
    cfg = W.SynthConfig("cfg3_stock", "stock", args.keys, args.mean, W.CONFIGS[3].seed,
                        key_base=dist.rank * args.keys)
    stream = N.synth_stream("stock", cfg.seed, cfg.n_keys, cfg.mean_events, cfg.key_base, device)
    q = N.Query(W.stock_query(args.variant).to_ir())
    sess = N.Session(q, device=device)
    el, kms, aux_ms = run_steps(sess, stream, args.steps, args.warmup, dist)
    n_m, digest = sess.digest(0)
    code, _ = sess.key_errors(0)
    n_err = int(np.count_nonzero(code))
    # pairs emitted (event ids): from the flat output of the last step
    m = N.Matches()
    N._check(N.lib().cep_poll_matches(sess.h, 0, N.CEP_MEM_DEVICE, N.C.byref(m)))
    n_pairs = m.n_pairs
    wm = dist.min_i64(sess.watermark())
    per = dist.gather([stream.n_events, n_m, n_pairs, el, kms, float(n_err)])
    checksum = dist.sum_u64(digest)  # wrapping sum of the shards' checksums (shard-local key ids)
    tot_ev, tot_m = per[:, 0].sum(), per[:, 1].sum()
    t_max = per[:, 3].max()

    if dist.rank == 0:
        alg = 8.0 * stream.n_events + 4.0 * n_pairs + 4.0 * n_m  # SURVEY §8(d), rank 0's launch
        achieved = alg / (kms * 1e-3) / 1e9
        out = {
            "metric": METRIC,
            "value": tot_ev * args.steps / t_max,
            "unit": "events/s",
            "matches_per_s": tot_m * args.steps / t_max,
            "n_gpus": dist.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * t_max / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic: SplitMix64 stock random walk (SURVEY §8d), generated in HBM",
            "config": {"workload": f"cfg3 README stock query SEQ(Stock+ a[], Stock b) skip_till_next, "
                                   f"folds avg/volume, WITHIN 1h ({args.variant} variant)",
                       "keys_per_gpu": args.keys, "events_per_gpu": int(stream.n_events),
                       "matches_per_gpu_step": int(n_m), "parallelism": f"key-sharded x{dist.world}",
                       "key_errors": int(per[:, 5].sum())},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": load_traffic("cep_nfa_jit"),
                         "kernel": "cep_nfa_jit", "kernel_ms": kms, "compaction_ms": aux_ms,
                         "algorithmic_bytes": alg},
            "watermark": wm,
            "checksum": f"{checksum:016x}",
        }
        if dist.world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(cfg, args.variant, args.cpu_threads, args.cpu_every)
        if dist.world == 1 and not args.no_secondary:
            out["secondary"] = secondary_strict(device, args.steps, args.warmup, dist)
        if dist.world == 1 and not args.no_e2e:
            sess.close()
            out["end_to_end"] = end_to_end(args, device, dist)
        if dist.world == 1 and not args.no_ingest:
            out["ingest"] = ingest(device, args.steps, args.other_keys, 0 if args.no_cpu_baseline else 100_000)
        if dist.world == 1 and not args.no_other:
            out["other_configs"] = other_configs(device, max(1, args.steps // 2), 1, dist, args.other_keys)
        print(json.dumps(out), flush=True)
    sess.close()
    dist.close()


if __name__ == "__main__":
    main()
