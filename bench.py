#!/usr/bin/env python3
"""bench.py — events/sec of the README stock Kleene+ query on 1/2/4/8 MI355X.

BASELINE.json metric: "events/sec (whole node) + matches/sec, stock Kleene+ query, 1M keys,
1/2/4/8 GPU" on config 3: 1e9 events over 1M keys.  One step = one pass of the matcher
(libcep.so: begin-hit bitmap, lane order, cep_nfa_jit, compaction) over one batch, inputs
already resident in HBM, every key starting from the NFA's initial state.

Multi-GPU: the 1M keys of ONE global stream are sharded by Kafka's
DefaultPartitioner over the key ids (kafkastreams-cep_amd/shard.py: murmur2 % n_gpus), each
rank gathering its keys' events on its GPU once before timing; N ranks share the fixed 1e9
events ("scaling": "strong", BASELINE's config).  --scaling weak gives every rank its own
1M keys instead.  There is no data-path collective: RCCL only all-gathers the per-rank
counts/checksums and reduces the watermark (min of the ranks' max event time).

    python bench.py                      # N=1, defaults finish in a few minutes
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N

Prints ONE JSON line on rank 0 (fields documented in DESIGN.md §7).  `roofline` prices
cep_nfa_jit at SURVEY §8(d)'s algorithmic bytes (columns read once + 4 B per emitted event id +
4 B per match) against 8 TB/s; `cpu_baseline` times the oracle (oracle/cep_oracle.cpp, the
literal restatement of the reference NFA) on a 1/8 key sample on this host's cores.  At N=1
the line also carries config 2 (`secondary`), the arrival-order end-to-end figure, the JSON
ingest figure and configs 4/5 (`other_configs`), each with key errors, emitted event ids,
roofline and a CPU baseline.
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
from kafkastreams_cep_amd import shard as SH  # noqa: E402
from kafkastreams_cep_amd import workloads as W  # noqa: E402

METRIC = "events/sec (whole node) + matches/sec, stock Kleene+ query, 1M keys, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
TS_BASE = 1_600_000_000_000  # ts = 1.6e12 + position (ms)
_T0 = time.time()


def cpu_share():
    """(host threads for the CPU baseline, nproc): the cgroup CPU quota when one is set (a
    GPU box's share of the machine), else every CPU this process may run on.  os.cpu_count()
    is reported beside it as `nproc`."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return max(1, n), os.cpu_count() or 1


def log(msg):
    """progress on stderr (the JSON line alone goes to stdout)"""
    print(f"[bench {time.time() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


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

            # ($CEP_BENCH_BACKEND=gloo with $CEP_BENCH_DEVICE=0: a rehearsal of the N-rank path
            # on a one-GPU box, every rank on the same card, the collectives on the CPU)
            self.backend = backend or os.environ.get("CEP_BENCH_BACKEND", "nccl")
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


def run_steps(sess, stream, steps, warmup, dist, ts=None):
    tsp = ts.ptr if ts is not None else None
    for _ in range(warmup):
        sess.push_device(stream, tsp)
    sess.timing_totals(0, reset=True)  # (syncs the stream)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        # NFA batches return after their kernels complete (retries need the counts); stencil
        # batches queue on the stream and return at once
        sess.push_device(stream, tsp)
    N.lib().cep_sync(sess.h)
    dist.barrier()
    el = time.perf_counter() - t0
    # HIP events of every timed batch on the session stream (read after the region)
    kern, aux, n = sess.timing_totals(0)
    assert n == steps, (n, steps)
    return el, kern / steps, aux / steps


def load_traffic(name):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            return json.load(f).get(name)
    except (OSError, ValueError):
        return None


def roofline(alg_bytes, kernel_ms, kernel, traffic_key=None, traffic_scale=1, **extra):
    """traffic: the committed PMC figure for one launch (x traffic_scale launches per priced
    interval, e.g. config 5's key-range batches per step)"""
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
    tr = load_traffic(traffic_key or kernel)
    r = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
         "traffic": tr * traffic_scale if tr is not None else None, "kernel": kernel, "kernel_ms": kernel_ms,
         "algorithmic_bytes": alg_bytes}
    r.update(extra)
    return r


def match_figures(sess, query, n_keys):
    """(matches, emitted event ids, keys with an error) of the last batch for one query"""
    m = N.Matches()
    N._check(N.lib().cep_poll_matches(sess.h, query, N.CEP_MEM_DEVICE, N.C.byref(m)))
    code, _ = sess.key_errors(query, n_keys)
    return int(m.n_matches), int(m.n_pairs), int(np.count_nonzero(code))


def global_digest(sess, key_ids):
    """Checksum of the last batch's matches with GLOBAL key ids (shard key i = key_ids[i]), so
    the wrapping sum over ranks equals a single GPU's checksum of the whole stream."""
    m = sess.matches(0)
    gk = key_ids[m["key"].astype(np.int64)] if key_ids is not None else m["key"]
    return W.match_digest(gk, m["emit_seq"], m["pair_off"], m["pair_seq"], m["pair_stage"])


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the checker / CPU baseline only

    return oracle


def cpu_baseline(cfg, queries, threads, every, gpu_check=None, extrapolated=False, semantic=False):
    """The oracle on keys 0, every, 2*every, ... of the same stream (the numpy generator = the
    GPU generator bit for bit), every query in turn.  events/s = sample events x queries /
    oracle time.  gpu_check(off, cols) -> per-query (n_matches, checksum) on the GPU for the
    same sample: the parity spot check."""
    oracle = _oracle()
    keys = np.arange(0, cfg.n_keys, every)
    off, cols = W.generate(cfg, keys)
    n_ev = int(off[-1])
    el, n_m, want = 0.0, 0, []
    for p in queries:
        r = oracle.run(p.to_ir(semantic_within=semantic), off, cols, threads=threads)
        el += r["elapsed_s"]
        n_m += r["n_matches"]
        emit = r["emit_pos"].astype(np.uint64) - off[r["key"].astype(np.int64)]
        pk = np.repeat(r["key"].astype(np.int64), np.diff(r["pair_off"].astype(np.int64)))
        pseq = r["pair_pos"].astype(np.uint64) - off[pk]
        want.append((r["n_matches"], W.match_digest(r["key"], emit, r["pair_off"], pseq, r["pair_stage"]),
                     int(np.count_nonzero(r["err_code"]))))
    out = {"value": n_ev * len(queries) / el, "unit": "events/s" if len(queries) == 1 else "query-events/s",
           "cores": r["threads"], "nproc": cpu_share()[1], "kind": "port",
           "sample": f"{len(keys)} of {cfg.n_keys} keys (every {every}th), {n_ev} events x {len(queries)} "
                     f"quer{'y' if len(queries) == 1 else 'ies'}, {n_m} matches, {el:.2f} s on {r['threads']} threads"
                     + (" (rate extrapolated to the full key set)" if extrapolated else ""),
           "matches_per_s": n_m / el}
    if gpu_check is not None:
        out["parity_on_sample"] = bool(gpu_check(off, cols) == want)
    return out


def gpu_digests(queries, device, semantic=False):
    """per query (n_matches, checksum, keys with an exception) of the GPU on the CPU sample"""
    def check(off, cols):
        qs = [N.Query(p.to_ir(semantic_within=semantic)) for p in queries]
        s = N.Session(qs, device=device)
        s.push(off, cols)
        got = [s.digest(i) + (int(np.count_nonzero(s.key_errors(i)[0])),) for i in range(len(qs))]
        s.close()
        return got
    return check


def secondary_strict(device, steps, warmup, dist, threads, cpu):
    """Config 2: strict SEQ(A,B,C), 1e8 events over 1e4 keys, the stencil passes.  CPU
    baseline: the oracle over the WHOLE stream on all host cores.  A step is
    0.12 ms, so it is timed over at least 50 steps after at least 5 warmup steps (a handful of
    steps is dominated by the first pushes' host work)."""
    steps, warmup = max(steps, 50), max(warmup, 5)
    cfg = W.CONFIGS[2]
    stream = N.synth_stream("abc", cfg.seed, cfg.n_keys, cfg.mean_events, 0, device)
    q = N.Query(W.strict_abc_query().to_ir())
    s = N.Session(q, device=device)
    el, kms, _ = run_steps(s, stream, steps, warmup, dist)
    n_m, dig = s.digest(0)
    _, n_pairs, n_err = match_figures(s, 0, cfg.n_keys)
    n_ev = stream.n_events
    alg = 4.0 * n_ev + 16.0 * n_m  # one int column + (key + 3 event ids) per match
    res = {"workload": "cfg2: strict SEQ(A,B,C) v<4 | 4<=v<8 | v>=8, 1e4 keys x 1e4 events",
           "value": n_ev * steps / el, "unit": "events/s", "matches_per_step": n_m, "pairs_per_step": n_pairs,
           "key_errors": n_err, "ms_per_step": 1e3 * el / steps, "steps": steps, "warmup": warmup,
           "roofline": roofline(alg, kms, "stencil_mask+stencil_emit", "stencil")}
    s.close()
    if cpu:
        oracle = _oracle()
        off, cols = stream.download()
        r = oracle.run(q.ir, off, cols, threads=threads)
        emit = r["emit_pos"].astype(np.uint64) - off[r["key"].astype(np.int64)]
        pk = np.repeat(r["key"].astype(np.int64), np.diff(r["pair_off"].astype(np.int64)))
        pseq = r["pair_pos"].astype(np.uint64) - off[pk]
        want = W.match_digest(r["key"], emit, r["pair_off"], pseq, r["pair_stage"])
        res["cpu_baseline"] = {"value": n_ev / r["elapsed_s"], "unit": "events/s", "cores": r["threads"],
                               "nproc": cpu_share()[1], "kind": "port", "sample": f"the whole stream ({n_ev} events, {r['n_matches']} matches), "
                                                         f"{r['elapsed_s']:.2f} s on {r['threads']} threads",
                               "parity_on_sample": bool((r["n_matches"], want) == (n_m, dig))}
    return res


def cfg4(device, stream, steps, warmup, dist, threads, cpu_every, stress=True):
    """Config 4: skip_till_any Kleene+ with folds and a 10 ms WITHIN over the cfg-3 stream (1M
    keys): run-explosion / versioned-buffer stress.  Reports buffer nodes per key.
    stress=True (the benched figure): workloads.any_kleene_query(carry_volume=True), the variant
    in which no key throws ("no Appendix-C exception path fires");
    stress=False: the query as written, the parity case, which throws NPE on about half of
    the keys in the reference itself (NFA.java:243, ValueStore.java:92-97)."""
    p = W.any_kleene_query(carry_volume=stress)
    q = N.Query(p.to_ir())
    s = N.Session(q, device=device)
    el, kms, _ = run_steps(s, stream, steps, warmup, dist)
    n_m, n_pairs, n_err = match_figures(s, 0, stream.n_keys)
    st = s.stats(0)
    s.close()
    alg = 8.0 * stream.n_events + 4.0 * n_pairs + 4.0 * n_m
    what = ("S1 also folds volume, S2 reads it with getOrElse: no key throws" if stress else
            "the query as written (parity case; NPE in the reference on the keys counted in key_errors)")
    # priced at step level, like cfg4_semantic: the step streams the
    # columns once (begin-hit bitmap), while cep_nfa_jit skips quiet words and keys that threw
    res = {"workload": f"cfg4: skip_till_any Kleene+ with folds avg/sum, within 10 ms, {what}; {stream.n_keys} keys x "
                       f"~1000 events ({stream.n_events} events) on 1 GPU",
           "value": stream.n_events * steps / el, "unit": "events/s", "ms_per_step": 1e3 * el / steps,
           "steps": steps, "warmup": warmup,
           "matches_per_step": n_m, "pairs_per_step": n_pairs, "key_errors": n_err,
           "buffer_nodes_per_key": st["nodes_used"] / max(1, stream.n_keys),
           "buffer_preds_per_key": st["preds_used"] / max(1, stream.n_keys),
           "retried_jobs": st["retried_jobs"],
           "roofline": roofline(alg, 1e3 * el / steps, "whole step (cep_nfa_bits, cep_nfa_est, lane order, "
                                "cep_nfa_jit, compaction)", "cfg4" + ("s" if stress else "") + "_step",
                                cep_nfa_jit_ms=st["main_ms"], step_kernels_ms=kms)}
    if cpu_every:
        cfg = W.SynthConfig("cfg4", "stock", stream.n_keys, 1000, W.CONFIGS[3].seed)
        res["cpu_baseline"] = cpu_baseline(cfg, [p], threads, cpu_every, gpu_digests([p], device), extrapolated=True)
    return res


def semantic_cfg4(device, stream, ts, steps, warmup, dist, threads, cpu_every):
    """config 4's query with its WITHIN 10 ms enforced (semantic mode,
    Pattern.to_ir(semantic_within=True); the reference's own WITHIN never prunes).  Event
    times are the stream's (1.6e12 + position: a key's events 1 ms apart), so a run expires
    ten events after its start instead of accumulating (config 4's run explosion)."""
    p = W.any_kleene_query()
    ir = p.to_ir(semantic_within=True)
    s = N.Session(N.Query(ir), device=device)
    el, kms, _ = run_steps(s, stream, steps, warmup, dist, ts)
    n_m, n_pairs, n_err = match_figures(s, 0, stream.n_keys)
    st = s.stats(0)
    s.close()
    # priced at step level: the step streams price + volume (begin-hit bitmap) and the
    # timestamps (watermark, expiry) once, but cep_nfa_jit itself skips most of those bytes
    # (quiet lanes jump 64 events per bitmap word), so a kernel-level price would overstate it
    alg = 16.0 * stream.n_events + 4.0 * n_pairs + 4.0 * n_m  # price, volume, ts
    res = {"workload": f"cfg4 query, semantic WITHIN 10 ms (runs expire), {stream.n_keys} keys x ~1000 events "
                       f"({stream.n_events} events), ts = 1.6e12 + position",
           "value": stream.n_events * steps / el, "unit": "events/s", "ms_per_step": 1e3 * el / steps,
           "steps": steps, "warmup": warmup,
           "matches_per_step": n_m, "pairs_per_step": n_pairs, "key_errors": n_err,
           "buffer_nodes_per_key": st["nodes_used"] / max(1, stream.n_keys),
           "roofline": roofline(alg, 1e3 * el / steps, "whole step (cep_nfa_bits, cep_nfa_est, lane order, "
                                "watermark max, cep_nfa_jit, compaction)", "cfg4_semantic_step",
                                cep_nfa_jit_ms=st["main_ms"], step_kernels_ms=kms)}
    if cpu_every:
        cfg = W.SynthConfig("cfg4s", "stock", stream.n_keys, 1000, W.CONFIGS[3].seed)
        res["cpu_baseline"] = cpu_baseline(cfg, [p], threads, cpu_every, gpu_digests([p], device, True),
                                           extrapolated=True, semantic=True)
    return res


def slice_stream(stream, slices):
    """The stream cut into `slices` consecutive batches per key: batch b holds key k's events
    j with n_k*b/slices <= j < n_k*(b+1)/slices (gathered on the device)."""
    off = stream.key_off.download(np.uint64, stream.n_keys + 1).astype(np.int64)
    n = np.diff(off)
    parts = []
    for b in range(slices):
        lo, hi = n * b // slices, n * (b + 1) // slices
        parts.append(N.gather_ranges(stream, (off[:-1] + lo).astype(np.uint64), (off[:-1] + hi).astype(np.uint64)))
    return parts


def streaming_cfg3(device, stream, slices, steps, dist, warmup=1, variant="readme"):
    """The path CEPProcessor uses (processor.py): a streaming session, each key's NFA carried
    from batch to batch (cep_opts.streaming; NFA.java:94-109 driven per record by
    CEPProcessor.java:155-163).  The cfg-3 stream is pushed as `slices` consecutive batches
    (about 1000/slices events per key each); a step = all of them, every key starting from the
    NFA's initial state.  Exactness at full size: the sum of the batches'
    checksums equals the per-batch session's checksum of the whole stream (the same matches
    with the same per-key sequence numbers), checked on one untimed pass."""
    parts = slice_stream(stream, slices)
    q = N.Query(W.stock_query(variant).to_ir())
    times, kern = [], []
    s = N.Session(q, device=device, streaming=True)
    for it in range(warmup + steps):
        s.reset()  # every key back to the initial state (the warmup sized the pools)
        dist.barrier()
        t0 = time.perf_counter()
        km = 0.0
        for p in parts:
            s.push_device(p)
            km += s.stats(0)["kernel_ms"]
        N.lib().cep_sync(s.h)
        el = time.perf_counter() - t0
        if it >= warmup:
            times.append(el)
            kern.append(km)
    # the untimed verification pass: matches, errors and checksums summed over the batches
    s.reset()
    n_m = n_p = 0
    dig = 0
    for p in parts:
        s.push_device(p)
        m, d = s.digest(0)
        _, pairs, _ = match_figures(s, 0, p.n_keys)
        n_m += m
        n_p += pairs
        dig = (dig + d) % (1 << 64)
    code, _ = s.key_errors(0, stream.n_keys)
    s.close()
    el = float(np.mean(times))
    return {"workload": f"cfg3 README stock query as {slices} consecutive batches of a streaming session "
                        f"({stream.n_keys} keys, ~{stream.n_events // max(1, stream.n_keys * slices)} events per key "
                        f"per batch, {stream.n_events} events per step)",
            "value": stream.n_events / el, "unit": "events/s", "ms_per_step": 1e3 * el, "steps": steps,
            "warmup": warmup, "kernel_ms_per_step": float(np.mean(kern)), "matches_per_step": n_m,
            "pairs_per_step": n_p, "key_errors": int(np.count_nonzero(code)), "checksum": f"{dig:016x}"}


def processor_throughput(device, n_keys=10_000, per_key=100, batch=65_536):
    """The reference's own entry point: CEPProcessor.process(key, value) (CEPProcessor.java:
    155-163) called once per record, as a Kafka stream task calls it, on the README query, for
    `n_keys` keys x `per_key` records of the cfg-3 generator interleaved round-robin (arrival
    order), then close() (the flush).  processor.py buffers `batch` records per GPU push (a
    streaming session's arrival-order batch) and forwards every Sequence in the reference's
    order.  records/s = records / wall time of the process() calls + close(), host work
    included: the Python host path, not the kernel, bounds this figure."""
    from kafkastreams_cep_amd import processor as P
    cfg = W.SynthConfig("proc", "stock", n_keys, per_key, W.CONFIGS[3].seed)
    off, (price, vol) = W.generate(cfg)
    off = off.astype(np.int64)
    lens = np.diff(off)
    order = []  # round-robin arrival: record r of every key before record r + 1 of any
    for r in range(int(lens.max())):
        ks = np.flatnonzero(lens > r)
        order.append(off[ks] + r)
    pos = np.concatenate(order)
    kid = np.searchsorted(off, pos, side="right") - 1
    recs = [(f"K{int(k)}", {"name": f"K{int(k)}", "price": int(price[p]), "volume": int(vol[p])}, int(i))
            for i, (k, p) in enumerate(zip(kid, pos))]
    ctx = P.RecordContext("StockEvents", 0)
    proc = P.CEPProcessor(W.stock_query("readme"), in_memory=True, batch_size=batch, max_keys=n_keys, device=device)
    proc.init(ctx)
    t0 = time.perf_counter()
    for k, v, ts in recs:
        ctx.send(k, v, ts)
    proc.close()
    el = time.perf_counter() - t0
    res = {"workload": f"CEPProcessor.process() per record, README query, {n_keys} keys x {per_key} records "
                       f"(round-robin arrival), batch {batch}, in_memory", "value": len(recs) / el,
           "unit": "records/s", "records": len(recs), "forwarded": len(ctx.forwarded),
           "matches_per_s": len(ctx.forwarded) / el, "seconds": el}
    res["latency"] = processor_latency(device, recs, n_keys)
    return res


def processor_latency(device, recs, n_keys, batch=None):
    """ Time from process() to forward at the processor's default batch
    size: a record is forwarded by the flush of the batch it lands in, so the newest record of a
    batch waits that flush (the GPU push, the match read-back and the Sequence forwarding) and
    the oldest the batch's fill time before it too.  Per flush: its wall time and the fill time
    since the previous flush ended."""
    from kafkastreams_cep_amd import processor as P
    ctx = P.RecordContext("StockEvents", 0)
    kw = {} if batch is None else {"batch_size": batch}
    proc = P.CEPProcessor(W.stock_query("readme"), in_memory=True, max_keys=n_keys, device=device, **kw)
    proc.init(ctx)
    flush_ms, fill_ms = [], []
    orig = proc.flush
    last = [time.perf_counter()]

    def timed_flush():
        t = time.perf_counter()
        orig()
        e = time.perf_counter()
        flush_ms.append(1e3 * (e - t))
        fill_ms.append(1e3 * (t - last[0]))
        last[0] = e
    proc.flush = timed_flush
    for k, v, ts in recs:
        ctx.send(k, v, ts)
    proc.close()
    f, g = np.array(flush_ms[:-1] or flush_ms), np.array(fill_ms[:-1] or fill_ms)  # (the last: close's partial batch)
    return {"batch_size": proc.batch_size, "flushes": len(flush_ms),
            "flush_ms_mean": float(f.mean()), "flush_ms_p99": float(np.percentile(f, 99)),
            "fill_ms_mean": float(g.mean()),
            "newest_record_ms": float(f.mean()), "oldest_record_ms": float((f + g).mean()),
            "note": "per record, process() to forward: between the newest (flush only) and the oldest (fill + flush) of its batch"}


def projected_scaling(device, cfg, stream, world, steps, dist, t1_ms=None):
    """SURVEY §8(e) strong scaling, projected on ONE GPU: every rank's murmur2 shard of the
    cfg-3 stream (shard.py, the same split bench.py makes at --gpus N) is run alone, one after
    the other; the projected N-GPU step is the slowest rank's, and the projected efficiency
    t1 / (N x that).  A projection, not a measured multi-GPU curve (no collective, no
    contention between GPUs)."""
    off = stream.key_off.download(np.uint64, stream.n_keys + 1)
    q = N.Query(W.stock_query("readme").to_ir())
    per = []
    for r in range(world):
        keys, loff = SH.shard_layout(off, world, r)
        sh, _ = N.shard_stream(stream, keys, loff)
        s = N.Session(q, device=device)
        el, kms, _ = run_steps(s, sh, steps, 1, dist)
        per.append({"rank": r, "keys": int(len(keys)), "events": int(sh.n_events), "ms_per_step": 1e3 * el / steps,
                    "kernel_ms": s.stats(0)["main_ms"]})
        s.close()
        del sh
    worst = max(p["ms_per_step"] for p in per)
    res = {"world": world, "per_rank": per, "projected_ms_per_step": worst,
           "note": "projection: each rank's shard run alone on one GPU, not a measured multi-GPU curve"}
    if t1_ms:
        res["t1_ms_per_step"] = t1_ms
        res["projected_efficiency"] = t1_ms / (world * worst)
    return res


def cfg5(device, n_keys, sub, steps, warmup, threads, cpu_every):
    """Config 5: the 64 stock-query variants in ONE session over the cfg-3 stream, 1M keys.  The
    queries differ only in literals, so libcep runs them as one kernel group (one launch per
    batch, lanes = (query, key), the columns read once for all 64).  The 1M keys are pushed as
    key-range batches of `sub` keys (the same stream: the generator is counter-based), so each
    batch's output (~2.5e9 event ids per 100k keys) stays within HBM; a step = all of them."""
    cfg = W.CONFIGS[3]
    parts = []
    for b in range(0, n_keys, sub):
        parts.append(N.synth_stream("stock", cfg.seed, min(sub, n_keys - b), 1000, b, device))
    queries = W.multi_queries(64)
    qs = [N.Query(p.to_ir()) for p in queries]
    s = N.Session(qs, device=device)
    tot = {"events": sum(p.n_events for p in parts), "matches": 0, "pairs": 0, "errors": 0, "kernel_ms": 0.0,
           "retried": 0, "wall": 0.0}
    for it in range(warmup + steps):
        timed = it >= warmup
        for bi, p in enumerate(parts):
            log(f"cfg5 {'step' if timed else 'warmup'} {it} batch {bi}")
            t0 = time.perf_counter()
            s.push_device(p)
            dt = time.perf_counter() - t0
            if not timed:
                continue
            tot["wall"] += dt
            st = s.stats(0)
            tot["kernel_ms"] += st["kernel_ms"]
            tot["retried"] += st["retried_jobs"]
            for i in range(len(qs)):
                n_m, n_p, n_e = match_figures(s, i, p.n_keys)
                tot["matches"] += n_m
                tot["pairs"] += n_p
                tot["errors"] += n_e
    s.close()
    ev_s = tot["events"] * steps / tot["wall"]
    alg = 8.0 * tot["events"] * steps + 4.0 * tot["pairs"] + 4.0 * tot["matches"]
    res = {"workload": f"cfg5: 64 stock-query variants, one session, one kernel group; {n_keys} keys x ~1000 events "
                       f"({tot['events']} events) on 1 GPU, pushed as {len(parts)} key-range batches of {sub} keys",
           "value": ev_s, "unit": "events/s", "query_events_per_s": ev_s * len(qs), "queries": len(qs),
           "ms_per_step": 1e3 * tot["wall"] / steps, "matches_per_step": tot["matches"] // steps,
           "pairs_per_step": tot["pairs"] // steps, "key_errors": tot["errors"] // steps,
           "retried_jobs": tot["retried"], "kernel_ms_per_step": tot["kernel_ms"] / steps,
           "roofline": roofline(alg, tot["kernel_ms"], "cep_nfa_jit (64-query group)", "cep_nfa_jit_cfg5",
                                traffic_scale=len(parts))}
    if cpu_every:
        log("cfg5 cpu baseline")
        c = W.SynthConfig("cfg5", "stock", n_keys, 1000, cfg.seed)
        res["cpu_baseline"] = cpu_baseline(c, queries, threads, cpu_every, gpu_digests(queries, device),
                                           extrapolated=True)
    return res


def end_to_end(args, device, dist):
    """SURVEY §8(d)'s secondary figure: the same cfg-3 workload handed over in arrival order
    (a key id per event, round-robin interleaved), so each step includes the device partition
    (csrc/partition.hip) before the NFA.  Per step the record keeps what the push spent (VERDICT
    r4 item 5: one round-4 run measured its NFA launches at 185 ms against the usual 31): the
    partition, the matching launch alone, bitmap + estimate + lane order, re-runs, and the device
    allocations the push made."""
    cfg = W.CONFIGS[3]
    st = N.synth_arrival_stream("stock", cfg.seed, args.keys, args.mean, 0, device)
    q = N.Query(W.stock_query(args.variant).to_ir())
    s = N.Session(q, device=device)
    for _ in range(max(1, args.warmup)):
        s.push_arrival_device(st)
    steps = []
    dist.barrier()
    N.lib().cep_sync(s.h)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        s.push_arrival_device(st)
        b = s.stats(0)
        steps.append({"partition_ms": _partition_ms(s), "nfa_kernel_ms": b["kernel_ms"], "main_ms": b["main_ms"],
                      "est_order_bits_ms": b["kernel_ms"] - b["main_ms"] - b["retry_ms"], "retry_ms": b["retry_ms"],
                      "retried_jobs": int(b["retried_jobs"]), "allocs": int(b["allocs"])})
    N.lib().cep_sync(s.h)
    el = time.perf_counter() - t0
    n_m, dig = s.digest(0)
    try:
        bal, _ = s.lane_balance(0)
    except N.CepError:
        bal = None
    s.close()
    mean = lambda k: float(np.mean([x[k] for x in steps]))  # noqa: E731
    return {"workload": "cfg3 stock query, arrival-order batches (partition on the GPU + NFA)",
            "value": st.n_events * args.steps / el, "unit": "events/s", "ms_per_step": 1e3 * el / args.steps,
            "partition_ms": mean("partition_ms"), "nfa_kernel_ms": mean("nfa_kernel_ms"), "main_ms": mean("main_ms"),
            "est_order_bits_ms": mean("est_order_bits_ms"), "retry_ms": mean("retry_ms"),
            "retried_jobs": sum(x["retried_jobs"] for x in steps), "allocs": sum(x["allocs"] for x in steps),
            "lane_balance": bal, "per_step": steps, "matches_per_step": n_m, "checksum": f"{dig:016x}"}


def ingest(device, steps, keys, cpu_sample):
    """the step before the matcher.  The cfg-3 stream at `keys` keys x ~1000
    events as StockEvent JSON record values back to back in HBM, in the serializer's own key
    order (json-simple JSONObject = HashMap: volume, price, name; StockEventSerDe.java:75-82),
    decoded by cep_decode_stock_json (csrc/ingest.hip) into the int32 price/volume columns the
    matcher reads.  Timed with HIP events on the launch stream; algorithmic bytes = record text
    + 8 B offset read + 4+4+4 B (price, volume, status) written per record.  CPU baseline:
    oracle/json_oracle.py (the json-simple restatement, 1 thread) on the first `cpu_sample`
    records."""
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
                       f"{batch.nbytes} bytes, json-simple key order)", "value": n / (ms * 1e-3),
           "unit": "records/s", "ms_per_step": ms, "bytes_per_s": batch.nbytes / (ms * 1e-3), "failed_records": bad,
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
    ap.add_argument("--keys", type=int, default=1_000_000, help="keys of the stream (strong) or per GPU (weak)")
    ap.add_argument("--mean", type=int, default=1000, help="mean events per key")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"])
    ap.add_argument("--variant", default="readme", choices=["readme", "test"])
    ap.add_argument("--cpu-threads", type=int, default=cpu_share()[0])
    ap.add_argument("--cpu-every", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the arrival-order end-to-end figure")
    ap.add_argument("--no-other", action="store_true", help="skip the cfg 4 / cfg 5 figures")
    ap.add_argument("--no-ingest", action="store_true", help="skip the JSON ingest figure")
    ap.add_argument("--no-projection", action="store_true", help="skip the projected 8-GPU strong scaling")
    ap.add_argument("--no-streaming", action="store_true", help="skip the streaming-session figure")
    ap.add_argument("--ingest-keys", type=int, default=100_000, help="keys of the JSON ingest figure")
    ap.add_argument("--cfg5-keys", type=int, default=1_000_000)
    ap.add_argument("--cfg5-batch", type=int, default=125_000, help="keys per pushed batch of config 5")
    args = ap.parse_args()

    dist = Dist()
    if dist.world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={dist.world}", file=sys.stderr)
    device = int(os.environ.get("CEP_BENCH_DEVICE", dist.local))
    strong = args.scaling == "strong"
    key_base = 0 if strong else dist.rank * args.keys
    cfg = W.SynthConfig("cfg3_stock", "stock", args.keys, args.mean, W.CONFIGS[3].seed, key_base=key_base)
    stream = N.synth_stream("stock", cfg.seed, cfg.n_keys, cfg.mean_events, key_base, device)
    ts = N.synth_ts(stream.n_events, TS_BASE, device)
    key_ids = None  # shard key i -> global key id
    if strong and dist.world > 1:  # this rank's shard of the one global stream (Kafka partitioner)
        keys, local_off = SH.shard_layout(W.key_offsets(cfg), dist.world, dist.rank)
        whole, whole_ts = stream, ts
        stream, ts = N.shard_stream(whole, keys, local_off, whole_ts)
        del whole, whole_ts
        key_ids = keys.astype(np.int64)
    elif not strong:
        key_ids = np.arange(args.keys, dtype=np.int64) + key_base
    q = N.Query(W.stock_query(args.variant).to_ir())
    sess = N.Session(q, device=device)
    log(f"cfg3: {stream.n_keys} keys, {stream.n_events} events on rank {dist.rank}")
    el, kms, aux_ms = run_steps(sess, stream, args.steps, args.warmup, dist, ts)
    log(f"cfg3: {1e3 * el / args.steps:.2f} ms per step")
    n_m, n_pairs, n_err = match_figures(sess, 0, stream.n_keys)
    st = sess.stats(0)
    try:
        bal_ordered, bal_identity = sess.lane_balance(0)
    except N.CepError:  # (no estimate ran: a shard of <= 64 keys)
        bal_ordered = bal_identity = None
    digest = global_digest(sess, key_ids)
    wm = dist.min_i64(sess.watermark())
    per = dist.gather([stream.n_events, n_m, n_pairs, el, kms, float(n_err), stream.n_keys])
    checksum = dist.sum_u64(digest)  # wrapping sum of the shards' checksums (global key ids)
    tot_ev, tot_m, tot_p = per[:, 0].sum(), per[:, 1].sum(), per[:, 2].sum()
    t_max = per[:, 3].max()

    if dist.rank == 0:
        alg = 8.0 * stream.n_events + 4.0 * n_pairs + 4.0 * n_m  # SURVEY §8(d), rank 0's launch
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
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic: SplitMix64 stock random walk (SURVEY §8d), generated in HBM; ts = 1.6e12 + position",
            "config": {"workload": f"cfg3 README stock query SEQ(Stock+ a[], Stock b) skip_till_next, "
                                   f"folds avg/volume, WITHIN 1h ({args.variant} variant)",
                       "keys": int(per[:, 6].sum()), "events": int(tot_ev), "keys_per_gpu": [int(x) for x in per[:, 6]],
                       "matches_per_step": int(tot_m), "pairs_per_step": int(tot_p),
                       "parallelism": f"key-sharded x{dist.world} (Kafka DefaultPartitioner: murmur2(key) % "
                                      f"{dist.world})" if strong else f"key ranges x{dist.world}",
                       "key_errors": int(per[:, 5].sum())},
            # the dominant kernel's own launch (cep_nfa_jit, HIP events around it on the session
            # stream; rocprofv3's average for it agrees, profiles/r02/); the step's other kernels
            # (work estimate + lane order + begin-hit bitmap, compaction) listed beside it
            "roofline": roofline(alg, st["main_ms"], "cep_nfa_jit", step_kernels_ms=kms, compaction_ms=aux_ms,
                                 est_order_bits_ms=st["kernel_ms"] - st["main_ms"] - st["retry_ms"],
                                 retry_ms=st["retry_ms"]),
            # north_star's wave divergence figure: sum over 64-lane waves of the busiest lane's
            # work estimate / the mean lane's, in the launch's lane order and in key order
            "lane_balance": {"wave_max_over_mean": bal_ordered, "without_lane_order": bal_identity},
            "watermark": wm,
            "checksum": f"{checksum:016x}",
        }
        one = dist.world == 1
        cpu = one and not args.no_cpu_baseline
        if cpu:
            log("cfg3 cpu baseline")
            out["cpu_baseline"] = cpu_baseline(cfg, [W.stock_query(args.variant)], args.cpu_threads, args.cpu_every,
                                               gpu_digests([W.stock_query(args.variant)], device))
        if one and not args.no_projection:
            log("projected strong scaling")
            out["projected_scaling"] = projected_scaling(device, cfg, stream, 8, args.steps, dist,
                                                         t1_ms=out["ms_per_step"])
        if one and not args.no_streaming:
            log("streaming")
            out["streaming"] = streaming_cfg3(device, stream, 10, max(1, min(args.steps, 5)), dist)
        if one and not args.no_streaming:
            log("processor")
            out["processor"] = processor_throughput(device)
        if one and not args.no_other:
            log("cfg4")
            # (a config-4 step is 5-10 ms: 10 timed steps after 3 warmup ones, the first of
            # which size the session's pools)
            ok, ow = max(10, args.steps), max(3, args.warmup)
            out["other_configs"] = {"cfg4": cfg4(device, stream, ok, ow, dist, args.cpu_threads, 64 if cpu else 0)}
            log("cfg4 as written")
            out["other_configs"]["cfg4_literal"] = cfg4(device, stream, ok, ow, dist, args.cpu_threads,
                                                        64 if cpu else 0, stress=False)
            log("cfg4 semantic WITHIN")
            out["other_configs"]["cfg4_semantic"] = semantic_cfg4(device, stream, ts, ok, ow, dist, args.cpu_threads,
                                                                   64 if cpu else 0)
        sess.close()
        del stream, ts
        if one and not args.no_secondary:
            log("cfg2")
            out["secondary"] = secondary_strict(device, args.steps, args.warmup, dist, args.cpu_threads, cpu)
        if one and not args.no_e2e:
            log("end to end")
            out["end_to_end"] = end_to_end(args, device, dist)
        if one and not args.no_ingest:
            log("ingest")
            out["ingest"] = ingest(device, args.steps, args.ingest_keys, 100_000 if cpu else 0)
        if one and not args.no_other:
            out["other_configs"]["cfg5"] = cfg5(device, args.cfg5_keys, args.cfg5_batch, 1, 1, args.cpu_threads,
                                                256 if cpu else 0)
        log("done")
        print(json.dumps(out), flush=True)
    else:
        sess.close()
    dist.close()


if __name__ == "__main__":
    main()
