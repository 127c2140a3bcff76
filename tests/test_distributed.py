"""Multi-rank path on the CPU: bench.py's key sharding (rank r owns keys [r K, (r+1) K) of
the same generator stream) and its gloo/RCCL reductions (all-gather of counts, wrapping
checksum sum, min watermark), with the oracle standing in for the per-GPU matcher.
The union of the shards must equal one rank running all keys."""
import os
import socket
import sys
import tempfile

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K, MEAN = 150, 300


def _shard_result(rank):
    import cepamd  # noqa: F401
    import oracle
    from kafkastreams_cep_amd import workloads as W

    cfg = W.SynthConfig("t", "stock", K, MEAN, W.CONFIGS[3].seed, key_base=rank * K)
    off, cols = W.generate(cfg)
    ir = W.stock_query("readme").to_ir()
    r = oracle.run(ir, off, cols, threads=2)
    emit = r["emit_pos"].astype(np.uint64) - off[r["key"].astype(np.int64)]
    pk = np.repeat(r["key"].astype(np.int64), np.diff(r["pair_off"].astype(np.int64)))
    pseq = r["pair_pos"].astype(np.uint64) - off[pk]
    return int(off[-1]), r["n_matches"], W.match_digest(r["key"], emit, r["pair_off"], pseq, r["pair_stage"])


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import bench

    dist = bench.Dist(backend="gloo")
    n_ev, n_m, dig = _shard_result(rank)
    per = dist.gather([n_ev, n_m])
    total = dist.sum_u64(dig)
    wm = dist.min_i64(1000 + rank)
    dist.barrier()
    if rank == 0:
        np.save(out, np.array([per[:, 0].sum(), per[:, 1].sum(), total >> 32, total & 0xFFFFFFFF, wm], np.int64))
    dist.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_sharding_matches_single_rank():
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.npy")
        mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
        got = np.load(out)
    # the same two shards computed in this process, and one rank owning all 2K keys
    shards = [_shard_result(r) for r in range(2)]
    import cepamd  # noqa: F401
    import oracle
    from kafkastreams_cep_amd import workloads as W

    cfg = W.SynthConfig("t", "stock", 2 * K, MEAN, W.CONFIGS[3].seed)
    off, cols = W.generate(cfg)
    whole = oracle.run(W.stock_query("readme").to_ir(), off, cols, threads=2)
    assert got[0] == sum(s[0] for s in shards) == int(off[-1])
    assert got[1] == sum(s[1] for s in shards) == whole["n_matches"] > 0
    assert (int(got[2]) << 32 | int(got[3])) == sum(s[2] for s in shards) % (1 << 64)
    assert got[4] == 1000
    # shard r's matches are exactly the whole run's matches on keys [r K, (r+1) K)
    n0 = int(np.count_nonzero(whole["key"] < K))
    assert (n0, whole["n_matches"] - n0) == (shards[0][1], shards[1][1])
