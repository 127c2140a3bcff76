"""Config 5's work distribution: each key-range batch of the 64-variant group pushed and timed on
its own, with the emitted event ids per (variant, key) job counted on the GPU (the walk work is
about proportional to them).  One JSON line per batch: kernel time, the heaviest jobs and keys,
and how concentrated the ids are.
    python profiles/cfg5_probe.py [--keys 1000000] [--batch 125000] [--only 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cepamd  # noqa: E402,F401
from kafkastreams_cep_amd import native as N  # noqa: E402
from kafkastreams_cep_amd import workloads as W  # noqa: E402


class _Dev:
    """a device array as torch sees one (__cuda_array_interface__)"""

    def __init__(self, ptr, n, typestr):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (int(ptr), False), "version": 2}


def job_pairs(s, q, n_keys):
    m = N.Matches()
    N._check(N.lib().cep_poll_matches(s.h, q, N.CEP_MEM_DEVICE, N.C.byref(m)))
    out = torch.zeros(n_keys, dtype=torch.int64, device="cuda")
    if m.n_matches == 0:
        return out, 0, 0
    key = torch.as_tensor(_Dev(N.C.cast(m.key, N.C.c_void_p).value, m.n_matches, "<u4"), device="cuda")
    if m.arity:
        per = torch.full((m.n_matches,), m.arity, dtype=torch.int64, device="cuda")
    else:
        off = torch.as_tensor(_Dev(N.C.cast(m.pair_off, N.C.c_void_p).value, m.n_matches + 1, "<u8"), device="cuda")
        off = off.view(torch.int64)
        per = off[1:] - off[:-1]
    out.index_add_(0, key.to(torch.int64), per)
    return out, int(m.n_matches), int(m.n_pairs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=125_000)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    cfg = W.CONFIGS[3]
    qs = [N.Query(p.to_ir()) for p in W.multi_queries(64)]
    s = N.Session(qs)
    only = [int(x) for x in args.only.split(",")] if args.only else None
    for bi, b in enumerate(range(0, args.keys, args.batch)):
        if only is not None and bi not in only:
            continue
        nk = min(args.batch, args.keys - b)
        p = N.synth_stream("stock", cfg.seed, nk, 1000, b)
        s.push_device(p)  # (warm)
        t0 = time.perf_counter()
        s.push_device(p)
        N.lib().cep_sync(s.h)
        wall = 1e3 * (time.perf_counter() - t0)
        st = s.stats(0)
        jp = torch.stack([job_pairs(s, q, nk)[0] for q in range(64)])  # [variant, key]
        flat = jp.flatten()
        tot = int(flat.sum())
        top = torch.topk(flat, 16)
        per_key = jp.sum(0)
        topk = torch.topk(per_key, 8)
        srt = torch.sort(flat, descending=True).values.double().cumsum(0)
        res = {"batch": bi, "first_key": b, "keys": nk, "wall_ms": wall, "kernel_ms": st["kernel_ms"],
               "pairs": tot,
               "top_jobs": [[int(i) // nk, b + int(i) % nk, int(v)] for v, i in zip(top.values, top.indices)],
               "top_keys": [[b + int(i), int(v), int((jp[:, int(i)] > 0).sum())] for v, i in zip(topk.values, topk.indices)],
               "share_top": {str(n): float(srt[n - 1] / max(tot, 1)) for n in (1, 16, 64, 256, 1024, 4096, 65536)},
               "per_variant": [int(x) for x in jp.sum(1)]}
        print(json.dumps(res), flush=True)
        del p


if __name__ == "__main__":
    main()
