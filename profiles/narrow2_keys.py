"""Which keys of the headline batch outgrow a 2-pair Dewey build, against the lane order's
work estimate: the 2-pair build runs with re-runs off ($CEP_DEWEY_PAIRS=2 $CEP_NO_RETRY=1,
measurement build), its KE_RETRY keys are read back, and the estimate (cep_nfa_est's formula:
sum over begin hits b of (n - b), plus n / 16 + 1) is recomputed on the host.  Prints, for the
top 2-20 % of keys by estimate, the share of the outgrowing keys they hold and their share of
the estimated work.
    CEP_MEASURE=1 python profiles/narrow2_keys.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import cepamd  # noqa: E402,F401
from kafkastreams_cep_amd import native as N  # noqa: E402
from kafkastreams_cep_amd import workloads as W  # noqa: E402

cfg = W.CONFIGS[3]
stream = N.synth_stream("stock", cfg.seed, cfg.n_keys, cfg.mean_events)
os.environ["CEP_DEWEY_PAIRS"] = "2"
q = N.Query(W.stock_query("readme").to_ir())
del os.environ["CEP_DEWEY_PAIRS"]
os.environ["CEP_NO_RETRY"] = "1"
s = N.Session(q)
s.push_device(stream)
code, _ = s.key_errors(0)
st = s.stats(0)
s.close()
bad = np.flatnonzero(code != 0)
off, (price, vol) = stream.download()
off = off.astype(np.int64)
n = np.diff(off)
hit = np.flatnonzero(vol > 1000)  # the README query's begin predicate (volume > 1000)
key = np.searchsorted(off, hit, side="right") - 1
est = np.bincount(key, weights=(off[key + 1] - hit).astype(np.float64), minlength=len(n)) + n // 16 + 1
order = np.argsort(-est, kind="stable")
rank = np.empty_like(order)
rank[order] = np.arange(len(order))
res = {"main_ms": st["main_ms"], "keys_outgrowing": int(len(bad)), "codes": sorted(set(int(c) for c in code[bad]))}
tot = est.sum()
for pct in (2, 5, 10, 15, 20, 30):
    top = int(len(n) * pct / 100)
    res[f"top{pct}"] = {"outgrowing_share": float((rank[bad] < top).mean()) if len(bad) else 0.0,
                        "work_share": float(est[order[:top]].sum() / tot)}
print(json.dumps(res))
