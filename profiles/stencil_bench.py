"""Config 2 (strict SEQ(A,B,C), 1e8 events / 1e4 keys, in HBM): the stencil passes alone, for
rocprofv3 kernel traces.  Usage (GPU box, repo root): python profiles/stencil_bench.py [--steps K]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cepamd  # noqa: E402,F401
from kafkastreams_cep_amd import native as N  # noqa: E402
from kafkastreams_cep_amd import workloads as W  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
args = ap.parse_args()
cfg = W.CONFIGS[2]
stream = N.synth_stream("abc", cfg.seed, cfg.n_keys, cfg.mean_events)
s = N.Session(N.Query(W.strict_abc_query().to_ir()))
ms = []
for _ in range(args.steps):
    s.push_device(stream)
    ms.append(s.timing(0)[0])
print(f"stencil kernel_ms min {min(ms):.4f} mean {sum(ms) / len(ms):.4f} matches {s.digest(0)[0]}")
