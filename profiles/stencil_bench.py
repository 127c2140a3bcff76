"""Config 2 (strict SEQ(A,B,C), 1e8 events / 1e4 keys, in HBM): the stencil passes alone, for
rocprofv3 kernel traces.  Pushes queue on the session stream (no host sync per batch); the
step time is the wall clock over all of them, the kernel time the HIP events of every batch.
Usage (GPU box, repo root): python profiles/stencil_bench.py [--steps K]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cepamd  # noqa: E402,F401
from kafkastreams_cep_amd import native as N  # noqa: E402
from kafkastreams_cep_amd import workloads as W  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=200)
args = ap.parse_args()
cfg = W.CONFIGS[2]
stream = N.synth_stream("abc", cfg.seed, cfg.n_keys, cfg.mean_events)
s = N.Session(N.Query(W.strict_abc_query().to_ir()))
for _ in range(5):
    s.push_device(stream)
s.timing_totals(0, reset=True)
t0 = time.perf_counter()
for _ in range(args.steps):
    s.push_device(stream)
N.lib().cep_sync(s.h)
el = time.perf_counter() - t0
kern, aux, n = s.timing_totals(0)
alg = 4.0 * stream.n_events + 16.0 * s.digest(0)[0]
print(f"stencil steps {n} ms/step {1e3 * el / n:.4f} kernel_ms {kern / n:.4f} setup_ms {aux / n:.4f} "
      f"kernel frac {alg / (kern / n * 1e-3) / 8e12:.3f} step frac {alg / (el / n) / 8e12:.3f} "
      f"matches {s.digest(0)[0]}")
