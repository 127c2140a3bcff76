"""NFA cost ablation on the bench workload (cfg 3: 1e6 keys x ~1000 events, in HBM).

Times cep_nfa_jit for stock-query variants that switch parts of the per-event work off:
  readme      the bench query (begins, takes, dips -> branch walks + match walks)
  no_dip      dip predicate never true: no branch, no match walk (takes/ignores only)
  no_begin    begin predicate never true: every lane stays in the quiet scan
The differences price the walks and the per-run step.  Usage (GPU box, repo root):
    python profiles/nfa_ablation.py [--keys N] [--precompile]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cepamd  # noqa: E402,F401
from kafkastreams_cep_amd import native as N  # noqa: E402
from kafkastreams_cep_amd import workloads as W  # noqa: E402

VARIANTS = {
    "readme": dict(),
    "no_dip": dict(dip_num=0),
    "no_begin": dict(begin_volume=10**9),
}


def _test_variant(take):
    """zeroOrMore ("test") stock query without dips; `take` = the Kleene stage's predicate"""
    from kafkastreams_cep_amd import QueryBuilder
    S = W.stock_query("test").schema
    return (QueryBuilder(S).select().where(lambda k, v, ts, s: v.volume > 1000).fold("avg", lambda k, v, c: v.price)
            .then().select().zeroOrMore().skipTillNextMatch().where(take)
            .fold("avg", lambda k, v, c: (c + v.price) / 2).fold("volume", lambda k, v, c: v.volume).then()
            .select().skipTillNextMatch().where(lambda k, v, ts, s: v.volume < 0 * s.getOrElse("volume", 0))
            .build())


def queries():
    qs = {k: W.stock_query("readme", **kw).to_ir() for k, kw in VARIANTS.items()}
    qs["test_nodip"] = _test_variant(lambda k, v, ts, s: v.price > s.get("avg")).to_ir()
    qs["test_notake"] = _test_variant(lambda k, v, ts, s: v.price > s.get("avg") + 1000000).to_ir()
    return qs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--precompile", action="store_true")
    ap.add_argument("--only", default=None, help="comma-separated variant names")
    args = ap.parse_args()
    if args.precompile:
        for ir in queries().values():
            N.Query(ir).precompile()
        return
    cfg = W.CONFIGS[3]
    stream = N.synth_stream("stock", cfg.seed, args.keys, cfg.mean_events)
    res = {}
    for name, ir in queries().items():
        if args.only and name not in args.only.split(","):
            continue
        s = N.Session(N.Query(ir))
        s.push_device(stream)
        ks = []
        for _ in range(args.steps):
            s.push_device(stream)
            ks.append(s.timing(0)[0])
        n, _ = s.digest(0)
        res[name] = {"kernel_ms": min(ks), "matches": n, "launches": s.timing(0)[2]}
        print(name, res[name], flush=True)
        s.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
