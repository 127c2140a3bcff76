"""NFA kernel variants on the bench workload (cfg 3 stream in HBM), selected by the JIT
generator's measurement knobs ($CEP_RING_LDS, $CEP_JIT_WAVES, $CEP_WALK_FLUSH, ...), each a
separately generated kernel.  Prints kernel ms and the checksum per variant (the checksums
must agree).  --precompile fills the JIT cache for every variant (no GPU needed).
    python profiles/nfa_env_sweep.py [--keys N] [--variants name=K:V,K:V;...] [--precompile]
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

KNOBS = ("CEP_RING_LDS", "CEP_JIT_WAVES", "CEP_WALK_FLUSH", "CEP_QUIET_CHUNK", "CEP_JOB_DRAIN", "CEP_NO_PERSIST",
         "CEP_DEWEY_PAIRS", "CEP_RING_LDS_SLOTS", "CEP_STREAM_PAIRS",
         "CEP_STREAM_LAYOUT", "CEP_STREAM_PUTLOG", "CEP_PARTIAL_DRAIN",
         # (session knobs, read at session creation)
         "CEP_NODE_CHUNK", "CEP_OUT_CHUNK", "CEP_WALK_CAP", "CEP_RESIDENT_WAVES")
SESSION_KNOBS = ("CEP_NODE_CHUNK", "CEP_OUT_CHUNK", "CEP_WALK_CAP", "CEP_RESIDENT_WAVES")
DEFAULT = "default=;nolds=CEP_RING_LDS:0;w2=CEP_JIT_WAVES:2"


def parse(spec):
    out = []
    for item in spec.split(";"):
        name, _, kv = item.partition("=")
        env = dict(x.split(":") for x in kv.split(",") if x)
        out.append((name, env))
    return out


def query(name, env, variant):
    for k in KNOBS:
        os.environ.pop(k, None)
    os.environ.update(env)
    if variant.startswith("mq"):  # one of config 5's variants, e.g. mq63
        ir = W.multi_queries(64)[int(variant[2:])].to_ir()
    else:
        ir = (W.any_kleene_query().to_ir() if variant == "any" else
              W.any_kleene_query(carry_volume=True).to_ir() if variant == "anys" else W.stock_query(variant).to_ir())
    q = N.Query(ir)
    for k in KNOBS:
        # (CEP_STREAM_*: read again when a streaming session builds its kernel; the session
        # knobs when the session is created - main() drops them after the variant's run)
        if not k.startswith("CEP_STREAM_") and k not in SESSION_KNOBS:
            os.environ.pop(k, None)
    return q


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--query", default="readme")
    ap.add_argument("--variants", default=DEFAULT)
    ap.add_argument("--precompile", action="store_true")
    ap.add_argument("--stream", action="store_true",
                    help="one push of the whole batch into a fresh streaming session per step (stream build)")
    args = ap.parse_args()
    vs = parse(args.variants)
    if args.precompile:
        for name, env in vs:
            print(name, query(name, env, args.query).precompile())
            for k in KNOBS:
                os.environ.pop(k, None)
        return
    cfg = W.CONFIGS[3]
    stream = N.synth_stream("stock", cfg.seed, args.keys, cfg.mean_events)
    res = {}
    for name, env in vs:
        qq = query(name, env, args.query)
        if "CEP_NO_PERSIST" in env:  # read by the session at each batch
            os.environ["CEP_NO_PERSIST"] = env["CEP_NO_PERSIST"]
        ks = []
        if args.stream:  # a stream carries its keys' runs: a fresh session per step
            for _ in range(args.steps + 1):
                s = N.Session(qq, streaming=True)
                s.push_device(stream)
                ks.append(s.timing(0)[0])
                if _ < args.steps:
                    s.close()
            ks = ks[1:]
        else:
            s = N.Session(qq)
            s.push_device(stream)
            for _ in range(args.steps):
                s.push_device(stream)
                ks.append(s.timing(0)[0])
        n, d = s.digest(0)
        code, _ = s.key_errors(0)
        os.environ.pop("CEP_NO_PERSIST", None)
        for k in KNOBS:
            os.environ.pop(k, None)
        res[name] = {"kernel_ms": min(ks), "all_ms": ks, "matches": n, "checksum": f"{d:016x}",
                     "key_errors": int((code != 0).sum()), "launches": s.timing(0)[2], "stats": s.stats(0)}
        print(name, json.dumps(res[name]), flush=True)
        s.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
