"""Walk hops by kind on the CPU lane build (tests/lane_cpu.py, the generated kernels run lane by
lane): branch hops, extraction hops, extraction hops that retrace a branch walk of the same key
and event (same node, same walker version), remove-only hops.  Config 5's 64 queries as the
kernel groups a session launches, and config 3's README query, on a sample of the stream's keys
(the full-size generator restricted to `--keys` keys spread over the key range).
    python profiles/r06/scripts/hop_retrace.py [--keys 256]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import cepamd  # noqa: E402,F401
import lane_cpu  # noqa: E402
from kafkastreams_cep_amd import native as N  # noqa: E402
from kafkastreams_cep_amd import workloads as W  # noqa: E402

HOPS = ("hops_branch", "hops_emit", "hops_emit_retrace", "hops_remove")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=256)
    args = ap.parse_args()
    cfg = W.CONFIGS[5]
    keys = np.linspace(0, cfg.n_keys - 1, args.keys).astype(np.int64)
    off, cols = W.generate(cfg, keys)
    out = {"keys": args.keys, "events": int(off[-1])}
    m = lane_cpu.run(W.stock_query("readme").to_ir(), off, cols)
    out["cfg3_readme"] = {k: m["stats"][k] for k in HOPS + ("walks", "walk_nodes")}
    out["cfg3_readme"]["matches"] = m["n_matches"]
    irs = [p.to_ir() for p in W.multi_queries(64)]
    tot = dict.fromkeys(HOPS, 0)
    matches = 0
    for g in N.group_plans([N.Query(ir) for ir in irs]):
        r = lane_cpu.run(irs[g["members"][0]], off, cols, _group=g)
        for k in HOPS:
            tot[k] += r["stats"][k]
        matches += r["n_matches"]
    out["cfg5_64_queries"] = dict(tot, matches=matches)
    for k in ("cfg3_readme", "cfg5_64_queries"):
        d = out[k]
        d["retrace_of_emit"] = d["hops_emit_retrace"] / max(1, d["hops_emit"])
        d["retrace_of_all"] = d["hops_emit_retrace"] / max(1, sum(d[h] for h in HOPS if h != "hops_emit_retrace"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
