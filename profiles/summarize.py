"""Summarise a profiles/profile.sh run: per-kernel mean duration (kernel trace) and mean PMC
values per dispatch, plus HBM traffic per launch with the gfx950 corrections of
MI355X_MICROARCH.md §HBM (FETCH_SIZE counts half the bytes of wide coalesced reads -> x2 as an
upper bound, see notes; sizes are KiB)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "").replace("cep::", "")


def main(d, out_json=None):
    stats = {}
    with open(os.path.join(d, "trace", "run_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            stats[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
    pmc = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(d, "pmc_*", "run_counter_collection.csv")):
        with open(path) as f:
            for r in csv.DictReader(f):
                pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, s in sorted(stats.items(), key=lambda kv: -kv[1]["avg_us"] * kv[1]["calls"]):
        row = dict(s)
        for c, v in pmc.get(k, {}).items():
            row[c] = sum(v) / len(v)
        if "FETCH_SIZE" in row:
            row["fetch_bytes"] = row["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in row:
            row["write_bytes"] = row["WRITE_SIZE"] * 1024
        res[k] = row
    for k, row in res.items():
        print(k, json.dumps({a: (round(b, 3) if isinstance(b, float) else b) for a, b in row.items()}))
    if out_json:
        with open(out_json, "w") as f:
            json.dump(res, f, indent=1)
    return res


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
