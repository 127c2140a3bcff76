"""HBM bytes per launch for bench.py's `roofline.traffic`, from rocprofv3 FETCH_SIZE and
WRITE_SIZE passes (separate runs, KiB per dispatch in run_counter_collection.csv).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of a wide
coalesced streaming read, so every kernel's fetch is doubled - applied to all kernels alike
(the NFA's reads are mostly per-lane 16-B quads; for narrower or scattered reads the doubled
figure is an upper bound).  WRITE_SIZE is taken as is (exact for 16-B stores).

Per kernel the median over its dispatches is taken (the first push of a session may run a
smaller or a re-run launch); a key may sum several kernels (a whole step).

usage: python profiles/traffic.py OUT.json KEY:FETCH_DIR:WRITE_DIR:KERNEL[+KERNEL...][/PUSHES] ...
  e.g. cep_nfa_jit_cfg4s:profiles/r03/pmc_cfg4s_FETCH_SIZE:profiles/r03/pmc_cfg4s_WRITE_SIZE:cep_nfa_jit
An existing OUT.json keeps its other keys.
"""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict


def per_kernel(d, pushes=0):
    """median bytes per dispatch of each kernel; pushes > 0: the sum over its dispatches / pushes
    (a push whose main launch is followed by re-run launches)"""
    acc = defaultdict(list)
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            acc[r["Kernel_Name"].split("(")[0].replace("cep::", "")].append(float(r["Counter_Value"]) * 1024)
    return {k: (sum(v) / pushes if pushes else statistics.median(v)) for k, v in acc.items()}


def main(out, specs):
    res = json.load(open(out)) if os.path.exists(out) else {}
    res["_unit"] = "bytes per launch (HBM, rocprofv3 PMC): traffic = 2 x FETCH_SIZE + WRITE_SIZE (gfx950 correction)"
    for spec in specs:
        key, fd, wd, kernels = spec.split(":")
        kernels, _, pushes = kernels.partition("/")
        fetch, write = per_kernel(fd, int(pushes or 0)), per_kernel(wd, int(pushes or 0))
        ks = kernels.split("+")
        f = sum(fetch[k] for k in ks)
        w = sum(write[k] for k in ks)
        res[key] = 2 * f + w
        res["_" + key] = {"kernels": ks, "fetch_raw": f, "write": w, "source": [fd, wd]}
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
