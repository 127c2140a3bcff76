"""HBM bytes per launch for bench.py's `roofline.traffic`, from a profiles/summarize.py
summary (rocprofv3 FETCH_SIZE / WRITE_SIZE passes, KiB per dispatch).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts half the bytes of wide
coalesced streaming reads -> x2 for the stencil passes (calibrated there: stencil_mask's
corrected fetch equals its 400 MB column + 12.5 MB bitmap).  The NFA kernel's reads are
per-lane scattered; the guide leaves such widths uncalibrated, so its FETCH_SIZE is taken
as is (a lower bound).  WRITE_SIZE is exact for 16-B stores and taken as is.

The JSON decoder stages its byte span with 16-B coalesced loads: FETCH_SIZE x 2 as for the
stencil.

usage: python profiles/traffic.py summary.json [more summaries...] > profiles/pmc_traffic.json
(a kernel is taken from the first summary that has it)
"""
import json
import sys

STENCIL = ("stencil_mask", "stencil_scan", "stencil_emit")


def main(paths):
    out = {"_source": " ".join(paths), "_unit": "bytes per launch (HBM, rocprofv3 PMC)"}
    for path in paths:
        s = json.load(open(path))
        for name, row in s.items():
            if name.startswith("cep_nfa_jit") and "FETCH_SIZE" in row and "cep_nfa_jit" not in out:
                out["cep_nfa_jit"] = row["FETCH_SIZE"] * 1024 + row["WRITE_SIZE"] * 1024
            if name == "decode_stock_json_kernel" and "FETCH_SIZE" in row and name not in out:
                out[name] = 2 * row["FETCH_SIZE"] * 1024 + row["WRITE_SIZE"] * 1024
        st = [row for name, row in s.items() if name.startswith(STENCIL) and "FETCH_SIZE" in row]
        if st and "stencil" not in out:
            out["stencil"] = sum(2 * r["FETCH_SIZE"] * 1024 + r["WRITE_SIZE"] * 1024 for r in st)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
