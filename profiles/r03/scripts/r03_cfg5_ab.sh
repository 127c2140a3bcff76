#!/bin/bash
# Config 5 A/B of round 3's scheduling changes (batches 0 and 3 of the 64-variant group).
# Measured at c1c66a4, where heavy-first was the default (CEP_NO_HEAVY_FIRST turned it off):
# profiles/r03/cfg5_ab/{default = heavy-first + partial drains, no_heavy_first, no_partial,
# neither}.json.  Since then heavy-first is opt-in ($CEP_HEAVY_FIRST=1); this script runs the
# same four cases under the current knobs.
# usage: bash profiles/r03/scripts/r03_cfg5_ab.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/cfg5_ab}
mkdir -p $OUT
CEP_HEAVY_FIRST=1 timeout -k 10 200 python3 profiles/cfg5_probe.py --only 0,3 > $OUT/default.json 2> $OUT/default.log || exit $?
timeout -k 10 200 python3 profiles/cfg5_probe.py --only 0,3 > $OUT/no_heavy_first.json 2> $OUT/no_heavy_first.log || exit $?
CEP_HEAVY_FIRST=1 CEP_PARTIAL_DRAIN=0 timeout -k 10 300 python3 profiles/cfg5_probe.py --only 0,3 > $OUT/no_partial.json 2> $OUT/no_partial.log || exit $?
CEP_PARTIAL_DRAIN=0 timeout -k 10 200 python3 profiles/cfg5_probe.py --only 0,3 > $OUT/neither.json 2> $OUT/neither.log || exit $?
