#!/bin/bash
# Round-4 probe: config 5's batches 0 and 3 with the CEP_PROF time split (nfa_lane.h): is a
# 64-query batch launch bound by its tail (the max wave lifetime) or by its total work?
# usage: bash profiles/r04/scripts/r04_cfg5prof.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_cfg5prof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 profiles/cfg5_probe.py --only 0,3 > $OUT/base.json 2> $OUT/base.log || exit $?
CEP_PROF=1 timeout -k 10 600 python3 profiles/cfg5_probe.py --only 0,3 > $OUT/prof.json 2> $OUT/prof.log || exit $?
echo done > $OUT/DONE
