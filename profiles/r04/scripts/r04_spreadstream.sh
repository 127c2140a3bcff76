#!/bin/bash
# Round-4 probe: a streamed batch spread over all its waves ($CEP_SPREAD_STREAM=1: every wave led
# by one of the heaviest keys, lighter ones beside it) against the lane order.
# (the knob was removed after this measurement: DESIGN.md §7, round 4)
# usage: bash profiles/r04/scripts/r04_spreadstream.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_spreadstream}
mkdir -p $OUT
export TMPDIR=/tmp
CEP_SPREAD_STREAM=1 timeout -k 10 120 python3 profiles/stream_probe.py > $OUT/s10_spread.json 2> $OUT/s10_spread.log || exit $?
CEP_SPREAD_STREAM=1 timeout -k 10 120 python3 profiles/stream_probe.py --slices 1 > $OUT/s1_spread.json 2> $OUT/s1_spread.log || exit $?
echo done > $OUT/DONE
