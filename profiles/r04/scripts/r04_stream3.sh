#!/bin/bash
# Round-4 streaming probe: the CEP_PROF time split (nfa_lane.h) of the stream build's launches,
# cfg 3 in 10 slices and in 1 (stderr: one cep_prof line per launch).
# usage: bash profiles/r04/scripts/r04_stream3.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_stream3}
mkdir -p $OUT
export TMPDIR=/tmp
CEP_PROF=1 timeout -k 10 300 python3 profiles/stream_probe.py > $OUT/p10.json 2> $OUT/p10.log || exit $?
CEP_PROF=1 timeout -k 10 300 python3 profiles/stream_probe.py --slices 1 > $OUT/p1.json 2> $OUT/p1.log || exit $?
echo done > $OUT/DONE
