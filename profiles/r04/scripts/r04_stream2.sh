#!/bin/bash
# Round-4 streaming probe: where the streamed cfg 3 loses against one per-batch launch - the
# stream build with the lane order (rings at key positions: scattered across a wave) and
# without it ($CEP_STREAM_NO_ORDER=1: rings coalesced), in 10 slices and in 1 slice.
# usage: bash profiles/r04/scripts/r04_stream2.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_stream2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python3 profiles/stream_probe.py > $OUT/s10.json 2> $OUT/s10.log || exit $?
CEP_STREAM_NO_ORDER=1 timeout -k 10 120 python3 profiles/stream_probe.py > $OUT/s10_no_order.json 2> $OUT/s10_no_order.log || exit $?
timeout -k 10 120 python3 profiles/stream_probe.py --slices 1 > $OUT/s1.json 2> $OUT/s1.log || exit $?
CEP_STREAM_NO_ORDER=1 timeout -k 10 120 python3 profiles/stream_probe.py --slices 1 > $OUT/s1_no_order.json 2> $OUT/s1_no_order.log || exit $?
echo done > $OUT/DONE
