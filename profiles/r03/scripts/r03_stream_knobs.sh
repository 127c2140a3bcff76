#!/bin/bash
# Streaming cfg 3 (10 slices, 1M keys) under the measurement knobs of session.cpp: the default
# (wide build, lane order), without the lane order (rings coalesced by key position), on the
# narrow build, and both.  usage: bash profiles/r03/scripts/r03_stream_knobs.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/stream_knobs}
mkdir -p $OUT
timeout -k 10 120 python3 profiles/stream_probe.py > $OUT/default.json 2> $OUT/default.log || exit $?
CEP_STREAM_NO_ORDER=1 timeout -k 10 120 python3 profiles/stream_probe.py > $OUT/no_order.json 2> $OUT/no_order.log || exit $?
CEP_STREAM_NARROW=1 timeout -k 10 120 python3 profiles/stream_probe.py > $OUT/narrow.json 2> $OUT/narrow.log || exit $?
CEP_STREAM_NARROW=1 CEP_STREAM_NO_ORDER=1 timeout -k 10 120 python3 profiles/stream_probe.py > $OUT/narrow_no_order.json 2> $OUT/narrow_no_order.log || exit $?
