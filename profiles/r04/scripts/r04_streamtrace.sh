#!/bin/bash
# Round-4: rocprofv3 kernel table of the streamed cfg 3 (profiles/stream_probe.py, default
# $CEP_STREAM_ISO): where a batch's time goes besides the matching launch.
# usage: bash profiles/r04/scripts/r04_streamtrace.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_streamtrace}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 profiles/stream_probe.py > $OUT/probe.json 2> $OUT/probe.log || exit $?
echo done > $OUT/DONE
