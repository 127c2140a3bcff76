#!/bin/bash
# Round-4: $CEP_STREAM_ISO around its optimum, each K twice (run-to-run spread), streamed cfg 3.
# usage: bash profiles/r04/scripts/r04_streamiso3.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_streamiso3}
mkdir -p $OUT
export TMPDIR=/tmp
for R in a b; do
  for K in 1024 1536 2048 3072; do
    CEP_STREAM_ISO=$K timeout -k 10 120 python3 profiles/stream_probe.py > $OUT/iso$K$R.json 2> $OUT/iso$K$R.log || exit $?
  done
done
echo done > $OUT/DONE
