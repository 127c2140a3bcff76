#!/bin/bash
# Round-4 probe: a stream's heaviest keys alone in their waves ($CEP_STREAM_ISO=K, lane order for
# the rest) on the streamed cfg 3 (10 batches; each lasts as long as its heaviest wave).
# usage: bash profiles/r04/scripts/r04_streamiso.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_streamiso}
mkdir -p $OUT
export TMPDIR=/tmp
for K in 0 64 256 1024 4096; do
  CEP_STREAM_ISO=$K timeout -k 10 120 python3 profiles/stream_probe.py > $OUT/iso$K.json 2> $OUT/iso$K.log || exit $?
done
echo done > $OUT/DONE
