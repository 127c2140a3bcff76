#!/bin/bash
# Round-4: the GPU suite and the bench with $CEP_STREAM_ISO's default (1024), then K = 512 / 2048
# on the streamed cfg 3 (profiles/stream_probe.py).
# usage: bash profiles/r04/scripts/r04_streamiso2.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_streamiso2}
mkdir -p $OUT
export TMPDIR=/tmp
bash profiles/r04/scripts/r04_final.sh $OUT tests bench || exit $?
for K in 512 2048; do
  CEP_STREAM_ISO=$K timeout -k 10 120 python3 profiles/stream_probe.py > $OUT/iso$K.json 2> $OUT/iso$K.log || exit $?
done
echo done > $OUT/DONE2
