#!/bin/bash
# Round-4 probe: the headline (per-batch cfg 3) launch with its K heaviest keys alone in their
# waves ($CEP_BATCH_ISO=K), bench headline figure only.
# usage: bash profiles/r04/scripts/r04_batchiso.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_batchiso}
mkdir -p $OUT
export TMPDIR=/tmp
for K in 0 256 2048 8192; do
  CEP_BATCH_ISO=$K timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-other --no-ingest --no-e2e --no-projection --no-streaming > $OUT/iso$K.json 2> $OUT/iso$K.log || exit $?
done
echo done > $OUT/DONE
