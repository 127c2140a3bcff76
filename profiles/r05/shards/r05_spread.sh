#!/bin/bash
# Round 5: the world-8 shards (each alone) with their spread launch over more waves than the
# chip holds at once ($CEP_SPREAD_WAVES, measurement build): fewer keys per wave.
# usage: bash profiles/r05/scripts/r05_spread.sh <outdir> [waves ...]
OUT=${1:-gpurun_out/r05_spread}; shift
mkdir -p $OUT
for W in ${@:-0 6144 12288 24576}; do
  CEP_MEASURE=1 CEP_SPREAD_WAVES=$W timeout -k 10 300 python -u profiles/workload.py shards --world 8 --steps 3 > $OUT/w$W.json 2> $OUT/w$W.log || exit 1
done
echo done > $OUT/DONE
