#!/bin/bash
# Round-4 probe: config 5's batches 0 and 3 with the heaviest keys' jobs run alone, one per wave,
# beside the persistent launch ($CEP_SOLO_KEYS=T: the T heaviest keys by the lane order).
# usage: bash profiles/r04/scripts/r04_solo.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_solo}
mkdir -p $OUT
export TMPDIR=/tmp
for T in ${SOLO_LIST:-0 8 24 48}; do
  CEP_SOLO_KEYS=$T timeout -k 10 300 python3 profiles/cfg5_probe.py --only 0,3 > $OUT/solo$T.json 2> $OUT/solo$T.log || exit $?
done
echo done > $OUT/DONE
