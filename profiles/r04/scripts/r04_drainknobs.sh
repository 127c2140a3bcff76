#!/bin/bash
# Round-4 probe: config 5's batches 0 and 3 under the walk-drain knobs (compile-time, variants
# precompiled in-tree): the drain threshold $CEP_WALK_FLUSH (default 24 queued walks) and
# $CEP_JOB_DRAIN (lanes at a job's end that make the wave drain, default 1).
# usage: bash profiles/r04/scripts/r04_drainknobs.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_drainknobs}
mkdir -p $OUT
export TMPDIR=/tmp
I=0
for V in "" "CEP_WALK_FLUSH=12" "CEP_WALK_FLUSH=48" "CEP_JOB_DRAIN=4" "CEP_JOB_DRAIN=16"; do
  env $V timeout -k 10 400 python3 profiles/cfg5_probe.py --only 0,3 > $OUT/v$I.json 2> $OUT/v$I.log || exit $?
  echo "$I $V" >> $OUT/index.txt
  I=$((I+1))
done
echo done > $OUT/DONE
