#!/bin/bash
# Round 5: config 5's time split ($CEP_PROF, measurement build) with the cooperative walk hops
# off (0) and at 2 / 8 walkers, node pool chunks of 64 (default) and 1024 nodes per lane; one
# batch of 125k keys, one timed push.
# usage: bash profiles/r05/scripts/r05_cfg5prof.sh <outdir> [configs "C:NC ..."]
set -o pipefail
OUT=${1:-gpurun_out/r05_cfg5prof}; shift
CONFS=${@:-0:64 2:64 8:64}
mkdir -p $OUT
export TMPDIR=/tmp
for X in $CONFS; do
  C=${X%%:*}; NC=${X##*:}
  CEP_MEASURE=1 CEP_PROF=1 CEP_COOP_WALKERS=$C CEP_NODE_CHUNK=$NC timeout -k 10 300 python -u profiles/workload.py cfg5 --keys 125000 --steps 1 > $OUT/c${C}_n$NC.json 2> $OUT/c${C}_n$NC.log || exit $?
done
echo done > $OUT/DONE
