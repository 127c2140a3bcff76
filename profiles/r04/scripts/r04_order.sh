#!/bin/bash
# Round-4 probe: cfg 3's cep_nfa_jit under the default lane order (sum over begin hits of the
# events after them) and under the span order ($CEP_EST_MODE=1: events after the first begin
# hit), plain and with the $CEP_PROF time split.  Run on the GPU box from the repo root.
# usage: bash profiles/r04/scripts/r04_order.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_order}
mkdir -p $OUT
export TMPDIR=/tmp
for MODE in 0 1; do
  CEP_EST_MODE=$MODE timeout -k 10 300 python3 profiles/workload.py cfg3 --steps 3 > $OUT/cfg3_est$MODE.json 2> $OUT/cfg3_est$MODE.log || exit $?
  CEP_EST_MODE=$MODE CEP_PROF=1 timeout -k 10 300 python3 profiles/workload.py cfg3 --steps 1 > $OUT/prof_est$MODE.json 2> $OUT/prof_est$MODE.log || exit $?
done
echo done > $OUT/DONE
