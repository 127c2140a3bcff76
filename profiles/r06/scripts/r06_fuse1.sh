#!/bin/bash
# Round 6: fused walks forced on for single-query builds ($CEP_JIT_OPTS=-DCEP_WALK_FUSE=1,
# measurement build) against the default, on the headline and the config 4 stress query.
# usage: bash profiles/r06/scripts/r06_fuse1.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r06_fuse1}
mkdir -p $OUT
export TMPDIR=/tmp
for Q in readme anys; do
  CEP_MEASURE=1 timeout -k 10 300 python -u profiles/nfa_env_sweep.py --query $Q --steps 3 --variants "default=" > $OUT/${Q}_default.txt 2>&1 || exit $?
  CEP_MEASURE=1 CEP_JIT_OPTS=-DCEP_WALK_FUSE=1 timeout -k 10 300 python -u profiles/nfa_env_sweep.py --query $Q --steps 3 --variants "fused=" > $OUT/${Q}_fused.txt 2>&1 || exit $?
done
echo done > $OUT/DONE
