#!/bin/bash
# Round 6: what 2 Dewey pairs in registers buy now that the narrow build no longer spills -
# the main launch with 3 (default) and 2 pairs (measurement build, $CEP_DEWEY_PAIRS; its keys
# that outgrow 2 pairs re-run), and the SQ instruction counts of both on the headline batch.
# usage: bash profiles/r06/scripts/r06_p2.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r06_p2}
mkdir -p $OUT
export TMPDIR=/tmp
CEP_MEASURE=1 timeout -k 10 300 python -u profiles/nfa_env_sweep.py --variants "default=;p2=CEP_DEWEY_PAIRS:2" > $OUT/sweep.txt 2>&1 || exit $?
for V in 3 2; do
  I=0
  for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES"; do
    CEP_MEASURE=1 CEP_DEWEY_PAIRS=$V CEP_NO_RETRY=1 timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/sq_p${V}_$I -o run --output-format csv -- python3 profiles/workload.py cfg3 --steps 1 > $OUT/sq_p${V}_$I.log 2>&1 || exit $?
    I=$((I+1))
  done
done
echo done > $OUT/DONE
