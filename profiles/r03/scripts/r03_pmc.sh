#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over one command: usage
#   bash profiles/r03/scripts/r03_pmc.sh <outdir> <python args...>
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
I=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES" FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_$I -o run --output-format csv -- python3 "$@" > $OUT/pmc_$I.log 2>&1 || exit $?
  I=$((I+1))
done
echo done > $OUT/DONE
