#!/bin/bash
# Round-3 evidence for the bench line (run on the GPU box from the repo root):
#   1. rocprofv3 --kernel-trace --stats over bench.py's cfg-3 + cfg-2 figures (the kernel
#      table the line's roofline must agree with)
#   2. separate FETCH_SIZE / WRITE_SIZE passes per workload (profiles/workload.py) -> traffic
#   3. SQ instruction / cycle counters for cfg 3
# usage: bash profiles/r03/scripts/r03_final.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r03_final}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 5 --no-cpu-baseline --no-other --no-ingest --no-e2e --no-projection --no-streaming > $OUT/trace_bench.json 2> $OUT/trace_bench.log || exit $?
for M in cfg3 cfg4 cfg4s cfg4sem "cfg5 --keys 125000 --steps 1"; do
  N=$(echo $M | cut -d' ' -f1)
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C -d $OUT/pmc_${N}_$C -o run --output-format csv -- python3 profiles/workload.py $M > $OUT/pmc_${N}_$C.log 2>&1 || exit $?
  done
done
I=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES"; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/sq_cfg3_$I -o run --output-format csv -- python3 profiles/workload.py cfg3 > $OUT/sq_cfg3_$I.log 2>&1 || exit $?
  I=$((I+1))
done
echo done > $OUT/DONE
