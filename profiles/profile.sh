#!/bin/bash
# Collects the rocprofv3 evidence for bench.py's kernels (run on the GPU box from the repo root):
#   1. --kernel-trace --stats  (per-kernel durations; must agree with bench.py's HIP events)
#   2. separate --pmc passes    (FETCH_SIZE, WRITE_SIZE, SQ counters), never combined with tracing
# usage: bash profiles/profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
ARGS=${@:---keys 200000 --steps 2 --warmup 1 --no-cpu-baseline}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit $?
for C in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  N=$(echo $C | tr ' ' '_')
  timeout -k 10 600 rocprofv3 --pmc $C -d $OUT/pmc_$N -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_$N.log 2>&1 || exit $?
done
echo done > $OUT/DONE
