#!/bin/bash
# Round-4 probe: compiler options for the generated NFA kernel ($CEP_JIT_OPTS, part of the JIT
# cache key; the variants are precompiled in-tree) on cfg 3.
# usage: bash profiles/r04/scripts/r04_jitopts.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_jitopts}
mkdir -p $OUT
export TMPDIR=/tmp
I=0
for O in "" "-mllvm -amdgpu-sched-strategy=max-ilp" "-mllvm -amdgpu-sched-strategy=max-memory-clause" "-mllvm -amdgpu-sched-strategy=iterative-ilp" "-O2" "-mllvm -amdgpu-early-ifcvt=1"; do
  CEP_JIT_OPTS="$O" timeout -k 10 300 python3 profiles/workload.py cfg3 --steps 3 > $OUT/opt$I.json 2> $OUT/opt$I.log || exit $?
  echo "$I $O" >> $OUT/index.txt
  I=$((I+1))
done
echo done > $OUT/DONE
