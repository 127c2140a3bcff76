#!/bin/bash
# Round-4 probe: stencil_mask's prefetch depth ($CEP_STENCIL_PF = 1, 2, 4 steps of 256 events in
# flight per wave) on cfg 2, under rocprofv3's kernel table.
# usage: bash profiles/r04/scripts/r04_stpf.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_stpf}
mkdir -p $OUT
export TMPDIR=/tmp
for PF in 1 2 4; do
  CEP_STENCIL_PF=$PF timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/pf$PF -o run --output-format csv -- python3 profiles/stencil_bench.py --steps 50 > $OUT/pf$PF.json 2> $OUT/pf$PF.log || exit $?
done
echo done > $OUT/DONE
