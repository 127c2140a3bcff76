#!/bin/bash
# Round-4: the begin-hit bitmap with its timestamp loads issued before the predicate's - GPU
# suite, bench, rocprofv3 kernel table of the bench's cfg-3 + cfg-2 figures.
# usage: bash profiles/r04/scripts/r04_bits.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_bits}
bash profiles/r04/scripts/r04_final.sh $OUT tests bench trace || exit $?
echo done > $OUT/DONE2
