#!/bin/bash
# Round-4: the work estimate with est_lanes() lanes per key - GPU suite, bench, streamed-cfg-3
# kernel table.
# usage: bash profiles/r04/scripts/r04_est.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_est}
mkdir -p $OUT
export TMPDIR=/tmp
bash profiles/r04/scripts/r04_final.sh $OUT tests bench || exit $?
bash profiles/r04/scripts/r04_streamtrace.sh $OUT/st || exit $?
echo done > $OUT/DONE2
