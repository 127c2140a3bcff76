#!/bin/bash
# Round-4 closing evidence for the last build: bench, its rocprofv3 kernel table, PMC traffic
# passes and SQ counters (profiles/r04/scripts/r04_final.sh parts bench trace pmc sq).
# usage: bash profiles/r04/scripts/r04_final5.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_final5}
bash profiles/r04/scripts/r04_final.sh $OUT bench trace pmc sq || exit $?
echo done > $OUT/DONE2
