#!/bin/bash
# Round-4: rocprofv3 kernel table of the arrival-order partition (e2e probe, 1e9 events).
# usage: bash profiles/r04/scripts/r04_parttrace.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_parttrace}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 profiles/e2e_probe.py --steps 3 > $OUT/e2e.json 2> $OUT/e2e.log || exit $?
echo done > $OUT/DONE
