#!/bin/bash
# Round-4: the partition with 4-tile, 16-B-load histograms - arrival-order parity tests, the
# e2e probe and its rocprofv3 kernel table.
# usage: bash profiles/r04/scripts/r04_hist.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_hist}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "arrival or partition or order or cfg3" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 profiles/e2e_probe.py > $OUT/e2e.json 2> $OUT/e2e.log || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 profiles/e2e_probe.py --steps 3 > $OUT/e2e_trace.json 2> $OUT/e2e_trace.log || exit $?
echo done > $OUT/DONE
