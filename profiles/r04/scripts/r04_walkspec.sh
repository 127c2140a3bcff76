#!/bin/bash
# Round-4 probe: speculative walk loads (kernel groups; node s - 1 loaded beside node s) on
# config 5's batches 0 and 3, against $CEP_NO_WALK_SPEC=1; then the GPU suite's group tests.
# (the speculation was reverted after this measurement: DESIGN.md §7, round 4)
# usage: bash profiles/r04/scripts/r04_walkspec.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_walkspec}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "cfg5 or group or heavy or solo" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 profiles/cfg5_probe.py --only 0,3 > $OUT/spec.json 2> $OUT/spec.log || exit $?
CEP_NO_WALK_SPEC=1 timeout -k 10 400 python3 profiles/cfg5_probe.py --only 0,3 > $OUT/nospec.json 2> $OUT/nospec.log || exit $?
echo done > $OUT/DONE
