#!/bin/bash
# Round-4 probe: the key-group tiled column gather (default) against the position-order one
# ($CEP_GATHER_PER=8), on cfg 3's arrival order (1e9 events); sort tiles of 3072 / 6144 events
# ($CEP_PART_ROUNDS=12 / 24) against 4096; the arrival-order parity tests.
# usage: bash profiles/r04/scripts/r04_gather.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_gather}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "arrival or partition" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 profiles/e2e_probe.py > $OUT/tr.json 2> $OUT/tr.log || exit $?
CEP_GATHER_PER=8 timeout -k 10 300 python3 profiles/e2e_probe.py > $OUT/pos8.json 2> $OUT/pos8.log || exit $?
CEP_PART_ROUNDS=12 timeout -k 10 300 python3 profiles/e2e_probe.py > $OUT/r12.json 2> $OUT/r12.log || exit $?
CEP_PART_ROUNDS=24 timeout -k 10 300 python3 profiles/e2e_probe.py > $OUT/r24.json 2> $OUT/r24.log || exit $?
echo done > $OUT/DONE
