#!/bin/bash
# Round-4 probe: the arrival-order partition with 8192-event sort tiles ($CEP_PART_ROUNDS=32, 2
# blocks per CU by LDS) against the 4096-event default (4 blocks per CU); the column gather at
# 4 / 8 / 16 positions per thread ($CEP_GATHER_PER); the arrival-order GPU parity tests.
# usage: bash profiles/r04/scripts/r04_part.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_part}
mkdir -p $OUT
export TMPDIR=/tmp
CEP_PART_ROUNDS=32 timeout -k 10 300 python3 profiles/e2e_probe.py > $OUT/part32.json 2> $OUT/part32.log || exit $?
timeout -k 10 300 python3 profiles/e2e_probe.py > $OUT/part16.json 2> $OUT/part16.log || exit $?
CEP_GATHER_PER=4 timeout -k 10 300 python3 profiles/e2e_probe.py > $OUT/gather4.json 2> $OUT/gather4.log || exit $?
CEP_GATHER_PER=16 timeout -k 10 300 python3 profiles/e2e_probe.py > $OUT/gather16.json 2> $OUT/gather16.log || exit $?
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "arrival or partition" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
echo done > $OUT/DONE
