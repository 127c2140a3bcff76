#!/bin/bash
# Round-4: the GPU streaming tests, the stream build's stop / wide-continuation case included.
# usage: bash profiles/r04/scripts/r04_widen.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_widen}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "streaming or knobs" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
echo done > $OUT/DONE
