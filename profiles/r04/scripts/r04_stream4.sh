#!/bin/bash
# Round-4 streaming: the GPU suite, then the streamed cfg 3 (10 slices) with the lane order
# blended across batches (KeyCarry.west, the default) and from each batch alone
# ($CEP_NO_EST_BLEND=1), then the bench's headline + streaming figures.
# usage: bash profiles/r04/scripts/r04_stream4.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_stream4}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
timeout -k 10 120 python3 profiles/stream_probe.py > $OUT/s10_blend.json 2> $OUT/s10_blend.log || exit $?
CEP_NO_EST_BLEND=1 timeout -k 10 120 python3 profiles/stream_probe.py > $OUT/s10_noblend.json 2> $OUT/s10_noblend.log || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-other --no-ingest --no-e2e --no-secondary --no-projection > $OUT/bench.json 2> $OUT/bench.log || exit $?
echo done > $OUT/DONE
