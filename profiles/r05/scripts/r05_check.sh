#!/bin/bash
# Round 5 check of a build: the GPU suite, the stencil probe, a short bench (cfg 3, cfg 2,
# projection, streaming, end to end) and the rocprofv3 kernel table of the cfg-3 + cfg-2 part.
# usage: bash profiles/r05/scripts/r05_check.sh <outdir> [notests]
set -o pipefail
OUT=${1:-gpurun_out/r05_check}
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "notests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
fi
timeout -k 10 120 ./profiles/micro/stencil_probe > $OUT/probe.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-other --no-ingest > $OUT/bench.json 2> $OUT/bench.log || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-other --no-ingest --no-e2e --no-projection --no-streaming > $OUT/trace_bench.json 2> $OUT/trace_bench.log || exit $?
echo done > $OUT/DONE
