#!/bin/bash
# Round 5: config 2's stencil passes.
#   1. the stencil GPU tests (parity vs the oracle, key boundaries, pipelined pushes)
#   2. the stencil probe (profiles/micro/stencil_probe: read floor, mask / emit passes alone)
#   3. bench config 2 (50 steps), twice; rocprofv3 kernel table of the same
# usage: bash profiles/r05/scripts/r05_stencil.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r05_stencil}
mkdir -p $OUT
export TMPDIR=/tmp
B="--steps 50 --warmup 5 --no-cpu-baseline --no-other --no-ingest --no-e2e --no-streaming --no-projection"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "stencil or strict or cfg2" > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 120 ./profiles/micro/stencil_probe > $OUT/probe.txt 2>&1 || exit $?
timeout -k 10 200 python -u bench.py $B > $OUT/bench.json 2> $OUT/bench.log || exit $?
timeout -k 10 200 python -u bench.py $B > $OUT/bench2.json 2> $OUT/bench2.log || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $B > $OUT/trace_bench.json 2> $OUT/trace_bench.log || exit $?
echo done > $OUT/DONE
