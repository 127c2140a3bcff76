#!/bin/bash
# Round-4 quick GPU check: the GPU suite, a short bench (cfg 3 + cfg 2), the rocprofv3 kernel
# table of the same bench, and the lane-order probe.  usage: bash profiles/r04/scripts/r04_quick.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_quick}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-other --no-ingest --no-e2e --no-streaming > $OUT/bench.json 2> $OUT/bench.log || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-other --no-ingest --no-e2e --no-projection --no-streaming > $OUT/trace_bench.json 2> $OUT/trace_bench.log || exit $?
bash profiles/r04/scripts/r04_order.sh $OUT/order || exit $?
echo done > $OUT/DONE
