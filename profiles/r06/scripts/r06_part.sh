#!/bin/bash
# Round 6, partition variants (first the onesweep form, then the prefetching gather): the GPU
# suite, the bench with the arrival-order end-to-end figure, and its kernel trace.
# usage: bash profiles/r06/scripts/r06_part.sh <outdir> [parts: tests bench trace]
set -o pipefail
OUT=${1:-gpurun_out/r06_part}; shift
PARTS=${@:-tests bench trace}
mkdir -p $OUT
export TMPDIR=/tmp
for P in $PARTS; do
  case $P in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
      ;;
    bench)
      timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-other --no-ingest --no-streaming > $OUT/bench.json 2> $OUT/bench.log || exit $?
      ;;
    trace)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-other --no-ingest --no-streaming --no-projection > $OUT/trace_bench.json 2> $OUT/trace_bench.log || exit $?
      ;;
  esac
done
echo done > $OUT/DONE
