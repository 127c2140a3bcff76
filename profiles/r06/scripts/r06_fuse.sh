#!/bin/bash
# Round 6, fused branch + extraction walks (kernel groups): the GPU suite, config 5 alone (one
# batch of 125k keys x 64 queries), the bench as the driver runs it, its kernel trace, and
# config 5's FETCH_SIZE / WRITE_SIZE passes.
# usage: bash profiles/r06/scripts/r06_fuse.sh <outdir> [parts: tests cfg5 bench trace pmc]
set -o pipefail
OUT=${1:-gpurun_out/r06_fuse}; shift
PARTS=${@:-tests cfg5 bench trace pmc}
mkdir -p $OUT
export TMPDIR=/tmp
for P in $PARTS; do
  case $P in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
      ;;
    cfg5)
      timeout -k 10 300 python -u profiles/workload.py cfg5 --keys 125000 --steps 2 > $OUT/cfg5.json 2> $OUT/cfg5.log || exit $?
      ;;
    bench)
      timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.log || exit $?
      ;;
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 5 --no-cpu-baseline --no-other --no-ingest --no-e2e --no-projection --no-streaming > $OUT/trace_bench.json 2> $OUT/trace_bench.log || exit $?
      ;;
    pmc)
      for C in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 300 rocprofv3 --pmc $C -d $OUT/pmc_cfg5_$C -o run --output-format csv -- python3 profiles/workload.py cfg5 --keys 125000 --steps 1 > $OUT/pmc_cfg5_$C.log 2>&1 || exit $?
      done
      ;;
  esac
done
echo done > $OUT/DONE
