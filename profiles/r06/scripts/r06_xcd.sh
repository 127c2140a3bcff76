#!/bin/bash
# Round 6, XCD-aware tile order of the partition's scatter passes: the GPU suite, the per-push
# partition time with and without it (measurement build, $CEP_PART_NO_XCD), the bench's
# arrival-order end-to-end figure and its kernel trace.
# usage: bash profiles/r06/scripts/r06_xcd.sh <outdir> [parts: tests ab bench trace]
set -o pipefail
OUT=${1:-gpurun_out/r06_xcd}; shift
PARTS=${@:-tests ab bench trace}
mkdir -p $OUT
export TMPDIR=/tmp
for P in $PARTS; do
  case $P in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
      ;;
    ab)
      for V in xcd noxcd xcd noxcd; do
        if [ $V = noxcd ]; then export CEP_PART_NO_XCD=1; else unset CEP_PART_NO_XCD; fi
        CEP_MEASURE=1 timeout -k 10 300 python -u profiles/e2e_probe.py --steps 4 > $OUT/ab_$V.jsonl 2>> $OUT/ab.log || exit $?
        cat $OUT/ab_$V.jsonl >> $OUT/ab_all_$V.jsonl
      done
      unset CEP_PART_NO_XCD
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
