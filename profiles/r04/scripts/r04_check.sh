#!/bin/bash
# Round-4 check of a build: GPU suite, bench (cfg 3 + cfg 2 + projection + streaming + processor),
# the cfg-3 time split ($CEP_PROF) and the lone heavy key.  usage: bash profiles/r04/scripts/r04_check.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_check}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-other --no-ingest --no-e2e > $OUT/bench.json 2> $OUT/bench.log || exit $?
CEP_PROF=1 timeout -k 10 300 python3 profiles/workload.py cfg3 --steps 1 > $OUT/prof_cfg3.json 2> $OUT/prof_cfg3.log || exit $?
timeout -k 10 120 python3 profiles/heavy_alone.py --steps 3 > $OUT/heavy.txt 2>&1 || exit $?
echo done > $OUT/DONE
# config 4 stress (the twin slots' target): timing, then FETCH_SIZE / WRITE_SIZE passes
if [ -n "$CFG4S" ]; then
  timeout -k 10 300 python3 profiles/workload.py cfg4s --steps 3 > $OUT/cfg4s.json 2> $OUT/cfg4s.log || exit $?
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $C -d $OUT/pmc_cfg4s_$C -o run --output-format csv -- python3 profiles/workload.py cfg4s --steps 1 > $OUT/pmc_cfg4s_$C.log 2>&1 || exit $?
  done
  echo done > $OUT/DONE4
fi
