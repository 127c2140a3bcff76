#!/bin/bash
# Round 6: HBM traffic of the arrival-order push's kernels (the partition after the gather
# change): separate FETCH_SIZE / WRITE_SIZE passes over profiles/workload.py arrival.
# usage: bash profiles/r06/scripts/r06_arrpmc.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r06_arrpmc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 profiles/workload.py arrival --steps 2 > $OUT/arrival.json 2> $OUT/arrival.log || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C -d $OUT/pmc_arrival_$C -o run --output-format csv -- python3 profiles/workload.py arrival --steps 1 > $OUT/pmc_arrival_$C.log 2>&1 || exit $?
done
echo done > $OUT/DONE
