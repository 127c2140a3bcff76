#!/bin/bash
# Round-4: HBM traffic of the partition kernels (FETCH_SIZE / WRITE_SIZE passes over the e2e
# probe, 1e9 arrival-order events; traffic = 2 x FETCH + WRITE per the gfx950 correction).
# usage: bash profiles/r04/scripts/r04_partpmc.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_partpmc}
mkdir -p $OUT
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C -d $OUT/pmc_$C -o run --output-format csv -- python3 profiles/e2e_probe.py --steps 2 > $OUT/pmc_$C.log 2>&1 || exit $?
done
echo done > $OUT/DONE
