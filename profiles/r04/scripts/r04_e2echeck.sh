#!/bin/bash
# Round-4 check: the arrival-order end-to-end figure alone (bench.py) and the e2e probe with its
# per-push stats.
# usage: bash profiles/r04/scripts/r04_e2echeck.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_e2echeck}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 profiles/e2e_probe.py --steps 6 > $OUT/probe.json 2> $OUT/probe.log || exit $?
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-other --no-ingest --no-projection --no-streaming --no-secondary > $OUT/bench.json 2> $OUT/bench.log || exit $?
echo done > $OUT/DONE
