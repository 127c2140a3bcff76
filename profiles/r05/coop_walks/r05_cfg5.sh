#!/bin/bash
# Round 5: wave-cooperative walk hops on config 5 (nfa_lane.h coop_hops).  The cfg 5 GPU
# parity tests, then batches 0 and 3 of the 64-variant group at the default threshold (8
# walkers) and, in the measurement build, at 0 (off), 2, 32 and 64.
# usage: bash profiles/r05/scripts/r05_cfg5.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r05_cfg5}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "cfg5 or heavy_key or group" > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 200 python -u profiles/cfg5_probe.py --only 0,3 > $OUT/probe_default.txt 2>&1 || exit $?
for C in 0 2 64; do
  CEP_MEASURE=1 CEP_COOP_WALKERS=$C timeout -k 10 200 python -u profiles/cfg5_probe.py --only 0,3 > $OUT/probe_c$C.txt 2>&1 || exit $?
done
echo done > $OUT/DONE
