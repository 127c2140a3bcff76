#!/bin/bash
# Round 6: occupancy variants of the headline kernel now that it no longer spills (measurement
# build knobs, profiles/nfa_env_sweep.py), and the world-8 shards at 2 and 3 waves per SIMD.
# usage: bash profiles/r06/scripts/r06_occ.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r06_occ}
mkdir -p $OUT
export TMPDIR=/tmp
CEP_MEASURE=1 timeout -k 10 400 python -u profiles/nfa_env_sweep.py --variants "default=;w4l1=CEP_JIT_WAVES:4,CEP_RING_LDS_SLOTS:1;l1=CEP_RING_LDS_SLOTS:1;w2=CEP_JIT_WAVES:2" > $OUT/sweep.txt 2>&1 || exit $?
timeout -k 10 300 python -u profiles/workload.py shards --steps 2 > $OUT/shards_w3.json 2> $OUT/shards_w3.log || exit $?
CEP_MEASURE=1 CEP_JIT_WAVES=2 timeout -k 10 300 python -u profiles/workload.py shards --steps 2 > $OUT/shards_w2.json 2> $OUT/shards_w2.log || exit $?
echo done > $OUT/DONE
