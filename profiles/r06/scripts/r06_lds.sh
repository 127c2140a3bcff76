#!/bin/bash
# Round 6: more run-queue slots in LDS per lane (3, 4) at the occupancy they leave (2 / 1 waves
# per SIMD), on the config 4 stress query (~20 live runs a key, 2 LDS slots by default) and the
# headline (measurement-build knobs, profiles/nfa_env_sweep.py).
# usage: bash profiles/r06/scripts/r06_lds.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r06_lds}
mkdir -p $OUT
export TMPDIR=/tmp
V="default=;w2=CEP_JIT_WAVES:2;l3w2=CEP_RING_LDS_SLOTS:3,CEP_JIT_WAVES:2;l4w1=CEP_RING_LDS_SLOTS:4,CEP_JIT_WAVES:1"
CEP_MEASURE=1 timeout -k 10 600 python -u profiles/nfa_env_sweep.py --query anys --steps 2 --variants "$V" > $OUT/sweep_cfg4s.txt 2>&1 || exit $?
V2="default=;l3w2=CEP_RING_LDS_SLOTS:3,CEP_JIT_WAVES:2"
CEP_MEASURE=1 timeout -k 10 600 python -u profiles/nfa_env_sweep.py --steps 2 --variants "$V2" > $OUT/sweep_cfg3.txt 2>&1 || exit $?
echo done > $OUT/DONE
