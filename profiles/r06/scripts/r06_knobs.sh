#!/bin/bash
# Round 6: the kernel's tuning knobs re-swept on the cfg-3 headline after the round's changes
# (measurement build; each variant its own generated kernel, compiled on the box).
# usage: bash profiles/r06/scripts/r06_knobs.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r06_knobs}
mkdir -p $OUT
export TMPDIR=/tmp
V="default=;qc8=CEP_QUIET_CHUNK:8;qc32=CEP_QUIET_CHUNK:32;wf16=CEP_WALK_FLUSH:16;wf40=CEP_WALK_FLUSH:40;pd0=CEP_PARTIAL_DRAIN:0;nc32=CEP_NODE_CHUNK:32;nc128=CEP_NODE_CHUNK:128;oc4=CEP_OUT_CHUNK:4;oc32=CEP_OUT_CHUNK:32"
CEP_MEASURE=1 timeout -k 10 1000 python -u profiles/nfa_env_sweep.py --variants "$V" > $OUT/sweep.txt 2>&1 || exit $?
echo done > $OUT/DONE
