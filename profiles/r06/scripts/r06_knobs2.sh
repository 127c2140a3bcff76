#!/bin/bash
# Round 6: the quiet-chunk constant (it also weighs the lane order's work estimate) and the
# session chunk knobs (applied this time: the first sweep dropped them before the session) on
# the headline, the config 4 stress query and one streaming push.
# usage: bash profiles/r06/scripts/r06_knobs2.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r06_knobs2}
mkdir -p $OUT
export TMPDIR=/tmp
V="default=;qc4=CEP_QUIET_CHUNK:4;qc8=CEP_QUIET_CHUNK:8;qc12=CEP_QUIET_CHUNK:12;qc8wf40=CEP_QUIET_CHUNK:8,CEP_WALK_FLUSH:40;nc128=CEP_NODE_CHUNK:128;oc4=CEP_OUT_CHUNK:4"
CEP_MEASURE=1 timeout -k 10 600 python -u profiles/nfa_env_sweep.py --variants "$V" > $OUT/sweep.txt 2>&1 || exit $?
V2="default=;qc4=CEP_QUIET_CHUNK:4;qc8=CEP_QUIET_CHUNK:8"
CEP_MEASURE=1 timeout -k 10 600 python -u profiles/nfa_env_sweep.py --query anys --steps 2 --variants "$V2" > $OUT/sweep_cfg4s.txt 2>&1 || exit $?
CEP_MEASURE=1 timeout -k 10 600 python -u profiles/nfa_env_sweep.py --stream --steps 2 --variants "$V2" > $OUT/sweep_stream.txt 2>&1 || exit $?
echo done > $OUT/DONE
