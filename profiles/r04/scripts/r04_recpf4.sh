#!/bin/bash
# Round-4 probe: software-pipelined record loads ($CEP_REC_PF=1) on the config-4 stress query,
# whose keys hold ~20 run records per event (cfg 3: ~1.3), at 3 and 2 waves per SIMD.
# usage: bash profiles/r04/scripts/r04_recpf4.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_recpf4}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 profiles/workload.py cfg4s --steps 3 > $OUT/base.json 2> $OUT/base.log || exit $?
CEP_REC_PF=1 timeout -k 10 400 python3 profiles/workload.py cfg4s --steps 3 > $OUT/pf.json 2> $OUT/pf.log || exit $?
CEP_REC_PF=1 CEP_JIT_WAVES=2 timeout -k 10 400 python3 profiles/workload.py cfg4s --steps 3 > $OUT/pf_w2.json 2> $OUT/pf_w2.log || exit $?
echo done > $OUT/DONE
