#!/bin/bash
# Round-4 probe: software-pipelined record loads ($CEP_REC_PF=1 at query compile: record i+1's
# quads loaded before record i's step) on cfg 3 per batch (3 and 2 waves per SIMD) and on the
# streamed cfg 3; the queries compile on the box (not in the JIT cache).
# usage: bash profiles/r04/scripts/r04_recpf.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_recpf}
mkdir -p $OUT
export TMPDIR=/tmp
CEP_REC_PF=1 timeout -k 10 400 python3 profiles/workload.py cfg3 --steps 3 > $OUT/cfg3_pf.json 2> $OUT/cfg3_pf.log || exit $?
CEP_REC_PF=1 CEP_JIT_WAVES=2 timeout -k 10 400 python3 profiles/workload.py cfg3 --steps 3 > $OUT/cfg3_pf_w2.json 2> $OUT/cfg3_pf_w2.log || exit $?
CEP_REC_PF=1 timeout -k 10 400 python3 profiles/stream_probe.py > $OUT/s10_pf.json 2> $OUT/s10_pf.log || exit $?
echo done > $OUT/DONE
