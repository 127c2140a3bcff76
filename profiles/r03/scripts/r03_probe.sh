#!/bin/bash
# Round-3 probes (run on the GPU box from the repo root):
#   1. the cep_nfa_jit time split ($CEP_PROF, nfa_lane.h) for cfg 3 at 1M keys and for each
#      rank's murmur2 shard of it (the projected 8-GPU strong scaling case)
#   2. the end-to-end (arrival-order) push breakdown
#   3. rocprofv3 kernel tables + FETCH_SIZE / WRITE_SIZE passes for cfg 4 (stress variant),
#      cfg 4 semantic and cfg 5 (one 125k-key batch of the 64-query group)
# usage: bash profiles/r03/scripts/r03_probe.sh <tag> [prof|e2e|rocprof ...]
set -o pipefail
TAG=${1:-r03}; shift
PARTS=${@:-prof e2e rocprof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for P in $PARTS; do
  case $P in
    prof)
      CEP_PROF=1 timeout -k 10 300 python3 profiles/workload.py cfg3 --steps 1 > $OUT/prof_cfg3.json 2> $OUT/prof_cfg3.log || exit $?
      CEP_PROF=1 timeout -k 10 300 python3 profiles/workload.py shards --world 8 --steps 1 > $OUT/prof_shards.json 2> $OUT/prof_shards.log || exit $?
      ;;
    e2e)
      timeout -k 10 300 python3 profiles/e2e_probe.py --steps 4 > $OUT/e2e.json 2> $OUT/e2e.log || exit $?
      ;;
    rocprof)
      for M in cfg4s cfg4sem "cfg5 --keys 125000 --steps 1"; do
        N=$(echo $M | cut -d' ' -f1)
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$N -o run --output-format csv -- python3 profiles/workload.py $M > $OUT/trace_$N.log 2>&1 || exit $?
        for C in FETCH_SIZE WRITE_SIZE; do
          timeout -k 10 300 rocprofv3 --pmc $C -d $OUT/pmc_${N}_$C -o run --output-format csv -- python3 profiles/workload.py $M > $OUT/pmc_${N}_$C.log 2>&1 || exit $?
        done
      done
      ;;
  esac
done
echo done > $OUT/DONE
