#!/bin/bash
# Round-4 probe: cfg 3's cep_nfa_jit with the wave-cooperative record pages (nfa_coop.h) and
# without ($CEP_NO_COOP), each in the default lane order and the span order ($CEP_EST_MODE=1),
# coop at 3 waves per SIMD ($CEP_JIT_WAVES=3, with spills), and the lone heaviest key.
# usage: bash profiles/r04/scripts/r04_coop.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_coop}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 profiles/workload.py cfg3 --steps 3 > $OUT/$name.json 2> $OUT/$name.log || exit $?
  env "$@" timeout -k 10 120 python3 profiles/heavy_alone.py --steps 3 > $OUT/heavy_$name.txt 2>&1 || exit $?
}
run coop
run nocoop CEP_NO_COOP=1
run coop_span CEP_EST_MODE=1
run nocoop_span CEP_NO_COOP=1 CEP_EST_MODE=1
run coop_w3 CEP_JIT_WAVES=3
timeout -k 10 300 python3 profiles/workload.py shards --world 8 --steps 2 > $OUT/shards_coop.json 2> $OUT/shards_coop.log || exit $?
CEP_NO_COOP=1 timeout -k 10 300 python3 profiles/workload.py shards --world 8 --steps 2 > $OUT/shards_nocoop.json 2> $OUT/shards_nocoop.log || exit $?
echo done > $OUT/DONE
