#!/bin/bash
# Round 5 probes: the stencil GPU tests and probe, config 2's bench figure, the NFA cost
# ablation (profiles/nfa_ablation.py) and SQ instruction counters for cfg 3.
# usage: bash profiles/r05/scripts/r05_probe.sh <outdir> [parts: stencil ablation sq]
set -o pipefail
OUT=${1:-gpurun_out/r05_probe}; shift
PARTS=${@:-stencil ablation sq}
mkdir -p $OUT
export TMPDIR=/tmp
for P in $PARTS; do
  case $P in
    stencil)
      timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
        -k "stencil or strict or cfg2 or allocates" > $OUT/tests.log 2>&1 || exit $?
      timeout -k 10 120 ./profiles/micro/stencil_probe > $OUT/probe.txt 2>&1 || exit $?
      timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-other --no-ingest --no-e2e --no-streaming --no-projection > $OUT/bench_cfg2.json 2> $OUT/bench_cfg2.log || exit $?
      ;;
    ablation)
      timeout -k 10 300 python -u profiles/nfa_ablation.py --steps 3 > $OUT/ablation.txt 2>&1 || exit $?
      ;;
    sq)
      I=0
      for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES"; do
        timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/sq_cfg3_$I -o run --output-format csv -- python3 profiles/workload.py cfg3 > $OUT/sq_cfg3_$I.log 2>&1 || exit $?
        I=$((I+1))
      done
      ;;
  esac
done
echo done > $OUT/DONE
