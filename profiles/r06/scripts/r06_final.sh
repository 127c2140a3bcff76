#!/bin/bash
# Round-6 evidence for the bench line (run on the GPU box from the repo root):
#   tests  the GPU suite
#   bench  the bench as the driver runs it (every figure, CPU baselines included)
#   trace  rocprofv3 --kernel-trace --stats over bench.py's cfg-3 + cfg-2 figures (the kernel
#          table the line's roofline must agree with)
#   pmc    separate FETCH_SIZE / WRITE_SIZE passes per workload (profiles/workload.py,
#          profiles/stencil_bench.py) -> profiles/traffic.py
#   sq     SQ instruction / cycle counters for cfg 3
# usage: bash profiles/r06/scripts/r06_final.sh <outdir> [parts: tests bench trace pmc sq]
set -o pipefail
OUT=${1:-gpurun_out/r06_final}; shift
PARTS=${@:-bench trace pmc sq}
mkdir -p $OUT
export TMPDIR=/tmp
for P in $PARTS; do
  case $P in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
      ;;
    bench)
      timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.log || exit $?
      ;;
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 5 --no-cpu-baseline --no-other --no-ingest --no-e2e --no-projection --no-streaming > $OUT/trace_bench.json 2> $OUT/trace_bench.log || exit $?
      ;;
    pmc)
      for M in cfg3 cfg4s cfg4 "cfg5 --keys 125000 --steps 1"; do
        N=$(echo $M | cut -d' ' -f1)
        for C in FETCH_SIZE WRITE_SIZE; do
          timeout -s KILL 300 rocprofv3 --pmc $C -d $OUT/pmc_${N}_$C -o run --output-format csv -- python3 profiles/workload.py $M > $OUT/pmc_${N}_$C.log 2>&1 || exit $?
        done
      done
      for C in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_cfg2_$C -o run --output-format csv -- python3 profiles/stencil_bench.py --steps 20 > $OUT/pmc_cfg2_$C.log 2>&1 || exit $?
      done
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
