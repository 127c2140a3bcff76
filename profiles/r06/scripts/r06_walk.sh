#!/bin/bash
# Round 6, after the record-load / walk-load changes (nfa_lane.h: one scalar LDS-or-HBM branch
# per record load, one branch per record store, a walk step's four loads in flight together):
# the GPU suite, the headline figure, occupancy variants, the world-8 shards at 3 and 2 waves
# per SIMD, and the config 4 stress / config 5 / streaming workloads on their own.
# usage: bash profiles/r06/scripts/r06_walk.sh <outdir> [parts: tests quick occ shards dist work]
set -o pipefail
OUT=${1:-gpurun_out/r06_walk}; shift
PARTS=${@:-tests quick occ shards work}
mkdir -p $OUT
export TMPDIR=/tmp
for P in $PARTS; do
  case $P in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
      ;;
    quick)
      timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-other --no-ingest --no-e2e --no-streaming > $OUT/quick.json 2> $OUT/quick.log || exit $?
      ;;
    occ)
      CEP_MEASURE=1 timeout -k 10 400 python -u profiles/nfa_env_sweep.py --variants "default=;w4l1=CEP_JIT_WAVES:4,CEP_RING_LDS_SLOTS:1;l1=CEP_RING_LDS_SLOTS:1;w2=CEP_JIT_WAVES:2" > $OUT/sweep.txt 2>&1 || exit $?
      ;;
    shards)
      CEP_MEASURE=1 CEP_JIT_WAVES=2 timeout -k 10 300 python -u profiles/workload.py shards --steps 2 > $OUT/shards_w2.json 2> $OUT/shards_w2.log || exit $?
      ;;
    dist)
      # the N-rank bench path rehearsed on this one GPU: every rank on cuda:0, the collectives
      # over gloo (the driver's N > 1 runs use RCCL, one rank per GPU); the union of the ranks'
      # checksums must equal the one-GPU checksum
      for NP in 2 4; do
        CEP_BENCH_BACKEND=gloo CEP_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $NP --master-addr 127.0.0.1 --master-port $((29510 + NP)) bench.py --gpus $NP --steps 3 --warmup 1 > $OUT/dist_n$NP.json 2> $OUT/dist_n$NP.log || exit $?
      done
      ;;
    work)
      timeout -k 10 300 python -u profiles/workload.py cfg4s --steps 2 > $OUT/cfg4s.json 2> $OUT/cfg4s.log || exit $?
      timeout -k 10 300 python -u profiles/workload.py stream --steps 2 > $OUT/stream.json 2> $OUT/stream.log || exit $?
      timeout -k 10 300 python -u profiles/workload.py cfg5 --keys 125000 --steps 1 > $OUT/cfg5.json 2> $OUT/cfg5.log || exit $?
      ;;
  esac
done
echo done > $OUT/DONE
