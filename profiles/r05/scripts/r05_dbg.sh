#!/bin/bash
# Round 5: the arrival-order flake (a repeated push's matches changing now and then).
#   1. every device buffer poisoned (0xA5, synchronously) on repeated CSR + arrival pushes
#   2. the stencil probe
#   3. the stencil / arrival GPU tests five times over (stop at the first failure: its message
#      carries every push's stats and the partition's checks)
# usage: bash profiles/r05/scripts/r05_dbg.sh <outdir>
OUT=${1:-gpurun_out/r05_dbg}
mkdir -p $OUT
export TMPDIR=/tmp
CEP_MEASURE=1 CEP_POISON=-1 CEP_POISON_BYTE=165 timeout -k 10 100 python -u profiles/arrival_repeat.py --pushes 4 --csr-first 2 > $OUT/poison.txt 2>&1
timeout -k 10 60 ./profiles/micro/stencil_probe > $OUT/probe.txt 2>&1 || exit 1
for i in 1 2 3 4 5; do
  timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 100 -k "stencil or strict or cfg2 or allocates or arrival" > $OUT/rel_$i.txt 2>&1 || break
done
echo done > $OUT/DONE
