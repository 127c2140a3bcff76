#!/bin/bash
# Round-4 stream build check: the GPU suite (streaming parity on the stream build and its wide
# continuation), the headline + projection + streaming bench figures, the streaming probe on the
# stream build and on the wide build ($CEP_STREAM_WIDE=1, the round-3 path), its rocprofv3
# kernel table, and the world-8 shards with the heaviest ranks isolated ($CEP_ISOLATE).
# usage: bash profiles/r04/scripts/r04_stream.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r04_stream}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
timeout -k 10 120 python3 profiles/stream_probe.py > $OUT/stream.json 2> $OUT/stream.log || exit $?
CEP_STREAM_WIDE=1 timeout -k 10 120 python3 profiles/stream_probe.py > $OUT/stream_wide.json 2> $OUT/stream_wide.log || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-other --no-ingest --no-e2e --no-secondary > $OUT/bench.json 2> $OUT/bench.log || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/trace_stream -o run --output-format csv -- python3 profiles/stream_probe.py > $OUT/trace_stream.json 2> $OUT/trace_stream.log || exit $?
timeout -k 10 300 python3 profiles/isolate_probe.py --iso 0,256,512,1024,2048 > $OUT/isolate.json 2> $OUT/isolate.log || exit $?
echo done > $OUT/DONE
