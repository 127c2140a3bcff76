#!/bin/bash
cd /root/repo
timeout -k 10 300 python bench.py --keys 100000 --steps 3 --no-cpu-baseline --no-secondary > gpurun_out/bench_small.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/bench_small.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench.py > gpurun_out/bench_full.log 2>&1
echo "rc=$?" >> gpurun_out/bench_full.log
