#!/bin/bash
cd /root/repo
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout=300 -p no:cacheprovider -x > gpurun_out/gpu_tests4.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests4.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench4.log 2>&1
echo "rc=$?" >> gpurun_out/bench4.log
