#!/bin/bash
cd /root/repo
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout=300 -p no:cacheprovider > gpurun_out/gpu_tests3.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests3.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash profiles/profile.sh r01a --keys 200000 --steps 2 --warmup 1 --no-cpu-baseline
