set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "kats or cfg3 or cfg4 or streaming or capacity or pool or long_strict or edge or error or arrival or cfg5" > gpurun_out/t2.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t2.log; tail -3 gpurun_out/t2.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u profiles/nfa_env_sweep.py --keys 1000000 --variants "default=;nolds=CEP_RING_LDS:0" > gpurun_out/sweep2.log 2>&1 || exit $?
timeout -k 10 300 python -u profiles/nfa_ablation.py --keys 1000000 > gpurun_out/abl3.log 2>&1 || exit $?
tail -1 gpurun_out/sweep2.log; tail -1 gpurun_out/abl3.log
