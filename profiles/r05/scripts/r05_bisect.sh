mkdir -p gpurun_out/r05_poison3
export CEP_MEASURE=1 CEP_POISON_BYTE=165
timeout -k 10 60 python -u profiles/poison_bisect.py --bit -2 > gpurun_out/r05_poison3/ref.txt 2>&1 || exit 1
CEP_HOST_TRACE=1 timeout -k 10 60 python -u profiles/poison_bisect.py --bit -2 > gpurun_out/r05_poison3/trace.txt 2>&1 || exit 1
for k in 11 12 7 8 9 10 5 13 14 15 16 17 6 2 3 4; do
  timeout -k 10 60 python -u profiles/poison_bisect.py --bit $k > gpurun_out/r05_poison3/b$k.txt 2>&1 || exit 1
done
echo done > gpurun_out/r05_poison3/DONE
