set -e
for v in base A B C; do
  if [ $v = base ]; then L=""; else L=flow-state_amd/flowstate/lib/variants/libflowstate_$v.so; fi
  FLOWSTATE_LIB=$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1
  echo $v $(grep -o '"kernel_ms[^}]*}' gpurun_out/ab_$v.log)
done
