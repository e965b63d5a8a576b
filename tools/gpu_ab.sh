#!/bin/bash
# A/B: default bench (f32 only) with the in-tree library, then with each variant
# named on the command line (tools/build_variant.sh); prints the per-kernel times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in base "$@"; do
  if [ $v = base ]; then L=""; else L=flow-state_amd/flowstate/lib/variants/$v/libflowstate.so; fi
  FLOWSTATE_LIB=$L timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-alt-precision --no-given-proposal --no-config2 ${AB_ARGS:-} > gpurun_out/ab_$v.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/ab_$v.log; exit $rc; }
  echo $v $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v.log | head -1) $(grep -o '"kernel_ms[^}]*}' gpurun_out/ab_$v.log)
done
