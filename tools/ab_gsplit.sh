#!/bin/bash
# A/B of the wide trunk modes on A1 N=16 / N=3 small batches: FS_WIDE_TRUNK16 = 3 (half-tile)
# vs 4 (column split, FS_GSPLIT workgroups per tile), main library and variants
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
T=$1; R=$2
for v in main $(ls flow-state_amd/flowstate/lib/variants 2>/dev/null); do
  if [ $v = main ]; then L=flow-state_amd/flowstate/lib/libflowstate.so; else L=flow-state_amd/flowstate/lib/variants/$v/libflowstate.so; fi
  for m in 3 4; do
    FS_WIDE_TRUNK16=$m FLOWSTATE_LIB=$L timeout -k 10 150 python -u tools/bench_wide.py $R > gpurun_out/${T}_${v}_t$m.log 2>&1 || { echo "fail $v $m"; tail -5 gpurun_out/${T}_${v}_t$m.log; exit 1; }
    grep A1-N16 gpurun_out/${T}_${v}_t$m.log | sed "s/^/$v t$m /"
  done
done
