#!/bin/bash
# A/B of the wide path: $1 = tag, $2 = rows list; every variant under
# flow-state_amd/flowstate/lib/variants/ (tools/build_variant.sh) and the main library
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
T=$1; R=$2
for v in $(ls flow-state_amd/flowstate/lib/variants 2>/dev/null) main; do
  if [ $v = main ]; then L=flow-state_amd/flowstate/lib/libflowstate.so; else L=flow-state_amd/flowstate/lib/variants/$v/libflowstate.so; fi
  FLOWSTATE_LIB=$L timeout -k 10 150 python -u tools/bench_wide.py $R > gpurun_out/${T}_bw_$v.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/${T}_bw_$v.log; exit 1; }
  grep A1-N16 gpurun_out/${T}_bw_$v.log | sed "s/^/$v /"
done
