#!/bin/bash
# tools/wide_variant_ab.py for the in-tree library and each named variant; $1 = tag
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=$1; shift
for v in base "$@" base; do
  if [ $v = base ]; then L=""; else L=flow-state_amd/flowstate/lib/variants/$v/libflowstate.so; fi
  FLOWSTATE_LIB=$L timeout -k 10 300 python tools/wide_variant_ab.py 300 >> gpurun_out/${T}_wide_ab.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/${T}_wide_ab.log; exit $rc; }
done
grep '^{' gpurun_out/${T}_wide_ab.log
