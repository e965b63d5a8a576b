#!/bin/bash
# tools/linbn_probe.py on the in-tree build, then on each variant named on the command line
# (tools/build_variant.sh <name> -D...); one JSON line per build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in base "$@"; do
  if [ $v = base ]; then L=""; else L=flow-state_amd/flowstate/lib/variants/$v/libflowstate.so; fi
  FLOWSTATE_LIB=$L timeout -k 10 120 python tools/linbn_probe.py > gpurun_out/probe_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/probe_$v.log; exit 1; }
  echo $v; tail -1 gpurun_out/probe_$v.log
done
