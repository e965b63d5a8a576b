#!/bin/bash
# r06 A/B probes: $1 = tag.  (1) the training ResidualBlock in-launch hand-off probe
# (tools/probes/block_fuse); (2) the column-split trunk with a tile's
# workgroups on one XCD (variant build "xcd", -DFS_GSPLIT_XCD=1) against the main build
# (VERDICT r05 item 6), propose passes of 16-256 rows.
set -u
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${1:-r06}
timeout -k 10 120 tools/probes/block_fuse 46 50 > gpurun_out/${T}_block_fuse.log 2>&1
rc=$?; echo "block_fuse rc=$rc"; tail -n 2 gpurun_out/${T}_block_fuse.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 tools/probes/block_fuse 2 400 > gpurun_out/${T}_block_fuse_2.log 2>&1
rc=$?; echo "block_fuse(2) rc=$rc"; tail -n 1 gpurun_out/${T}_block_fuse_2.log
[ $rc -le 1 ] || exit $rc
for round in 1 2; do
  for v in main xcd; do
    if [ $v = main ]; then L=flow-state_amd/flowstate/lib/libflowstate.so; else L=flow-state_amd/flowstate/lib/variants/$v/libflowstate.so; fi
    FLOWSTATE_LIB=$L timeout -k 10 200 python -u tools/bench_wide.py 16,64,128,256 > gpurun_out/${T}_bw_${v}_$round.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/${T}_bw_${v}_$round.log; exit 1; }
    grep A1-N16 gpurun_out/${T}_bw_${v}_$round.log | sed "s/^/$v $round /"
  done
done
