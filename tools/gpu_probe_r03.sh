#!/bin/bash
# measurement probes: graph-branch concurrency (tools/graph_branch_probe.py) and a kernel
# trace of one Algorithm-2 refeed (tools/prof_refeed.py + tools/trace_window.py); $1 = tag
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${1:-probe}
export TMPDIR=/tmp
timeout -k 10 120 python tools/graph_branch_probe.py > gpurun_out/${T}_graph_branch.log 2>&1
rc=$?; echo "branch probe rc=$rc"; tail -n 3 gpurun_out/${T}_graph_branch.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_prof_refeed -o run -- python3 tools/prof_refeed.py > gpurun_out/${T}_prof_refeed.log 2>&1
rc=$?; echo "refeed rocprof rc=$rc"; tail -n 5 gpurun_out/${T}_prof_refeed.log; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/${T}_prof_refeed -name "*kernel_trace.csv" | head -1)
python3 tools/trace_window.py "$f" 1 > gpurun_out/${T}_refeed_window.json && head -c 3000 gpurun_out/${T}_refeed_window.json
