#!/bin/bash
# rehearsal of the driver's round end: the GPU suite, smoke and the driver's bench
# command (tools/gpu_check_round.sh), the bench's rocprofv3 stats + per-grid kernel times + PMC
# traffic (tools/gpu_prof.sh), then a kernel trace of the A2 training graph's replays;
# $1 = tag.  Every GPU step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r03}
bash tools/gpu_check_round.sh $T full || exit $?
bash tools/gpu_prof.sh $T || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_prof_graph -o run -- python3 tools/prof_train_graph.py > gpurun_out/${T}_prof_graph.log 2>&1
rc=$?; echo "train rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_prof_graph.log; exit $rc; }
f=$(find gpurun_out/${T}_prof_graph -name "*kernel_trace.csv" | head -1)
python3 tools/trace_window.py "$f" 10 > gpurun_out/${T}_a2_graph_replay_window.json && head -c 600 gpurun_out/${T}_a2_graph_replay_window.json
