#!/bin/bash
# kernel census of the graphed A2 training step (tools/prof_train_graph.py under rocprofv3
# --kernel-trace, summarised by tools/trace_window.py); $1 = tag
set -u
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${1:-r06}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_prof_graph -o run -- python3 tools/prof_train_graph.py > gpurun_out/${T}_prof_graph.log 2>&1 || exit $?
f=$(find gpurun_out/${T}_prof_graph -name "*kernel_trace.csv" | head -1)
python3 tools/trace_window.py $f 10 seq > gpurun_out/${T}_a2_graph_replay_window.json || exit $?
rm -rf gpurun_out/${T}_prof_graph
python3 -c "
import json;d=json.load(open('gpurun_out/${T}_a2_graph_replay_window.json'))
print(d['kernels_per_replay'], d['busy_ms_per_replay'], d['span_ms_per_replay'])
for t in d['top'][:8]: print(round(t['ms_per_replay']*1e3/t['calls_per_replay'],2),'us', t['calls_per_replay'], round(t['ms_per_replay'],3), t['kernel'][:60])
"
