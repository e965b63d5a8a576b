#!/bin/bash
# kernel census of the captured A2 training step's replays (rocprofv3 kernel trace); $1 = tag
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${1:-census}
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_prof_graph -o run -- python3 tools/prof_train_graph.py > gpurun_out/${T}_prof_graph.log 2>&1
rc=$?; echo "train rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_prof_graph.log; exit $rc; }
f=$(find gpurun_out/${T}_prof_graph -name "*kernel_trace.csv" | head -1)
python3 tools/trace_window.py "$f" 10 > gpurun_out/${T}_a2_graph_replay_window.json && python3 - "$T" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/{sys.argv[1]}_a2_graph_replay_window.json"))
print({k: v for k, v in d.items() if k != "top"})
for r in d["top"][:12]:
    print(f"{r['calls_per_replay']:6.1f} {r['ms_per_replay']*1e3:8.1f}us {r['kernel'][:90]}")
PY
