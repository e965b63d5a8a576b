#!/bin/bash
# training tests, a kernel trace of A2 training-step replays (with the last replay's
# kernel sequence), then tools/bench_train.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_paired.py tests/test_gpu_train.py tests/test_gpu_train_fused.py tests/test_gpu_train_graph.py tests/test_gpu_algorithm2.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG:-r04v}_pytest_train.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/${TAG:-r04v}_pytest_train.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_graph -o run -- python3 tools/prof_train_graph.py > gpurun_out/prof_graph.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_graph.log; exit $rc; }
f=$(find gpurun_out/prof_graph -name "*kernel_trace.csv" | head -1)
python3 tools/trace_window.py "$f" 10 seq > gpurun_out/${TAG:-r04v}_a2_graph_replay_window.json && head -c 300 gpurun_out/${TAG:-r04v}_a2_graph_replay_window.json
timeout -k 10 240 python tools/bench_train.py > gpurun_out/${TAG:-r04v}_bench_train.log 2>&1
rc=$?; echo "bench_train rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/${TAG:-r04v}_bench_train.log
