#!/bin/bash
# training-path tests, then a rocprofv3 kernel trace of graph replays of the A2 step, summarised
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_fused.py tests/test_gpu_train_graph.py tests/test_gpu_algorithm2.py tests/test_gpu_spline_grad.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_train.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/pytest_train.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_graph -o run -- python3 tools/prof_train_graph.py > gpurun_out/prof_graph.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_graph.log; exit $rc; }
f=$(find gpurun_out/prof_graph -name "*kernel_trace.csv" | head -1)
python3 tools/trace_window.py "$f" 10 > gpurun_out/a2_graph_replay_window.json && head -c 400 gpurun_out/a2_graph_replay_window.json
timeout -k 10 240 python tools/bench_train.py > gpurun_out/bench_train.log 2>&1
rc=$?; echo "bench_train rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/bench_train.log
