#!/bin/bash
# round 4: each residual block's second BatchNorm backward folded into the backward pairs
# around it (FS_FOLD_BN) -- training tests (the A2 reference golden included), the step with
# the fold on and off, config 5, and a census of the graphed step.  $1 = tag.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04p}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_paired.py tests/test_gpu_train.py tests/test_gpu_train_fused.py tests/test_gpu_train_graph.py tests/test_gpu_algorithm2.py > gpurun_out/${T}_pytest_train.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest_train.log; [ $rc -eq 0 ] || exit $rc
for c in 1 0; do
  FS_FOLD_BN=$c timeout -k 10 240 python tools/bench_train.py > gpurun_out/${T}_bench_train_f$c.log 2>&1
  rc=$?; echo "bench_train fold=$c rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/${T}_bench_train_f$c.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python tools/bench_a2.py > gpurun_out/${T}_bench_a2.log 2>&1
rc=$?; echo "bench_a2 rc=$rc"; grep '^{' gpurun_out/${T}_bench_a2.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_prof_graph -o run -- python3 tools/prof_train_graph.py > gpurun_out/${T}_prof_graph.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_prof_graph.log; exit $rc; }
f=$(find gpurun_out/${T}_prof_graph -name "*kernel_trace.csv" | head -1)
python3 tools/trace_window.py "$f" 10 > gpurun_out/${T}_a2_graph_replay_window.json && head -c 300 gpurun_out/${T}_a2_graph_replay_window.json
