#!/bin/bash
# training-path GPU tests, then the A2 step and cycle benches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_fused.py tests/test_gpu_train_graph.py tests/test_gpu_algorithm2.py tests/test_gpu_spline_grad.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_train.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_train.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python tools/bench_train.py > gpurun_out/bench_train.log 2>&1
rc=$?; echo "bench_train rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/bench_train.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python tools/bench_a2.py > gpurun_out/bench_a2.log 2>&1
rc=$?; echo "bench_a2 rc=$rc"; grep -o '"value": [0-9.]*\|"phase_ms": {[^}]*}' gpurun_out/bench_a2.log
