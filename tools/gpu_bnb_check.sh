#!/bin/bash
# BatchNorm-backward-between-pairs check: its unit test and the training suites, then the
# training step bench and the A2 cycle bench; $1 = tag
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${1:-bnb}
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_graph.py tests/test_gpu_paired.py tests/test_gpu_train_fused.py tests/test_gpu_algorithm2.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_named.log 2>&1
rc=$?; echo "named rc=$rc"; tail -n 4 gpurun_out/${T}_named.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python tools/bench_train.py > gpurun_out/${T}_train_$i.log 2>&1
  rc=$?; echo "bench_train $i rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/${T}_train_$i.log | head -1)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python tools/bench_a2.py > gpurun_out/${T}_bench_a2.log 2>&1
rc=$?; echo "a2 rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/${T}_bench_a2.log | head -1)"; exit $rc
