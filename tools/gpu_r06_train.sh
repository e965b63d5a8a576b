#!/bin/bash
# r06 training-step check: the forward-product chain timing (tools/train_lin_chain.py),
# the graphed training step (tools/bench_train.py), the training tests; then a kernel trace
# of the Algorithm-1 regime (tools/regime_run.py).  $1 = tag.
set -u
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${1:-r06}
timeout -k 10 120 python -u tools/train_lin_chain.py > gpurun_out/${T}_lin_chain.log 2>&1 || exit $?
tail -n 1 gpurun_out/${T}_lin_chain.log
timeout -k 10 200 python -u tools/bench_train.py > gpurun_out/${T}_bench_train.log 2>&1 || exit $?
tail -c 600 gpurun_out/${T}_bench_train.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_train.py \
  tests/test_gpu_train_fused.py tests/test_gpu_train_graph.py tests/test_gpu_paired.py tests/test_gpu_algorithm2.py \
  > gpurun_out/${T}_pytest_train.log 2>&1
rc=$?; tail -n 2 gpurun_out/${T}_pytest_train.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_regime -o regime -- python3 tools/regime_run.py 100 \
  > gpurun_out/${T}_regime_prof.log 2>&1
rc=$?; tail -n 2 gpurun_out/${T}_regime_prof.log; exit $rc
