#!/bin/bash
# round 4: the whole GPU suite (the ResidualNet fragment order changed under every flow
# kernel; reciprocal-based spline normalisation in the training kernels), the wide path's
# pass times with the 16-row trunk on and off, the training step, and the driver's bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04d}
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for t in 1 0; do
  FS_WIDE_TRUNK16=$t timeout -k 10 300 python tools/bench_wide.py 200,1024,4096,8192 > gpurun_out/${T}_bench_wide_t$t.log 2>&1
  rc=$?; echo "bench_wide trunk16=$t rc=$rc"; grep '^{' gpurun_out/${T}_bench_wide_t$t.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python tools/bench_train.py > gpurun_out/${T}_bench_train.log 2>&1
rc=$?; echo "bench_train rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/${T}_bench_train.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 300 gpurun_out/${T}_bench.log
