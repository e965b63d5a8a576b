#!/bin/bash
# full GPU test suite, then a rocprofv3 kernel-trace of the bf16x6 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_x6 -o run -- python bench.py --steps 5 --warmup 1 --precision bf16x6 --no-cpu-baseline > gpurun_out/bench_x6.log 2>&1
rc=$?; echo "rocprof bf16x6 rc=$rc"; tail -c 1500 gpurun_out/bench_x6.log
[ $rc -eq 0 ] || exit $rc
find gpurun_out/prof_x6 -name "*kernel_stats.csv" | head -3
