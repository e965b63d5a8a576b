#!/bin/bash
# split-bf16 path: parity tests, then the bench (headline f32 + alt precisions)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python tools/split/debug_split.py > gpurun_out/dbg4.log 2>&1; grep "N=" gpurun_out/dbg4.log | head -8
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -v --timeout 300 --timeout-method thread > gpurun_out/split_tests.log 2>&1
rc=$?; echo "split tests rc=$rc"; tail -n 30 gpurun_out/split_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 5 --warmup 1 --cpu-budget 5 > gpurun_out/bench_split.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_split.log
