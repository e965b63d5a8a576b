#!/bin/bash
# proposal bank: parity tests, then the Algorithm-1 cycle on small batches with and without it
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mh.py tests/test_gpu_driver.py tests/test_gpu_algorithm2.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_bank.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 4 gpurun_out/pytest_bank.log; [ $rc -eq 0 ] || exit $rc
for args in "--N 16 --C 4096 --cycles 16 --interval 1000" "--N 16 --C 4096 --cycles 16 --interval 1000 --single" \
            "--N 64 --C 4096 --cycles 16 --interval 1000" "--N 64 --C 4096 --cycles 16 --interval 1000 --single" \
            "--N 64 --C 65536 --cycles 3"; do
  timeout -k 10 300 python tools/bench_hybrid.py $args >> gpurun_out/bench_hybrid_bank.log 2>&1
  rc=$?; echo "bench_hybrid $args rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
grep -o '"metric": "[^"]*", "value": [0-9.]*\|"big_move_ms_per_cycle": [0-9.]*\|"proposal_bank_steps": [0-9]*' gpurun_out/bench_hybrid_bank.log
timeout -k 10 300 python tools/bench_a2.py > gpurun_out/bench_a2_bank.log 2>&1
rc=$?; echo "bench_a2 rc=$rc"; tail -c 600 gpurun_out/bench_a2_bank.log
