#!/bin/bash
# round-end rehearsal: GPU suite, smoke(), default bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 2 gpurun_out/smoke_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_final.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*, "unit": "steps/s"[^}]*"ms_per_step": [0-9.]*' gpurun_out/bench_final.log
