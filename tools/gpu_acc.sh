set -u
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 200 python tools/acc_uncond.py && timeout -k 10 200 python tools/acc_layers.py && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-alt-precision > gpurun_out/bench.log 2>&1; rc=$?; echo bench rc=$rc; grep -o '"value": [0-9.]*\|"acceptance_match": {[^}]*}[^}]*}\|"kernel_ms": {[^}]*}' gpurun_out/bench.log
