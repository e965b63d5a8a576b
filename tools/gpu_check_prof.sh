#!/bin/bash
# full GPU test suite + smoke, then the default bench's rocprofv3 stats and PMC traffic
# passes (tools/gpu_prof.sh); $1 = tag
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${1:-prof}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/${T}_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 2 gpurun_out/${T}_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/${T}_bench.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh $T
