#!/bin/bash
# r06: dtype-sorted local-move workgroups (FS_LOCAL_SORT): the local-move and driver tests, then
# the Algorithm-1 regime's pipeline timeline sorted (default) and unsorted; $1 = tag
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${1:-r06zy}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_local.py tests/test_gpu_driver.py > gpurun_out/${T}_tests.log 2>&1 || exit 1
for x in 1 0 1 0; do
  FS_LOCAL_SORT=$x timeout -k 10 200 python -u tools/regime_gpu_timeline.py 1000 2 >> gpurun_out/${T}_regime_sort$x.log 2>&1 || exit 1
done
