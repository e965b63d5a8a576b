#!/bin/bash
# round 4: the two-waves-per-pair final phase (bit-identity tests, refeed-size pass times with
# it on and off) and config 5's cycle.  $1 = tag.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04g}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_mh.py tests/test_gpu_algorithm2.py > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
for f2 in 1 0; do
  FS_WIDE_FINAL2=$f2 timeout -k 10 300 python tools/bench_wide.py 200,1024,4096 > gpurun_out/${T}_bench_wide_f$f2.log 2>&1
  rc=$?; echo "bench_wide final2=$f2 rc=$rc"; grep '^{' gpurun_out/${T}_bench_wide_f$f2.log | grep A2 | cut -c1-200; [ $rc -eq 0 ] || exit $rc
  FS_WIDE_FINAL2=$f2 timeout -k 10 300 python tools/bench_a2.py > gpurun_out/${T}_bench_a2_f$f2.log 2>&1
  rc=$?; echo "bench_a2 final2=$f2 rc=$rc"; grep -o '"value": [0-9.]*\|"refeed": [0-9.]*' gpurun_out/${T}_bench_a2_f$f2.log; [ $rc -eq 0 ] || exit $rc
done
