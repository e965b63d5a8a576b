#!/bin/bash
# round 4: the start phase merged into the 16-row trunk launch (FS_WIDE_TRUNK16=2) -- the wide
# path's bit-identity tests, pass times and config 5 with it on (2) and off (1), the refeed
# census, and the driver's bench.  $1 = tag.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04i}
PYTESTS=${PYTESTS:-tests/test_gpu_wide.py tests/test_gpu_mh.py}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread $PYTESTS > gpurun_out/${T}_pytest_wide.log 2>&1
rc=$?; echo "pytest wide rc=$rc"; tail -3 gpurun_out/${T}_pytest_wide.log; [ $rc -eq 0 ] || exit $rc
for t in ${TLIST:-2 1}; do
  FS_WIDE_TRUNK16=$t timeout -k 10 300 python tools/bench_wide.py 200,1024,4096 > gpurun_out/${T}_bench_wide_t$t.log 2>&1
  rc=$?; echo "bench_wide trunk16=$t rc=$rc"; grep '^{' gpurun_out/${T}_bench_wide_t$t.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
  FS_WIDE_TRUNK16=$t timeout -k 10 300 python tools/bench_a2.py > gpurun_out/${T}_bench_a2_t$t.log 2>&1
  rc=$?; echo "bench_a2 trunk16=$t rc=$rc"; grep '^{' gpurun_out/${T}_bench_a2_t$t.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_prof_refeed -o run -- python3 tools/prof_refeed.py > gpurun_out/${T}_prof_refeed.log 2>&1
rc=$?; echo "refeed rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_prof_refeed.log; exit $rc; }
f=$(find gpurun_out/${T}_prof_refeed -name "*kernel_trace.csv" | head -1)
python3 tools/trace_window.py "$f" 1 > gpurun_out/${T}_refeed_window.json && head -c 1500 gpurun_out/${T}_refeed_window.json
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 300 gpurun_out/${T}_bench.log
