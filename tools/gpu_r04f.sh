#!/bin/bash
# config 5's cycle alone (tools/bench_a2.py, 10 cycles) with the 16-row trunk on and off,
# and a kernel census of the refeed.  $1 = tag.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04f}
mkdir -p gpurun_out
for t in 1 0 1; do
  FS_WIDE_TRUNK16=$t timeout -k 10 300 python tools/bench_a2.py > gpurun_out/${T}_bench_a2_t$t.log 2>&1
  rc=$?; echo "bench_a2 trunk16=$t rc=$rc"; grep '^{' gpurun_out/${T}_bench_a2_t$t.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_prof_refeed -o run -- python3 tools/prof_refeed.py > gpurun_out/${T}_prof_refeed.log 2>&1
rc=$?; echo "refeed rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_prof_refeed.log; exit $rc; }
f=$(find gpurun_out/${T}_prof_refeed -name "*kernel_trace.csv" | head -1)
python3 tools/trace_window.py "$f" 1 > gpurun_out/${T}_refeed_window.json && head -c 1200 gpurun_out/${T}_refeed_window.json; tail -3 gpurun_out/${T}_prof_refeed.log
