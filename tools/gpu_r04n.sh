#!/bin/bash
# round 4, HEAD: the whole GPU suite, smoke, the driver's bench, and the secondary
# measurements last taken in r02 (local moves, the Algorithm-1 cycle at config 3 and
# config 2 sizes).  $1 = tag.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04n}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 1 gpurun_out/${T}_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 300 gpurun_out/${T}_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_local.py > gpurun_out/${T}_bench_local.log 2>&1
rc=$?; echo "bench_local rc=$rc"; grep '^{' gpurun_out/${T}_bench_local.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_hybrid.py > gpurun_out/${T}_bench_hybrid.log 2>&1
rc=$?; echo "bench_hybrid rc=$rc"; grep '^{' gpurun_out/${T}_bench_hybrid.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
for s in "" "--single"; do
  timeout -k 10 300 python tools/bench_hybrid.py --N 16 --C 4096 --cycles 16 $s > gpurun_out/${T}_bench_hybrid_c2$s.log 2>&1
  rc=$?; echo "bench_hybrid c2 $s rc=$rc"; grep '^{' gpurun_out/${T}_bench_hybrid_c2$s.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
done
