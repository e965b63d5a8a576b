#!/bin/bash
# round 4: the wide path's 16-row trunk (bit-identity tests, pass times with it on and off),
# the training tests (lean GEMMs incl. the split-K group) and a kernel census of the graphed
# training step, then its steps/s.  $1 = tag.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04c}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_algorithm2.py tests/test_gpu_train.py tests/test_gpu_train_fused.py tests/test_gpu_paired.py tests/test_gpu_train_graph.py tests/test_gpu_spline_grad.py tests/test_gpu_wide.py > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
for t in 1 0; do
  FS_WIDE_TRUNK16=$t timeout -k 10 300 python tools/bench_wide.py 200,1024,4096,8192 > gpurun_out/${T}_bench_wide_t$t.log 2>&1
  rc=$?; echo "bench_wide trunk16=$t rc=$rc"; grep '^{' gpurun_out/${T}_bench_wide_t$t.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_prof_graph -o run -- python3 tools/prof_train_graph.py > gpurun_out/${T}_prof_graph.log 2>&1
rc=$?; echo "train rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_prof_graph.log; exit $rc; }
f=$(find gpurun_out/${T}_prof_graph -name "*kernel_trace.csv" | head -1)
python3 tools/trace_window.py "$f" 10 > gpurun_out/${T}_a2_graph_replay_window.json && head -c 2500 gpurun_out/${T}_a2_graph_replay_window.json
timeout -k 10 300 python tools/bench_train.py > gpurun_out/${T}_bench_train.log 2>&1
rc=$?; echo "bench_train rc=$rc"; tail -c 300 gpurun_out/${T}_bench_train.log
