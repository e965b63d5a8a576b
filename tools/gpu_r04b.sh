#!/bin/bash
# round 4: training tests (lean GEMMs, A2 reference golden, sticky NaN), the wide path
# (16-row trunk) and fused-step tests, the float64 evidence test, the training cold-start
# probe and graphed-step timing with the lean and the generic GEMMs, then the driver's
# bench and a 2-rank gloo rehearsal.  $1 = tag.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04b}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_train.py \
  tests/test_gpu_train_fused.py tests/test_gpu_paired.py tests/test_gpu_train_graph.py tests/test_gpu_algorithm2.py \
  tests/test_gpu_wide.py tests/test_gpu_mh.py \
  "tests/test_gpu_flow.py::test_a1_flow_samples_closer_to_float64_than_reference_f32" -s > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "worst|vs float64" gpurun_out/${T}_pytest.log; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in lean nolean; do
  lean=1; [ $v = nolean ] && lean=0
  FS_LEAN_GEMM=$lean timeout -k 10 200 python tools/icache_probe.py > gpurun_out/${T}_icache_$v.log 2>&1
  rc=$?; echo "probe $v rc=$rc"; tail -c 700 gpurun_out/${T}_icache_$v.log; [ $rc -eq 0 ] || exit $rc
  FS_LEAN_GEMM=$lean timeout -k 10 300 python tools/bench_train.py > gpurun_out/${T}_bench_train_$v.log 2>&1
  rc=$?; echo "bench_train $v rc=$rc"; tail -c 400 gpurun_out/${T}_bench_train_$v.log; [ $rc -eq 0 ] || exit $rc
done
for t in 1 0; do
  FS_WIDE_TRUNK16=$t timeout -k 10 300 python tools/bench_wide.py 200,1024,4096,8192 > gpurun_out/${T}_bench_wide_t$t.log 2>&1
  rc=$?; echo "bench_wide trunk16=$t rc=$rc"; cat gpurun_out/${T}_bench_wide_t$t.log | cut -c1-220; [ $rc -eq 0 ] || exit $rc
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_prof_refeed -o run -- python3 tools/prof_refeed.py > gpurun_out/${T}_prof_refeed.log 2>&1
rc=$?; echo "refeed rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_prof_refeed.log; exit $rc; }
f=$(find gpurun_out/${T}_prof_refeed -name "*kernel_trace.csv" | head -1)
python3 tools/trace_window.py "$f" 1 > gpurun_out/${T}_refeed_window.json && head -c 1500 gpurun_out/${T}_refeed_window.json
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_bench.log; exit $rc; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo > gpurun_out/${T}_dist2_gloo.log 2>&1
rc=$?; echo "dist rehearsal rc=$rc"; tail -c 300 gpurun_out/${T}_dist2_gloo.log
