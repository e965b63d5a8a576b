#!/bin/bash
# round 4, first box run: the changed GPU tests, the driver's bench command, and the
# 2-rank gloo rehearsal of the multi-GPU line (per-rank attribution).  $1 = tag.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04a}
mkdir -p gpurun_out
timeout -k 10 60 ./tools/probes/mfma_order > gpurun_out/${T}_mfma_order.log 2>&1; echo "mfma order rc=$?"; cat gpurun_out/${T}_mfma_order.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_algorithm2.py \
  tests/test_gpu_train.py tests/test_gpu_train_graph.py tests/test_gpu_paired.py \
  "tests/test_gpu_flow.py::test_a1_flow_samples_closer_to_float64_than_reference_f32" -s > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_bench.log; exit $rc; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo > gpurun_out/${T}_dist2_gloo.log 2>&1
rc=$?; echo "dist rehearsal rc=$rc"; tail -c 600 gpurun_out/${T}_dist2_gloo.log
timeout -k 10 200 python tools/icache_probe.py > gpurun_out/${T}_icache_probe.log 2>&1
rc=$?; echo "icache probe rc=$rc"; tail -c 800 gpurun_out/${T}_icache_probe.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/${T}_counters.txt 2>&1; echo "counters rc=$?"
