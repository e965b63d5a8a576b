#!/bin/bash
# A/B of the in-launch ends of the training step (split-K tile reduction, BatchNorm backward
# on the pair's last strip tile): named tests, then tools/bench_train.py per variant; $1 = tag
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${1:-ab}
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_named.log 2>&1
rc=$?; echo "named rc=$rc"; tail -n 3 gpurun_out/${T}_named.log; [ $rc -eq 0 ] || exit $rc
for v in "0 0" "1 1" "0 1" "1 0"; do
  set -- $v
  FS_AB_NO_GROUP_EX=$1 FS_AB_NO_PAIR_BN=$2 timeout -k 10 200 python tools/bench_train.py > gpurun_out/${T}_train_g$1_b$2.log 2>&1
  rc=$?; echo "no_group_ex=$1 no_pair_bn=$2 rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/${T}_train_g$1_b$2.log | head -1)"
  [ $rc -eq 0 ] || exit $rc
done
