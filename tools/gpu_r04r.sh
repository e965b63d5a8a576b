#!/bin/bash
# round 4, HEAD: the whole GPU suite, smoke, the driver's bench, and a 2-rank gloo rehearsal
# of the multi-GPU bench (both ranks on the one GPU).  $1 = tag.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04r}
mkdir -p gpurun_out
bash tools/gpu_check_round.sh $T full || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo > gpurun_out/${T}_dist2_gloo.log 2>&1
rc=$?; echo "dist rehearsal rc=$rc"; tail -c 300 gpurun_out/${T}_dist2_gloo.log
exit $rc
