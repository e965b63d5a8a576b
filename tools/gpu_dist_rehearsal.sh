#!/bin/bash
# bench.py as the driver launches it for N>1 (torch.distributed.run, one process per
# rank), rehearsed with 2 ranks sharing the one GPU over gloo (RCCL needs one GPU per rank)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --chains 16384 --backend gloo > gpurun_out/dist2.log 2>&1
rc=$?; echo "dist rehearsal rc=$rc"; tail -c 1500 gpurun_out/dist2.log
