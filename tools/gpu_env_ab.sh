#!/bin/bash
# HIP runtime launch knobs against the training step (tools/bench_train.py, latency-bound:
# ~460 small kernels per graph replay); $1 = tag
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${1:-envab}
run() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python tools/bench_train.py > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/${T}_${name}.log | head -1)"
  return $rc
}
run base X_NONE=1 && run devkernarg1 HIP_FORCE_DEV_KERNARG=1 && run devkernarg0 HIP_FORCE_DEV_KERNARG=0 && \
run pktcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && run pktcap1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 && run base2 X_NONE=1
