#!/bin/bash
# A/B of the training GEMM's reduction split (tools/build_variant.sh builds): bench_train per build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-base all8 s8m16 s16m16 s8m8pf1 base}; do
  if [ $v = base ]; then lib=""; else lib=flow-state_amd/flowstate/lib/variants/$v/libflowstate.so; fi
  FLOWSTATE_LIB=$lib timeout -k 10 240 python tools/bench_train.py > gpurun_out/train_$v.log 2>&1
  rc=$?; echo "$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/train_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
