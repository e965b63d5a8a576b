#!/bin/bash
# Phase-timer builds of the split kernel with experiment macros:
#   tools/split/build_variants.sh name "-DMACRO=1 ..." [name "flags"] ...
# -> flow-state_amd/flowstate/lib/variants/libflowstate_prof_<name>.so
set -e
cd "$(dirname "$0")/../../flow-state_amd/csrc"
make -s prof
OUT=../flowstate/lib/variants
mkdir -p $OUT
OBJS=$(ls ../flowstate/lib/obj_prof/*.o | grep -v flow_split_kernels)
while [ $# -gt 1 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-function -fno-gpu-rdc -munsafe-fp-atomics \
    -DFS_PROF $flags -c flow_split_kernels.hip -o $OUT/split_$name.o 2>&1 | grep -v "argument unused" || true
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libflowstate_prof_$name.so $OBJS $OUT/split_$name.o
  rm -f $OUT/split_$name.o
done
