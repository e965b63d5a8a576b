#!/bin/bash
# Build an A/B variant of libflowstate.so: $1 = name, rest = -D switches.
# Output: flow-state_amd/flowstate/lib/variants/$1/libflowstate.so (load with FLOWSTATE_LIB=...)
set -e
cd "$(dirname "$0")/../flow-state_amd/csrc"
name=$1; shift
make -s -j8 OUT=../flowstate/lib/variants/$name EXTRA="$*"
