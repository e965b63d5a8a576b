#!/bin/bash
# run tools/flow_phases.py on each prof variant built by build_variants.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/variants
prec=${PREC:-bf16x6}
for v in "$@"; do
  FS_PROF_LIB=flow-state_amd/flowstate/lib/variants/libflowstate_prof_$v.so timeout -k 10 120 python tools/flow_phases.py $prec \
    > gpurun_out/variants/$v.json 2> gpurun_out/variants/$v.err || { echo "$v failed rc=$?"; tail -5 gpurun_out/variants/$v.err; exit 1; }
  python3 -c "
import json,sys
d=json.load(open('gpurun_out/variants/$v.json'))
for k in ('density','sample'):
    s=d[k]['share']; print('$v', k, '%.2f ms'%d[k]['ms'], ' '.join('%s=%.3f'%(a[:8],b) for a,b in s.items() if b>0.004))
"
done
