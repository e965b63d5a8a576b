#!/bin/bash
# PMC passes (one counter set per run) over a short bf16x6 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-alt-precision --precision ${PREC:-bf16x6}"
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA -d gpurun_out/pmc_${PREC:-bf16x6}_a -o run --output-format csv -- $B > gpurun_out/pmc_a.log 2>&1 || { echo "pass a rc=$?"; tail -5 gpurun_out/pmc_a.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS -d gpurun_out/pmc_${PREC:-bf16x6}_b -o run --output-format csv -- $B > gpurun_out/pmc_b.log 2>&1 || { echo "pass b rc=$?"; tail -5 gpurun_out/pmc_b.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc_${PREC:-bf16x6}_a gpurun_out/pmc_${PREC:-bf16x6}_b > gpurun_out/pmc_${PREC:-bf16x6}.json 2>gpurun_out/pmc_sum.err || { ls -R gpurun_out/pmc_${PREC:-bf16x6}_a | head; cat gpurun_out/pmc_sum.err; }
python3 -c "
import json; d=json.load(open('gpurun_out/pmc_${PREC:-bf16x6}.json'))
for k,v in d.items():
    if 'split' in k or 'flow_pass' in k: print(k[:60], json.dumps(v.get('derived')), 'coexec', v.get('SQ_VALU_MFMA_COEXEC_CYCLES'), 'gui', v.get('GRBM_GUI_ACTIVE'))
"
