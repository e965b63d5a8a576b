#!/bin/bash
# flow kernel diagnostics: SQ counter passes (one rocprofv3 --pmc run each) over a
# 1-step f32 bench, then the phase-timer build (tools/flow_phases.py); $1 = tag
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-pmc}
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for cs in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
          "SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM"; do
  i=$((i+1)); d=gpurun_out/${T}_sq$i
  timeout -s KILL 240 rocprofv3 --pmc $cs --output-format csv -d $d -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-alt-precision --no-given-proposal > $d.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $d.log; exit $rc; }
  f=$(find $d -name "*counter_collection.csv" | head -1); [ "$f" = "$d/run_counter_collection.csv" ] || cp "$f" $d/run_counter_collection.csv
done
python3 tools/pmc_summary.py gpurun_out/${T}_sq1 gpurun_out/${T}_sq2 > gpurun_out/${T}_sq.json
if [ -f flow-state_amd/flowstate/lib/libflowstate_prof.so ]; then
  timeout -k 10 300 python3 tools/flow_phases.py f32 > gpurun_out/${T}_phases.json 2>&1; echo "phases rc=$?"
fi
