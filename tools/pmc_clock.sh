#!/bin/bash
# Effective shader clock of the headline flow kernels (MI355X_MICROARCH.md: GRBM_GUI_ACTIVE / 8 /
# kernel wall time) and their MFMA busy share, f32 and bf16x6: $1 = tag
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
T=$1
for prec in f32 bf16x6; do
  d=gpurun_out/${T}_pmc_$prec
  FS_PREC=$prec timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $d -o run -- python3 tools/variant_time.py base > $d.log 2>&1
  rc=$?; echo "pmc $prec rc=$rc"; [ $rc -eq 0 ] || { tail -5 $d.log; exit $rc; }
  f=$(find $d -name "*counter_collection.csv" | head -1); [ -z "$f" ] || mv "$f" $d/run_counter_collection.csv
  k=$(find $d -name "*kernel_trace.csv" | head -1); [ -z "$k" ] || mv "$k" $d/run_kernel_trace.csv
  find $d -type f ! -name "run_*.csv" -delete
done
