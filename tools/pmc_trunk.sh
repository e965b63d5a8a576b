set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 -L > gpurun_out/r05n_counters.txt 2>&1; echo "list rc=$?"
for R in 4096 16; do
  d=gpurun_out/r05n_pmc_sq_$R
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $d -o run -- python3 tools/wide_pmc_driver.py 16 $R 3 > $d.log 2>&1
  rc=$?; echo "pmc $R rc=$rc"; [ $rc -eq 0 ] || { tail -5 $d.log; exit $rc; }
  f=$(find $d -name "*counter_collection.csv" | head -1); [ -z "$f" ] || mv "$f" $d/run_counter_collection.csv
done
python3 tools/pmc_summary.py gpurun_out/r05n_pmc_sq_4096 > gpurun_out/r05n_sq_4096.json 2>&1
python3 tools/pmc_summary.py gpurun_out/r05n_pmc_sq_16 > gpurun_out/r05n_sq_16.json 2>&1
find gpurun_out/r05n_pmc_sq_4096 gpurun_out/r05n_pmc_sq_16 -type f ! -name "*counter_collection.csv" -delete
exit 0
