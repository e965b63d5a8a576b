#!/bin/bash
# rocprofv3 kernel stats of the default bench, then HBM traffic from separate
# FETCH_SIZE / WRITE_SIZE --pmc passes; $1 = tag (output under gpurun_out/<tag>_*)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-prof}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_stats -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-alt-precision --no-given-proposal --no-config2 --no-config5 --no-single-pass --no-algorithm1-regime > gpurun_out/${T}_bench_under_rocprof.log 2>&1
rc=$?; echo "rocprof stats rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_bench_under_rocprof.log; exit $rc; }
f=$(find gpurun_out/${T}_stats -name "*kernel_stats.csv" | head -1)
if [ -n "$f" ]; then cp "$f" gpurun_out/${T}_kernel_stats.csv; else python3 tools/rocpd_stats.py $(find gpurun_out/${T}_stats -name "*.db" | head -1) gpurun_out/${T}_kernel_stats.csv; fi
 head -4 gpurun_out/${T}_kernel_stats.csv | cut -c1-200
python3 tools/kernel_grid_stats.py gpurun_out/${T}_stats > gpurun_out/${T}_kernel_grid_stats.json && head -c 1200 gpurun_out/${T}_kernel_grid_stats.json
for c in FETCH_SIZE WRITE_SIZE; do
  d=gpurun_out/${T}_pmc_$c
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $d -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-alt-precision --no-given-proposal --no-config2 --no-config5 --no-single-pass --no-algorithm1-regime > $d.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 $d.log; exit $rc; }
  f=$(find $d -name "*counter_collection.csv" | grep -v "^$d/run_counter_collection.csv$" | head -1); [ -z "$f" ] || mv "$f" $d/run_counter_collection.csv
done
python3 tools/pmc_traffic.py gpurun_out/${T}_pmc_FETCH_SIZE gpurun_out/${T}_pmc_WRITE_SIZE > gpurun_out/${T}_traffic.json && grep -A3 "flow_pass_kernel<256, 32, 0>" gpurun_out/${T}_traffic.json | head -4
# keep the summaries, drop the raw traces (gpurun copies back at most 64 MiB)
rm -rf gpurun_out/${T}_stats
for c in FETCH_SIZE WRITE_SIZE; do find gpurun_out/${T}_pmc_$c -type f ! -name run_counter_collection.csv -delete; done
exit 0
