#!/bin/bash
# v9 HBM traffic: FETCH_SIZE and WRITE_SIZE in separate --pmc passes over a short f32 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  d=gpurun_out/v9_pmc_$c
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $d -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $d.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 $d.log; exit $rc; }
  f=$(find $d -name "*counter_collection.csv" | head -1); echo "$f"; cp "$f" $d/run_counter_collection.csv 2>/dev/null || true
done
python3 tools/pmc_traffic.py gpurun_out/v9_pmc_FETCH_SIZE gpurun_out/v9_pmc_WRITE_SIZE > gpurun_out/v9_traffic.json && cat gpurun_out/v9_traffic.json
