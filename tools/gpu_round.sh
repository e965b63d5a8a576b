#!/bin/bash
# One gpurun call: each GPU step under its own time limit; continue past plain
# test failures (rc 1) but stop at anything that looks like a fault/abort/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for step in "$@"; do
  case "$step" in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 900 python -m pytest tests -m gpu -q -rf ;;
    bench) run bench 600 python bench.py ;;
    tests_local) run pytest_local 600 python -m pytest tests/test_gpu_local.py -q -rf -x ;;
    bench_local) run bench_local 400 python tools/bench_local.py ;;
    pmc_flow1) run pmc_flow1 600 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc_flow1 -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    pmc_flow2) run pmc_flow2 600 rocprofv3 --pmc SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM -d gpurun_out/pmc_flow2 -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    pmc_local) run pmc_local 400 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/pmc_local -o run --output-format csv -- python tools/bench_local.py --steps 2 --no-cpu-baseline ;;
    pmc_local_wait) run pmc_local_wait 400 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_local_wait -o run --output-format csv -- python tools/bench_local.py --steps 2 --no-cpu-baseline ;;
    bench_hybrid) run bench_hybrid 400 python tools/bench_hybrid.py ;;
    bench_train) run bench_train 400 python tools/bench_train.py ;;
    bench_a2) run bench_a2 400 python tools/bench_a2.py ;;
    prof_graph) run rocprof_graph 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_graph -o run --output-format csv -- python tools/prof_train_graph.py; python tools/trace_window.py gpurun_out/prof_graph/run_kernel_trace.csv 10 > gpurun_out/graph_window.json; head -c 3000 gpurun_out/graph_window.json; rm -f gpurun_out/prof_graph/run_kernel_trace.csv ;;
    prof_train) run rocprof_train 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o run --output-format csv -- python tools/bench_train.py && rm -f gpurun_out/prof_train/run_kernel_trace.csv ;;
    phases) run phases 300 python tools/flow_phases.py ;;
    prof_local) run rocprof_local 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_local -o run --output-format csv -- python tools/bench_local.py --steps 3 --no-cpu-baseline ;;
    bench_short) run bench_short 400 python bench.py --steps 3 --warmup 1 --cpu-budget 10 ;;
    prof) run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    counters) run counters 120 rocprofv3 -L ;;
    pmc_fetch) run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    pmc_write) run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    pmc_sq) run pmc_sq 600 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/pmc_sq -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    pmc_wait) run pmc_wait 600 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_wait -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
