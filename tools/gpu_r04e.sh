#!/bin/bash
# round 4 profile: wide-path tests (trunk crossover, variant-keyed graph cache), the bench's
# rocprofv3 kernel stats + PMC traffic (tools/gpu_prof.sh), a kernel census of the graphed
# training step, then the driver's bench command.  $1 = tag.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04e}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_wide.py > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh $T || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_prof_graph -o run -- python3 tools/prof_train_graph.py > gpurun_out/${T}_prof_graph.log 2>&1
rc=$?; echo "train rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_prof_graph.log; exit $rc; }
f=$(find gpurun_out/${T}_prof_graph -name "*kernel_trace.csv" | head -1)
python3 tools/trace_window.py "$f" 10 > gpurun_out/${T}_a2_graph_replay_window.json && head -c 300 gpurun_out/${T}_a2_graph_replay_window.json
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 300 gpurun_out/${T}_bench.log
