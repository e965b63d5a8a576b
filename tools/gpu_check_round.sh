#!/bin/bash
# GPU check of a round: the named tests first, then the whole GPU suite, smoke and the
# driver's bench command; $1 = tag, $2 = "quick" to stop after the named tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${1:-r03}
shift || true
MODE=${1:-full}
shift || true
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/${T}_named.log 2>&1
  rc=$?; echo "named rc=$rc"; tail -n 15 gpurun_out/${T}_named.log
  [ $rc -eq 0 ] || exit $rc
fi
[ "$MODE" = quick ] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/${T}_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 2 gpurun_out/${T}_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/${T}_bench.log
exit $rc
