"""bench.py's algorithm1_regime leg at a chosen number of attempts (default 50), for
rocprofv3 --kernel-trace --stats: where an attempt's time goes.
Usage: python tools/regime_run.py [attempts]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "flow-state_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import bench  # noqa: E402

if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    print(json.dumps(bench.algorithm1_regime(attempts=n)))
