"""A/B of the final layer's GEMM route in training: run tools/bench_train.py with the
hipBLASLt width threshold (autograd_flow._WIDE) set from argv[1] (e.g. 1000000000 keeps
every Linear on fs_linear_f32)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "flow-state_amd"), os.path.join(REPO, "tools")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from flowstate.normflows import autograd_flow  # noqa: E402

autograd_flow._WIDE = int(sys.argv[1])
import bench_train  # noqa: E402

bench_train.main()
