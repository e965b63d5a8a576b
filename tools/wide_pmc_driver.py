"""A short, profiler-friendly run of the wide path (for rocprofv3 --pmc passes): the A1 flow
at N (default 16) on R rows (default 4096, BASELINE config 2's batch), density and propose
passes, a few repetitions each.  Usage: python tools/wide_pmc_driver.py [N] [R] [reps]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "flow-state_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from flowstate import _lib  # noqa: E402
from flowstate.models import A1, flow_from_state_dict, half_box  # noqa: E402
from oracle import flow as OF  # noqa: E402  (seeded weights only)


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    dims = OF.FlowDims(N=N, B=half_box(N), **A1)
    m = flow_from_state_dict(OF.random_state_dict(dims, seed=3), N, bound=dims.B, **A1)
    L = _lib.load()
    x = ((torch.rand((R, dims.D), device="cuda") * 2 - 1) * dims.B).contiguous()
    cfg = torch.empty_like(x)
    lq = torch.empty(R, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    for _ in range(reps):
        m.log_prob(x)
        _lib.check(L.fs_flow_propose_lq(m.dims(), _lib.ptr(m.packed()), R, 5, 0, 0, float(dims.B), _lib.ptr(cfg),
                                        None, None, _lib.ptr(lq), _lib.ptr(err), _lib.stream_ptr()))
    torch.cuda.synchronize()
    print("ok", N, R, reps)


if __name__ == "__main__":
    main()
