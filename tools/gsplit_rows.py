"""Column-split trunk (fs_set_wide_trunk16 4) against the half-tile trunk (3) by batch size:
density and propose passes through the raw ABI (no host sync per call), the default
choice (5) beside them; prints one JSON line per row count (ms per pass).
Usage: python tools/gsplit_rows.py [rows,...] [A1-N16 | A2-N64]"""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "flow-state_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)
from flowstate import _lib  # noqa: E402
from flowstate.models import A1, A2, flow_from_state_dict, half_box  # noqa: E402
from oracle import flow as OF  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    L = _lib.load()
    flow = sys.argv[2] if len(sys.argv) > 2 else "A1-N16"
    N, kw = (16, A1) if flow == "A1-N16" else (64, A2)
    dims = OF.FlowDims(N=N, B=half_box(N), **kw)
    m = flow_from_state_dict(OF.random_state_dict(dims, seed=3), N, bound=dims.B, **kw)
    pk = m.packed()
    rows = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "16,64,256,384,512").split(",")]
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    for R in rows:
        x = ((torch.rand((R, dims.D), device="cuda") * 2 - 1) * dims.B).contiguous()
        lq = torch.empty(R, device="cuda")
        cfg = torch.empty_like(x)
        out = {"flow": flow, "rows": R}
        for t in (5, 4, 3):
            prev = L.fs_set_wide_trunk16(t)
            out[f"t{t}_density_ms"] = round(timed(lambda: L.fs_flow_log_prob(
                m.dims(), _lib.ptr(pk), _lib.ptr(x), R, _lib.ptr(lq), None, _lib.ptr(err), _lib.stream_ptr())), 3)
            out[f"t{t}_propose_ms"] = round(timed(lambda: L.fs_flow_propose(
                m.dims(), _lib.ptr(pk), R, 5, 0, 0, float(dims.B), _lib.ptr(cfg), None, None, _lib.ptr(err),
                _lib.stream_ptr())), 3)
            L.fs_set_wide_trunk16(prev)
        torch.cuda.synchronize()
        out["err"] = int(err.item())
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
