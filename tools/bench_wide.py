"""Fused kernel vs wide path (phase-by-phase) flow-pass times for small batches:
log_prob (density pass) and propose (sampling pass) at A1 N=16 / N=64 and A2 N=64 over
a sweep of row counts; prints one JSON line per (flow, rows) with both times (ms) and
whether the outputs are bit-identical."""
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


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    L = _lib.load()
    rows_list = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else
                                  "64,128,256,512,1024,2048,4096,8192,16384".split(","))]
    for name, N, kw in (("A1-N16", 16, A1), ("A1-N64", 64, A1), ("A2-N64", 64, A2)):
        dims = OF.FlowDims(N=N, B=half_box(N), **kw)
        m = flow_from_state_dict(OF.random_state_dict(dims, seed=3), N, bound=dims.B, **kw)
        for R in rows_list:
            if name == "A1-N64" and R > 8192:
                continue
            x = ((torch.rand((R, dims.D), device="cuda") * 2 - 1) * dims.B).contiguous()
            out = {}
            res = {}
            for path, lim in (("fused", 0), ("wide", 65536)):
                L.fs_set_wide_rows(lim)
                reps = 3 if R * kw["nb"] >= 65536 else 10
                out[path + "_log_prob_ms"] = timed(lambda: m.log_prob(x), reps)
                cfg = torch.empty_like(x)
                lq = torch.empty(R, device="cuda")
                err = torch.zeros(1, dtype=torch.int32, device="cuda")
                out[path + "_propose_ms"] = timed(lambda: L.fs_flow_propose_lq(
                    m.dims(), _lib.ptr(m.packed()), R, 5, 0, 0, float(dims.B), _lib.ptr(cfg), None, None,
                    _lib.ptr(lq), _lib.ptr(err), _lib.stream_ptr()), reps)
                res[path] = (m.log_prob(x).clone(), lq.clone())
            L.fs_set_wide_rows(-1 if False else 8192)
            out["bit_identical"] = bool(torch.equal(res["fused"][0], res["wide"][0])
                                        and torch.equal(res["fused"][1], res["wide"][1]))
            print(json.dumps({"flow": name, "rows": R, **out}), flush=True)


if __name__ == "__main__":
    main()
