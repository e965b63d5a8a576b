"""Timing-only A/B of flow-kernel builds: the density and propose passes at the bench
shape (A1, N=64, 65536 chains) through each library given on the command line (paths;
'base' = the in-tree build), on one packed image.  Results of timing-only builds are
wrong by design and are not checked."""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flow-state_amd"))
sys.path.insert(0, REPO)
from flowstate import _lib  # noqa: E402
from bench import synthetic_model  # noqa: E402

N, C = 64, 65536
model = synthetic_model(N, torch.device("cuda")).set_precision(os.environ.get("FS_PREC", "f32"))
dims, packed = model.dims(), model.packed()
x = ((torch.rand((C, 2 * N), device="cuda") * 2 - 1) * 23.0).contiguous()
lq = torch.empty(C, device="cuda")
cfg = torch.empty_like(x)
cen = torch.empty_like(x)
err = torch.zeros(1, dtype=torch.int32, device="cuda")
out = {}
for arg in sys.argv[1:]:
    L = _lib.load() if arg == "base" else _lib.load(os.path.join(REPO, "flow-state_amd/flowstate/lib/variants", arg,
                                                                  "libflowstate.so"))
    res = {}
    for mode in ("density", "propose"):
        def run():
            if mode == "density":
                L.fs_flow_log_prob(dims, _lib.ptr(packed), _lib.ptr(x), C, _lib.ptr(lq), None, _lib.ptr(err),
                                   _lib.stream_ptr())
            else:
                L.fs_flow_propose(dims, _lib.ptr(packed), C, 1234, 0, 0, 23.0, _lib.ptr(cfg), _lib.ptr(cen), None,
                                  _lib.ptr(err), _lib.stream_ptr())
        run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(4):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        res[mode] = round(min(ts), 3)
    if os.environ.get("FS_CHECK"):  # bit-compare the density pass and the proposals with the base build
        Lb = _lib.load()
        outs = []
        for LL in (Lb, L):
            q = torch.empty(C, device="cuda")
            cf = torch.empty_like(x)
            LL.fs_flow_log_prob(dims, _lib.ptr(packed), _lib.ptr(x), C, _lib.ptr(q), None, _lib.ptr(err),
                                _lib.stream_ptr())
            LL.fs_flow_propose(dims, _lib.ptr(packed), C, 77, 3, 0, 23.0, _lib.ptr(cf), _lib.ptr(cen), None,
                               _lib.ptr(err), _lib.stream_ptr())
            torch.cuda.synchronize()
            outs.append((q.clone(), cf.clone()))
        res["log_q_bit_identical"] = bool(torch.equal(outs[0][0], outs[1][0]))
        res["proposals_bit_identical"] = bool(torch.equal(outs[0][1], outs[1][1]))
    out[arg] = res
    print(arg, res, flush=True)
print(json.dumps(out))
