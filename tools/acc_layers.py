"""Accuracy diagnostic (not a test): per-layer error of the HIP density pass vs the
oracle's float32 and float64 restatements, on flow-sampled inputs at A1, N=64.
Each layer gets the SAME float32 input (the float64 trace's input, rounded); the
float64 reference of that layer runs on the same (upcast) input."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "flow-state_amd")]
from flowstate.models import A1, flow_from_state_dict, half_box  # noqa: E402
from oracle import flow as OF  # noqa: E402

N = int(os.environ.get("ACC_N", 64))
C = int(os.environ.get("ACC_C", 256))
dims = OF.FlowDims(N=N, B=half_box(N), **A1)
sd = OF.random_state_dict(dims, seed=7)
sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
m = flow_from_state_dict(sd, N, bound=dims.B, **A1).set_precision(os.environ.get("ACC_PREC", "f32"))
g = torch.Generator().manual_seed(5)
z = (torch.rand((C, dims.D), generator=g) * 2 - 1) * dims.B
x = m.forward(z.cuda()).cpu()
_, _, trace = OF.log_prob(sd64, x.double(), dims, per_layer=True)
ins = [x.double()] + [t[0] for t in trace[:-1]]
print("layer | ident-half max|d| gpu ref32 | transform-half max|d| gpu ref32 | logdet max|d| gpu ref32 |"
      " logdet median|d| gpu ref32")
h = dims.D // 2
unroll = lambda o: torch.cat([o[:, h:], o[:, :h]], dim=1)
tot = {"gpu": 0.0, "ref": 0.0}
for k, i in enumerate(range(dims.L - 1, -1, -1)):
    u32 = ins[k].float()
    lp32, lp64 = OF.layer_params(sd, i), OF.layer_params(sd64, i)
    o64, l64 = OF.coupling_density(lp64, u32.double(), dims)
    o32, l32 = OF.coupling_density(lp32, u32.clone(), dims)
    og, lg = m.flows[i].inverse(u32.cuda())
    og, lg = og.cpu().double(), lg.cpu().double()
    d = lambda a, b: (a.double() - b).abs()
    idf, trf = lp32["idf"], lp32["trf"]
    eg, er = d(unroll(og), unroll(o64)), d(unroll(o32), unroll(o64))
    print(f"{i:5d} | {eg[:, idf].max():.2e} {er[:, idf].max():.2e} | {eg[:, trf].max():.2e} {er[:, trf].max():.2e}"
          f" | {d(lg, l64).max():.2e} {d(l32, l64).max():.2e}"
          f" | {d(lg, l64).median():.2e} {d(l32, l64).median():.2e}")
