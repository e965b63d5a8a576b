"""Locate the largest GPU-vs-oracle log q difference on the bench's own proposals:
per chain relative difference, then for the worst chains the per-layer log-det and
latent differences (GPU per-layer API vs oracle per_layer trace) and a float64 oracle
evaluation, to tell float32 noise from a discrepancy."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flow-state_amd"))
sys.path.insert(0, REPO)
from bench import Stepper, synthetic_model, synthetic_states  # noqa: E402
from flowstate.MCMC import BatchedMonteCarlo, Physics  # noqa: E402
from flowstate.models import A1, half_box  # noqa: E402
from oracle import flow as OF  # noqa: E402

N, C, S = 64, 65536, int(os.environ.get("FS_WORST_S", "2048"))
dev = torch.device("cuda")
model = synthetic_model(N, dev)
init, L = synthetic_states(N, C, 0)
bmc = BatchedMonteCarlo(model, init, Physics(L, L), np.arange(42, 42 + C, dtype=np.uint64), device=dev)
st = Stepper(bmc)
for _ in range(3):
    st.step(timed=False)
torch.cuda.synchronize()
cen = st.centered[:S].clone()
lq_gpu = model.log_prob(cen).double().cpu().numpy()
sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
dims = OF.FlowDims(N=N, B=half_box(N), **A1)
lq_o = OF.log_prob(sd, cen.cpu().clone(), dims).double().numpy()
rel = np.abs(lq_gpu - lq_o) / np.abs(lq_o)
order = np.argsort(-rel)[:4]
out = {"S": S, "max_rel": float(rel.max()), "p99_rel": float(np.quantile(rel, 0.99)),
       "median_rel": float(np.median(rel)), "worst": []}
sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
for c in order:
    x = cen[c:c + 1]
    lq64 = float(OF.log_prob(sd64, x.cpu().double(), dims)[0])
    _, _, tr_o = OF.log_prob(sd, x.cpu().clone(), dims, per_layer=True)
    _, _, tr64 = OF.log_prob(sd64, x.cpu().double(), dims, per_layer=True)
    z = x
    layers = []
    for k, i in enumerate(range(dims.L - 1, -1, -1)):
        z, ld = model.flows[i].inverse(z)
        zo, ldo = tr_o[k]
        z64, ld64 = tr64[k]
        layers.append({"layer": i, "ld_gpu": float(ld[0]), "ld_oracle32": float(ldo[0]), "ld_f64": float(ld64[0]),
                       "max_dz_gpu_f64": float((z.double().cpu() - z64).abs().max()),
                       "max_dz_o32_f64": float((zo.double() - z64).abs().max()),
                       "n_near_B": int(((z64.abs() - dims.B).abs() < 1e-4).sum())})
    out["worst"].append({"chain": int(c), "rel": float(rel[c]), "lq_gpu": float(lq_gpu[c]), "lq_o32": float(lq_o[c]),
                         "lq_f64": lq64, "x_absmax": float(x.abs().max()), "layers": layers})
print(json.dumps(out, indent=1))
