"""Where the GPU's float32 log q error against the exact value comes from.

On S flow samples prepared as the bench prepares them (the fused step's own proposals,
fl32(config - half_width)), A1 flow, N=64:
  gpu      the fused density pass (the product);
  f64      the oracle in float64 (the exact value), with its per-layer, per-feature
           log-dets along the exact trajectory;
  emu32    those exact per-feature log-dets, each rounded to float32, summed in the fused
           kernel's float32 order (per wave: the layer's conditional features j = w, w+8, ..,
           then its unconditional partial; waves summed in order; + the float32 base term):
           the error the float32 ACCUMULATION alone makes;
  emu64    the same terms summed in double, + the double base term;
  layers   the GPU's per-layer API (one L=1 launch per layer, its latents), each layer's
           log-det against the float64 layer evaluated on the GPU's own input latent
           (local error) and against the exact trajectory (propagated latent error).
Prints a JSON summary (quantiles of |log q|, and of each error relative to |log q|).
Test infrastructure only: imports the oracle.  FLOWSTATE_LIB selects a variant build."""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flow-state_amd"))
sys.path.insert(0, REPO)
from bench import Stepper, decorrelate, synthetic_model, synthetic_states  # noqa: E402
from flowstate.MCMC import BatchedMonteCarlo, Physics  # noqa: E402
from flowstate.models import A1, half_box  # noqa: E402
from oracle import flow as OF  # noqa: E402

N, C, S = 64, 65536, int(os.environ.get("FS_SPLIT_S", "8192"))
dev = torch.device("cuda")
model = synthetic_model(N, dev)
init, L = synthetic_states(N, C, 0)
bmc = BatchedMonteCarlo(model, init, Physics(L, L), np.arange(42, 42 + C, dtype=np.uint64), device=dev)
decorrelate(bmc)
st = Stepper(bmc)
for _ in range(3):
    st.step(timed=False)
torch.cuda.synchronize()
cen = st.centered[:S].clone()
lq_gpu = model.log_prob(cen).double().cpu().numpy()

sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
dims = OF.FlowDims(N=N, B=half_box(N), **A1)
lps = [OF.layer_params(sd64, i) for i in range(dims.L)]


def layer_terms(lp, u):
    """coupling_density (oracle) in float64 with the per-feature log-dets kept."""
    ident, trans = u[:, lp["idf"]], u[:, lp["trf"]]
    params = OF.conditioner(lp, ident, dims.B).reshape(len(u), N, -1)
    K, H = dims.K, dims.H
    uw, uh, ud = params[..., :K] / np.sqrt(H), params[..., K:2 * K] / np.sqrt(H), params[..., 2 * K:]
    t_out, lc = OF.rqs(trans, uw, uh, ud, dims.B, inverse=False)
    n = len(u)
    i_out, lu = OF.rqs(ident, lp["uw"][None].expand(n, *lp["uw"].shape), lp["uh"][None].expand(n, *lp["uh"].shape),
                       lp["ud"][None].expand(n, *lp["ud"].shape), dims.B, inverse=False)
    out = torch.empty_like(u)
    out[:, lp["idf"]] = i_out
    out[:, lp["trf"]] = t_out
    return torch.cat([out[:, N:], out[:, :N]], dim=1), lc, lu


t0 = time.perf_counter()
z = cen.cpu().double()
cond, unc, traj = [], [], []
with torch.no_grad():
    for i in range(dims.L - 1, -1, -1):
        traj.append(z)
        z, lc, lu = layer_terms(lps[i], z)
        cond.append(lc.numpy())
        unc.append(lu.numpy())
inb = ((z >= -dims.B) & (z <= dims.B)).all(dim=1).numpy()
base64 = -dims.D * np.log(2 * dims.B)
base32 = np.float32(-dims.D * np.float32(np.log(np.float32(2 * dims.B))))
lq64 = sum(c.sum(1) + u.sum(1) for c, u in zip(cond, unc)) + np.where(inb, base64, -np.inf)

# the fused kernel's float32 accumulation order over the exact terms
f = np.float32
ldw = np.zeros((8, S), f)
for c, u in zip(cond, unc):
    c32, u32 = c.astype(f), u.astype(f)
    for w in range(8):
        for j in range(w, N, 8):
            ldw[w] = ldw[w] + c32[:, j]
        part = np.zeros(S, f)
        for j in range(w, N, 8):
            part = part + u32[:, j]
        ldw[w] = ldw[w] + part
tot = np.zeros(S, f)
for w in range(8):
    tot = tot + ldw[w]
emu32 = (tot + base32).astype(np.float64)
emu64 = sum(c.astype(f).astype(np.float64).sum(1) + u.astype(f).astype(np.float64).sum(1)
            for c, u in zip(cond, unc)) + base64

# per-layer: the GPU's own latents, local vs propagated error
zg = cen
local = np.zeros(S)
prop = np.zeros(S)
ldsum_gpu = np.zeros(S)
zulp_id, zulp_tr = [], []  # identity (unconditional spline) / transform (conditional) features
zulp = []  # per layer: |z_out(GPU) - z_out(f64, GPU's input)| in ulps of the f32 output
with torch.no_grad():
    for k, i in enumerate(range(dims.L - 1, -1, -1)):
        zin = zg.double().cpu()
        zg, ldg = model.flows[i].inverse(zg)
        z64o, lc, lu = layer_terms(lps[i], zin)
        zo = zg.cpu().numpy()
        u = np.spacing(np.abs(zo).astype(np.float32)).astype(np.float64)
        e = np.abs(zo.astype(np.float64) - z64o.numpy()) / u
        e = np.concatenate([e[:, N:], e[:, :N]], 1)  # un-roll: the layer's own feature order
        zulp.append(e)
        zulp_id.append(e[:, lps[i]["idf"].numpy()])
        zulp_tr.append(e[:, lps[i]["trf"].numpy()])
        loc64 = (lc.sum(1) + lu.sum(1)).numpy()
        ldg = ldg.double().cpu().numpy()
        ldsum_gpu += ldg
        local += ldg - loc64
        prop += loc64 - (cond[k].sum(1) + unc[k].sum(1))
t_o = time.perf_counter() - t0

fin = np.isfinite(lq64) & np.isfinite(lq_gpu)
a = np.abs(lq64[fin])


def q(x):
    x = np.abs(x[fin]) / a
    return {"max": float(x.max()), "p999": float(np.quantile(x, 0.999)), "p99": float(np.quantile(x, 0.99)),
            "median": float(np.median(x)), "beyond_1e-5": int((x > 1e-5).sum())}


worst = np.argsort(-(np.abs(lq_gpu - lq64) / np.abs(lq64)))[:8]
out = {"S": S, "rows": int(fin.sum()), "lib": os.environ.get("FLOWSTATE_LIB", "default"),
       "abs_log_q": {"min": float(a.min()), "median": float(np.median(a)), "max": float(a.max())},
       "gpu_vs_f64": q(lq_gpu - lq64),
       "emu32_accumulation_vs_f64_sum": q(emu32 - emu64),
       "base_term_f32_abs_err": float(base32 - base64),
       "gpu_layer_api_local": q(local),
       "gpu_layer_api_propagated": q(prop),
       "gpu_fused_vs_layer_api_sum": q(lq_gpu - (ldsum_gpu + base64)),
       "layer_z_out_err_ulps": {"what": "GPU layer output vs the float64 layer on the GPU's own input, in ulps of "
                                        "the float32 output (0.5 = correctly rounded)",
                                "mean": float(np.mean(zulp)), "p99": float(np.quantile(np.concatenate(zulp), 0.99)),
                                "max": float(np.max(zulp)),
                                "frac_above_half_ulp": float(np.mean(np.concatenate(zulp) > 0.5)),
                                "identity_mean": float(np.mean(zulp_id)), "transform_mean": float(np.mean(zulp_tr)),
                                "identity_p99": float(np.quantile(np.concatenate(zulp_id), 0.99)),
                                "transform_p99": float(np.quantile(np.concatenate(zulp_tr), 0.99))},
       "worst": [{"row": int(r), "rel": float(abs(lq_gpu[r] - lq64[r]) / abs(lq64[r])), "lq64": float(lq64[r]),
                  "err_gpu": float(lq_gpu[r] - lq64[r]), "err_emu32": float(emu32[r] - emu64[r]),
                  "local": float(local[r]), "prop": float(prop[r]),
                  "fused_vs_layers": float(lq_gpu[r] - ldsum_gpu[r] - base64)} for r in worst],
       "oracle_s": t_o}
print(json.dumps(out, indent=1))
