"""ORACLE (test infrastructure only): torch-CPU float32 restatement of the
circular rational-quadratic-spline coupling flow on the hot path.

Written against a reference-format ``state_dict`` (keys of
NF/normflows/flows/neural_spline/wrapper.py:98-275 modules), so the same
tensors drive the reference, this oracle and the HIP product.  The op
sequence (and the masked-select shapes) follow the reference so that torch's
CPU kernels see the same shapes and the restatement is bit-identical to the
reference on CPU (pinned by tests/test_oracle_golden.py).

References (paths relative to the reference root):
  rqs_core            NF/normflows/utils/splines.py:91-222
  rqs (circular tails) NF/normflows/utils/splines.py:16-88 (branch :35-39)
  conditioner          NF/normflows/nets/resnet.py:7-104, utils/nn.py:120-137
  coupling_density     NF/normflows/flows/neural_spline/coupling.py:71-102, 156-170, 335-368
  coupling_sample      NF/normflows/flows/neural_spline/coupling.py:104-134
  log_prob             NF/normflows/core.py:198-214 + Energy/Uniform.py:50-74
  sample (given z)     NF/normflows/core.py:178-196
"""
import math
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F

MIN_W = 1e-3  # splines.py:6-8
MIN_H = 1e-3
MIN_D = 1e-3


@dataclass
class FlowDims:
    N: int   # particles; D = 2N
    L: int   # coupling layers
    H: int   # hidden units
    nb: int  # residual blocks
    K: int   # spline bins
    B: float  # tail bound = HALF_BOX

    @property
    def D(self):
        return 2 * self.N


def dims_from_state_dict(sd, tail_bound):
    L = 1 + max(int(k.split(".")[1]) for k in sd if k.startswith("flows."))
    p = "flows.0.prqct."
    N = sd[p + "identity_features"].numel()
    H = sd[p + "transform_net.initial_layer.weight"].shape[0]
    nb = len({k.split(".")[5] for k in sd if k.startswith(p + "transform_net.blocks.")})
    K = sd[p + "unconditional_transform.unnormalized_widths"].shape[1]
    return FlowDims(N=N, L=L, H=H, nb=nb, K=K, B=float(tail_bound))


def rqs_core(x, uw, uh, ud, left, right, bottom, top, inverse):
    """rational_quadratic_spline (splines.py:91-222), float32."""
    K = uw.shape[-1]
    w = F.softmax(uw, dim=-1)
    w = MIN_W + (1 - MIN_W * K) * w
    cw = torch.cumsum(w, dim=-1)
    cw = F.pad(cw, pad=(1, 0), mode="constant", value=0.0)
    cw = (right - left) * cw + left
    cw[..., 0] = left
    cw[..., -1] = right
    w = cw[..., 1:] - cw[..., :-1]

    d = MIN_D + F.softplus(ud)

    h = F.softmax(uh, dim=-1)
    h = MIN_H + (1 - MIN_H * K) * h
    ch = torch.cumsum(h, dim=-1)
    ch = F.pad(ch, pad=(1, 0), mode="constant", value=0.0)
    ch = (top - bottom) * ch + bottom
    ch[..., 0] = bottom
    ch[..., -1] = top
    h = ch[..., 1:] - ch[..., :-1]

    knots = ch if inverse else cw
    knots[..., -1] += 1e-6  # searchsorted eps, in place (splines.py:11-13)
    b = (torch.sum(x[..., None] >= knots, dim=-1) - 1)[..., None]

    icw = cw.gather(-1, b)[..., 0]
    ibw = w.gather(-1, b)[..., 0]
    ich = ch.gather(-1, b)[..., 0]
    delta = h / w
    idl = delta.gather(-1, b)[..., 0]
    id0 = d.gather(-1, b)[..., 0]
    id1 = d[..., 1:].gather(-1, b)[..., 0]
    ih = h.gather(-1, b)[..., 0]

    if inverse:
        s = id0 + id1 - 2 * idl
        a = (x - ich) * s + ih * (idl - id0)
        bb = ih * id0 - (x - ich) * s
        c = -idl * (x - ich)
        disc = abs(bb.pow(2) - 4 * a * c)
        if torch.isnan(disc).any():
            raise ValueError("Discriminant computation resulted in NaN.")
        root = (2 * c) / (-bb - torch.sqrt(disc))
        out = root * ibw + icw
        tomt = root * (1 - root)
        den = idl + (id0 + id1 - 2 * idl) * tomt
        dnum = idl.pow(2) * (id1 * root.pow(2) + 2 * idl * tomt + id0 * (1 - root).pow(2))
        lad = torch.log(dnum) - 2 * torch.log(den)
        return out, -lad, b[..., 0]
    theta = (x - icw) / ibw
    tomt = theta * (1 - theta)
    num = ih * (idl * theta.pow(2) + id0 * tomt)
    den = idl + (id0 + id1 - 2 * idl) * tomt
    out = ich + num / den
    dnum = idl.pow(2) * (id1 * theta.pow(2) + 2 * idl * tomt + id0 * (1 - theta).pow(2))
    lad = torch.log(dnum) - 2 * torch.log(den)
    return out, lad, b[..., 0]


def rqs(x, uw, uh, ud, B, inverse, return_bins=False):
    """unconstrained_rational_quadratic_spline, circular-tail branch (splines.py:16-88).

    ud has K+1 columns; the circular pad writes index K+1, which is never read
    (only bin and bin+1 <= K are gathered) — reproduced as-is.
    """
    inside = (x >= -B) & (x <= B)
    outside = ~inside
    out = torch.zeros_like(x)
    lad = torch.zeros_like(x)
    ud_ = F.pad(ud, pad=(0, 1))
    ud_[..., -1] = ud_[..., 0]
    out[outside] = x[outside]
    lad[outside] = 0
    o, l, b = rqs_core(x[inside], uw[inside, :], uh[inside, :], ud_[inside, :],
                       -B, B, -B, B, inverse)
    out[inside] = o
    lad[inside] = l
    if return_bins:
        bins = torch.full_like(x, -1, dtype=torch.long)
        bins[inside] = b
        return out, lad, bins
    return out, lad


def layer_params(sd, i):
    p = f"flows.{i}.prqct."
    g = lambda k: sd[p + k]
    blocks = []
    nb = len({k.split(".")[5] for k in sd if k.startswith(p + "transform_net.blocks.")})
    for j in range(nb):
        q = f"transform_net.blocks.{j}."
        blocks.append(dict(
            bn0=[g(q + f"batch_norm_layers.0.{n}") for n in ("running_mean", "running_var", "weight", "bias")],
            lin0=(g(q + "linear_layers.0.weight"), g(q + "linear_layers.0.bias")),
            bn1=[g(q + f"batch_norm_layers.1.{n}") for n in ("running_mean", "running_var", "weight", "bias")],
            lin1=(g(q + "linear_layers.1.weight"), g(q + "linear_layers.1.bias")),
        ))
    return dict(
        idf=g("identity_features"), trf=g("transform_features"),
        w_in=g("transform_net.initial_layer.weight"), b_in=g("transform_net.initial_layer.bias"),
        blocks=blocks,
        w_f=g("transform_net.final_layer.weight"), b_f=g("transform_net.final_layer.bias"),
        uw=g("unconditional_transform.unnormalized_widths"),
        uh=g("unconditional_transform.unnormalized_heights"),
        ud=g("unconditional_transform.unnormalized_derivatives"),
    )


def conditioner(lp, ident, B):
    """ResidualNet (resnet.py:92-104) with PeriodicFeaturesElementwise (nn.py:120-137)."""
    scale = np.pi / B
    t = torch.cat([torch.cos(scale * ident), torch.sin(scale * ident)], dim=-1)
    t = F.linear(t, lp["w_in"], lp["b_in"])
    for blk in lp["blocks"]:
        m, v, w, b = blk["bn0"]
        u = F.batch_norm(t, m, v, w, b, training=False, momentum=0.0, eps=1e-3)
        u = F.relu(u)
        u = F.linear(u, *blk["lin0"])
        m, v, w, b = blk["bn1"]
        u = F.batch_norm(u, m, v, w, b, training=False, momentum=0.0, eps=1e-3)
        u = F.relu(u)
        u = F.linear(u, *blk["lin1"])
        t = t + u
    return F.linear(t, lp["w_f"], lp["b_f"])


def _cond_spline(lp, trans, params, H, K, B, inverse):
    b, d = trans.shape
    params = params.reshape(b, d, -1)
    uw = params[..., :K]
    uh = params[..., K:2 * K]
    ud = params[..., 2 * K:]
    uw /= np.sqrt(H)
    uh /= np.sqrt(H)
    out, lad = rqs(trans, uw, uh, ud, B, inverse)
    return out, torch.sum(lad, dim=[1])


def _uncond_spline(lp, ident, B, inverse):
    n = ident.shape[0]
    uw = lp["uw"][None, ...].expand(n, *lp["uw"].shape)
    uh = lp["uh"][None, ...].expand(n, *lp["uh"].shape)
    ud = lp["ud"][None, ...].expand(n, *lp["ud"].shape)
    out, lad = rqs(ident, uw, uh, ud, B, inverse)
    return out, torch.sum(lad, dim=[1])


def coupling_density(lp, u, dims):
    """Coupling.forward (coupling.py:71-102) == CircularCoupled...inverse (wrapper.py:273-275)."""
    ident = u[:, lp["idf"]]
    trans = u[:, lp["trf"]]
    params = conditioner(lp, ident, dims.B)
    trans, lad = _cond_spline(lp, trans, params, dims.H, dims.K, dims.B, inverse=False)
    ident, lad_u = _uncond_spline(lp, ident, dims.B, inverse=False)
    lad = lad + lad_u
    out = torch.empty_like(u)
    out[:, lp["idf"]] = ident
    out[:, lp["trf"]] = trans
    split = int(dims.D / 2)
    return torch.cat([out[:, split:], out[:, :split]], dim=1), lad


def coupling_sample(lp, u, dims):
    """Coupling.inverse (coupling.py:104-134) == CircularCoupled...forward (wrapper.py:269-271)."""
    split = int(dims.D / 2)
    u = torch.cat([u[:, split:], u[:, :split]], dim=1)
    ident = u[:, lp["idf"]]
    trans = u[:, lp["trf"]]
    ident, lad = _uncond_spline(lp, ident, dims.B, inverse=True)
    params = conditioner(lp, ident, dims.B)
    trans, lad_s = _cond_spline(lp, trans, params, dims.H, dims.K, dims.B, inverse=True)
    lad = lad + lad_s
    out = torch.empty_like(u)
    out[:, lp["idf"]] = ident
    out[:, lp["trf"]] = trans
    return out, lad


def base_log_prob(z, dims):
    """UniformParticle.log_prob (Energy/Uniform.py:50-74)."""
    inb = ((z >= -dims.B) & (z <= dims.B)).all(dim=1)
    const = -dims.D * torch.log(torch.tensor(2 * dims.B))
    lp = torch.full((z.size(0),), const, device=z.device, dtype=z.dtype)
    lp[~inb] = -float("inf")
    return lp


@torch.no_grad()
def log_prob(sd, x, dims, per_layer=False):
    """NormalizingFlow.log_prob (core.py:198-214): layers L-1..0 in the density direction."""
    lps = [layer_params(sd, i) for i in range(dims.L)]
    log_q = torch.zeros(len(x), dtype=x.dtype, device=x.device)
    z = x
    trace = []
    for i in range(dims.L - 1, -1, -1):
        z, ld = coupling_density(lps[i], z, dims)
        log_q += ld.view(-1)
        if per_layer:
            trace.append((z.clone(), ld.clone()))
    log_q += base_log_prob(z, dims)
    if per_layer:
        return log_q, z, trace
    return log_q


@torch.no_grad()
def sample_from(sd, z, dims, with_logdet=False):
    """NormalizingFlow.sample (core.py:178-196) with the base draw z supplied."""
    lps = [layer_params(sd, i) for i in range(dims.L)]
    ld_tot = torch.zeros(len(z), dtype=z.dtype)
    for i in range(dims.L):
        z, ld = coupling_sample(lps[i], z, dims)
        ld_tot += ld.view(-1)
    if with_logdet:
        return z, ld_tot
    return z


def flops_per_pass(dims):
    """Conditioner GEMM FLOP per chain per pass."""
    N, H, nb, K, L = dims.N, dims.H, dims.nb, dims.K, dims.L
    return 2 * L * (2 * N * H + 2 * nb * H * H + H * N * (3 * K + 1))


def half_box(N, rho=0.03, dim=2):
    """HALF_BOX of main_algorithm_1.py:50."""
    return ((N / rho) ** (1 / dim)) / 2


def random_state_dict(dims, seed=0, final_std=0.01, uncond_std=0.3):
    """Seeded reference-format weights (the SURVEY §8(d) synthetic recipe).

    Produces exactly the keys/shapes/dtypes of the reference model's
    state_dict (NormalizingFlow of CircularCoupledRationalQuadraticSpline
    layers, wrapper.py:98-275): nn.Linear-style U(+-1/sqrt(fan_in)) weights,
    the residual blocks' second linear U(+-1e-3) (resnet.py:33-35), final
    layers N(0, final_std) on top of the identity-init bias (wrapper.py:181-185),
    unconditional widths/heights N(0, uncond_std), and mildly perturbed
    BatchNorm affine/running statistics so the eval-mode BN is exercised.
    Final/unconditional perturbations keep log_prob from being the constant
    -D*log(2B) of the identity initialisation.
    """
    N, L, H, nb, K, D = dims.N, dims.L, dims.H, dims.nb, dims.K, dims.D
    g = torch.Generator().manual_seed(int(seed))
    U = lambda shape, a: (torch.rand(shape, generator=g) * 2 - 1) * a
    Nrm = lambda shape, s: torch.randn(shape, generator=g) * s
    id_bias = float(np.log(np.exp(1 - MIN_D) - 1))
    sd = {}
    for i in range(L):
        p = f"flows.{i}.prqct."
        sd[p + "identity_features"] = torch.arange(D)[0::2].clone()
        sd[p + "transform_features"] = torch.arange(D)[1::2].clone()
        q = p + "transform_net."
        sd[q + "preprocessing.weights"] = torch.ones(N, 2)
        sd[q + "preprocessing.ind"] = torch.arange(N)
        sd[q + "preprocessing.ind_"] = torch.zeros(0, dtype=torch.long)
        sd[q + "preprocessing.inv_perm"] = torch.arange(N)
        sd[q + "initial_layer.weight"] = U((H, D), 1 / math.sqrt(D))
        sd[q + "initial_layer.bias"] = U((H,), 1 / math.sqrt(D))
        for j in range(nb):
            r = q + f"blocks.{j}."
            for t in range(2):
                sd[r + f"batch_norm_layers.{t}.weight"] = 1.0 + Nrm((H,), 0.05)
                sd[r + f"batch_norm_layers.{t}.bias"] = Nrm((H,), 0.05)
                sd[r + f"batch_norm_layers.{t}.running_mean"] = Nrm((H,), 0.05)
                sd[r + f"batch_norm_layers.{t}.running_var"] = 1.0 + torch.rand((H,), generator=g) * 0.2
                sd[r + f"batch_norm_layers.{t}.num_batches_tracked"] = torch.tensor(0)
            sd[r + "linear_layers.0.weight"] = U((H, H), 1 / math.sqrt(H))
            sd[r + "linear_layers.0.bias"] = U((H,), 1 / math.sqrt(H))
            sd[r + "linear_layers.1.weight"] = U((H, H), 1e-3)
            sd[r + "linear_layers.1.bias"] = U((H,), 1e-3)
        sd[q + "final_layer.weight"] = Nrm((N * (3 * K + 1), H), final_std)
        sd[q + "final_layer.bias"] = id_bias + Nrm((N * (3 * K + 1),), 0.05)
        u = p + "unconditional_transform."
        sd[u + "unnormalized_widths"] = Nrm((N, K), uncond_std)
        sd[u + "unnormalized_heights"] = Nrm((N, K), uncond_std)
        sd[u + "unnormalized_derivatives"] = id_bias + Nrm((N, K + 1), uncond_std)
    return sd
