"""CircularCoupledRationalQuadraticSpline — parameter holder + HIP execution.

Reference: NF/normflows/flows/neural_spline/wrapper.py:98-275 (layer),
coupling.py:16-368 (coupling + spline parameterisation), nets/resnet.py:7-104
(conditioner), utils/nn.py:64-137 (periodic features), utils/masks.py:4-17.

The module tree reproduces the reference's so that ``state_dict()`` keys,
shapes and dtypes are identical (a reference checkpoint loads with
``strict=True``) and so that, under the same ``torch.manual_seed``, the
parameter initialisation consumes the RNG in the same order.  Execution never
uses these modules' forward(): the whole coupling stack runs in
libflowstate.so from a packed (MFMA-fragment-ordered) copy of the parameters.
"""
import numpy as np
import torch
from torch import nn

from .. import _lib

DEFAULT_MIN_DERIVATIVE = 1e-3  # splines.py:8
# Conditioner GEMM arithmetic of the fused passes (fs_flow_dims.precision, include/flowstate.h):
#   "f32"    the reference's float32 products and sums (exact-f32 MFMA), the default;
#   "bf16x6" f32 operands as three bf16 planes, the six plane products above 2^-24 (f32-level error);
#   "bf16x3" two planes, three products (16 significant bits per operand).
PRECISIONS = {"f32": 0, "bf16x6": 1, "bf16x3": 2}


def _alternating_mask(features, even):
    """create_alternating_binary_mask (masks.py:4-17)."""
    mask = torch.zeros(features).byte()
    mask[(0 if even else 1)::2] += 1
    return mask


class _PeriodicFeaturesElementwise(nn.Module):
    """Buffers/parameter of PeriodicFeaturesElementwise (nn.py:64-118); the fork's
    forward is cos/sin of scale*x over all identity features (nn.py:120-137)."""

    def __init__(self, ndim, ind, scale):
        super().__init__()
        self.ndim = ndim
        self.register_buffer("ind", torch.tensor(list(ind), dtype=torch.long))
        ind_ = [i for i in range(ndim) if i not in set(int(v) for v in self.ind)]
        self.register_buffer("ind_", torch.tensor(ind_, dtype=torch.long))
        perm = torch.cat((self.ind, self.ind_))
        inv = torch.zeros_like(perm)
        for i in range(ndim):
            inv[perm[i]] = i
        self.register_buffer("inv_perm", inv)
        self.weights = nn.Parameter(torch.ones(len(self.ind), 2))
        self.scale = scale


class _ResidualBlock(nn.Module):
    """Parameter layout of ResidualBlock (resnet.py:7-50), BatchNorm eps 1e-3."""

    def __init__(self, features):
        super().__init__()
        self.batch_norm_layers = nn.ModuleList([nn.BatchNorm1d(features, eps=1e-3) for _ in range(2)])
        self.linear_layers = nn.ModuleList([nn.Linear(features, features) for _ in range(2)])
        nn.init.uniform_(self.linear_layers[-1].weight, -1e-3, 1e-3)
        nn.init.uniform_(self.linear_layers[-1].bias, -1e-3, 1e-3)


class _ResidualNet(nn.Module):
    """Parameter layout of ResidualNet (resnet.py:53-104) with preprocessing."""

    def __init__(self, in_features, out_features, hidden_features, num_blocks, preprocessing):
        super().__init__()
        self.hidden_features = hidden_features
        self.preprocessing = preprocessing
        self.initial_layer = nn.Linear(in_features, hidden_features)
        self.blocks = nn.ModuleList([_ResidualBlock(hidden_features) for _ in range(num_blocks)])
        self.final_layer = nn.Linear(hidden_features, out_features)


class _PiecewiseRationalQuadraticCDF(nn.Module):
    """Unconditional spline parameters (coupling.py:176-221), identity init,
    list-valued tails -> K+1 derivatives."""

    def __init__(self, features, num_bins):
        super().__init__()
        self.unnormalized_widths = nn.Parameter(torch.zeros(features, num_bins))
        self.unnormalized_heights = nn.Parameter(torch.zeros(features, num_bins))
        c = np.log(np.exp(1 - DEFAULT_MIN_DERIVATIVE) - 1)
        self.unnormalized_derivatives = nn.Parameter(c * torch.ones(features, num_bins + 1))


class _PRQCoupling(nn.Module):
    """PiecewiseRationalQuadraticCoupling (coupling.py:268-368) parameter layout."""

    def __init__(self, num_input_channels, num_blocks, num_hidden_channels, num_bins, tail_bound, mask):
        super().__init__()
        fv = torch.arange(num_input_channels)
        self.register_buffer("identity_features", fv.masked_select(mask <= 0))
        self.register_buffer("transform_features", fv.masked_select(mask > 0))
        n_id = len(self.identity_features)
        n_tr = len(self.transform_features)
        pf = _PeriodicFeaturesElementwise(n_id, list(range(n_id)), np.pi / tail_bound)
        self.transform_net = _ResidualNet(2 * n_id, n_tr * (3 * num_bins + 1), num_hidden_channels,
                                          num_blocks, pf)
        nn.init.constant_(self.transform_net.final_layer.weight, 0.0)
        nn.init.constant_(self.transform_net.final_layer.bias, np.log(np.exp(1 - DEFAULT_MIN_DERIVATIVE) - 1))
        self.unconditional_transform = _PiecewiseRationalQuadraticCDF(n_id, num_bins)


class CircularCoupledRationalQuadraticSpline(nn.Module):
    """Same constructor signature as the reference (wrapper.py:103-119).

    Supported configuration (the one every driver uses): residual conditioner,
    all coordinates circular, alternating mask, no context, no dropout in
    eval.  Anything else raises instead of silently computing something else.
    """

    def __init__(self, num_input_channels, num_blocks, num_hidden_channels, ind_circ, num_heads=4,
                 num_context_channels=None, num_bins=8, tail_bound=3.0, net_type="residual",
                 activation=nn.ReLU, dropout_probability=0.0, reverse_mask=False, mask=None,
                 init_identity=True):
        super().__init__()
        if num_context_channels is not None:
            raise NotImplementedError("context channels are not on the hot path")
        if net_type != "residual":
            raise NotImplementedError(f"net_type={net_type!r}: only the residual conditioner is built")
        if torch.is_tensor(tail_bound):
            raise NotImplementedError("per-coordinate tail bounds are not on the hot path")
        if sorted(int(i) for i in ind_circ) != list(range(num_input_channels)):
            raise NotImplementedError("all coordinates must be circular (main_algorithm_1.py:282-283)")
        if activation is not nn.ReLU:
            raise NotImplementedError("ReLU conditioner only (wrapper.py:113)")
        if num_input_channels % 2:
            raise NotImplementedError("odd flow dimension: the half-roll is not invertible (SURVEY §4)")
        if mask is None:
            mask = _alternating_mask(num_input_channels, even=reverse_mask)
        if reverse_mask or not torch.equal(torch.as_tensor(mask), _alternating_mask(num_input_channels, False)):
            raise NotImplementedError("only the default alternating mask (even=False) is built")
        self.num_input_channels = num_input_channels
        self.num_blocks = num_blocks
        self.num_hidden_channels = num_hidden_channels
        self.num_bins = num_bins
        self.tail_bound = float(tail_bound)
        self.dropout_probability = dropout_probability
        self.prqct = _PRQCoupling(num_input_channels, num_blocks, num_hidden_channels, num_bins,
                                  self.tail_bound, mask)
        if not init_identity:
            raise NotImplementedError("init_identity=False is not used by the drivers")

    # -- raw canonical buffer (include/flowstate.h: fs_flow_raw_floats) ------------
    def raw_param_tensors(self):
        t = self.prqct.transform_net
        out = [t.initial_layer.weight, t.initial_layer.bias]
        for blk in t.blocks:
            for i in range(2):
                bn = blk.batch_norm_layers[i]
                out += [bn.weight, bn.bias, bn.running_mean, bn.running_var]
                lin = blk.linear_layers[i]
                out += [lin.weight, lin.bias]
        out += [t.final_layer.weight, t.final_layer.bias]
        u = self.prqct.unconditional_transform
        out += [u.unnormalized_widths, u.unnormalized_heights, u.unnormalized_derivatives]
        return out

    def dims(self, L=1):
        d = _lib.FlowDims()
        d.N = self.num_input_channels // 2
        d.L = L
        d.H = self.num_hidden_channels
        d.nb = self.num_blocks
        d.K = self.num_bins
        d.precision = PRECISIONS[getattr(self, "_fs_precision", "f32")]
        d.tail_bound = self.tail_bound
        return d

    def same_shape(self, other):
        return (self.num_input_channels, self.num_blocks, self.num_hidden_channels, self.num_bins,
                self.tail_bound) == (other.num_input_channels, other.num_blocks, other.num_hidden_channels,
                                      other.num_bins, other.tail_bound)

    # -- per-layer API (wrapper.py:269-275) -------------------------------------
    def forward(self, z, context=None):
        """Sampling direction (= prqct.inverse = Coupling.inverse): (z, log_det)."""
        from .core import _run_stack
        return _run_stack([self], z, direction="forward")

    def inverse(self, z, context=None):
        """Density direction (= prqct = Coupling.forward): (z, log_det)."""
        from .core import _run_stack
        return _run_stack([self], z, direction="inverse")
