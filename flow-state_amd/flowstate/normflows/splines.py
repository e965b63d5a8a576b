"""Drop-in for ``normflows.utils.splines`` on the hot path (reference:
NF/normflows/utils/splines.py:16-222): the circular-tail rational-quadratic spline
as one fused HIP kernel each way (csrc/spline_autograd.hip, fs_rqs_forward /
fs_rqs_backward), differentiable.

Only what the path uses is supported, and everything else raises instead of computing
something different: ``tails`` a list/tuple whose first entry is "circular" (the
circular branch, splines.py:35-39: identity and log-det 0 outside [-tail_bound,
tail_bound]; the derivative pad ties nothing, index K+1 is never read), the default
minimum bin width / height / derivative (1e-3), K in the instantiated set, device tensors.
"""
import torch

from . import autograd_flow as AF

DEFAULT_MIN_BIN_WIDTH = 1e-3  # splines.py:6-8
DEFAULT_MIN_BIN_HEIGHT = 1e-3
DEFAULT_MIN_DERIVATIVE = 1e-3


def unconstrained_rational_quadratic_spline(inputs, unnormalized_widths, unnormalized_heights,
                                            unnormalized_derivatives, inverse=False, tails="linear",
                                            tail_bound=1.0, min_bin_width=DEFAULT_MIN_BIN_WIDTH,
                                            min_bin_height=DEFAULT_MIN_BIN_HEIGHT,
                                            min_derivative=DEFAULT_MIN_DERIVATIVE):
    """splines.py:16-88 with circular tails: (outputs, logabsdet), both shaped like inputs.
    unnormalized_widths / _heights: [..., K]; unnormalized_derivatives: [..., K+1]."""
    if isinstance(tails, str) or not len(tails) or tails[0] != "circular":
        raise NotImplementedError("flowstate supports the circular tails of the hot path only "
                                  "(CircularCoupledRationalQuadraticSpline); got tails=%r" % (tails,))
    if (min_bin_width, min_bin_height, min_derivative) != (DEFAULT_MIN_BIN_WIDTH, DEFAULT_MIN_BIN_HEIGHT,
                                                           DEFAULT_MIN_DERIVATIVE):
        raise NotImplementedError("non-default minimum bin width / height / derivative")
    K = unnormalized_widths.shape[-1]
    if unnormalized_heights.shape[-1] != K or unnormalized_derivatives.shape[-1] != K + 1:
        raise ValueError("widths / heights need K entries and derivatives K+1 (circular tails)")
    if not inputs.is_cuda:
        raise RuntimeError("flowstate's spline runs on the device (fs_rqs_forward); move the tensors to cuda")
    if K not in AF._HIP_K:
        raise NotImplementedError(f"K={K}: instantiated spline bin counts are {AF._HIP_K}")
    out, lad = AF.circular_rqs(inputs, unnormalized_widths, unnormalized_heights, unnormalized_derivatives,
                               float(tail_bound), bool(inverse))
    AF.check_nan_flags()  # splines.py:176-183 raises on a NaN discriminant
    return out, lad
