"""Differentiable (PyTorch autograd) coupling-layer math for training (SURVEY §8(f)
row 4: Algorithm 2's forward_kld / reverse_kld, hybrid_NF_MCMC/main_algorithm_2.py:314-331).

Training needs gradients and train-mode BatchNorm (batch statistics + running
statistics updates), which the fused inference kernels (eval mode, forward only)
do not provide.  This module evaluates the same layers with torch ops on the
layers' own nn.Modules (nn.Linear / nn.BatchNorm1d, so train/eval semantics and
running-statistics updates are torch's), on the device the parameters live on
(PyTorch-ROCm on MI355X: hipBLASLt GEMMs + elementwise kernels).  After an
optimizer step the inference kernels pick the new parameters up through the
packed-image cache (tensor version counters).

Reference math (paths relative to the reference root):
  Coupling.forward / inverse          NF/normflows/flows/neural_spline/coupling.py:71-134
  _piecewise_cdf (/ sqrt(H) scaling)   coupling.py:335-368
  PiecewiseRationalQuadraticCDF       coupling.py:176-265 (K+1 derivatives, shared over the batch)
  unconstrained RQS, circular branch  NF/normflows/utils/splines.py:16-88
  rational_quadratic_spline           splines.py:91-222
  ResidualNet / ResidualBlock         NF/normflows/nets/resnet.py:7-104 (dropout p = 0)
  PeriodicFeaturesElementwise         NF/normflows/utils/nn.py:120-137
"""
import ctypes

import os

import numpy as np
import torch
import torch.nn.functional as F

MIN_BIN_WIDTH = 1e-3  # splines.py:6-8
MIN_BIN_HEIGHT = 1e-3
MIN_DERIVATIVE = 1e-3


def _knots(unnorm, min_size, lo, hi):
    """softmax -> min-size affine -> cumsum -> [lo, hi] with pinned ends (splines.py:117-127)."""
    K = unnorm.shape[-1]
    s = F.softmax(unnorm, dim=-1)
    s = min_size + (1 - min_size * K) * s
    c = torch.cumsum(s, dim=-1)
    c = F.pad(c, pad=(1, 0), mode="constant", value=0.0)
    c = (hi - lo) * c + lo
    c = torch.cat([torch.full_like(c[..., :1], lo), c[..., 1:-1], torch.full_like(c[..., :1], hi)], dim=-1)
    return c, c[..., 1:] - c[..., :-1]


def rational_quadratic_spline(x, uw, uh, ud, inverse, left, right, bottom, top):
    """splines.py:91-222 (inputs already inside [left, right])."""
    cw, w = _knots(uw, MIN_BIN_WIDTH, left, right)
    d = MIN_DERIVATIVE + F.softplus(ud)
    ch, h = _knots(uh, MIN_BIN_HEIGHT, bottom, top)
    knots = (ch if inverse else cw).detach().clone()
    knots[..., -1] += 1e-6  # searchsorted eps (splines.py:11-13)
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
        disc = torch.abs(bb.pow(2) - 4 * a * c)
        _nan_flags.append(torch.isnan(disc).any())  # splines.py:176-183, raised after the pass
        root = (2 * c) / (-bb - torch.sqrt(disc))
        out = root * ibw + icw
        tomt = root * (1 - root)
        den = idl + (id0 + id1 - 2 * idl) * tomt
        dnum = idl.pow(2) * (id1 * root.pow(2) + 2 * idl * tomt + id0 * (1 - root).pow(2))
        return out, -(torch.log(dnum) - 2 * torch.log(den))
    theta = (x - icw) / ibw
    tomt = theta * (1 - theta)
    num = ih * (idl * theta.pow(2) + id0 * tomt)
    den = idl + (id0 + id1 - 2 * idl) * tomt
    out = ich + num / den
    dnum = idl.pow(2) * (id1 * theta.pow(2) + 2 * idl * tomt + id0 * (1 - theta).pow(2))
    return out, torch.log(dnum) - 2 * torch.log(den)


_nan_flags = []
_defer_nan = False  # set while a training step is captured in a graph (train.py)
# While a training step is captured (train.py): the graph's sticky NaN word (int32 [1] on the
# device, never cleared inside the graph).  The shared-launch sampling pass ORs its spline
# flags straight into it and the deferred running-statistics update skips on it, so a step
# after (and including) the first NaN writes no BatchNorm statistics.
_sticky_nan = None


# Set by paired_kld when its spline flags went straight into the captured graph's sticky
# word (nothing appended to _nan_flags); kld_loss then writes "sticky word set" as a bool
# in its own launch (_sticky_flag_out) and reduce_nan_flags returns that.
_flags_in_sticky = False
_sticky_flag_out = None


def reduce_nan_flags(device):
    """All pending NaN flags as one device bool (graph-capturable, no host read).  Returns
    (flag, only_sticky): only_sticky when the flag is the sticky word's own state, so the
    caller need not OR it back in."""
    global _flags_in_sticky, _sticky_flag_out
    flags = [f.reshape(()).to(device) for f in _nan_flags]
    _nan_flags.clear()
    only_sticky = _flags_in_sticky and not flags
    if _flags_in_sticky:
        flags.append(_sticky_flag_out if _sticky_flag_out is not None else _sticky_nan[0] != 0)
    _flags_in_sticky, _sticky_flag_out = False, None
    if not flags:
        return torch.zeros((), dtype=torch.bool, device=device), False
    if len(flags) == 1:
        return flags[0], only_sticky
    return torch.stack(flags).any(), False


class _KldLoss(torch.autograd.Function):
    """loss = -mean(log_q) + 0 * (mean(energy) + mean(lq_rev)) (main_algorithm_2.py:316-318,
    ALPHA = 1) in one launch each way (fs_kld_loss / fs_kld_loss_backward) instead of
    torch's seven forward and three backward kernels; the gradient is torch's
    (-g) * (1 / B) per row, bit for bit."""

    @staticmethod
    def forward(ctx, log_q, energy, lq_rev):
        global _sticky_flag_out
        from .. import _lib

        loss = torch.empty((), device=log_q.device)
        word = _sticky_nan if _flags_in_sticky else None
        if word is not None:
            _sticky_flag_out = torch.empty((), dtype=torch.bool, device=log_q.device)
        _lib.check(_lib.load().fs_kld_loss(_lib.ptr(log_q), log_q.shape[0], _lib.ptr(energy), _lib.ptr(lq_rev),
                                           lq_rev.shape[0], _lib.ptr(word), _lib.ptr(loss),
                                           _lib.ptr(_sticky_flag_out if word is not None else None),
                                           _lib.stream_ptr()), "fs_kld_loss")
        ctx.B = log_q.shape[0]
        return loss

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g):
        from .. import _lib

        g = g.detach().contiguous()
        gq = torch.empty(ctx.B, device=g.device)
        _lib.check(_lib.load().fs_kld_loss_backward(_lib.ptr(g), ctx.B, _lib.ptr(gq), _lib.stream_ptr()),
                   "fs_kld_loss_backward")
        return gq, None, None


def kld_loss(log_q, energy, lq_rev):
    """The ALPHA = 1 training loss from forward_kld's log q and reverse_kld's energies and
    log q (_KldLoss) for float32 device vectors; the torch expression otherwise."""
    ok = all(t.is_cuda and t.dtype == torch.float32 and t.dim() == 1 and t.is_contiguous()
             for t in (log_q, energy, lq_rev)) and log_q.shape[0] >= 1 and energy.shape == lq_rev.shape \
        and energy.shape[0] >= 1 and not energy.requires_grad and not lq_rev.requires_grad
    if ok:
        from .. import _lib

        with _lib.on_device(log_q):
            return _KldLoss.apply(log_q, energy, lq_rev)
    return -torch.mean(log_q) + 0.0 * (torch.mean(energy) + torch.mean(lq_rev))


def check_nan_flags():
    """Raise the reference's discriminant error if any inverse spline of the pass hit
    a NaN (one device->host read per pass instead of one per layer)."""
    if _defer_nan:
        return
    flags = list(_nan_flags)
    _nan_flags.clear()
    if flags and bool(torch.stack([f.reshape(()).to(flags[0].device) for f in flags]).any()):
        raise ValueError("Discriminant computation resulted in NaN.")


_HIP_K = (5, 8, 15, 32)


class _CircularRQS(torch.autograd.Function):
    """The circular RQS of M elements as one HIP kernel each way (csrc/spline_autograd.hip:
    fs_rqs_forward / fs_rqs_backward) instead of ~100 small torch kernels."""

    @staticmethod
    def forward(ctx, x, uw, uh, ud, B, inverse):
        from .. import _lib

        x, uw, uh, ud = (t.detach().contiguous().float() for t in (x, uw, uh, ud))
        M, K = x.numel(), uw.shape[-1]
        out = torch.empty_like(x)
        lad = torch.empty_like(x)
        flag = torch.zeros(1, dtype=torch.int32, device=x.device)
        L = _lib.load()
        with _lib.on_device(x):
            _lib.require_device(x, uw, uh, ud)
            _lib.check(L.fs_rqs_forward(M, K, int(inverse), _lib.ptr(x), _lib.ptr(uw), _lib.ptr(uh), _lib.ptr(ud),
                                        float(B), _lib.ptr(out), _lib.ptr(lad), _lib.ptr(flag), _lib.stream_ptr()),
                       "fs_rqs_forward")
        _nan_flags.append(flag[0] != 0)
        ctx.save_for_backward(x, uw, uh, ud)
        ctx.B, ctx.inverse = float(B), int(inverse)
        return out, lad

    @staticmethod
    def backward(ctx, g_out, g_lad):
        from .. import _lib

        x, uw, uh, ud = ctx.saved_tensors
        M, K = x.numel(), uw.shape[-1]
        go = g_out.contiguous().float() if g_out is not None else None
        gl = g_lad.contiguous().float() if g_lad is not None else None
        gx = torch.empty_like(x)
        guw = torch.empty_like(uw)
        guh = torch.empty_like(uh)
        gud = torch.empty_like(ud)
        L = _lib.load()
        with _lib.on_device(x):
            _lib.require_device(x, go, gl)
            _lib.check(L.fs_rqs_backward(M, K, ctx.inverse, _lib.ptr(x), _lib.ptr(uw), _lib.ptr(uh), _lib.ptr(ud),
                                         ctx.B, _lib.ptr(go), _lib.ptr(gl), _lib.ptr(gx), _lib.ptr(guw),
                                         _lib.ptr(guh), _lib.ptr(gud), _lib.stream_ptr()), "fs_rqs_backward")
        return gx, guw, guh, gud, None, None


def circular_rqs(x, uw, uh, ud, B, inverse):
    """Dispatch: the fused HIP spline for device tensors, the torch restatement below for
    CPU tensors (tests and host-side use).  A device tensor with a bin count K the HIP
    spline does not instantiate raises (DESIGN.md 'The path and its boundary': unsupported
    options raise instead of computing something else)."""
    if x.is_cuda:
        if uw.shape[-1] not in _HIP_K:
            from .. import _lib

            raise _lib.FlowStateError(f"the HIP spline is instantiated for K in {sorted(_HIP_K)}, "
                                      f"not K={uw.shape[-1]}")
        shp = x.shape
        K = uw.shape[-1]
        out, lad = _CircularRQS.apply(x.reshape(-1), uw.reshape(-1, K), uh.reshape(-1, K), ud.reshape(-1, K + 1),
                                      B, inverse)
        return out.reshape(shp), lad.reshape(shp)
    return circular_rqs_torch(x, uw, uh, ud, B, inverse)


def circular_rqs_torch(x, uw, uh, ud, B, inverse):
    """unconstrained_rational_quadratic_spline, circular tails (splines.py:16-88): identity
    outside [-B, B]; the derivative pad writes index K+1, which is never read.  Evaluated
    on every element with the outside ones parked at 0 (so their unused branch stays
    finite and contributes exact zeros to the gradient) and selected with where: no
    data-dependent shapes, no host synchronisation."""
    inside = (x >= -B) & (x <= B)
    xin = torch.where(inside, x, torch.zeros_like(x))
    o, l = rational_quadratic_spline(xin, uw, uh, ud, inverse, -B, B, -B, B)
    return torch.where(inside, o, x), torch.where(inside, l, torch.zeros_like(l))


# The conditioner's final layer (n (3K+1) columns, 2944 at A2) runs on fs_linear_f32 like
# every other Linear: its forward over 736 output tiles, its input gradient (K = 2944 over 32
# tiles) as split-K chunks plus an ordered reduction (csrc/train_kernels.hip); in r02 these
# two went to hipBLASLt, whose macro tiles beat the single-phase kernel there.

def _gemm_desc(x, w, b, r, y):
    """fs_gemm_f32 of nn.Linear's forward y = x W^T + b (+ r)."""
    from .. import _lib

    M, K = x.shape
    N = w.shape[0]
    p = _lib.ptr
    return _lib.GemmF32(M, N, K, p(x), K, 1, p(w), 1, K, p(b), p(r), N, p(y), N, None)


_GRAD_HOMES = {}


def register_grad_home(flat, flat_grad):
    """Parameters that are views of `flat` (train.GraphedTrainStep re-homes them so) get
    their gradients written straight into the same offsets of `flat_grad` by the backward
    kernels; autograd hands such a view to p.grad as is, so no gather copies them."""
    import weakref

    _GRAD_HOMES[flat.untyped_storage().data_ptr()] = (weakref.ref(flat), flat.data_ptr(), flat_grad)


_direct_grads = False  # set by paired_kld around its forward: one gradient contribution per parameter
# the block's second BatchNorm backward folded into the backward pairs around it
# (fs_linear_f32_pair_bn; _BnFoldLink) in the graphs paired_kld builds; FS_FOLD_BN=0 turns it off
_fold_bn = os.environ.get("FS_FOLD_BN", "1") != "0"
# The final Linear's input gradient (split-K over n (3K+1)) left as unreduced partials in the
# same graphs: its first reader, the last block's second Linear backward, sums them on load as
# its A and writes the sum out for the other (the block's first BatchNorm fold, dx_add), so the
# reduction launch goes; FS_DEFER_SPLITK=0 turns it off.  {placeholder data_ptr: (placeholder, workspace, chunks)}: the placeholder is
# what autograd carries; whoever cannot sum on load materialises it first (_sk_materialise).
_defer_splitk = os.environ.get("FS_DEFER_SPLITK", "1") != "0"
_splitk_pending = {}
_sk_deferred = 0  # forwards that took the deferral (tests: the handshake is met on the product path)


def _sk_get(t, pop=False):
    """(workspace, chunks) when t is a pending split-K placeholder (pop: its last reader)."""
    if t is None or not _splitk_pending:
        return None
    e = _splitk_pending.get(t.data_ptr())
    if e is None or e[0].shape != t.shape:
        return None
    if pop:
        del _splitk_pending[t.data_ptr()]
    return e[1], e[2]


def _sk_materialise(t):
    """Write a pending placeholder's reduction into it (fs_splitk_sum); no-op otherwise."""
    from .. import _lib

    e = _sk_get(t, pop=True)
    if e is not None:
        ws, ch = e
        n = t.numel()
        _lib.check(_lib.load().fs_splitk_sum(_lib.ptr(ws), ch, n, n, _lib.ptr(t), _lib.stream_ptr()), "fs_splitk_sum")
    return t


def _pair_bn(g0, g1, fi, fo, a_sk=None, add_sk=None):
    """fs_linear_f32_pair_bn, or its split-K-operand form (fs_linear_f32_pair_bn_sk)."""
    from .. import _lib

    L = _lib.load()
    if a_sk is None and add_sk is None:
        _lib.check(L.fs_linear_f32_pair_bn(g0, g1, fi, fo, _lib.stream_ptr()), "fs_linear_f32_pair_bn")
        return
    ach, astr = (a_sk[1], g0.M * g0.K) if a_sk is not None else (1, 0)
    dch, dstr = (add_sk[1], fi.B * fi.H) if add_sk is not None else (1, 0)
    _lib.check(L.fs_linear_f32_pair_bn_sk(g0, g1, fi, fo, ach, astr, dch, dstr, _lib.stream_ptr()),
               "fs_linear_f32_pair_bn_sk")


_ZERO = {}


def _zero_grad_placeholder(dev, M, K):
    """A [M, K] zero view of one cached scalar: what autograd sees for dy when it is folded."""
    z = _ZERO.get(dev)
    if z is None:
        z = _ZERO[dev] = torch.zeros((), dtype=torch.float32, device=dev)
    return z.expand(M, K)


class _BnFoldLink:
    """Carries a BatchNorm backward between the two Linear backward pairs around it
    (fs_linear_f32_pair_bn): the producer, the Linear that applies the BatchNorm to its
    input, computes its output gradient gu and the per-tile sums (fout); the consumer, the
    Function whose output the BatchNorm normalises, loads the BatchNorm's input gradient dy
    from them (+ the block's residual gradient for a block's first BatchNorm, fin) and writes
    that BatchNorm's dgamma / dbeta: the BatchNorm-backward launches and dy disappear.  A side
    channel like _ResidualGrad: the producer hands autograd a zero placeholder for dy, so it
    is only built where the whole backward runs through the conditioner (paired_kld's
    graphs); the consumer takes the BatchNorm's gamma and beta as extra inputs to return
    their gradients, and writes dy out where the residual needs it (a_out)."""

    __slots__ = ("pending", "consumer_ok")

    def __init__(self):
        self.pending = None
        self.consumer_ok = False  # set by the consuming Function's forward (it runs first)


def _grad_out(*ps, direct=False):
    """The gradient buffer of parameters ps (consecutive in memory when several): their
    slice of a registered flat gradient buffer when the Function was built by paired_kld
    (direct: each parameter enters that graph once, ALPHA = 1) and none of them holds a
    gradient yet, else a new tensor.  autograd makes the slice p.grad as is.  A parameter
    with two contributions in one backward (ALPHA != 1: the sampling pass is
    differentiable too) must not share a slice, since the second Function's backward may
    run before autograd has stored the first; those get new tensors."""
    n = sum(q.numel() for q in ps)
    home = _GRAD_HOMES.get(ps[0].untyped_storage().data_ptr()) if (_GRAD_HOMES and direct) else None
    if home is not None and all(q.grad is None for q in ps):
        flat = home[0]()
        if flat is not None and flat.untyped_storage().data_ptr() == ps[0].untyped_storage().data_ptr():
            off = (ps[0].data_ptr() - home[1]) // 4
            end = off
            for q in ps:  # every piece where the flat layout puts it
                if q.untyped_storage().data_ptr() != flat.untyped_storage().data_ptr() or \
                        (q.data_ptr() - home[1]) // 4 != end or not q.is_contiguous():
                    break
                end += q.numel()
            else:
                g = home[2][off:end]
                return g.view_as(ps[0]) if len(ps) == 1 else g
    if len(ps) == 1:
        return torch.empty_like(ps[0])
    return torch.empty((n,), dtype=ps[0].dtype, device=ps[0].device)


def _gemm(g, device):
    """One fs_linear_f32 product; long reductions over few tiles take the split-K path with
    a torch-allocated partial-tile workspace (graph-capture safe: the caching allocator)."""
    from .. import _lib

    L = _lib.load()
    n = L.fs_linear_f32_splitk_floats(g)
    if n > 0:
        ws = torch.empty(n, dtype=torch.float32, device=device)
        _lib.check(L.fs_linear_f32_splitk(g, _lib.ptr(ws), n, _lib.stream_ptr()), "fs_linear_f32_splitk")
    else:
        _lib.check(L.fs_linear_f32(g.M, g.N, g.K, g.A, g.sam, g.sak, g.B, g.sbk, g.sbn, g.bias, g.R, g.ldr, g.C,
                                   g.ldc, g.rowsum_a, _lib.stream_ptr()), "fs_linear_f32")


class _Linear(torch.autograd.Function):
    """nn.Linear (+ an optional residual added to the output) through fs_linear_f32
    (csrc/train_kernels.hip): y = x W^T + b (+ r); backward: dx = dy W and dW = dy^T x,
    db = column sums of dy, in one launch (fs_linear_f32_pair) unless dx is a long
    reduction (the 2944-wide final layer), which takes the split-K path."""

    @staticmethod
    def forward(ctx, x, w, b, r, res=None, pair=None):
        from .. import _lib

        x = x.contiguous()
        M, K = x.shape
        ctx.save_for_backward(x, w)
        ctx.bias = b
        ctx.direct = _direct_grads
        ctx.has_r = r is not None
        ctx.res = res
        y = torch.empty((M, w.shape[0]), dtype=torch.float32, device=x.device)
        _lib.require_device(x, w, b, r)
        g = _gemm_desc(x, w, b, r, y)
        if pair is not None and _lib.load().fs_linear_f32_splitk_floats(g) == 0:
            gs, _, _ = pair.gemm("final")
            _lib.check(_lib.load().fs_linear_f32_ex2(g, None, None, gs, None, None, _lib.stream_ptr()),
                       "fs_linear_f32_ex2")
            pair.commit()
        else:
            _gemm(g, x.device)
            if pair is not None:
                pair.gemm_alone("final")
        return y

    @staticmethod
    def backward(ctx, gy):
        from .. import _lib

        x, w = ctx.saved_tensors
        gy = _sk_materialise(gy.contiguous())
        M, K = x.shape
        N = w.shape[0]
        L = _lib.load()
        p = _lib.ptr
        gx = gw = gb = None
        need_x = ctx.needs_input_grad[0]
        need_w = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        if need_x:
            gx = torch.empty_like(x)
            g0 = _lib.GemmF32(M, K, N, p(gy), N, 1, p(w), K, 1, None, None, 0, p(gx), K, None)
        if need_w:
            gw = _grad_out(w, direct=ctx.direct)
            gb = _grad_out(ctx.bias, direct=ctx.direct) if ctx.bias is not None else torch.empty((N,), dtype=torch.float32, device=x.device)
            g1 = _lib.GemmF32(N, K, M, p(gy), 1, N, p(x), K, 1, None, None, 0, p(gw), K, p(gb))
        if need_x and need_w and L.fs_linear_f32_splitk_floats(g0) == 0:
            _lib.check(L.fs_linear_f32_pair(g0, g1, _lib.stream_ptr()), "fs_linear_f32_pair")
        else:
            if need_x:
                _gemm(g0, x.device)
            if need_w:
                _gemm(g1, x.device)
        if ctx.res is not None and ctx.needs_input_grad[3]:
            # the residual's gradient goes to the block's first BatchNorm backward, which
            # adds it in its own launch (no autograd accumulation kernel)
            if ctx.res.g is not None:
                raise RuntimeError("residual gradient stash was never consumed by its BatchNorm backward")
            ctx.res.g = gy
            return gx, gw, gb, None, None, None
        return gx, gw, gb, (gy if ctx.has_r and ctx.needs_input_grad[3] else None), None, None


class _BnRelu(torch.autograd.Function):
    """relu(BatchNorm1d(x)) in train mode through fs_bn_relu_train_fwd / _bwd: batch
    statistics, the module's running statistics and num_batches_tracked updated in the
    same launch (torch.nn.BatchNorm1d.forward, momentum form)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, bn, res=None):
        from .. import _lib

        x = x.contiguous()
        M, H = x.shape
        y = torch.empty_like(x)
        mean = torch.empty((H,), dtype=torch.float32, device=x.device)
        invstd = torch.empty_like(mean)
        L = _lib.load()
        _lib.require_device(x, gamma, beta)
        _lib.check(L.fs_bn_relu_train_fwd(M, H, _lib.ptr(x), _lib.ptr(gamma), _lib.ptr(beta),
                                          _lib.ptr(bn.running_mean), _lib.ptr(bn.running_var),
                                          _lib.ptr(bn.num_batches_tracked), float(bn.momentum), float(bn.eps),
                                          _lib.ptr(y), _lib.ptr(mean), _lib.ptr(invstd), _lib.stream_ptr()),
                   "fs_bn_relu_train_fwd")
        ctx.save_for_backward(x, y, gamma, mean, invstd)
        ctx.beta = beta
        ctx.direct = _direct_grads
        ctx.res = res
        return y

    @staticmethod
    def backward(ctx, gy):
        from .. import _lib

        x, y, gamma, mean, invstd = ctx.saved_tensors
        gy = gy.contiguous()
        M, H = x.shape
        gx = torch.empty_like(x)
        gg = _grad_out(gamma, direct=ctx.direct)
        gb = _grad_out(ctx.beta, direct=ctx.direct)
        add = None
        if ctx.res is not None and ctx.res.g is not None:
            add, ctx.res.g = ctx.res.g, None
            if add.shape != x.shape:
                raise RuntimeError("residual gradient does not match the block input")
        _lib.check(_lib.load().fs_bn_relu_train_bwd(M, H, _lib.ptr(x), _lib.ptr(y), _lib.ptr(gy), _lib.ptr(gamma),
                                                    _lib.ptr(mean), _lib.ptr(invstd), _lib.ptr(gx), _lib.ptr(add),
                                                    _lib.ptr(gg), _lib.ptr(gb), _lib.stream_ptr()),
                   "fs_bn_relu_train_bwd")
        return gx, gg, gb, None, None


class _LinearStats(torch.autograd.Function):
    """_Linear whose epilogue also writes each 32-row tile's column statistics of y (the
    batch statistics of the BatchNorm that consumes y, fs_linear_f32_ex stats_out)."""

    @staticmethod
    def forward(ctx, x, w, b, pair=None, fold_in=None, gamma2=None, beta2=None):
        from .. import _lib

        x = x.contiguous()
        M, K = x.shape
        N = w.shape[0]
        y = torch.empty((M, N), dtype=torch.float32, device=x.device)
        st = torch.empty(((M + 31) // 32, N, 2), dtype=torch.float32, device=x.device)
        ok = fold_in is not None and _fold_ok(M, K, N)  # the first block's first BatchNorm folded in here
        ctx.fold_in = fold_in if ok else None
        if fold_in is not None:
            fold_in.consumer_ok = ok
        ctx.gparams2 = (gamma2, beta2)
        _lib.require_device(x, w, b)
        if pair is None:
            _lib.check(_lib.load().fs_linear_f32_ex(_gemm_desc(x, w, b, None, y), None, _lib.ptr(st),
                                                    _lib.stream_ptr()), "fs_linear_f32_ex")
        else:
            gs, bs, sts = pair.gemm("init")
            _lib.check(_lib.load().fs_linear_f32_ex2(_gemm_desc(x, w, b, None, y), None, _lib.ptr(st), gs, bs,
                                                     _lib.ptr(sts), _lib.stream_ptr()), "fs_linear_f32_ex2")
            pair.commit()
        ctx.save_for_backward(x, w)
        ctx.bias = b
        ctx.direct = _direct_grads
        ctx.mark_non_differentiable(st)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for st (a fill kernel per call)
        return y, st

    @staticmethod
    def backward(ctx, gy, gst):
        from .. import _lib

        x, w = ctx.saved_tensors
        if gy is None:  # y unused by the loss
            return None, None, None, None, None, None, None
        fin = ctx.fold_in.pending if ctx.fold_in is not None else None
        M, K = x.shape
        N = w.shape[0]
        gx, gw = torch.empty_like(x), _grad_out(w, direct=ctx.direct)
        gb = _grad_out(ctx.bias, direct=ctx.direct)
        p = _lib.ptr
        if fin is not None:  # dy of the first block's first BatchNorm, loaded on the fly
            ctx.fold_in.pending = None
            gu2, u2, y2, mean2, invstd2, gamma2, part2, add2 = fin
            gg2 = _grad_out(ctx.gparams2[0], direct=ctx.direct)
            gbeta2 = _grad_out(ctx.gparams2[1], direct=ctx.direct)
            g0 = _lib.GemmF32(M, K, N, p(gu2), N, 1, p(w), K, 1, None, None, 0, p(gx), K, None)
            g1 = _lib.GemmF32(N, K, M, p(gu2), 1, N, p(x), K, 1, None, None, 0, p(gw), K, p(gb))
            add_sk = _sk_get(add2, pop=True)  # the residual gradient as split-K partials
            fi = _lib.BnFold(p(gu2), p(u2), p(y2), p(mean2), p(invstd2), p(gamma2), p(part2), p(gg2), p(gbeta2),
                             p(add_sk[0] if add_sk else add2), None, M, N)
            _pair_bn(g0, g1, fi, None, add_sk=add_sk)
            return gx, gw, gb, None, None, gg2, gbeta2
        gy = _sk_materialise(gy.contiguous())
        g0 = _lib.GemmF32(M, K, N, p(gy), N, 1, p(w), K, 1, None, None, 0, p(gx), K, None)
        g1 = _lib.GemmF32(N, K, M, p(gy), 1, N, p(x), K, 1, None, None, 0, p(gw), K, p(gb))
        _lib.check(_lib.load().fs_linear_f32_pair(g0, g1, _lib.stream_ptr()), "fs_linear_f32_pair")
        return gx, gw, gb, None, None, None, None


class _BnReluLinear(torch.autograd.Function):
    """Linear(relu(BatchNorm1d_train(x))) (+ r) in one launch: the BatchNorm's batch
    statistics come from the producer's tile statistics (x_stats), the normalisation and
    ReLU are applied to the GEMM's A operand as it is loaded, running statistics and
    num_batches_tracked are updated as torch does, and y's own tile statistics are written
    for the next BatchNorm (fs_linear_f32_ex).  u = relu(BN(x)) is written once for the
    backward, which is the weight / input gradient pair on u and then the BatchNorm + ReLU
    backward (fs_bn_relu_train_bwd, with the block's residual gradient added there as in
    _BnRelu)."""

    @staticmethod
    def forward(ctx, x, x_stats, gamma, beta, bn, w, b, r, res=None, pair=None, op=None, fold_in=None, fold_out=None,
                gamma2=None, beta2=None):
        from .. import _lib

        x = x.contiguous()
        M, K = x.shape
        N = w.shape[0]
        y = torch.empty((M, N), dtype=torch.float32, device=x.device)
        st = torch.empty(((M + 31) // 32, N, 2), dtype=torch.float32, device=x.device)
        invstd = torch.empty((K,), dtype=torch.float32, device=x.device)
        u = torch.empty_like(x) if any(ctx.needs_input_grad) else None
        # fold_out: this Linear's own BatchNorm (applied to x); fold_in: the BatchNorm that
        # normalises y (gamma2, beta2, their gradients returned here).  The lean kernels'
        # limits: widths <= 256, the weight gradients reduce over the batch in quads.
        ok = _fold_ok(M, K, N)
        ctx.fold_in = fold_in if ok else None
        if fold_in is not None:
            fold_in.consumer_ok = ok
        ctx.fold_out = fold_out if ok else None
        ctx.gparams2 = (gamma2, beta2)
        p = _lib.ptr
        _lib.require_device(x, x_stats, gamma, beta, w, b, r)
        if pair is None:
            mean = torch.empty((K,), dtype=torch.float32, device=x.device)
            bi = _lib.BnIn(p(x_stats), (M + 31) // 32, M, p(gamma), p(beta), float(bn.eps), float(bn.momentum),
                           p(bn.running_mean), p(bn.running_var), p(bn.num_batches_tracked), p(mean), p(invstd),
                           p(u), None)
            _lib.check(_lib.load().fs_linear_f32_ex(_gemm_desc(x, w, b, r, y), bi, p(st), _lib.stream_ptr()),
                       "fs_linear_f32_ex")
        else:
            # running statistics deferred to the end of the pass pair (_SamplingRider)
            mean, var = pair.bn_slots(bn, 1)
            bi = _lib.BnIn(p(x_stats), (M + 31) // 32, M, p(gamma), p(beta), float(bn.eps), float(bn.momentum),
                           None, None, None, p(mean), p(invstd), p(u), p(var))
            gs, bs, sts = pair.gemm(op)
            _lib.check(_lib.load().fs_linear_f32_ex2(_gemm_desc(x, w, b, r, y), bi, p(st), gs, bs, p(sts),
                                                     _lib.stream_ptr()), "fs_linear_f32_ex2")
            pair.commit()
        ctx.save_for_backward(x, u, gamma, mean, invstd, w)
        ctx.gparams = (beta, b)
        ctx.direct = _direct_grads
        ctx.has_r = r is not None
        ctx.res = res
        ctx.mark_non_differentiable(st)
        ctx.set_materialize_grads(False)
        if r is not None and res is not None and ctx.fold_out is not None:
            # handshake with _FinalSplines: this backward can take y's gradient as split-K
            # partials (summed on load, written out for the residual's reader)
            y._fs_splitk_reader = True
        return y, st

    @staticmethod
    def backward(ctx, gy, gst):
        from .. import _lib

        x, u, gamma, mean, invstd, w = ctx.saved_tensors
        if gy is None:
            return (None,) * 15
        M, K = x.shape
        N = w.shape[0]
        L = _lib.load()
        p = _lib.ptr
        # dy of the BatchNorm that normalises y, not materialised (its producer folded it)
        fin = ctx.fold_in.pending if ctx.fold_in is not None else None
        if fin is not None:
            ctx.fold_in.pending = None
        fout = ctx.fold_out if (ctx.fold_out is not None and ctx.fold_out.consumer_ok) else None
        gw = _grad_out(w, direct=ctx.direct)
        gb = _grad_out(ctx.gparams[1], direct=ctx.direct)
        add = None  # the block's residual gradient, for its first BatchNorm (this Linear's own)
        if ctx.res is not None and ctx.res.g is not None:
            add, ctx.res.g = ctx.res.g, None
        a_sk = None  # gy as split-K partials, summed on load (the placeholder goes on as the residual)
        if fin is None:
            gy = gy.contiguous()
            a_sk = _sk_get(gy)
            if a_sk is not None and not (fout is not None and ctx.res is not None and ctx.has_r
                                         and ctx.needs_input_grad[7]):
                a_sk = None
                _sk_materialise(gy)
        if fout is None:
            _sk_materialise(add)  # read by fs_bn_relu_train_bwd below
        dy = fin[0] if fin is not None else gy  # (fin: only the layout, gu of the folded BatchNorm)
        pa = p(a_sk[0]) if a_sk is not None else p(dy)
        gu = torch.empty_like(u)
        g0 = _lib.GemmF32(M, K, N, pa, N, 1, p(w), K, 1, None, None, 0, p(gu), K, None)
        g1 = _lib.GemmF32(N, K, M, pa, 1, N, p(u), K, 1, None, None, 0, p(gw), K, p(gb))
        gg2 = gbeta2 = a_out = None
        fi = fo = None
        add_sk = None
        if fin is not None:
            gu2, u2, y2, mean2, invstd2, gamma2, part2, add2 = fin
            add_sk = _sk_get(add2, pop=True)  # the residual gradient as split-K partials
            if add_sk is not None:
                add2 = add_sk[0]
            gg2 = _grad_out(ctx.gparams2[0], direct=ctx.direct)
            gbeta2 = _grad_out(ctx.gparams2[1], direct=ctx.direct)
            if ctx.has_r and ctx.needs_input_grad[7]:
                a_out = torch.empty((M, N), dtype=torch.float32, device=x.device)  # dy for the residual
            fi = _lib.BnFold(p(gu2), p(u2), p(y2), p(mean2), p(invstd2), p(gamma2), p(part2), p(gg2), p(gbeta2),
                             p(add2), p(a_out), M, N)
        if fout is not None:
            part = torch.empty(((M + 31) // 32, K, 2), dtype=torch.float32, device=x.device)
            # (a_sk) the pair also writes the reduced gy into its placeholder (a_out) for the
            # residual's reader
            fo = _lib.BnFold(p(gu), p(u), p(x), p(mean), p(invstd), p(gamma), p(part), None, None, None,
                             p(gy) if a_sk is not None else None, M, K)
        # the input / weight gradient pair over 48 workgroups, then the BatchNorm + ReLU
        # backward unless it is folded into the pair before (r04): 10.9 us per layer in a
        # graph, against 18.1 us for one launch whose column strips own the BatchNorm sums
        # (profiles/r03/r03k_linbn_probe.log), and 148 against 239
        # steps/s for the BatchNorm backward run by each strip's last tile in the pair's launch
        # (device-scope fences; DESIGN "Training", profiles/r03/r03v_*)
        if fi is not None or fo is not None:
            _pair_bn(g0, g1, fi, fo, a_sk=a_sk, add_sk=add_sk)
            if a_sk is not None:
                _sk_get(gy, pop=True)  # materialised by the pair: its other reader loads it plainly
        else:
            _lib.check(L.fs_linear_f32_pair(g0, g1, _lib.stream_ptr()), "fs_linear_f32_pair")
        gr = None
        if ctx.has_r and ctx.needs_input_grad[7]:
            g_out = a_out if fin is not None else gy
            if ctx.res is not None:
                ctx.res.g = g_out  # to the block's first BatchNorm backward (its dx_add)
            else:
                gr = g_out
        if fout is not None:
            fout.pending = (gu, u, x, mean, invstd, gamma, part, add)
            gx = _zero_grad_placeholder(x.device, M, K)  # the placeholder for this BatchNorm's dy
            return gx, None, None, None, None, gw, gb, gr, None, None, None, None, None, gg2, gbeta2
        gx = torch.empty_like(x)
        gg = _grad_out(gamma, direct=ctx.direct)
        gbeta = _grad_out(ctx.gparams[0], direct=ctx.direct)
        _lib.check(L.fs_bn_relu_train_bwd(M, K, p(x), p(u), p(gu), p(gamma), p(mean), p(invstd), p(gx), p(add),
                                          p(gg), p(gbeta), _lib.stream_ptr()), "fs_bn_relu_train_bwd")
        return gx, None, gg, gbeta, None, gw, gb, gr, None, None, None, None, None, gg2, gbeta2


def _fold_ok(M, K, N):
    """A BatchNorm-backward fold applies to a Linear of this shape (lean kernels, widths <= 256,
    batch a multiple of 4) in the graphs paired_kld builds."""
    from .. import _lib

    return (_fold_bn and _direct_grads and N <= 256 and K <= 256 and M % 4 == 0
            and _lib.load().fs_set_lean_gemm(-1) == 1)


def _fused_ok(net, t):
    """The fused train-mode conditioner applies: f32 device activations, every BatchNorm
    in train mode with affine parameters, running statistics and a momentum, batch >= 2
    (torch raises on a batch of one in train mode: that case keeps torch's modules)."""
    if not (t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.shape[0] >= 2):
        return False
    for blk in net.blocks:
        for bn in blk.batch_norm_layers:
            if not (bn.training and bn.affine and bn.track_running_stats and bn.momentum is not None
                    and bn.running_mean is not None):
                return False
    return True


class _ResidualGrad:
    """Carries a block input's residual-branch gradient from the block's second Linear
    (whose backward runs first: the chain l1 -> bn1 -> l0 -> bn0 orders them) to its first
    BatchNorm's backward, which adds it in its own launch (fs_bn_relu_train_bwd dx_add)
    instead of autograd summing the two branches in a separate kernel.

    A side channel: autograd sees None for that gradient, so it is correct only when the
    gradient reaches the consuming BatchNorm's backward, as in loss.backward() through
    the whole conditioner (_conditioner_fused).  Checking these Functions in isolation
    (gradcheck, or autograd.grad on an intermediate that skips the block's first BatchNorm)
    must construct them with res=None, which returns the residual gradient normally.
    A stash still unconsumed when the next one is written raises."""

    __slots__ = ("g",)

    def __init__(self):
        self.g = None


def _conditioner_fused(net, t, pair=None, final=True):
    """ResidualNet.forward (resnet.py:82-104, blocks :35-51) in train mode: every Linear
    on fs_linear_f32 kernels; each BatchNorm + ReLU applied inside the Linear that consumes
    it (its statistics from the producing Linear's epilogue, _BnReluLinear), the block's
    residual add fused into its second Linear; backward: input / weight gradient pairs,
    BatchNorm backward with the residual gradient added by the block's first one."""
    li = net.initial_layer
    if _bn_in_load_ok(net):
        blocks = list(net.blocks)
        links0 = [_BnFoldLink() for _ in blocks]  # each block's first BatchNorm
        first = blocks[0].batch_norm_layers[0] if blocks else None
        t, st = _LinearStats.apply(t, li.weight, li.bias, pair, links0[0] if blocks else None,
                                   first.weight if blocks else None, first.bias if blocks else None)
        for i, blk in enumerate(blocks):
            bn0, bn1 = blk.batch_norm_layers
            l0, l1 = blk.linear_layers
            res = _ResidualGrad()
            link1 = _BnFoldLink()  # its second BatchNorm
            u, su = _BnReluLinear.apply(t, st, bn0.weight, bn0.bias, bn0, l0.weight, l0.bias, None, res, pair, (i, 0),
                                        link1, links0[i], bn1.weight, bn1.bias)
            nxt = blocks[i + 1].batch_norm_layers[0] if i + 1 < len(blocks) else None
            t, st = _BnReluLinear.apply(u, su, bn1.weight, bn1.bias, bn1, l1.weight, l1.bias, t, res, pair, (i, 1),
                                        links0[i + 1] if nxt is not None else None, link1,
                                        nxt.weight if nxt is not None else None, nxt.bias if nxt is not None else None)
        if not final:  # the caller fuses the final Linear into its next Function (_FinalSplines)
            return t
        lf = net.final_layer
        return _Linear.apply(t, lf.weight, lf.bias, None, None, pair)
    if pair is not None:
        raise ValueError("the paired passes need the BatchNorm-in-load conditioner")
    t = _Linear.apply(t, li.weight, li.bias, None)
    for blk in net.blocks:
        bn0, bn1 = blk.batch_norm_layers
        l0, l1 = blk.linear_layers
        res = _ResidualGrad()
        u = _BnRelu.apply(t, bn0.weight, bn0.bias, bn0, res)
        u = _Linear.apply(u, l0.weight, l0.bias, None)
        u = _BnRelu.apply(u, bn1.weight, bn1.bias, bn1)
        t = _Linear.apply(u, l1.weight, l1.bias, t, res)
    lf = net.final_layer
    return _Linear.apply(t, lf.weight, lf.bias, None)


def _bn_in_load_ok(net):
    """The BatchNorm-in-load GEMM's limit: hidden width <= 256 (its per-column statistics
    live in LDS)."""
    return net.initial_layer.weight.shape[0] <= 256


def conditioner(net, ident, B):
    """ResidualNet.forward with PeriodicFeaturesElementwise (fork: cos/sin of all identity
    features, nn.py:120-137); BatchNorm modules in their current train/eval mode."""
    scale = np.pi / B
    t = torch.cat([torch.cos(scale * ident), torch.sin(scale * ident)], dim=-1)
    if _fused_ok(net, t):
        return _conditioner_fused(net, t)
    t = net.initial_layer(t)
    for blk in net.blocks:
        u = blk.batch_norm_layers[0](t)
        u = F.relu(u)
        u = blk.linear_layers[0](u)
        u = blk.batch_norm_layers[1](u)
        u = F.relu(u)
        u = blk.linear_layers[1](u)
        t = t + u
    return net.final_layer(t)


def _cond_spline(layer, trans, params, inverse):
    K = layer.num_bins
    b, d = trans.shape
    params = params.reshape(b, d, -1)
    sq = np.sqrt(layer.num_hidden_channels)
    uw = params[..., :K] / sq
    uh = params[..., K:2 * K] / sq
    ud = params[..., 2 * K:]
    out, lad = circular_rqs(trans, uw, uh, ud, layer.tail_bound, inverse)
    return out, lad.sum(dim=1)


def _uncond_spline(layer, ident, inverse):
    u = layer.prqct.unconditional_transform
    n = ident.shape[0]
    uw = u.unnormalized_widths[None].expand(n, *u.unnormalized_widths.shape)
    uh = u.unnormalized_heights[None].expand(n, *u.unnormalized_heights.shape)
    ud = u.unnormalized_derivatives[None].expand(n, *u.unnormalized_derivatives.shape)
    out, lad = circular_rqs(ident, uw, uh, ud, layer.tail_bound, inverse)
    return out, lad.sum(dim=1)


def coupling_density(layer, x):
    """Coupling.forward (coupling.py:71-102) = the layer's inverse (density direction)."""
    p = layer.prqct
    ident = x[:, p.identity_features]
    trans = x[:, p.transform_features]
    params = conditioner(p.transform_net, ident, layer.tail_bound)
    trans, lad = _cond_spline(layer, trans, params, inverse=False)
    ident, lad_u = _uncond_spline(layer, ident, inverse=False)
    lad = lad + lad_u
    out = torch.empty_like(x)
    out = out.index_copy(1, p.identity_features, ident).index_copy(1, p.transform_features, trans)
    split = layer.num_input_channels // 2
    return torch.cat([out[:, split:], out[:, :split]], dim=1), lad


def coupling_sample(layer, z):
    """Coupling.inverse (coupling.py:104-134) = the layer's forward (sampling direction)."""
    p = layer.prqct
    split = layer.num_input_channels // 2
    z = torch.cat([z[:, split:], z[:, :split]], dim=1)
    ident = z[:, p.identity_features]
    trans = z[:, p.transform_features]
    ident, lad = _uncond_spline(layer, ident, inverse=True)
    params = conditioner(p.transform_net, ident, layer.tail_bound)
    trans, lad_s = _cond_spline(layer, trans, params, inverse=True)
    lad = lad + lad_s
    out = torch.empty_like(z)
    out = out.index_copy(1, p.identity_features, ident).index_copy(1, p.transform_features, trans)
    return out, lad


# ---------------------------------------------------------------------------
# Whole coupling layers on the device (csrc/spline_autograd.hip, fs_coupling_*): the
# gather, periodic features, both splines, half-roll and log-det sums of one layer in one
# launch on each side of the conditioner.


def _coupling_desc(layer, rows):
    from .. import _lib

    p = layer.prqct
    c = _lib.Coupling()
    c.rows = rows
    c.D = layer.num_input_channels
    c.K = layer.num_bins
    c.hidden = layer.num_hidden_channels
    c.identity_features = p.identity_features.data_ptr()
    c.transform_features = p.transform_features.data_ptr()
    c.tail_bound = layer.tail_bound
    return c


def _check_shapes(layer, rows, params, uw, uh, ud):
    """The kernels index params [rows][n][3K+1] (None: not yet computed) and the
    unconditional [n][K], [n][K], [n][K+1] from the layer's sizes: refuse anything else
    before launching."""
    n, K = layer.num_input_channels // 2, layer.num_bins
    want = [(uw, (n, K)), (uh, (n, K)), (ud, (n, K + 1))]
    if params is not None:
        want.append((params, (rows, n * (3 * K + 1))))
    for t, shp in want:
        if tuple(t.shape) != shp or t.dtype != torch.float32:
            raise ValueError(f"coupling operand of shape {tuple(t.shape)} / {t.dtype}, expected {shp} float32")


def fused_coupling_ok(layer, x):
    """Device f32 rows, an instantiated K, index buffers on the same device."""
    p = layer.prqct
    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.shape[1] == layer.num_input_channels
            and layer.num_bins in _HIP_K and p.identity_features.device == x.device
            and p.identity_features.dtype == torch.int64 and p.transform_features.dtype == torch.int64)


class _Features(torch.autograd.Function):
    """t = [cos(s x_id), sin(s x_id)] (nn.py:120-137) and its adjoint."""

    @staticmethod
    def forward(ctx, x, layer, res=None, pair=None):
        from .. import _lib

        x = x.contiguous()
        t = torch.empty_like(x)
        c = _coupling_desc(layer, x.shape[0])
        _lib.require_device(x)
        if pair is None:
            _lib.check(_lib.load().fs_coupling_features_fwd(ctypes.byref(c), _lib.ptr(x), _lib.ptr(t),
                                                            _lib.stream_ptr()), "fs_coupling_features_fwd")
        else:
            pair.pre(c, x, t)
        ctx.save_for_backward(x)
        ctx.layer = layer
        ctx.res = res
        # x is the previous layer's output (the training step's density pass): the backward
        # leaves its launch to that layer's spline backward, which carries it
        # (fs_coupling_bwd_step); the previous layer passed x's spline gradient through the
        # res stash, so autograd hands the placeholder gradient on unchanged
        ctx.defer = (pair is not None and res is not None and x.grad_fn is not None
                     and type(x.grad_fn).__name__ in ("_FinalSplinesBackward", "_DensitySplinesBackward"))
        return t

    @staticmethod
    def backward(ctx, gt):
        from .. import _lib

        (x,) = ctx.saved_tensors
        gt = gt.contiguous()
        gx = torch.empty_like(x)
        add = None
        if ctx.res is not None and ctx.res.g is not None:
            add, ctx.res.g = ctx.res.g, None
            if add.shape != x.shape:
                raise RuntimeError("spline gradient does not match the layer input")
        if ctx.defer:
            _pending_features_bwd[gx.data_ptr()] = (ctx.layer, x, gt, add, gx)
            return gx, None, None, None
        c = _coupling_desc(ctx.layer, x.shape[0])
        _lib.check(_lib.load().fs_coupling_features_bwd(ctypes.byref(c), _lib.ptr(x), _lib.ptr(gt), _lib.ptr(gx),
                                                        _lib.ptr(add), _lib.stream_ptr()), "fs_coupling_features_bwd")
        return gx, None, None, None


# Features backward launches left to the next spline backward (the previous layer's):
# {placeholder gradient's data_ptr: (layer, x, g_t, gx_add, placeholder)}.  Each entry holds
# its placeholder, so no other tensor can take its address meanwhile.
_pending_features_bwd = {}


def _density_bwd(c, x, params, uw, uh, ud, g_out, g_lq, gx, gp, gu):
    """fs_coupling_density_bwd, or, when g_out is a features backward's pending placeholder,
    fs_coupling_bwd_step (that backward and this one in one launch)."""
    from .. import _lib

    L, p = _lib.load(), _lib.ptr
    q = _pending_features_bwd.pop(g_out.data_ptr(), None) if g_out is not None else None
    if q is not None and q[4].shape == g_out.shape:
        layer_f, xf, gt, add, gxf = q
        cf = _coupling_desc(layer_f, xf.shape[0])
        _lib.check(L.fs_coupling_bwd_step(ctypes.byref(cf), p(xf), p(gt), p(gxf), p(add), ctypes.byref(c), p(x),
                                          p(params), p(uw), p(uh), p(ud), p(g_lq), p(gx), p(gp), p(gu),
                                          _lib.stream_ptr()), "fs_coupling_bwd_step")
        return
    if q is not None:  # not this layer's: launch it on its own first
        layer_f, xf, gt, add, gxf = q
        cf = _coupling_desc(layer_f, xf.shape[0])
        _lib.check(L.fs_coupling_features_bwd(ctypes.byref(cf), p(xf), p(gt), p(gxf), p(add), _lib.stream_ptr()),
                   "fs_coupling_features_bwd")
    _lib.check(L.fs_coupling_density_bwd(ctypes.byref(c), p(x), p(params), p(uw), p(uh), p(ud), p(g_out), p(g_lq),
                                         p(gx), p(gp), p(gu), _lib.stream_ptr()), "fs_coupling_density_bwd")


def flush_features_bwd():
    """Launch every features backward still pending (none after a complete backward)."""
    from .. import _lib

    L, p = _lib.load(), _lib.ptr
    _splitk_pending.clear()  # (an interrupted backward's; their placeholders are unreachable)
    while _pending_features_bwd:
        _, (layer_f, xf, gt, add, gxf) = _pending_features_bwd.popitem()
        cf = _coupling_desc(layer_f, xf.shape[0])
        _lib.check(L.fs_coupling_features_bwd(ctypes.byref(cf), p(xf), p(gt), p(gxf), p(add), _lib.stream_ptr()),
                   "fs_coupling_features_bwd")


class _DensitySplines(torch.autograd.Function):
    """Coupling.forward after the conditioner (coupling.py:71-102): conditional spline of the
    transform half, unconditional spline of the identity half, half-roll, and
    lq_out = lq_in + both log-det sums; backward through both splines."""

    @staticmethod
    def forward(ctx, x, params, uw, uh, ud, lq_in, layer, res=None, pair=None):
        from .. import _lib

        x = x.contiguous()
        params = params.contiguous()
        uw, uh, ud = uw.contiguous(), uh.contiguous(), ud.contiguous()
        _check_shapes(layer, x.shape[0], params, uw, uh, ud)
        if lq_in is not None and tuple(lq_in.shape) != (x.shape[0],):
            raise ValueError("log_q must be [rows]")
        out = torch.empty_like(x)
        lq = torch.empty((x.shape[0],), dtype=torch.float32, device=x.device)
        c = _coupling_desc(layer, x.shape[0])
        _lib.require_device(x, params, uw, lq_in)
        if pair is None:
            _lib.check(_lib.load().fs_coupling_density_fwd(ctypes.byref(c), _lib.ptr(x), _lib.ptr(params),
                                                           _lib.ptr(uw), _lib.ptr(uh), _lib.ptr(ud), _lib.ptr(lq_in),
                                                           _lib.ptr(out), _lib.ptr(lq), _lib.stream_ptr()),
                       "fs_coupling_density_fwd")
        else:
            pair.post(c, x, params, uw, uh, ud, lq_in, out, lq)
        ctx.save_for_backward(x, params, uw, uh, ud)
        ctx.direct = _direct_grads
        ctx.layer = layer
        ctx.has_lq = lq_in is not None
        ctx.res = res
        ctx.set_materialize_grads(False)  # the last layer's out has no gradient: no zero fill
        return out, lq

    @staticmethod
    def backward(ctx, g_out, g_lq):
        from .. import _lib

        x, params, uw, uh, ud = ctx.saved_tensors
        layer = ctx.layer
        K = layer.num_bins
        g_out = g_out.contiguous() if g_out is not None else None
        g_lq = g_lq.contiguous() if g_lq is not None else None
        gx = torch.empty_like(x)
        gp = torch.empty_like(params)
        n = x.shape[1] // 2
        gu = torch.empty((x.shape[0], n * (3 * K + 1)), dtype=torch.float32, device=x.device)
        c = _coupling_desc(layer, x.shape[0])
        _density_bwd(c, x, params, uw, uh, ud, g_out, g_lq, gx, gp, gu)
        # the unconditional parameters are shared by every row: their gradient is the column
        # sum of gu, taken as fs_linear_f32's row sum of gu^T (N = 0: no product), which
        # spreads it over (n(3K+1))/32 workgroups (torch's reduction took 16 us at batch 256)
        P = n * (3 * K + 1)
        gs = _grad_out(uw, uh, ud, direct=ctx.direct)  # [uw | uh | ud] gradients, one row sum
        _lib.check(_lib.load().fs_linear_f32(P, 0, x.shape[0], _lib.ptr(gu), 1, P, None, 0, 0, None, None, 0, None, 0,
                                             _lib.ptr(gs), _lib.stream_ptr()), "fs_linear_f32")
        # [uw | uh | ud] back to back: contiguous views, no copies when the gradients are gathered
        guw = gs[:n * K].view(n, K)
        guh = gs[n * K:2 * n * K].view(n, K)
        gud = gs[2 * n * K:].view(n, K + 1)
        if ctx.res is not None and ctx.needs_input_grad[0]:
            # x's spline gradient is added by the features backward of the same layer, which
            # runs after this one (it needs the conditioner's adjoint, which needs gp)
            ctx.res.g = gx
            gx = None
        return (gx, gp, guw, guh, gud, g_lq if ctx.has_lq else None, None, None, None)


class _FinalSplines(torch.autograd.Function):
    """The conditioner's final Linear (params = h W^T + b, nn.Linear) and the layer's
    density-direction splines (as _DensitySplines) in one Function, so that the backward's
    three products run as one group launch (fs_linear_f32_group): dh = dparams W (split-K
    over the n (3K+1) columns), dW = dparams^T h with db, and the unconditional spline
    parameters' gradient (the row sum of the per-row adjoints).  Values are those of
    _Linear + _DensitySplines."""

    @staticmethod
    def forward(ctx, h, w, b, x, uw, uh, ud, lq_in, layer, res=None, pair=None):
        from .. import _lib

        h = h.contiguous()
        x = x.contiguous()
        uw, uh, ud = uw.contiguous(), uh.contiguous(), ud.contiguous()
        L = _lib.load()
        params = torch.empty((h.shape[0], w.shape[0]), dtype=torch.float32, device=h.device)
        _lib.require_device(h, w, b, x, uw, lq_in)
        g = _gemm_desc(h, w, b, None, params)
        if pair is not None and L.fs_linear_f32_splitk_floats(g) == 0:
            gs, _, _ = pair.gemm("final")
            _lib.check(L.fs_linear_f32_ex2(g, None, None, gs, None, None, _lib.stream_ptr()), "fs_linear_f32_ex2")
            pair.commit()
        else:
            _gemm(g, h.device)
            if pair is not None:
                pair.gemm_alone("final")
        _check_shapes(layer, x.shape[0], params, uw, uh, ud)
        if lq_in is not None and tuple(lq_in.shape) != (x.shape[0],):
            raise ValueError("log_q must be [rows]")
        out = torch.empty_like(x)
        lq = torch.empty((x.shape[0],), dtype=torch.float32, device=x.device)
        c = _coupling_desc(layer, x.shape[0])
        if pair is None:
            _lib.check(L.fs_coupling_density_fwd(ctypes.byref(c), _lib.ptr(x), _lib.ptr(params), _lib.ptr(uw),
                                                 _lib.ptr(uh), _lib.ptr(ud), _lib.ptr(lq_in), _lib.ptr(out),
                                                 _lib.ptr(lq), _lib.stream_ptr()), "fs_coupling_density_fwd")
        else:
            pair.post(c, x, params, uw, uh, ud, lq_in, out, lq)
        ctx.save_for_backward(h, w, x, params, uw, uh, ud)
        ctx.bias = b
        ctx.direct = _direct_grads
        # dh left as split-K partials for its readers (decided here: _direct_grads is a
        # forward-time setting)
        # Only when h's producer said in its forward that its backward sums the partials on
        # load (_BnReluLinear, _fs_splitk_reader) and nothing else is registered to read gh
        # (retain_grad, tensor hooks): any other reader would see the unreduced placeholder.
        ctx.defer = (_defer_splitk and _fold_ok(h.shape[0], h.shape[1], h.shape[1])
                     and getattr(h, "_fs_splitk_reader", False) and not h.retains_grad
                     and not getattr(h, "_backward_hooks", None))
        if ctx.defer:
            global _sk_deferred
            _sk_deferred += 1
        ctx.layer = layer
        ctx.has_lq = lq_in is not None
        ctx.res = res
        ctx.set_materialize_grads(False)  # the last layer's out has no gradient: no zero fill
        return out, lq

    @staticmethod
    def backward(ctx, g_out, g_lq):
        from .. import _lib

        h, w, x, params, uw, uh, ud = ctx.saved_tensors
        layer = ctx.layer
        K = layer.num_bins
        L = _lib.load()
        p = _lib.ptr
        g_out = g_out.contiguous() if g_out is not None else None
        g_lq = g_lq.contiguous() if g_lq is not None else None
        M, H = h.shape
        n = x.shape[1] // 2
        P = n * (3 * K + 1)
        gx = torch.empty_like(x)
        gp = torch.empty_like(params)
        gu = torch.empty((M, P), dtype=torch.float32, device=x.device)
        c = _coupling_desc(layer, M)
        _density_bwd(c, x, params, uw, uh, ud, g_out, g_lq, gx, gp, gu)
        gh, gw = torch.empty_like(h), _grad_out(w, direct=ctx.direct)
        gb = _grad_out(ctx.bias, direct=ctx.direct)
        gs = _grad_out(uw, uh, ud, direct=ctx.direct)  # [uw | uh | ud] gradients, one row sum
        descs = [_lib.GemmF32(M, H, P, p(gp), P, 1, p(w), H, 1, None, None, 0, p(gh), H, None),  # dh = dparams W
                 _lib.GemmF32(P, H, M, p(gp), 1, P, p(h), H, 1, None, None, 0, p(gw), H, p(gb)),  # dW, db
                 _lib.GemmF32(P, 0, M, p(gu), 1, P, None, 0, 0, None, None, 0, None, 0, p(gs))]  # row sum of gu
        nws = sum(max(0, L.fs_linear_f32_splitk_floats(d)) for d in descs)
        ws = torch.empty((max(nws, 1),), dtype=torch.float32, device=x.device)
        arr = (ctypes.POINTER(_lib.GemmF32) * 3)(*[ctypes.pointer(d) for d in descs])
        # re-checked now: a retain_grad() or tensor hook registered on h after the forward
        # would otherwise receive the unreduced placeholder
        if ctx.defer and not (h.retains_grad or getattr(h, "_backward_hooks", None)):
            # dh's partials left for its readers (_sk_get): the reduction launch goes
            ch = ctypes.c_int32(1)
            _lib.check(L.fs_linear_f32_group_partial(arr, 3, p(ws), nws, 3, ctypes.byref(ch), _lib.stream_ptr()),
                       "fs_linear_f32_group_partial")
            if ch.value > 1:
                _splitk_pending[gh.data_ptr()] = (gh, ws, ch.value)
        else:
            _lib.check(L.fs_linear_f32_group(arr, 3, p(ws), nws, _lib.stream_ptr()), "fs_linear_f32_group")
        guw = gs[:n * K].view(n, K)
        guh = gs[n * K:2 * n * K].view(n, K)
        gud = gs[2 * n * K:].view(n, K + 1)
        if ctx.res is not None and ctx.needs_input_grad[3]:
            ctx.res.g = gx  # added by the layer's features backward (as _DensitySplines)
            gx = None
        return (gh, gw, gb, gx, guw, guh, gud, g_lq if ctx.has_lq else None, None, None, None)


def conditioner_from_features(net, t, pair=None):
    """ResidualNet.forward from the periodic features t (the rest of conditioner())."""
    if _fused_ok(net, t):
        return _conditioner_fused(net, t, pair)
    if pair is not None:
        raise ValueError("the paired passes need the fused train-mode conditioner")
    t = net.initial_layer(t)
    for blk in net.blocks:
        u = blk.batch_norm_layers[0](t)
        u = F.relu(u)
        u = blk.linear_layers[0](u)
        u = blk.batch_norm_layers[1](u)
        u = F.relu(u)
        u = blk.linear_layers[1](u)
        t = t + u
    return net.final_layer(t)


def density_step(layer, x, log_q, pair=None):
    """One layer of forward_kld on the device: (z, log_q + log_det), differentiable.
    pair: a _SamplingRider whose sampling-pass layer runs in the same launches."""
    p = layer.prqct
    # x feeds the features and the splines: the features backward adds the splines' x
    # gradient in its own launch (no autograd accumulation kernel)
    res = _ResidualGrad() if x.requires_grad and torch.is_grad_enabled() else None
    t = _Features.apply(x, layer, res, pair)
    u = p.unconditional_transform
    net = p.transform_net
    if _fused_ok(net, t) and _bn_in_load_ok(net):
        h = _conditioner_fused(net, t, pair, final=False)
        lf = net.final_layer
        return _FinalSplines.apply(h, lf.weight, lf.bias, x, u.unnormalized_widths, u.unnormalized_heights,
                                   u.unnormalized_derivatives, log_q, layer, res, pair)
    params = conditioner_from_features(net, t, pair)
    return _DensitySplines.apply(x, params, u.unnormalized_widths, u.unnormalized_heights,
                                 u.unnormalized_derivatives, log_q, layer, res, pair)


@torch.no_grad()
def sample_step(layer, z, log_q, nan_flag):
    """One layer of reverse_kld's sampling direction on the device, without autograd:
    (z, log_q - log_det); nan_flag (int32 [1]) |= 1 on a NaN discriminant."""
    from .. import _lib

    p = layer.prqct
    z = z.contiguous()
    rows = z.shape[0]
    u = p.unconditional_transform
    uw, uh, ud = (v.detach().contiguous() for v in (u.unnormalized_widths, u.unnormalized_heights,
                                                      u.unnormalized_derivatives))
    _check_shapes(layer, rows, None, uw, uh, ud)
    t = torch.empty_like(z)
    out = torch.empty_like(z)
    lad_u = torch.empty((rows,), dtype=torch.float32, device=z.device)
    c = _coupling_desc(layer, rows)
    L = _lib.load()
    _lib.require_device(z, uw, log_q, nan_flag)
    _lib.check(L.fs_coupling_sample_pre(ctypes.byref(c), _lib.ptr(z), _lib.ptr(uw), _lib.ptr(uh), _lib.ptr(ud),
                                        _lib.ptr(t), _lib.ptr(out), _lib.ptr(lad_u), _lib.ptr(nan_flag),
                                        _lib.stream_ptr()), "fs_coupling_sample_pre")
    params = conditioner_from_features(p.transform_net, t).contiguous()
    _check_shapes(layer, rows, params, uw, uh, ud)
    if log_q is not None and tuple(log_q.shape) != (rows,):
        raise ValueError("log_q must be [rows]")
    lq = torch.empty_like(lad_u)
    _lib.check(L.fs_coupling_sample_post(ctypes.byref(c), _lib.ptr(params), _lib.ptr(lad_u), _lib.ptr(log_q),
                                         _lib.ptr(out), _lib.ptr(lq), _lib.ptr(nan_flag), _lib.stream_ptr()),
               "fs_coupling_sample_post")
    return out, lq


# ---------------------------------------------------------------------------
# The training step's two passes in shared launches.  With ALPHA = 1 a step runs
# reverse_kld's sampling pass (no autograd: its loss only gates the step and its
# BatchNorms update their running statistics) and then forward_kld's density pass
# (main_algorithm_2.py:446-447).  The two are independent apart from those running
# statistics, and each launch of either is a few dozen workgroups on a 256-CU chip, so
# they run side by side: at step s the sampling pass is at layer s and the density pass at
# layer L-1-s, and every launch carries one problem of each (fs_linear_f32_ex2,
# fs_coupling_pair_pre / _post).  Each problem is computed exactly as alone.  The
# running-statistics updates, whose order the interleaving would change, are deferred:
# the batch mean / variance of every BatchNorm of both passes go to one buffer and
# fs_bn_running_update applies them at the end, sampling pass first, as the reference.


class FlatBatchNorm:
    """Every BatchNorm1d of a flow with its running buffers re-homed as rows of flat
    buffers (values unchanged), so that fs_bn_running_update can update all of them in one
    launch.  Needs one width and one momentum for all of them (the ResidualNets of a flow)."""

    def __init__(self, model):
        bns = [m for m in model.modules() if isinstance(m, torch.nn.BatchNorm1d)]
        if not bns:
            raise ValueError("no BatchNorm1d in the model")
        H, mom = bns[0].num_features, bns[0].momentum
        for bn in bns:
            if (bn.num_features != H or bn.momentum != mom or mom is None or not bn.track_running_stats
                    or bn.running_mean is None or not bn.affine):
                raise ValueError("BatchNorms of one width, one momentum, with running statistics")
        with torch.no_grad():
            self.rm = torch.stack([bn.running_mean.detach() for bn in bns]).contiguous()
            self.rv = torch.stack([bn.running_var.detach() for bn in bns]).contiguous()
            self.nbt = torch.stack([bn.num_batches_tracked.detach().reshape(()) for bn in bns]).contiguous()
        for i, bn in enumerate(bns):  # through register_buffer: the packed-image cache sees the new tensors
            bn.running_mean = self.rm[i]
            bn.running_var = self.rv[i]
            bn.num_batches_tracked = self.nbt[i]
        self.bns = bns
        self.index = {id(bn): i for i, bn in enumerate(bns)}
        self.H, self.momentum = H, float(mom)

    @classmethod
    def try_build(cls, model):
        try:
            return cls(model)
        except ValueError:
            return None

    def intact(self):
        """Still the flat buffers (a .to() to another device re-allocates them)."""
        return all(bn.running_mean.data_ptr() == self.rm[i].data_ptr() and
                   bn.running_var.data_ptr() == self.rv[i].data_ptr() and
                   bn.num_batches_tracked.data_ptr() == self.nbt[i].data_ptr() for i, bn in enumerate(self.bns))

    def update(self, stats, rows0, rows1, skip=None):
        """skip (int32 [1] device word, nullable): nothing is written when it is non-zero."""
        from .. import _lib

        _lib.check(_lib.load().fs_bn_running_update(len(self.bns), self.H, _lib.ptr(self.rm), _lib.ptr(self.rv),
                                                    _lib.ptr(self.nbt), _lib.ptr(stats), 2, int(rows0), int(rows1),
                                                    self.momentum, _lib.ptr(skip), _lib.stream_ptr()),
                   "fs_bn_running_update")

    def buffers(self):
        return [self.rm, self.rv, self.nbt]


class _SamplingRider:
    """reverse_kld's sampling pass, carried by the density pass's launches (see above):
    holds its state (rows z, log q, NaN flag, the current layer's activations) and builds
    its half of each shared launch."""

    def __init__(self, z, flat_bn):
        self.z = z.contiguous()
        self.lq = None
        # inside a captured training step: the graph's sticky word (train.py), never cleared
        self.nan_flag = _sticky_nan if _sticky_nan is not None else torch.zeros(1, dtype=torch.int32, device=z.device)
        self.fbn = flat_bn
        # [pass][BatchNorm][mean | biased variance][H]; pass 0 sampling, 1 density
        self.bnstats = torch.empty((2, len(flat_bn.bns), 2, flat_bn.H), dtype=torch.float32, device=z.device)
        self.layer = None
        self._post = None  # the last layers' post launch, carried by the next pre launch

    def bn_slots(self, bn, p):
        i = self.fbn.index[id(bn)]
        return self.bnstats[p, i, 0], self.bnstats[p, i, 1]

    def begin(self, layer):
        self.layer = layer
        u = layer.prqct.unconditional_transform
        self.u = tuple(v.detach().contiguous() for v in (u.unnormalized_widths, u.unnormalized_heights,
                                                         u.unnormalized_derivatives))
        _check_shapes(layer, self.z.shape[0], None, *self.u)

    def pre(self, c_density, x, t_density):
        """fs_coupling_sample_pre of this layer + fs_coupling_features_fwd of the density's;
        with the previous layers' post launch still pending, both in one launch
        (fs_coupling_pair_step)."""
        from .. import _lib

        z = self.z
        self.t = torch.empty_like(z)
        self.out = torch.empty_like(z)
        self.lad_u = torch.empty((z.shape[0],), dtype=torch.float32, device=z.device)
        self.cs = _coupling_desc(self.layer, z.shape[0])
        p = _lib.ptr
        q, self._post = self._post, None
        if (q is not None and q["out_d"].data_ptr() == x.data_ptr() and q["out"].data_ptr() == z.data_ptr()
                and x.is_contiguous() and z.is_contiguous()):
            _lib.check(_lib.load().fs_coupling_pair_step(
                ctypes.byref(q["cs"]), p(q["params"]), p(q["lad_u"]), p(q["lq_in"]), p(q["out"]), p(q["lq_out"]),
                p(self.nan_flag), ctypes.byref(self.cs), p(self.u[0]), p(self.u[1]), p(self.u[2]), p(self.t),
                p(self.out), p(self.lad_u), ctypes.byref(q["cd"]), p(q["x"]), p(q["params_d"]), p(q["uw"]),
                p(q["uh"]), p(q["ud"]), p(q["lq_in_d"]), p(q["out_d"]), p(q["lq_out_d"]), ctypes.byref(c_density),
                p(t_density), _lib.stream_ptr()), "fs_coupling_pair_step")
        else:
            if q is not None:
                self._launch_post(q)
            _lib.check(_lib.load().fs_coupling_pair_pre(ctypes.byref(self.cs), p(z), p(self.u[0]), p(self.u[1]),
                                                        p(self.u[2]), p(self.t), p(self.out), p(self.lad_u),
                                                        p(self.nan_flag), ctypes.byref(c_density), p(x), p(t_density),
                                                        _lib.stream_ptr()), "fs_coupling_pair_pre")
        self.h, self.hst = self.t, None

    def gemm(self, op):
        """This pass's half of a shared conditioner launch: (descriptor, BatchNorm or None,
        statistics output or None); commit() takes the result after the launch."""
        from .. import _lib

        net = self.layer.prqct.transform_net
        p = _lib.ptr
        bi = None
        r = None
        if op == "init":
            lin, x = net.initial_layer, self.h
        elif op == "final":
            lin, x = net.final_layer, self.h
        else:
            b, j = op
            blk = net.blocks[b]
            lin, bn = blk.linear_layers[j], blk.batch_norm_layers[j]
            x, xs = (self.h, self.hst) if j == 0 else (self.u0, self.u0st)
            if j == 1:
                r = self.h
            mean, var = self.bn_slots(bn, 0)
            M = x.shape[0]
            bi = _lib.BnIn(p(xs), (M + 31) // 32, M, p(bn.weight), p(bn.bias), float(bn.eps), float(bn.momentum),
                           None, None, None, p(mean), None, None, p(var))
        M, N = x.shape[0], lin.weight.shape[0]
        y = torch.empty((M, N), dtype=torch.float32, device=x.device)
        st = None if op == "final" else torch.empty(((M + 31) // 32, N, 2), dtype=torch.float32, device=x.device)
        self._pending = (op, y, st)
        return _gemm_desc(x, lin.weight.detach(), lin.bias.detach(), r, y), bi, st

    def commit(self):
        op, y, st = self._pending
        self._pending = None
        if op == "final":
            self.params = y
        elif op == "init" or op[1] == 1:
            self.h, self.hst = y, st
        else:
            self.u0, self.u0st = y, st

    def gemm_alone(self, op):
        """The final Linear on its own when the density's takes another path (split-K)."""
        from .. import _lib

        g, _, _ = self.gemm(op)
        _gemm(g, self.z.device)
        self.commit()

    def post(self, c_density, x, params, uw, uh, ud, lq_in, out, lq):
        """fs_coupling_sample_post of this layer + fs_coupling_density_fwd of the density's:
        left pending, so that the next layers' pre launch carries it (fs_coupling_pair_step);
        flush() launches it alone after the last layer.  The outputs are allocated here."""
        params_s = self.params.contiguous()
        _check_shapes(self.layer, self.z.shape[0], params_s, *self.u)
        lq_s = torch.empty_like(self.lad_u)
        self.flush()
        # every operand referenced until the launch
        self._post = dict(cs=self.cs, params=params_s, lad_u=self.lad_u, lq_in=self.lq, out=self.out, lq_out=lq_s,
                          cd=c_density, x=x, params_d=params, uw=uw, uh=uh, ud=ud, lq_in_d=lq_in, out_d=out,
                          lq_out_d=lq)
        self.z, self.lq = self.out, lq_s
        self.t = self.out = self.h = self.hst = self.u0 = self.u0st = self.params = None

    def _launch_post(self, q):
        from .. import _lib

        p = _lib.ptr
        _lib.check(_lib.load().fs_coupling_pair_post(ctypes.byref(q["cs"]), p(q["params"]), p(q["lad_u"]),
                                                     p(q["lq_in"]), p(q["out"]), p(q["lq_out"]), p(self.nan_flag),
                                                     ctypes.byref(q["cd"]), p(q["x"]), p(q["params_d"]), p(q["uw"]),
                                                     p(q["uh"]), p(q["ud"]), p(q["lq_in_d"]), p(q["out_d"]),
                                                     p(q["lq_out_d"]), _lib.stream_ptr()), "fs_coupling_pair_post")

    def flush(self):
        """Launch a pending post launch on its own (after the last layers)."""
        q, self._post = self._post, None
        if q is not None:
            self._launch_post(q)


_last_paired = False  # set by paired_kld (train.py reads it after a warm-up step)


def paired_ok(model, x, z, flat_bn):
    """The shared-launch passes apply: device f32 rows, every layer on the fused coupling
    kernels with the BatchNorm-in-load conditioner, one layer shape throughout, the flat
    BatchNorm buffers intact."""
    if flat_bn is None or not flat_bn.intact() or not torch.is_grad_enabled():
        return False
    flows = list(model.flows)
    if not flows or z.shape[0] < 2 or x.shape[0] < 2:
        return False
    f0 = flows[0]
    for f in flows:
        net = f.prqct.transform_net
        if not (fused_coupling_ok(f, x) and fused_coupling_ok(f, z) and _bn_in_load_ok(net)):
            return False
        if (f.num_bins, f.num_input_channels, f.num_hidden_channels, len(net.blocks)) != \
                (f0.num_bins, f0.num_input_channels, f0.num_hidden_channels, len(f0.prqct.transform_net.blocks)):
            return False
        for blk in net.blocks:
            for bn in blk.batch_norm_layers:
                if not (bn.training and id(bn) in flat_bn.index):
                    return False
    return True


def paired_kld(model, x, z, flat_bn, reduce=True):
    """forward_kld(x) (differentiable) and reverse_kld's sampling pass of the base draws z
    (no autograd) in shared launches; returns (forward_kld loss, samples, their log q), or
    with reduce=False forward_kld's per-row log q in place of the loss."""
    from .. import _lib

    flows = model.flows
    L = len(flows)
    rider = _SamplingRider(z, flat_bn)
    flush_features_bwd()  # nothing may be pending from an interrupted backward
    log_q = None
    xd = x
    global _direct_grads
    with _lib.on_device(x):
        _direct_grads = True  # the density pass is the only differentiable one here
        try:
            for s in range(L):
                rider.begin(flows[s])
                xd, log_q = density_step(flows[L - 1 - s], xd, log_q, pair=rider)
        finally:
            _direct_grads = False
        rider.flush()
        # the sampling pass's spline flags are in the sticky word already when captured:
        # the failing step and every later one leave the running statistics alone
        flat_bn.update(rider.bnstats, z.shape[0], x.shape[0], skip=_sticky_nan)
    global _last_paired, _flags_in_sticky
    _last_paired = True
    if _defer_nan and _sticky_nan is not None and rider.nan_flag is _sticky_nan:
        _flags_in_sticky = True  # the rider's flags are in the sticky word already
    else:
        _nan_flags.append(rider.nan_flag[0] != 0)
    check_nan_flags()
    return (-torch.mean(log_q) if reduce else log_q), rider.z, rider.lq
