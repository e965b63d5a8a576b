"""The fused train-mode conditioner (csrc/train_kernels.hip: fs_linear_f32,
fs_bn_relu_train_fwd / _bwd) against torch's own nn.Linear / nn.BatchNorm1d / ReLU
modules on the same device: outputs, every gradient, running statistics and
num_batches_tracked (ResidualNet in train mode, NF/normflows/nets/resnet.py:35-104).
Tolerance: f32 with different summation orders (rtol 1e-4 on values scaled by their
largest magnitude)."""
import copy

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from flowstate import _lib
from flowstate.normflows import autograd_flow as AF
from flowstate.normflows.flows import _ResidualNet

pytestmark = pytest.mark.gpu


def close(a, b, rtol=1e-4, what=""):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    if b.numel() == 0:
        return
    scale = max(1.0, float(b.abs().max()))
    err = float((a - b).abs().max())
    assert err <= rtol * scale, (what, err, scale)


def gemm(M, N, K, A, sam, sak, B, sbk, sbn, bias=None, R=None, rowsum=None):
    C = torch.empty((M, N), device="cuda")
    _lib.check(_lib.load().fs_linear_f32(M, N, K, _lib.ptr(A), sam, sak, _lib.ptr(B), sbk, sbn, _lib.ptr(bias),
                                         _lib.ptr(R), N, _lib.ptr(C), N, _lib.ptr(rowsum), _lib.stream_ptr()),
               "fs_linear_f32")
    return C


@pytest.mark.parametrize("M,N,K", [(256, 128, 128), (256, 2944, 128), (37, 45, 13), (1, 1, 1), (64, 32, 3000),
                                   (300, 70, 0)])
def test_linear_f32_layouts(M, N, K):
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K)
    x = torch.randn(M, K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g)
    b = torch.randn(N, device="cuda", generator=g)
    r = torch.randn(M, N, device="cuda", generator=g)
    ref = (x.double() @ w.double().t() + b.double() + r.double())
    close(gemm(M, N, K, x, K, 1, w, 1, K, b, r), ref, 1e-5, "forward")
    dy = torch.randn(M, N, device="cuda", generator=g)
    close(gemm(M, K, N, dy, N, 1, w, K, 1), dy.double() @ w.double(), 1e-5, "input grad")
    rs = torch.empty(N, device="cuda")
    close(gemm(N, K, M, dy, 1, N, x, K, 1, rowsum=rs), dy.double().t() @ x.double(), 1e-5, "weight grad")
    close(rs, dy.double().sum(0), 1e-5, "bias grad")


@pytest.mark.parametrize("M,N,K", [(256, 128, 2944), (40, 24, 2051), (64, 32, 3000)])
def test_linear_f32_splitk(M, N, K):
    """The split-K path (long reductions over few tiles: the final layer's input gradient)
    against float64, with bias and residual; too small a workspace falls back to the
    single-phase kernel."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    x = torch.randn(M, K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g)
    b = torch.randn(N, device="cuda", generator=g)
    r = torch.randn(M, N, device="cuda", generator=g)
    ref = x.double() @ w.double().t() + b.double() + r.double()
    L, p = _lib.load(), _lib.ptr
    outs = []
    for short in (False, True):
        y = torch.empty((M, N), device="cuda")
        d = _lib.GemmF32(M, N, K, p(x), K, 1, p(w), 1, K, p(b), p(r), N, p(y), N, None)
        n = L.fs_linear_f32_splitk_floats(d)
        assert n > 0
        ws = torch.empty(n, device="cuda")
        _lib.check(L.fs_linear_f32_splitk(d, p(ws), n - 1 if short else n, _lib.stream_ptr()))
        close(y, ref, 1e-5, "split-K" if not short else "fallback")
        outs.append(y)


def module_path(net, t):
    """The reference's ResidualNet.forward on torch modules (resnet.py:37-50, 92-104)."""
    t = net.initial_layer(t)
    for blk in net.blocks:
        u = F.relu(blk.batch_norm_layers[0](t))
        u = blk.linear_layers[0](u)
        u = F.relu(blk.batch_norm_layers[1](u))
        u = blk.linear_layers[1](u)
        t = t + u
    return net.final_layer(t)


@pytest.mark.parametrize("batch", [256, 64, 2, 37])
def test_conditioner_fused_matches_modules(batch):
    torch.manual_seed(batch)
    net = _ResidualNet(128, 64 * 46, 128, 2, None).cuda()
    for blk in net.blocks:  # non-trivial BatchNorm affine parameters and running stats
        for bn in blk.batch_norm_layers:
            with torch.no_grad():
                bn.weight.uniform_(0.5, 1.5)
                bn.bias.uniform_(-0.2, 0.2)
                bn.running_mean.uniform_(-0.1, 0.1)
                bn.running_var.uniform_(0.5, 1.5)
        with torch.no_grad():
            blk.linear_layers[1].weight.normal_(0, 0.05)
    with torch.no_grad():
        net.final_layer.weight.normal_(0, 0.05)
    ref = copy.deepcopy(net)
    net.train()
    ref.train()
    t = torch.randn(batch, 128, device="cuda")
    t1 = t.clone().requires_grad_(True)
    t2 = t.clone().requires_grad_(True)
    assert AF._fused_ok(net, t1)
    y1 = AF._conditioner_fused(net, t1)
    y2 = module_path(ref, t2)
    close(y1, y2, 1e-4, "output")
    gy = torch.randn_like(y1)
    (y1 * gy).sum().backward()
    (y2 * gy).sum().backward()
    close(t1.grad, t2.grad, 1e-4, "input grad")
    for (n, p1), (_, p2) in zip(net.named_parameters(), ref.named_parameters()):
        close(p1.grad, p2.grad, 1e-4, n)
    for (n, b1), (_, b2) in zip(net.named_buffers(), ref.named_buffers()):
        if b1.dtype == torch.int64:
            assert torch.equal(b1, b2), n
        else:
            close(b1, b2, 1e-5, n)
    # under no_grad (reverse_kld with ALPHA = 1): same values, statistics still updated
    with torch.no_grad():
        close(AF._conditioner_fused(net, t), module_path(ref, t), 1e-4, "no-grad output")
    for (n, b1), (_, b2) in zip(net.named_buffers(), ref.named_buffers()):
        if b1.dtype == torch.int64:
            assert int(b1) == int(b2) == 2, n


def test_conditioner_falls_back_outside_train_mode():
    net = _ResidualNet(128, 64 * 46, 128, 2, None).cuda()
    t = torch.randn(8, 128, device="cuda")
    net.eval()
    assert not AF._fused_ok(net, t)
    net.train()
    assert AF._fused_ok(net, t)
    assert not AF._fused_ok(net, t[:1])  # torch raises on a batch of one in train mode


def a2_layer(seed, N=64, K=15, H=128):
    from flowstate.models import build_flow, half_box

    torch.manual_seed(seed)
    m = build_flow(N, bound=half_box(N), device="cpu", L=1, H=H, nb=2, K=K)
    layer = m.flows[0]
    with torch.no_grad():  # leave the identity init: non-trivial splines and BatchNorm
        for prm in layer.parameters():
            prm.add_(0.05 * torch.randn_like(prm))
    return layer.cuda()


@pytest.mark.parametrize("K", [15, 8])
def test_density_step_matches_torch_ops(K):
    """density_step (fs_coupling_features_* + fs_coupling_density_*) against
    coupling_density over torch ops: outputs, log q, input and parameter gradients,
    running statistics; rows include coordinates outside [-B, B] (identity tails)."""
    layer = a2_layer(5, K=K)
    ref = copy.deepcopy(layer)
    layer.train()
    ref.train()
    B = layer.tail_bound
    g = torch.Generator(device="cuda").manual_seed(1)
    x = (torch.rand(256, layer.num_input_channels, device="cuda", generator=g) * 2 - 1) * B
    x[:8, :5] = B * 1.5  # outside the tails: identity, log-det 0
    lq0 = torch.randn(256, device="cuda", generator=g)
    x1 = x.clone().requires_grad_(True)
    x2 = x.clone().requires_grad_(True)
    assert AF.fused_coupling_ok(layer, x1)
    z1, lq1 = AF.density_step(layer, x1, lq0)
    z2, ld2 = AF.coupling_density(ref, x2)
    lq2 = lq0 + ld2
    close(z1, z2, 1e-5, "z")
    close(lq1, lq2, 1e-5, "log q")
    gz = torch.randn_like(z1)
    gl = torch.randn_like(lq1)
    ((z1 * gz).sum() + (lq1 * gl).sum()).backward()
    ((z2 * gz).sum() + (lq2 * gl).sum()).backward()
    close(x1.grad, x2.grad, 1e-4, "x grad")
    for (n, p1), (_, p2) in zip(layer.named_parameters(), ref.named_parameters()):
        if p2.grad is None:
            assert p1.grad is None or not p1.grad.abs().max().item(), n
            continue
        close(p1.grad, p2.grad, 1e-4, n)
    for (n, b1), (_, b2) in zip(layer.named_buffers(), ref.named_buffers()):
        if b1.dtype == torch.int64:
            assert torch.equal(b1, b2), n
        else:
            close(b1, b2, 1e-5, n)


def test_sample_step_matches_torch_ops():
    """sample_step (fs_coupling_sample_pre / _post) against coupling_sample, no autograd."""
    layer = a2_layer(6)
    ref = copy.deepcopy(layer)
    layer.train()
    ref.train()
    B = layer.tail_bound
    g = torch.Generator(device="cuda").manual_seed(2)
    z = (torch.rand(256, layer.num_input_channels, device="cuda", generator=g) * 2 - 1) * B
    z[3:6, 7:9] = -B * 1.2
    lq0 = torch.randn(256, device="cuda", generator=g)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    with torch.no_grad():
        z1, lq1 = AF.sample_step(layer, z, lq0, flag)
        z2, ld2 = AF.coupling_sample(ref, z)
        AF._nan_flags.clear()
    close(z1, z2, 1e-5, "z")
    close(lq1, lq0 - ld2, 1e-5, "log q")
    assert int(flag.item()) == 0
    for (n, b1), (_, b2) in zip(layer.named_buffers(), ref.named_buffers()):
        if b1.dtype == torch.int64:
            assert torch.equal(b1, b2), n
        else:
            close(b1, b2, 1e-5, n)
