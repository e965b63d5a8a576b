"""The training step's two passes in shared launches (autograd_flow.paired_kld,
fs_linear_f32_ex2, fs_coupling_pair_pre / _post, fs_bn_running_update): reverse_kld's
sampling pass rides along forward_kld's density pass.  Every problem is computed as it
is alone and the BatchNorm running statistics are applied afterwards in the reference's
order (sampling pass first, main_algorithm_2.py:446-447), so a step must give exactly
what the separate passes give: loss, every gradient, running statistics and counters."""
import ctypes

import numpy as np
import pytest
import torch

from flowstate import _lib
from flowstate.models import A2, build_flow, half_box
from flowstate.normflows import autograd_flow as AF
from flowstate.normflows.Energy import DoubleWellLJ
from flowstate.normflows.train import GraphedTrainStep, step_loss

pytestmark = pytest.mark.gpu


def _model(N, kw, seed=0):
    torch.manual_seed(seed)
    B = half_box(N)
    m = build_flow(N, bound=B, device="cpu", **kw)
    m.p = DoubleWellLJ(2 * N, N, 1.0, B, V0_list=[-10.0, -10.5], r0=1.2, k=15)
    m = m.cuda().train()
    m.q0.device = torch.device("cuda")
    return m


def _batch(N, rows, seed=3):
    B = half_box(N)
    g = np.random.default_rng(seed)
    return torch.from_numpy(((g.random((rows, 2 * N)) * 2 - 1) * B * 0.9).astype(np.float32)).cuda()


def _state(m):
    return [t.detach().clone() for t in list(m.parameters()) + list(m.buffers())]


@pytest.fixture
def no_fold():
    """The paired graphs without the BatchNorm-backward fold, so that their gradients are
    bit-comparable with the separate passes' (the fold reassociates the column sums)."""
    prev = AF._fold_bn
    AF._fold_bn = False
    yield
    AF._fold_bn = prev


@pytest.mark.parametrize("N,kw,rows", [(16, dict(L=4, H=64, nb=2, K=8), 96), (64, A2, 256), (16, dict(L=3, H=32, nb=1,
                                                                                                     K=5), 37)],
                         ids=["n16-h64", "a2-n64", "n16-ragged"])
def test_paired_step_matches_separate_passes(N, kw, rows, no_fold):
    ma, mb = _model(N, kw), _model(N, kw)
    fbn = AF.FlatBatchNorm(mb)
    x = _batch(N, rows)
    z = mb.q0(rows).cuda()
    assert AF.paired_ok(mb, x, z, fbn)
    for m in (ma, mb):
        for p in m.parameters():
            p.grad = None
    torch.cuda.manual_seed(11)
    la = step_loss(ma, x, rows, 1.0)
    la.backward()
    torch.cuda.manual_seed(11)
    lb = step_loss(mb, x, rows, 1.0, fbn)
    lb.backward()
    torch.cuda.synchronize()
    # the paired step's loss head (fs_kld_loss) sums in its own order: the loss within
    # float32 rounding, its gradient (-1 / rows per row) and so every parameter's exact
    torch.testing.assert_close(la, lb, rtol=2e-6, atol=0)
    for (na, pa), (nb_, pb) in zip(ma.named_parameters(), mb.named_parameters()):
        assert (pa.grad is None) == (pb.grad is None), na
        if pa.grad is not None:
            assert torch.equal(pa.grad, pb.grad), na
    for (na, ba), (nb_, bb) in zip(ma.named_buffers(), mb.named_buffers()):
        assert torch.equal(ba, bb), na  # running statistics in the reference's order, counters +2
    assert int(fbn.nbt[0]) == 2


def test_paired_graphed_steps_match_separate(no_fold):
    """GraphedTrainStep with the shared launches (the default) against paired=False over a
    few replays: parameters, Adam moments and BatchNorm buffers identical (the BatchNorm
    backward fold, which reassociates its column sums, off: test_bn_fold_matches_unfolded)."""
    N, rows = 16, 128
    kw = dict(L=4, H=64, nb=2, K=8)
    out = []
    for paired in (True, False):
        m = _model(N, kw, seed=4)
        x = _batch(N, rows, seed=5)
        torch.cuda.manual_seed(7)
        g = GraphedTrainStep(m, rows, lr=1e-3, weight_decay=1e-4, alpha=1.0, example=x, paired=paired)
        assert (g.flat_bn is not None) == paired
        for k in range(3):
            g.step(_batch(N, rows, seed=10 + k))
        torch.cuda.synchronize()
        out.append(_state(m) + [t.clone() for t in g._state_tensors])
    for a, b in zip(*out):
        assert torch.equal(a, b)


def test_paired_launch_count():
    """The paired step's forward half: per layer step 7 launches carry both passes
    (6 conditioner + one coupling launch that holds this layer's post and the next layer's
    pre, fs_coupling_pair_step; one more after the last layer), against 16 when the passes
    run one after the other."""
    from torch.profiler import ProfilerActivity, profile

    N, rows = 16, 64
    kw = dict(L=4, H=64, nb=2, K=8)
    m = _model(N, kw)
    fbn = AF.FlatBatchNorm(m)
    x = _batch(N, rows)
    counts = {}
    for mode in ("paired", "separate"):
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            loss = step_loss(m, x, rows, 1.0, fbn if mode == "paired" else None)
            torch.cuda.synchronize()
        names = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
        if not names:
            pytest.skip("the profiler recorded no device kernels")
        counts[mode] = sum(1 for n in names if "gemm" in n or "coupling" in n)
        del loss
    L = kw["L"]
    assert counts["paired"] == 7 * L + 1, counts
    assert counts["separate"] == 16 * L, counts


class coupling_waves:
    """The training step's coupling launches with each row's splines on two / four waves
    (1) or on one / two (0), for a block."""

    def __init__(self, on):
        self.on = on

    def __enter__(self):
        self.prev = _lib.load().fs_set_coupling_waves(self.on)

    def __exit__(self, *exc):
        _lib.load().fs_set_coupling_waves(self.prev)


@pytest.mark.parametrize("N,kw,rows", [(16, dict(L=4, H=64, nb=2, K=8), 96), (64, A2, 256), (16, dict(L=3, H=32, nb=1,
                                                                                                     K=5), 37),
                                       (8, dict(L=3, H=32, nb=1, K=32), 50)],
                         ids=["n16-h64", "a2-n64", "n16-ragged", "n8-k32"])
def test_coupling_waves_bit_identical(N, kw, rows):
    """fs_coupling_pair_step / fs_coupling_bwd_step with each row's knot sets built on
    separate waves against one wave per spline: loss, every gradient and BatchNorm buffer
    identical, with inputs outside the tail bound on some coordinates (identity branches)."""
    outs = []
    for on in (1, 0):
        with coupling_waves(on):
            m = _model(N, kw, seed=2)
            fbn = AF.FlatBatchNorm(m)
            x = _batch(N, rows, seed=6)
            x[::7, ::5] *= 1.2  # beyond the bound: the identity branches
            for p in m.parameters():
                p.grad = None
            torch.cuda.manual_seed(13)
            loss = step_loss(m, x, rows, 1.0, fbn)
            loss.backward()
            torch.cuda.synchronize()
            outs.append([loss.detach().clone()] + [p.grad.clone() for p in m.parameters() if p.grad is not None]
                        + [b.clone() for b in m.buffers()])
    assert len(outs[0]) == len(outs[1])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("N,kw,rows", [(16, dict(L=4, H=64, nb=2, K=8), 96), (64, A2, 256), (16, dict(L=3, H=32, nb=1,
                                                                                                     K=5), 37),
                                       (16, dict(L=2, H=256, nb=3, K=8), 64), (64, A2, 232)],
                         ids=["n16-h64", "a2-n64", "n16-ragged", "n16-h256-nb3", "a2-n64-232"])
def test_bn_fold_matches_unfolded(N, kw, rows):
    """Every BatchNorm backward of the conditioner folded into the backward pairs around it
    (fs_linear_f32_pair_bn: per-tile sums in the producing pair's epilogue, dy loaded on the
    fly by the consuming pair, + the residual gradient for a block's first BatchNorm, whose
    consumer is the previous block's second Linear or the initial layer) against the
    separate fs_bn_relu_train_bwd launches: the same loss and buffers, every gradient within
    float32 reassociation (the BatchNorms' column sums are taken per 32-row tile, then over
    tiles), and no BatchNorm-backward launch left (batches that are a multiple of 4; the
    ragged one keeps them all)."""
    from torch.profiler import ProfilerActivity, profile

    outs, counts = [], []
    prev = AF._fold_bn
    try:
        for fold in (True, False):
            AF._fold_bn = fold
            m = _model(N, kw, seed=2)
            fbn = AF.FlatBatchNorm(m)
            x = _batch(N, rows, seed=6)
            for p in m.parameters():
                p.grad = None
            torch.cuda.manual_seed(13)
            with profile(activities=[ProfilerActivity.CUDA]) as prof:
                loss = step_loss(m, x, rows, 1.0, fbn)
                loss.backward()
                torch.cuda.synchronize()
            names = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
            counts.append(sum(1 for n in names if "bn_relu_train_bwd" in n))
            outs.append((loss.detach().clone(), {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None},
                         [b.clone() for b in m.buffers()]))
    finally:
        AF._fold_bn = prev
    (la, ga, ba), (lb, gb, bb) = outs
    assert torch.equal(la, lb)
    assert ga.keys() == gb.keys()
    for n in ga:
        scale = float(gb[n].abs().max()) + 1e-30
        torch.testing.assert_close(ga[n], gb[n], rtol=1e-4, atol=2e-5 * scale, msg=n)
    for a, b in zip(ba, bb):
        assert torch.equal(a, b)
    if counts[1]:  # the profiler saw device kernels
        L, nb = kw["L"], kw["nb"]
        folded = rows % 4 == 0  # the lean weight-gradient kernels reduce the batch in quads
        assert counts == [0 if folded else 2 * L * nb, 2 * L * nb], counts


@pytest.mark.parametrize("B,R", [(256, 256), (37, 37), (1, 5), (1000, 300)])
def test_kld_loss_head(B, R):
    """fs_kld_loss / fs_kld_loss_backward (autograd_flow._KldLoss) against the torch
    expression of main_algorithm_2.py:316-318 at ALPHA = 1: the value within float32
    rounding (ordered tree sums), the gradient bit for bit, NaN / inf of the zero-weighted
    reverse term kept, and the sticky word's state written as a bool."""
    g = torch.Generator().manual_seed(B)
    lq = (torch.randn(B, generator=g) * 40 - 100).cuda().requires_grad_(True)
    E = (torch.randn(R, generator=g) * 1e3).cuda()
    lqs = (torch.randn(R, generator=g) * 40).cuda()
    want = -torch.mean(lq) + 0.0 * (torch.mean(E) + torch.mean(lqs))
    (gw,) = torch.autograd.grad(want, lq)
    got = AF.kld_loss(lq, E, lqs)
    assert got.grad_fn is not None and "KldLoss" in type(got.grad_fn).__name__
    (gg,) = torch.autograd.grad(got, lq)
    torch.testing.assert_close(got, want, rtol=2e-6, atol=0)
    assert torch.equal(gg, gw)
    (gg2,) = torch.autograd.grad(AF.kld_loss(lq, E, lqs), lq, torch.tensor(3.5, device="cuda"))
    (gw2,) = torch.autograd.grad(-torch.mean(lq) + 0.0 * E.sum(), lq, torch.tensor(3.5, device="cuda"))
    assert torch.equal(gg2, gw2)
    for bad in (float("inf"), float("nan")):
        E2 = E.clone()
        E2[R // 2] = bad
        assert torch.isnan(AF.kld_loss(lq.detach(), E2, lqs))
    L = _lib.load()
    for word in (0, 4):
        w = torch.tensor([word], dtype=torch.int32, device="cuda")
        loss = torch.empty((), device="cuda")
        flag = torch.full((), True, dtype=torch.bool, device="cuda") if word == 0 else \
            torch.zeros((), dtype=torch.bool, device="cuda")
        _lib.check(L.fs_kld_loss(_lib.ptr(lq), B, _lib.ptr(E), _lib.ptr(lqs), R, _lib.ptr(w), _lib.ptr(loss),
                                 _lib.ptr(flag), _lib.stream_ptr()))
        assert bool(flag) == (word != 0)
        torch.testing.assert_close(loss, want.detach(), rtol=2e-6, atol=0)


@pytest.mark.parametrize("N,kw,rows", [(16, dict(L=4, H=64, nb=2, K=8), 96), (64, A2, 256),
                                       (16, dict(L=3, H=32, nb=1, K=5), 64), (16, dict(L=2, H=256, nb=3, K=8), 64)],
                         ids=["n16-h64", "a2-n64", "n16-nb1", "n16-h256-nb3"])
def test_deferred_splitk_matches_reduced(N, kw, rows):
    """The final Linear's input gradient left as split-K partials (fs_linear_f32_group_partial)
    and summed on load by its two readers (the last block's second Linear backward as A, the
    block's first BatchNorm fold as dx_add; fs_linear_f32_pair_bn_sk) against the reduction
    launch: the same loss, every gradient and buffer bit for bit, and no splitk_reduce_kernel
    left when the reduction input is the split product (K = n (3K+1) >= 2048)."""
    from torch.profiler import ProfilerActivity, profile

    outs, counts = [], []
    prev = AF._defer_splitk
    try:
        for defer in (True, False):
            AF._defer_splitk = defer
            m = _model(N, kw, seed=3)
            fbn = AF.FlatBatchNorm(m)
            x = _batch(N, rows, seed=8)
            for p in m.parameters():
                p.grad = None
            torch.cuda.manual_seed(17)
            with profile(activities=[ProfilerActivity.CUDA]) as prof:
                loss = step_loss(m, x, rows, 1.0, fbn)
                registered = []
                AF._splitk_pending = _Recording(registered)
                try:
                    loss.backward()
                    assert not AF._splitk_pending  # every placeholder consumed by its last reader
                finally:
                    AF._splitk_pending = {}
                torch.cuda.synchronize()
            split = N * (3 * kw["K"] + 1) >= 2048  # n (3K+1), n = D / 2 = N features
            assert len(registered) == (kw["L"] if defer and split else 0)  # one deferred dh per layer
            names = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
            counts.append(sum(1 for n in names if "splitk_reduce" in n))
            outs.append((loss.detach().clone(), {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None},
                         [b.clone() for b in m.buffers()]))
    finally:
        AF._defer_splitk = prev
    (la, ga, ba), (lb, gb, bb) = outs
    assert torch.equal(la, lb)
    assert ga.keys() == gb.keys()
    for n in ga:
        assert torch.equal(ga[n], gb[n]), n
    for a, b in zip(ba, bb):
        assert torch.equal(a, b)
    if counts[1]:  # the profiler saw device kernels
        assert counts[0] == (0 if split else counts[1]), counts


class _Recording(dict):
    """AF._splitk_pending that records every placeholder registered."""

    def __init__(self, log):
        super().__init__()
        self.log = log

    def __setitem__(self, k, v):
        self.log.append(k)
        super().__setitem__(k, v)


def test_splitk_partial_entry_points():
    """fs_linear_f32_group_partial + fs_splitk_sum give fs_linear_f32_group's values bit for
    bit; fs_linear_f32_pair_bn_sk with A as 3 partials equals fs_linear_f32_pair_bn on the
    reduced A, and writes that reduced A out (fout->a_out)."""
    L = _lib.load()
    p = _lib.ptr
    g = torch.Generator().manual_seed(5)
    M, H, P = 256, 128, 2944
    gp = torch.randn((M, P), generator=g).cuda()
    w = torch.randn((P, H), generator=g).cuda() * 0.05
    outs = []
    for partial in (False, True):
        gh = torch.full((M, H), float("nan"), device="cuda")
        d = _lib.GemmF32(M, H, P, p(gp), P, 1, p(w), H, 1, None, None, 0, p(gh), H, None)
        nws = L.fs_linear_f32_splitk_floats(d)
        ws = torch.empty((nws,), device="cuda")
        arr = (ctypes.POINTER(_lib.GemmF32) * 1)(ctypes.pointer(d))
        if partial:
            ch = ctypes.c_int32(0)
            _lib.check(L.fs_linear_f32_group_partial(arr, 1, p(ws), nws, 3, ctypes.byref(ch), _lib.stream_ptr()))
            assert ch.value == 3 and torch.isnan(gh).all()  # C not written: its partials are in ws
            _lib.check(L.fs_splitk_sum(p(ws), ch.value, M * H, M * H, p(gh), _lib.stream_ptr()))
            outs.append((gh, ws, ch.value))
        else:
            _lib.check(L.fs_linear_f32_group(arr, 1, p(ws), nws, _lib.stream_ptr()))
            outs.append((gh, ws, 1))
    torch.cuda.synchronize()
    # the chunking differs (3 partials against the plan's), so the sums agree within rounding
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-5, atol=1e-5)
    gh, ws, ch = outs[1]
    # the pair on the reduced A against the pair summing the partials on load
    K2 = 128
    u = torch.rand((M, K2), generator=g).cuda()
    wl = torch.randn((H, K2), generator=g).cuda() * 0.1
    x = torch.randn((M, K2), generator=g).cuda()
    mean, invstd = x.mean(0), torch.rsqrt(x.var(0, unbiased=False) + 1e-5)
    gamma = torch.rand(K2, generator=g).cuda() + 0.5
    res = []
    for sk in (False, True):
        gu = torch.empty((M, K2), device="cuda")
        gw = torch.empty((H, K2), device="cuda")
        gb = torch.empty((H,), device="cuda")
        part = torch.empty(((M + 31) // 32, K2, 2), device="cuda")
        a = p(ws) if sk else p(gh)
        g0 = _lib.GemmF32(M, K2, H, a, H, 1, p(wl), K2, 1, None, None, 0, p(gu), K2, None)
        g1 = _lib.GemmF32(H, K2, M, a, 1, H, p(u), K2, 1, None, None, 0, p(gw), K2, p(gb))
        aout = torch.full((M, H), float("nan"), device="cuda")
        fo = _lib.BnFold(p(gu), p(u), p(x), p(mean), p(invstd), p(gamma), p(part), None, None, None,
                         p(aout) if sk else None, M, K2)
        if sk:
            _lib.check(L.fs_linear_f32_pair_bn_sk(g0, g1, None, fo, ch, M * H, 1, 0, _lib.stream_ptr()))
        else:
            _lib.check(L.fs_linear_f32_pair_bn(g0, g1, None, fo, _lib.stream_ptr()))
        res.append((gu, gw, gb, part))
    torch.cuda.synchronize()
    for a, b in zip(*res):
        assert torch.equal(a, b)
    assert torch.equal(aout, gh)  # the reduced A written out (fout->a_out) for its other readers


def test_splitk_dx_add_consumer():
    """fs_linear_f32_pair_bn_sk's consumer form: the folded BatchNorm's residual gradient
    dx_add given as 3 split-K partials (add_chunks) against the same pair on the reduced
    dx_add: input / weight / bias gradients, dgamma / dbeta and dy written out, bit for bit."""
    L = _lib.load()
    p = _lib.ptr
    g = torch.Generator().manual_seed(9)
    M, H, P, K3 = 256, 128, 2944, 128
    gp = torch.randn((M, P), generator=g).cuda()
    w = torch.randn((P, H), generator=g).cuda() * 0.05
    gh = torch.empty((M, H), device="cuda")
    d = _lib.GemmF32(M, H, P, p(gp), P, 1, p(w), H, 1, None, None, 0, p(gh), H, None)
    nws = L.fs_linear_f32_splitk_floats(d)
    ws = torch.empty((nws,), device="cuda")
    ch = ctypes.c_int32(0)
    arr = (ctypes.POINTER(_lib.GemmF32) * 1)(ctypes.pointer(d))
    _lib.check(L.fs_linear_f32_group_partial(arr, 1, p(ws), nws, 3, ctypes.byref(ch), _lib.stream_ptr()))
    _lib.check(L.fs_splitk_sum(p(ws), ch.value, M * H, M * H, p(gh), _lib.stream_ptr()))
    gu2 = torch.randn((M, H), generator=g).cuda()
    y2 = torch.randn((M, H), generator=g).cuda()
    u2 = torch.relu(y2 + 0.1)
    mean2, invstd2 = y2.mean(0), torch.rsqrt(y2.var(0, unbiased=False) + 1e-5)
    gamma2 = (torch.rand(H, generator=g) + 0.5).cuda()
    part2 = torch.randn(((M + 31) // 32, H, 2), generator=g).cuda()
    w3 = torch.randn((H, K3), generator=g).cuda() * 0.1
    x3 = torch.randn((M, K3), generator=g).cuda()
    res = []
    for sk in (False, True):
        gx = torch.empty((M, K3), device="cuda")
        gw3 = torch.empty((H, K3), device="cuda")
        gb3 = torch.empty((H,), device="cuda")
        dg = torch.empty((H,), device="cuda")
        db = torch.empty((H,), device="cuda")
        aout = torch.empty((M, H), device="cuda")
        g0 = _lib.GemmF32(M, K3, H, p(gu2), H, 1, p(w3), K3, 1, None, None, 0, p(gx), K3, None)
        g1 = _lib.GemmF32(H, K3, M, p(gu2), 1, H, p(x3), K3, 1, None, None, 0, p(gw3), K3, p(gb3))
        fi = _lib.BnFold(p(gu2), p(u2), p(y2), p(mean2), p(invstd2), p(gamma2), p(part2), p(dg), p(db),
                         p(ws) if sk else p(gh), p(aout), M, H)
        if sk:
            _lib.check(L.fs_linear_f32_pair_bn_sk(g0, g1, fi, None, 1, 0, ch.value, M * H, _lib.stream_ptr()))
        else:
            _lib.check(L.fs_linear_f32_pair_bn(g0, g1, fi, None, _lib.stream_ptr()))
        res.append((gx, gw3, gb3, dg, db, aout))
    torch.cuda.synchronize()
    for a, b in zip(*res):
        assert torch.isfinite(a).all() and torch.equal(a, b)
