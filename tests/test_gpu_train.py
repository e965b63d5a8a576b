"""Algorithm-2 training on the MI355X (PyTorch-ROCm autograd over the layers) against
the reference's values, and the hand-off to the HIP inference kernels: after an Adam
step the packed image is rebuilt and the fused log_prob matches the autograd
path's eval-mode density."""
import numpy as np
import pytest
import torch

from test_train_cpu import build, check_training

pytestmark = pytest.mark.gpu


def test_training_step_matches_reference_gpu():
    check_training("cuda", rtol_loss=2e-5, rtol_grad=2e-3, atol_grad=2e-5)


def test_inference_kernels_see_trained_parameters():
    from flowstate.normflows import autograd_flow as AF

    m, f = build("cuda")
    x = torch.from_numpy(f["x"]).cuda()
    m.eval()
    before = m.log_prob(x).clone()
    m.train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-2)
    for _ in range(3):
        opt.zero_grad()
        m.forward_kld(x).backward()
        opt.step()
    m.eval()
    after = m.log_prob(x)
    assert (after - before).abs().max().item() > 1e-3  # the kernels picked up the new weights
    with torch.no_grad():
        z, lq = x, torch.zeros(len(x), device=x.device)
        for i in range(len(m.flows) - 1, -1, -1):
            z, ld = AF.coupling_density(m.flows[i], z)
            lq += ld
        lq += m.q0.log_prob(z)
    np.testing.assert_allclose(after.cpu().numpy(), lq.cpu().numpy(), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("N", [4, 16, 64])
def test_target_energy_kernel_matches_reference(N):
    """DoubleWellLJ._energy on the device runs fs_target_energy (csrc/target_kernels.hip):
    energies and dE/dx against the reference's (tests/golden/target_energy.npz)."""
    from test_train_cpu import _target_case, check_target_energy

    f, mod = _target_case(N)
    x = torch.from_numpy(f[f"N{N}_x"]).cuda().requires_grad_(True)
    E = mod._energy(x)
    assert "TargetEnergy" in type(E.grad_fn).__name__  # the HIP kernel, not the torch restatement
    (gx,) = torch.autograd.grad(E.sum(), x)
    check_target_energy(mod, f, N, x, E, gx)
    with torch.no_grad():
        E2 = mod._energy(x.detach())
    # the energy-only launch (target_energy_only_kernel): the same float32 pair energies,
    # summed in double in another order, rounded once: equal up to that last rounding
    torch.testing.assert_close(E2, E.detach(), rtol=1.2e-7, atol=0)
    check_target_energy(mod, f, N, x, E2, gx)


def test_linear_residual_path_gradcheck():
    """_Linear's residual input r with res=None (no side channel) returns its gradient to
    autograd: numerical gradcheck in float32 with float32-sized steps."""
    from flowstate.normflows.autograd_flow import _Linear

    g = torch.Generator().manual_seed(0)
    x = torch.randn((40, 24), generator=g).cuda().requires_grad_(True)
    w = (torch.randn((16, 24), generator=g) * 0.3).cuda().requires_grad_(True)
    b = torch.randn(16, generator=g).cuda().requires_grad_(True)
    r = torch.randn((40, 16), generator=g).cuda().requires_grad_(True)
    assert torch.autograd.gradcheck(lambda *t: _Linear.apply(*t, None), (x, w, b, r), eps=1e-2, atol=2e-2,
                                    rtol=1e-2, nondet_tol=1e-5)
    y = _Linear.apply(x, w, b, r, None)
    (gr,) = torch.autograd.grad(y.sum() * 2.0, r)
    torch.testing.assert_close(gr, torch.full_like(r, 2.0))


def test_linear_pair_launch_matches_two_launches():
    """fs_linear_f32_pair (nn.Linear's backward in one launch) gives exactly what the two
    fs_linear_f32 calls give, at the A2 training shapes and a ragged one."""
    from flowstate import _lib

    L, p = _lib.load(), _lib.ptr
    g = torch.Generator().manual_seed(1)
    for M, K, N in ((256, 128, 128), (232, 128, 128), (256, 128, 96), (37, 40, 24)):
        x = torch.randn((M, K), generator=g).cuda()
        w = torch.randn((N, K), generator=g).cuda()
        gy = torch.randn((M, N), generator=g).cuda()
        outs = []
        for pair in (True, False):
            gx, gw, gb = torch.empty_like(x), torch.empty_like(w), torch.empty(N, device="cuda")
            g0 = _lib.GemmF32(M, K, N, p(gy), N, 1, p(w), K, 1, None, None, 0, p(gx), K, None)
            g1 = _lib.GemmF32(N, K, M, p(gy), 1, N, p(x), K, 1, None, None, 0, p(gw), K, p(gb))
            if pair:
                _lib.check(L.fs_linear_f32_pair(g0, g1, _lib.stream_ptr()))
            else:
                for gg in (g0, g1):
                    _lib.check(L.fs_linear_f32(gg.M, gg.N, gg.K, gg.A, gg.sam, gg.sak, gg.B, gg.sbk, gg.sbn, None,
                                               None, 0, gg.C, gg.ldc, gg.rowsum_a, _lib.stream_ptr()))
            outs.append((gx, gw, gb))
        for a, b in zip(*outs):
            assert torch.equal(a, b)
        torch.testing.assert_close(outs[0][0], gy @ w, rtol=1e-5, atol=1e-4)
        torch.testing.assert_close(outs[0][1], gy.t() @ x, rtol=1e-5, atol=1e-4)
        torch.testing.assert_close(outs[0][2], gy.sum(0), rtol=1e-5, atol=1e-4)


def test_linear_group_launch_matches_single_launches():
    """fs_linear_f32_group (the final Linear's backward + the unconditional row sum in one
    launch, split-K included) gives exactly what the products give one by one."""
    import ctypes

    from flowstate import _lib

    L, p = _lib.load(), _lib.ptr
    g = torch.Generator().manual_seed(2)
    for M, H, P in ((256, 128, 2944), (100, 64, 1040), (37, 24, 300)):
        h = torch.randn((M, H), generator=g).cuda()
        w = torch.randn((P, H), generator=g).cuda()
        gp = torch.randn((M, P), generator=g).cuda()
        gu = torch.randn((M, P), generator=g).cuda()
        outs = []
        for grouped in (True, False):
            gh, gw = torch.empty_like(h), torch.empty_like(w)
            gb, gs = torch.empty(P, device="cuda"), torch.empty(P, device="cuda")
            descs = [_lib.GemmF32(M, H, P, p(gp), P, 1, p(w), H, 1, None, None, 0, p(gh), H, None),
                     _lib.GemmF32(P, H, M, p(gp), 1, P, p(h), H, 1, None, None, 0, p(gw), H, p(gb)),
                     _lib.GemmF32(P, 0, M, p(gu), 1, P, None, 0, 0, None, None, 0, None, 0, p(gs))]
            nws = sum(max(0, L.fs_linear_f32_splitk_floats(d)) for d in descs)
            ws = torch.empty((max(nws, 1),), device="cuda")
            if grouped:
                arr = (ctypes.POINTER(_lib.GemmF32) * 3)(*[ctypes.pointer(d) for d in descs])
                _lib.check(L.fs_linear_f32_group(arr, 3, p(ws), nws, _lib.stream_ptr()))
            else:
                for d in descs:
                    f = L.fs_linear_f32_splitk_floats(d)
                    if f > 0:
                        _lib.check(L.fs_linear_f32_splitk(d, p(ws), f, _lib.stream_ptr()))
                    else:
                        _lib.check(L.fs_linear_f32(d.M, d.N, d.K, d.A, d.sam, d.sak, d.B, d.sbk, d.sbn, None, None, 0,
                                                   d.C, d.ldc, d.rowsum_a, _lib.stream_ptr()))
            outs.append((gh, gw, gb, gs))
        for a, b in zip(*outs):
            assert torch.equal(a, b)
        torch.testing.assert_close(outs[0][0], gp @ w, rtol=1e-5, atol=2e-3)
        torch.testing.assert_close(outs[0][1], gp.t() @ h, rtol=1e-5, atol=2e-3)
        torch.testing.assert_close(outs[0][2], gp.sum(0), rtol=1e-5, atol=1e-3)
        torch.testing.assert_close(outs[0][3], gu.sum(0), rtol=1e-5, atol=1e-3)




@pytest.mark.parametrize("n", [4096 + 3, 1000])
def test_fused_adam_matches_torch_capturable_adam(n):
    """fs_adam_step (csrc/optim_kernels.hip) against torch.optim.Adam(capturable=True) with
    L2 weight decay (main_algorithm_2.py:310) over several steps, including a step whose
    loss is NaN (nothing written, the step count kept: main_algorithm_2.py:324-326) and one
    whose skip word is set (a graphed epoch's sticky spline-NaN flag)."""
    from flowstate import _lib

    L, p = _lib.load(), _lib.ptr
    g = torch.Generator(device="cuda").manual_seed(n)
    lr, betas, eps, wd = 5.4351e-4, (0.9, 0.999), 1e-8, 9.5857e-5
    ref = torch.nn.Parameter(torch.randn(n, device="cuda", generator=g))
    opt = torch.optim.Adam([ref], lr=lr, betas=betas, eps=eps, weight_decay=wd, capturable=True)
    par = ref.detach().clone()
    m, v = torch.zeros_like(par), torch.zeros_like(par)
    step = torch.zeros((), device="cuda")
    for it in range(6):
        grad = torch.randn(n, device="cuda", generator=g) * (10.0 ** (it % 3 - 1))
        loss = torch.tensor([float("nan") if it == 3 else 1.0], device="cuda")
        skip = torch.tensor([1 if it == 4 else 0], dtype=torch.int32, device="cuda")
        if it not in (3, 4):
            ref.grad = grad.clone()
            opt.step()
        before = (par.clone(), m.clone(), v.clone(), step.clone())
        _lib.check(L.fs_adam_step(p(par), p(grad), p(m), p(v), n, p(step), p(loss), p(skip), lr, betas[0], betas[1],
                                  eps, wd, _lib.stream_ptr()))
        torch.cuda.synchronize()
        if it in (3, 4):
            for a, b in zip((par, m, v, step), before):
                assert torch.equal(a, b)
            continue
        st = opt.state[ref]
        assert float(step) == float(st["step"])
        torch.testing.assert_close(m, st["exp_avg"], rtol=1e-6, atol=1e-9)
        torch.testing.assert_close(v, st["exp_avg_sq"], rtol=1e-6, atol=1e-12)
        torch.testing.assert_close(par, ref.detach(), rtol=1e-6, atol=1e-8)


@pytest.mark.parametrize("M,K,N,bn,res", [(256, 128, 128, True, True), (232, 128, 128, True, False),
                                          (256, 128, 2944, False, False), (100, 64, 96, False, True),
                                          (256, 256, 128, True, False), (37, 192, 32, True, True)])
def test_lean_forward_product_matches_generic_kernel(M, K, N, bn, res):
    """nn.Linear's forward layout takes gemm_lin_kernel (32-bit buffer offsets, rows past M
    read as zero); the generic gemm_bn_f32_kernel / gemm_f32_kernel take the same product
    with W handed over transposed (strided along k), and with the lean kernels switched off
    (fs_set_lean_gemm).  All must agree bit for bit: output, tile statistics,
    u = relu(BN(x)) and the BatchNorm outputs.  Then fs_linear_f32_ex2 (two problems, one
    launch) against the two products alone."""
    from flowstate import _lib

    L, p, st = _lib.load(), _lib.ptr, _lib.stream_ptr
    g = torch.Generator().manual_seed(M + K + N)
    x = torch.randn((M, K), generator=g).cuda()
    w = (torch.randn((N, K), generator=g) * 0.1).cuda()
    wt = w.t().contiguous()
    b = torch.randn(N, generator=g).cuda()
    r = torch.randn((M, N), generator=g).cuda() if res else None
    gam, bet = (torch.rand(K, generator=g) + 0.5).cuda(), (torch.randn(K, generator=g) * 0.1).cuda()
    xst = torch.empty(((M + 31) // 32, K, 2), device="cuda")
    if bn:  # the producer's tile statistics of x
        wi = torch.eye(K, device="cuda")
        xx = torch.empty_like(x)
        _lib.check(L.fs_linear_f32_ex(_lib.GemmF32(M, K, K, p(x), K, 1, p(wi), 1, K, None, None, 0, p(xx), K, None),
                                      None, p(xst), st()))
        x = xx
    outs = []
    for lean, tr in ((True, False), (False, True), (False, False)):
        prev = L.fs_set_lean_gemm(1 if lean else 0)
        y = torch.empty((M, N), device="cuda")
        sto = torch.empty(((M + 31) // 32, N, 2), device="cuda")
        u = torch.empty_like(x)
        mo, io, vo = (torch.empty(K, device="cuda") for _ in range(3))
        rm, rv = torch.zeros(K, device="cuda"), torch.ones(K, device="cuda")
        nbt = torch.zeros(1, dtype=torch.int64, device="cuda")
        gd = (_lib.GemmF32(M, N, K, p(x), K, 1, p(wt), N, 1, p(b), p(r), N, p(y), N, None) if tr else
              _lib.GemmF32(M, N, K, p(x), K, 1, p(w), 1, K, p(b), p(r), N, p(y), N, None))
        bi = _lib.BnIn(p(xst), (M + 31) // 32, M, p(gam), p(bet), 1e-5, 0.1, p(rm), p(rv), p(nbt), p(mo), p(io),
                       p(u), p(vo)) if bn else None
        _lib.check(L.fs_linear_f32_ex(gd, bi, p(sto), st()))
        L.fs_set_lean_gemm(prev)
        outs.append([y, sto] + ([u, mo, io, vo, rm, rv, nbt] if bn else []))
    torch.cuda.synchronize()
    for a, c, d in zip(*outs):
        assert torch.equal(a, c) and torch.equal(a, d)
    ref = (torch.relu(torch.nn.functional.batch_norm(x, None, None, gam, bet, True, 0.1, 1e-5)) if bn else x) @ w.t() + b
    if res:
        ref = ref + r
    torch.testing.assert_close(outs[0][0], ref, rtol=1e-4, atol=1e-4)
    # two problems in one launch (the second a copy of the first on other buffers)
    y2 = [torch.empty((M, N), device="cuda") for _ in range(2)]
    s2 = [torch.empty(((M + 31) // 32, N, 2), device="cuda") for _ in range(2)]
    gds = [_lib.GemmF32(M, N, K, p(x), K, 1, p(w), 1, K, p(b), p(r), N, p(y2[i]), N, None) for i in range(2)]
    bis = [_lib.BnIn(p(xst), (M + 31) // 32, M, p(gam), p(bet), 1e-5, 0.1, None, None, None, None, None, None, None)
           if bn else None for _ in range(2)]
    _lib.check(L.fs_linear_f32_ex2(gds[0], bis[0], p(s2[0]), gds[1], bis[1], p(s2[1]), st()))
    torch.cuda.synchronize()
    for i in range(2):
        assert torch.equal(y2[i], outs[0][0]) and torch.equal(s2[i], outs[0][1])


@pytest.mark.parametrize("M,K,N", [(256, 128, 128), (232, 128, 128), (256, 128, 2944), (100, 64, 96), (36, 512, 40)])
def test_lean_backward_products_match_generic_kernel(M, K, N):
    """nn.Linear's backward on gemm_ling_kernel (32-bit buffer offsets, loads past the
    operands read as zero): the input / weight gradient pair in one launch
    (fs_linear_f32_pair), the weight gradient with its bias row sum alone, and a row sum
    without product (the unconditional spline's batch sum), each against the generic
    kernels (fs_set_lean_gemm(0)) bit for bit, and against torch."""
    from flowstate import _lib

    L, p, st = _lib.load(), _lib.ptr, _lib.stream_ptr
    g = torch.Generator().manual_seed(M * 7 + N)
    x = torch.randn((M, K), generator=g).cuda()   # the layer input
    w = (torch.randn((N, K), generator=g) * 0.1).cuda()
    gy = torch.randn((M, N), generator=g).cuda()  # dL/dy
    outs = []
    for lean in (1, 0):
        prev = L.fs_set_lean_gemm(lean)
        gx, gw, gb = torch.empty_like(x), torch.empty_like(w), torch.empty(N, device="cuda")
        g0 = _lib.GemmF32(M, K, N, p(gy), N, 1, p(w), K, 1, None, None, 0, p(gx), K, None)
        g1 = _lib.GemmF32(N, K, M, p(gy), 1, N, p(x), K, 1, None, None, 0, p(gw), K, p(gb))
        if N <= 512:
            _lib.check(L.fs_linear_f32_pair(g0, g1, st()))
        else:  # a long input-gradient reduction takes the split-K path; the weight gradient alone
            _lib.check(L.fs_linear_f32(g1.M, g1.N, g1.K, g1.A, g1.sam, g1.sak, g1.B, g1.sbk, g1.sbn, None, None, 0,
                                       g1.C, g1.ldc, g1.rowsum_a, st()))
            gx.zero_()
        gs = torch.empty(N, device="cuda")
        _lib.check(L.fs_linear_f32(N, 0, M, p(gy), 1, N, None, 0, 0, None, None, 0, None, 0, p(gs), st()))
        L.fs_set_lean_gemm(prev)
        outs.append((gx, gw, gb, gs))
    torch.cuda.synchronize()
    for a, c in zip(*outs):
        assert torch.equal(a, c)
    if N <= 512:
        torch.testing.assert_close(outs[0][0], gy @ w, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(outs[0][1], gy.t() @ x, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(outs[0][2], gy.sum(0), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(outs[0][3], gy.sum(0), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("M", [2, 33, 179, 256])
def test_batchnorm_combine_on_ill_conditioned_columns(M):
    """The BatchNorm-in-load combine (lin_bn_prologue: Chan's update over the producer's
    32-row tile statistics, tiles in order) on columns whose variance is ~1e-9 of their
    squared mean, on ragged batches (a partial last tile): the batch variance stays
    non-negative, invstd finite, the mean within 1e-5 and the variance within 1e-2 relative of
    float64 statistics (the float32 tile means' rounding, ~3e-5 here, against tile-mean
    differences of ~2e-3)
    of the same float32 inputs, for the lean and the generic kernels alike.  A combine that
    folds the per-tile updates into sum(x^2)/n - mean^2 (one way to constant-fold its
    divisions) cancels catastrophically here: negative variances, NaN invstd, the NaN
    discriminant of r05ak (DESIGN_HISTORY.md r06; tests/test_train_cpu.py shows the
    mechanism on the same statistics)."""
    from flowstate import _lib

    L, p, st = _lib.load(), _lib.ptr, _lib.stream_ptr
    K, N = 64, 32
    g = torch.Generator().manual_seed(M)
    scale = torch.cat([torch.full((K // 2,), 300.0), torch.ones(K // 2)])
    spread = torch.cat([torch.full((K // 2,), 1e-2), torch.ones(K // 2)])
    x = (scale + spread * torch.randn((M, K), generator=g)).float().cuda()
    w = (torch.randn((N, K), generator=g) * 0.1).cuda()
    gam, bet = torch.ones(K, device="cuda"), torch.zeros(K, device="cuda")
    xst = torch.empty(((M + 31) // 32, K, 2), device="cuda")
    xx = torch.empty_like(x)
    wi = torch.eye(K, device="cuda")
    _lib.check(L.fs_linear_f32_ex(_lib.GemmF32(M, K, K, p(x), K, 1, p(wi), 1, K, None, None, 0, p(xx), K, None),
                                  None, p(xst), st()))
    x64 = xx.double().cpu()
    mean64 = x64.mean(0)
    var64 = ((x64 - mean64) ** 2).mean(0)
    for lean in (1, 0):
        prev = L.fs_set_lean_gemm(lean)
        y = torch.empty((M, N), device="cuda")
        sto = torch.empty(((M + 31) // 32, N, 2), device="cuda")
        u = torch.empty_like(x)
        mo, io, vo = (torch.empty(K, device="cuda") for _ in range(3))
        bi = _lib.BnIn(p(xst), (M + 31) // 32, M, p(gam), p(bet), 1e-5, 0.1, None, None, None, p(mo), p(io), p(u),
                       p(vo))
        _lib.check(L.fs_linear_f32_ex(_lib.GemmF32(M, N, K, p(xx), K, 1, p(w), 1, K, None, None, 0, p(y), N, None),
                                      bi, p(sto), st()))
        L.fs_set_lean_gemm(prev)
        torch.cuda.synchronize()
        var, mean, inv = vo.double().cpu(), mo.double().cpu(), io.double().cpu()
        assert (var >= 0).all() and torch.isfinite(inv).all() and torch.isfinite(y).all(), (lean, var.min())
        assert ((mean - mean64).abs() <= 1e-5 * mean64.abs() + 1e-6).all(), lean
        assert ((var - var64).abs() <= 1e-2 * var64 + 1e-9).all(), (lean, ((var - var64).abs() / var64).max())
