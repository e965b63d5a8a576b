"""The fused training spline (fs_rqs_forward / fs_rqs_backward) against the torch
restatement of splines.py (autograd_flow.circular_rqs_torch) on the MI355X: values,
log-dets and gradients with respect to the input and all three parameter sets, in
both directions, with elements inside, on and outside the interval."""
import numpy as np
import pytest
import torch

from flowstate.normflows import autograd_flow as AF

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("K", [5, 8, 15, 32])
@pytest.mark.parametrize("inverse", [False, True])
def test_fused_spline_matches_torch(K, inverse):
    g = torch.Generator().manual_seed(K + 7 * int(inverse))
    M, B = 4096, 3.0
    x = (torch.rand(M, generator=g) * 2 - 1) * B * 1.05  # ~5 % outside
    x[:4] = torch.tensor([B, -B, 0.0, B * 1.2])
    uw = torch.randn(M, K, generator=g) * 0.7
    uh = torch.randn(M, K, generator=g) * 0.7
    ud = torch.randn(M, K + 1, generator=g) * 0.7
    ud[:8, 0] = 25.0  # softplus above its threshold
    wo = torch.randn(M, generator=g)
    wl = torch.randn(M, generator=g)
    res = {}
    for dev in ("cuda", "cpu"):
        ts = [t.to(dev).clone().requires_grad_(True) for t in (x, uw, uh, ud)]
        if dev == "cuda":
            out, lad = AF.circular_rqs(*ts, B, inverse)
        else:
            out, lad = AF.circular_rqs_torch(*ts, B, inverse)
        loss = (out * wo.to(dev)).sum() + (lad * wl.to(dev)).sum()
        grads = torch.autograd.grad(loss, ts)
        res[dev] = [out.detach().cpu(), lad.detach().cpu()] + [gr.cpu() for gr in grads]
    AF.check_nan_flags()
    # element-wise tolerance; a handful of ill-conditioned elements (minimum-width bins,
    # the near-degenerate inverse root) may exceed it by float32 rounding alone
    names = ["out", "lad", "g_x", "g_uw", "g_uh", "g_ud"]
    for n, a, b in zip(names, res["cuda"], res["cpu"]):
        a, b = a.numpy().reshape(len(a), -1), b.numpy().reshape(len(b), -1)
        scale = max(1.0, float(np.abs(b).max()))
        bad = ~np.isclose(a, b, rtol=2e-4, atol=2e-5 * scale)
        rows = np.nonzero(bad.any(1))[0]
        assert len(rows) <= 4, (n, len(rows), a[rows[:3]], b[rows[:3]])
        np.testing.assert_allclose(a, b, rtol=5e-2, atol=5e-3 * scale, err_msg=n)


@pytest.mark.parametrize("K", [5, 8, 15, 32])
def test_fused_spline_forward_inverse_consistent(K):
    """The reference's own splines_test.py (unconstrained RQS forward / inverse
    consistency, inputs partly outside the interval) on the fused HIP spline, circular
    tails on [-B, B]: inputs recovered to 1e-4, log-dets cancel to 1e-3."""
    from flowstate.normflows.autograd_flow import circular_rqs

    torch.manual_seed(K)
    shape, B = (2, 3, 4), 3.0
    uw = torch.randn(*shape, K, device="cuda")
    uh = torch.randn(*shape, K, device="cuda")
    ud = torch.randn(*shape, K + 1, device="cuda")
    x = torch.randn(*shape, device="cuda") * 2  # some outside [-B, B]: identity, log-det 0
    y, ld = circular_rqs(x, uw, uh, ud, B, inverse=False)
    x2, ld2 = circular_rqs(y, uw, uh, ud, B, inverse=True)
    torch.testing.assert_close(x2, x, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(ld + ld2, torch.zeros_like(ld), atol=1e-3, rtol=1e-3)
    out = x.abs() > B
    assert torch.equal(y[out], x[out]) and torch.equal(ld[out], torch.zeros_like(ld[out]))


@pytest.mark.parametrize("K", [5, 8, 32])
@pytest.mark.parametrize("inverse", [False, True])
def test_splines_dropin_matches_reference_golden(K, inverse):
    """flowstate.normflows.splines.unconstrained_rational_quadratic_spline against the
    reference's own outputs (tests/golden/spline.npz, splines.py:16-222, circular tails,
    elements inside, on and outside the interval)."""
    import os

    from flowstate.normflows import splines as S

    f = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "spline.npz"))
    x, uw, uh, ud = (torch.from_numpy(f[f"K{K}_{n}"]).cuda() for n in ("x", "uw", "uh", "ud"))
    B = float(f[f"K{K}_B"])
    out, lad = S.unconstrained_rational_quadratic_spline(x, uw, uh, ud, inverse=inverse,
                                                         tails=["circular"] * len(x), tail_bound=B)
    tag = f"K{K}_{'inv' if inverse else 'fwd'}"
    o, l = f[tag + "_out"], f[tag + "_lad"]
    out, lad = out.cpu().numpy(), lad.cpu().numpy()
    print(tag, "max |d out|", np.abs(out - o).max(), "max |d lad|", np.abs(lad - l).max())
    outside = np.abs(f[f"K{K}_x"]) > B
    np.testing.assert_array_equal(out[outside], o[outside])
    assert (lad[outside] == 0).all()
    # measured on MI355X: |d out| <= 2.1e-5 (1.8e-6 B), |d lad| <= 6.9e-5 over all K, both ways
    np.testing.assert_allclose(out, o, rtol=0, atol=1e-5 * B)
    np.testing.assert_allclose(lad, l, rtol=1e-4, atol=2e-4)
