"""Algorithm-2 training path (forward_kld / reverse_kld / one Adam step in train
mode, main_algorithm_2.py:314-331) against the reference's own values
(tests/golden/train.npz).  The training path is PyTorch autograd over the layers'
modules (flowstate/normflows/autograd_flow.py), so it runs on CPU tensors too;
tests/test_gpu_train.py repeats it on the MI355X."""
import os

import numpy as np
import pytest
import torch

G = os.path.join(os.path.dirname(__file__), "golden")


def build(device):
    from flowstate.models import build_flow
    from flowstate.normflows.Energy import DoubleWellLJ
    from oracle import flow as OF

    f = np.load(os.path.join(G, "train.npz"))
    dims = OF.FlowDims(N=4, L=2, H=32, nb=2, K=5, B=OF.half_box(4))
    sd = OF.random_state_dict(dims, seed=5, final_std=0.05)
    m = build_flow(4, L=2, H=32, nb=2, K=5, bound=dims.B, device="cpu")
    m.load_state_dict(sd, strict=True)
    m.p = DoubleWellLJ(dims.D, dims.N, 1.0, dims.B, V0_list=[-10.0, -10.5], r0=1.2, k=15)
    m = m.to(device)
    z0 = torch.from_numpy(f["z0"]).to(device)
    m.q0.forward = lambda n: z0[:n].clone()
    m.train()
    return m, f


def check_training(device, rtol_loss, rtol_grad, atol_grad):
    torch.manual_seed(0)
    m, f = build(device)
    names = [str(n) for n in f["names"]]
    assert names == [n for n, _ in m.named_parameters()]
    x = torch.from_numpy(f["x"]).to(device)
    lf = m.forward_kld(x)
    np.testing.assert_allclose(lf.item(), float(f["fkld"]), rtol=rtol_loss)
    gf = torch.autograd.grad(lf, list(m.parameters()), allow_unused=True)
    for n, g in zip(names, gf):
        ref = f["gf/" + n]
        if ref.size == 0:
            assert g is None or not g.abs().max().item()
            continue
        np.testing.assert_allclose(g.cpu().numpy(), ref, rtol=rtol_grad, atol=atol_grad, err_msg=n)
    for k, v in m.state_dict().items():
        if "running" in k:
            np.testing.assert_allclose(v.cpu().numpy(), f["bn_after_f/" + k], rtol=1e-5, atol=1e-6, err_msg=k)
    m, _ = build(device)
    lr_, zr = m.reverse_kld(64)
    np.testing.assert_allclose(lr_.item(), float(f["rkld"]), rtol=rtol_loss)
    np.testing.assert_allclose(zr.detach().cpu().numpy(), f["rkld_z"], rtol=1e-5, atol=5e-4 * 1.0)
    gr = torch.autograd.grad(lr_, list(m.parameters()), allow_unused=True)
    for n, g in zip(names, gr):
        ref = f["gr/" + n]
        if ref.size == 0:
            continue
        scale = max(1.0, float(np.abs(ref).max()))
        np.testing.assert_allclose(g.cpu().numpy(), ref, rtol=rtol_grad, atol=atol_grad * scale, err_msg=n)
    m, _ = build(device)
    opt = torch.optim.Adam(m.parameters(), lr=0.000543510751759681, weight_decay=9.5857178422352e-05)
    opt.zero_grad()
    energy_loss, _ = m.reverse_kld(64)
    sample_loss = m.forward_kld(x)
    loss = 1.0 * sample_loss + (1 - 1.0) * energy_loss
    np.testing.assert_allclose(loss.item(), float(f["step_loss"]), rtol=rtol_loss)
    assert bool(~(torch.isnan(loss) | torch.isinf(loss)))
    loss.backward()
    opt.step()
    for k, v in m.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), f["after_step/" + k], rtol=1e-5, atol=1e-6, err_msg=k)


def test_training_step_matches_reference_cpu():
    torch.set_num_threads(4)
    check_training("cpu", rtol_loss=1e-6, rtol_grad=1e-4, atol_grad=1e-6)


def test_torch_spline_forward_inverse_consistent():
    """The reference's splines_test.py consistency check on the torch restatement used
    on CPU tensors (autograd_flow.circular_rqs_torch)."""
    from flowstate.normflows.autograd_flow import circular_rqs_torch

    torch.manual_seed(0)
    shape, K, B = (2, 3, 4), 10, 3.0
    uw, uh, ud = torch.randn(*shape, K), torch.randn(*shape, K), torch.randn(*shape, K + 1)
    x = torch.randn(*shape) * 2
    y, ld = circular_rqs_torch(x, uw, uh, ud, B, False)
    x2, ld2 = circular_rqs_torch(y, uw, uh, ud, B, True)
    torch.testing.assert_close(x2, x, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(ld + ld2, torch.zeros_like(ld), atol=1e-3, rtol=1e-3)


def _target_case(N):
    from flowstate.normflows.Energy import DoubleWellLJ

    f = np.load(os.path.join(G, "target_energy.npz"))
    mod = DoubleWellLJ(2 * N, N, 1.0, float(f[f"N{N}_B"]), V0_list=[-10.0, -10.5], r0=1.2, k=15)
    return f, mod


def check_target_energy(mod, f, N, x, E, gx):
    ref_E, ref_g = f[f"N{N}_E"], f[f"N{N}_grad"]
    E = E.detach().double().cpu().numpy()
    assert np.all(np.abs(E - ref_E) <= 1e-5 * np.abs(ref_E) + 1e-4), np.abs(E - ref_E).max()
    gx = gx.double().cpu().numpy()
    # the reference's NaN gradients (coinciding particles: torch.where's pow branch) kept
    np.testing.assert_array_equal(np.isnan(gx), np.isnan(ref_g))
    ok = ~np.isnan(ref_g).any(axis=1)
    assert ok.sum() >= len(ok) - 3
    g, r = gx[ok], ref_g[ok]
    scale = np.abs(r).max(axis=1, keepdims=True)
    assert np.all(np.abs(g - r) <= 1e-5 * scale + 1e-4 * np.abs(r)), np.abs(g - r).max()


@pytest.mark.parametrize("N", [4, 16, 64])
def test_target_energy_restatement_matches_reference(N):
    """The torch restatement of DoubleWellLJ._energy (CPU tensors) against the
    reference's values and gradients (tests/golden/target_energy.npz)."""
    f, mod = _target_case(N)
    x = torch.from_numpy(f[f"N{N}_x"]).requires_grad_(True)
    E = mod._energy(x)
    (gx,) = torch.autograd.grad(E.sum(), x)
    check_target_energy(mod, f, N, x, E, gx)
