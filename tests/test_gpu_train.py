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
    torch.testing.assert_close(E2, E.detach(), rtol=0, atol=0)  # energy-only launch, same values
