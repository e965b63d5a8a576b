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
