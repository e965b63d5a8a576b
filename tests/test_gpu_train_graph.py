"""The HIP-graph training step (flowstate.normflows.train.GraphedTrainStep) against the
eager reference loop (main_algorithm_2.py:314-331) with the same base draws, and the
reference's skip-on-non-finite-loss rule."""
import numpy as np
import pytest
import torch

from test_train_cpu import build

pytestmark = pytest.mark.gpu


def _eager(m, opt, x, alpha):
    opt.zero_grad()
    e, _ = m.reverse_kld(64)
    s = m.forward_kld(x)
    loss = alpha * s + (1 - alpha) * e
    if bool(~(torch.isnan(loss) | torch.isinf(loss))):
        loss.backward()
        opt.step()
    return loss


@pytest.mark.parametrize("alpha", [1.0, 0.7])
def test_graphed_step_matches_eager(alpha):
    from flowstate.normflows.train import GraphedTrainStep

    lr, wd = 5e-3, 1e-4
    m1, f = build("cuda")
    m2, _ = build("cuda")
    x = torch.from_numpy(f["x"]).cuda()
    opt = torch.optim.Adam(m1.parameters(), lr=lr, weight_decay=wd)
    g = GraphedTrainStep(m2, 64, lr, wd, alpha=alpha, example=x)
    p0 = {k: v.clone() for k, v in m1.state_dict().items()}
    for sd1, sd2 in zip(m1.state_dict().values(), m2.state_dict().values()):
        assert torch.equal(sd1, sd2)  # capture left the model untouched
    if alpha == 1.0:
        # the backward kernels wrote every parameter's gradient into its slice of the flat
        # buffer Adam reads (no gather copies): p.grad is that slice
        base = g._flat_grad.data_ptr()
        assert all(p.grad is not None and p.grad.data_ptr() == base + 4 * o for p, o in zip(g.params, g._goffs))
    for i in range(4):
        xb = x.roll(i, 0)
        l1 = _eager(m1, opt, xb, alpha)
        l2 = g.step(xb)
        np.testing.assert_allclose(l2.item(), l1.item(), rtol=1e-4)
    # Adam normalises each coordinate, so a near-zero gradient turns float32 noise between
    # the capturable and the default implementation into an lr-sized difference on that
    # coordinate: compare the updates per tensor in norm
    for (k, v1), v2 in zip(m1.state_dict().items(), m2.state_dict().values()):
        if not v1.is_floating_point():
            assert torch.equal(v1, v2), k
            continue
        moved = (v1 - p0[k]).norm().item()
        diff = (v2 - v1).norm().item()
        assert diff <= 2e-2 * moved + 1e-6, (k, diff, moved)


def test_graphed_step_skips_non_finite_loss():
    from flowstate.normflows.train import GraphedTrainStep

    m, f = build("cuda")
    x = torch.from_numpy(f["x"]).cuda()
    g = GraphedTrainStep(m, 64, 1e-2, 0.0, alpha=1.0, example=x)
    g.step(x)
    before = {k: v.clone() for k, v in m.state_dict().items() if "running" not in k and "num_batches" not in k}
    bad = x.clone()
    bad[0, 0] = float("nan")
    loss = g.step(bad)
    assert torch.isnan(loss).item()
    for k, v in before.items():
        assert torch.equal(m.state_dict()[k], v), k


def test_graphed_step_updates_inference_image():
    """Graph replays write parameters / BN statistics without bumping tensor versions;
    the eval-mode HIP passes must still see the trained weights."""
    from flowstate.normflows.train import GraphedTrainStep

    m, f = build("cuda")
    x = torch.from_numpy(f["x"]).cuda()
    m.eval()
    lp0 = m.log_prob(x)  # packs the initial weights
    g = GraphedTrainStep(m, 64, 1e-2, 0.0, alpha=1.0, example=x)
    for i in range(3):
        g.step(x.roll(i, 0))
    m.eval()
    lp1 = m.log_prob(x)
    fresh, _ = build("cuda")
    fresh.load_state_dict(m.state_dict())
    fresh.eval()
    assert not torch.equal(lp0, lp1)
    assert torch.equal(lp1, fresh.log_prob(x))


def test_graph_replays_write_only_memory_they_own():
    """Every tensor a captured training step reads or writes outside its own pool lives as
    long as the graph (train._Captured.keep).  r06 found the BatchNorm snapshot buffers of the
    non-paired path (ALPHA != 1) freed after capture: the caching allocator handed their
    blocks to later tensors (another model's Adam state in
    test_graphed_step_matches_eager[0.7], whose NaN discriminant it caused) and every replay
    overwrote them.  Here small sentinel tensors allocated after the capture (the freed
    blocks' size class) must come through several replays unchanged."""
    from flowstate.normflows.train import GraphedTrainStep

    m, f = build("cuda")
    x = torch.from_numpy(f["x"]).cuda()
    g = GraphedTrainStep(m, 64, 5e-3, 1e-4, alpha=0.7, example=x)
    torch.cuda.synchronize()
    sentinels = [torch.full((32,), 1234.5, device="cuda") for _ in range(50000)]
    for i in range(3):
        g.step(x.roll(i, 0))
    torch.cuda.synchronize()
    bad = sum(int((s != 1234.5).any()) for s in sentinels)
    assert bad == 0, f"{bad} sentinel tensors overwritten by graph replays"
