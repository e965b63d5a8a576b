"""Algorithm-2 update cycle on the GPU (flowstate.algorithm2): the graphed training
epoch against the reference's epoch (tests/golden/train_cycle.npz, ALPHA = 1: the
shuffle order and the partial last batch are the reference's; parameters compared as
per-tensor update norms because Adam turns float32 noise on near-zero gradients into
lr-sized steps), and a full production -> training -> refeed cycle whose refeed sees
the trained weights."""
import os

import numpy as np
import pytest
import torch

from flowstate.algorithm2 import Algorithm2
from flowstate.MCMC import BatchedMonteCarlo, Physics, initialise_low_left, initialise_low_right
from flowstate.models import flow_from_state_dict
from flowstate.normflows.Energy import DoubleWellLJ
from oracle import flow as OF
from test_algorithm2_cpu import _model

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class _NoEngine:
    C = 100


def test_graphed_training_epoch_matches_reference():
    f = np.load(os.path.join(G, "train_cycle.npz"))
    m = _model().cuda()
    p0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    a = Algorithm2(_NoEngine(), m, batch_size=256, alpha=1.0, graphed=True)
    assert a.graphed
    a.training_data = torch.tensor(f["data"], dtype=torch.float32).reshape(600, -1).cuda()
    torch.manual_seed(23)
    avg = a.train()
    np.testing.assert_allclose(avg, float(f["a10_avg"]), rtol=1e-4)
    for k, v in m.state_dict().items():
        if "running" in k or not v.is_floating_point():
            continue  # reverse_kld's base draws (CUDA generator) only feed the BN statistics at ALPHA = 1
        ref = torch.from_numpy(f["a10/" + k]).cuda()
        moved = (ref - p0[k]).norm().item()
        assert (v - ref).norm().item() <= 3e-2 * moved + 1e-6, k


def _cycle_model():
    dims = OF.FlowDims(N=3, L=2, H=32, nb=2, K=8, B=OF.half_box(3))  # an instantiated (H, K) of the HIP passes
    sd = OF.random_state_dict(dims, seed=29, final_std=0.05)
    m = flow_from_state_dict(sd, 3, L=2, H=32, nb=2, K=8, bound=dims.B)
    m.p = DoubleWellLJ(dims.D, dims.N, 1.0, dims.B, V0_list=[-10.0, -10.5], r0=1.2, k=15)
    return m


def test_update_cycle_refeeds_with_trained_weights():
    N, runs = 3, 100
    m = _cycle_model()
    B = float(m.flows[0].tail_bound)
    init = np.array([(initialise_low_left if i % 2 == 0 else initialise_low_right)(N, 0.03, 1.0)[0]
                     for i in range(runs)])
    phys = Physics(2 * B)
    bmc = BatchedMonteCarlo(None, init, phys, [42 + i for i in range(runs)], device="cuda",
                            initial_max_displacement=0.65)
    bmc.local_moves(500, adjust_every=100)
    a = Algorithm2(bmc, m, batch_size=256, alpha=1.0, sampling_frequency=10, update_num_samples=1000)
    assert a.production_runs == 100
    torch.manual_seed(0)
    for _ in range(2):
        snap, loss, acc, p = a.cycle()
        assert snap.xy.shape == (runs, 10, N, 2)
        assert a.training_data.shape == (1000, 2 * N)
        assert np.isfinite(loss) and 0.0 <= p <= 1.0
    assert a.total_mcmc_steps == 2 * 100 * runs
    assert len(a.loss_history) == 2 and len(a.p_acc_history) == 2
    # the cached old NLL after the refeed is -log q(state) under the TRAINED weights
    fresh = _cycle_model()
    fresh.load_state_dict(m.state_dict())
    fresh.eval()
    x = (bmc.state - phys.half_width).to(torch.float32).reshape(runs, -1)
    torch.testing.assert_close(bmc.nll_old, -fresh.log_prob(x).double(), rtol=0, atol=0)


def test_config5_cycle_at_reference_sizes():
    """BASELINE config 5's cycle at the reference's sizes (main_algorithm_2.py:33-52,
    393-577): A2 flow (L=23, H=128, 2 blocks, K=15), N=64, NUM_MC_RUNS=100,
    UPDATE_NUM_SAMPLES=1000 (100 local moves per run, sample() every 10), one epoch of
    batch 256 (3 full batches + 1 of 232), ALPHA=1, then the refeed.
    Checked: the epoch's invariants (every BatchNorm counted 2 forwards per step, as the
    reference's forward_kld + reverse_kld in train mode; 4 Adam steps; parameters moved
    and finite) and the graphed epoch against the eager one from the same start; then
    all 100 refeed decisions against the oracle's restatement of nf_big_move with the
    trained weights (old NLL re-derived from the moved states, the running energy of the
    local moves in the ratio, the kernel's own proposals, each run's PCG64 stream), the
    energies a reject writes back, and the cached NLL."""
    from flowstate.MCMC import initialise_fcc
    from flowstate.models import A2, build_flow, half_box
    from oracle import physics as OP

    N, runs = 64, 100
    torch.manual_seed(0)
    B = half_box(N)
    m = build_flow(N, bound=B, device="cpu", **A2)
    m.p = DoubleWellLJ(2 * N, N, 1.0, B, V0_list=[-10.0, -10.5], r0=1.2, k=15)
    m = m.cuda()
    m.q0.device = torch.device("cuda", torch.cuda.current_device())
    base, box = initialise_fcc(num_particles=N, rho=0.03, aspect_ratio=1.0)
    phys = Physics(box.box_size_x, box.box_size_y)
    bmc = BatchedMonteCarlo(None, np.repeat(base[None], runs, 0), phys, [42 + i for i in range(runs)],
                            device="cuda", initial_max_displacement=0.65)
    bmc.local_moves(10 * N, adjust_every=5 * N)
    a = Algorithm2(bmc, m, batch_size=256, alpha=1.0, sampling_frequency=10, update_num_samples=1000)
    assert a.production_runs == 100
    a.production()
    assert a.training_data.shape == (1000, 2 * N)

    # --- training epoch: invariants + graphed vs eager from the same start
    twin = build_flow(N, bound=B, device="cpu", **A2)
    twin.p = DoubleWellLJ(2 * N, N, 1.0, B, V0_list=[-10.0, -10.5], r0=1.2, k=15)
    twin = twin.cuda()
    twin.load_state_dict(m.state_dict())
    twin.q0.device = m.q0.device
    before = {k: v.detach().clone() for k, v in m.state_dict().items()}
    torch.manual_seed(5)
    loss = a.train()
    assert np.isfinite(loss)
    assert int(a._step.opt.state[a._step._flat_param]["step"].item()) == 4
    sd = m.state_dict()
    for k, v in sd.items():
        if k.endswith("num_batches_tracked"):
            assert int(v) - int(before[k]) == 2 * 4, k
        elif v.is_floating_point():
            assert torch.isfinite(v).all(), k
    moved = [k for k in sd if "final_layer.weight" in k and not torch.equal(sd[k], before[k])]
    assert len(moved) == len(m.flows)
    b2 = Algorithm2(type("E", (), {"C": runs})(), twin, batch_size=256, alpha=1.0, graphed=False)
    b2.training_data = a.training_data
    torch.manual_seed(5)
    loss2 = b2.train()
    np.testing.assert_allclose(loss, loss2, rtol=1e-4)
    # the graphed epoch runs torch's capturable Adam arithmetic (fs_adam_step: float32 bias
    # corrections) and the paired passes' summation orders, the eager one torch's default
    # Adam (bias corrections in double): updates differ at float32 noise per step, which
    # Adam's near-sign(g) step turns into a full +-lr on elements whose gradient sits at the
    # noise level.  Measured at r05 (tools/a2_drift_bisect.py, profiles/r05/r05g_drift.log):
    # worst tensor 0.70 % of its update (a 128-element BatchNorm bias), median 0.007 %, the
    # same with every kernel-variant switch (FS_FOLD_BN, FS_DEFER_SPLITK, FS_LEAN_GEMM,
    # FS_COUPLING_WAVES) off.  Bound: 2 %.  The reference itself is pinned by
    # test_graphed_step_matches_reference_at_config5_size
    for k, v in twin.state_dict().items():
        if "running" in k or not v.is_floating_point():
            continue
        step = (sd[k] - before[k]).norm().item()
        assert (v - sd[k]).norm().item() <= 2e-2 * step + 1e-6, k

    # --- refeed against the oracle
    hw = phys.half_width
    state0 = bmc.state.cpu().numpy()
    f32 = bmc.state_is_f32.cpu().numpy().astype(bool)
    E_run = bmc.E_old.cpu().numpy().copy()
    pcg = bmc.pcg.cpu().numpy().view(np.uint64).copy()
    acc, p = a.refeed()
    torch.cuda.synchronize()
    bmc.check_errors()
    cfg = bmc.last_proposals().cpu().numpy()
    acc = acc.cpu().numpy().astype(bool)
    E_after = bmc.E_old.cpu().numpy()
    nll_after = bmc.nll_old.cpu().numpy()
    sd_cpu = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    dims = OF.FlowDims(N=N, B=B, **A2)
    ophys = OP.make_phys(N)
    nll_old = -OF.log_prob(sd_cpu, torch.from_numpy((state0 - hw).astype(np.float32).reshape(runs, -1)),
                           dims).numpy().astype(np.float64)
    lq = OF.log_prob(sd_cpu, torch.from_numpy((cfg.astype(np.float64) - hw).astype(np.float32).reshape(runs, -1)),
                     dims).numpy().astype(np.float64)
    E_new = OP.total_energy_batch(cfg, ophys)[0]
    acc_o, u = OP.mh_accept(E_run, E_new, nll_old, -lq, pcg.copy())
    acc_o = acc_o.astype(bool)
    with np.errstate(over="ignore", invalid="ignore", divide="ignore"):
        log_ratio = -(E_new - E_run) - (-lq - nll_old)
        border = (log_ratio < 0) & (np.abs(np.log(u) - log_ratio) < 1e-2)
    assert ((acc == acc_o) | border).all(), (np.flatnonzero(acc != acc_o), border.sum())
    assert border.sum() <= 2
    E_state = np.where(f32, OP.total_energy_batch(state0.astype(np.float32), ophys)[0],
                       OP.total_energy_batch(state0, ophys)[0])
    want_E = np.where(acc, E_new, E_state)
    fin = np.isfinite(want_E)
    assert np.array_equal(np.isfinite(E_after), fin)
    np.testing.assert_allclose(E_after[fin], want_E[fin], rtol=1e-12)
    want_nll = np.where(acc, -lq, nll_old)
    np.testing.assert_allclose(nll_after, want_nll, rtol=1e-5, atol=1e-4)
    assert p == acc.mean()


def test_graphed_step_matches_reference_at_config5_size():
    """The graphed HIP training step (GraphedTrainStep: shared-launch reverse_kld sampling
    pass + forward_kld density pass, their backward, the deferred BatchNorm running
    statistics, fs_adam_step) on config 5's own shapes (A2 flow, N=64, batch 256, ALPHA = 1)
    against the reference's own step (tests/golden/train_a2.npz, made by importing the
    reference): the loss, every parameter gradient, every running statistic, the Adam
    update.  Tolerances: test_train_cpu.A2_TOL (written out there)."""
    from flowstate.normflows import autograd_flow as AF
    from flowstate.normflows.train import GraphedTrainStep
    from test_train_cpu import A2_LR, A2_WD, build_a2, check_a2_step

    m, f = build_a2("cuda")
    before = {n: p.detach().clone() for n, p in m.named_parameters()}
    step = GraphedTrainStep(m, 256, A2_LR, A2_WD, alpha=1.0)
    assert step.flat_bn is not None and step._fused_adam_ok()
    x = torch.from_numpy(f["x"]).cuda()
    loss = step.step(x)
    torch.cuda.synchronize()
    assert AF._last_paired  # the shared-launch passes ran (captured after warm-up)
    names = {id(p): n for n, p in m.named_parameters()}
    grads = {names[id(p)]: step._flat_grad[o:o + p.numel()].view_as(p).clone()
             for p, o in zip(step.params, step._goffs)}
    check_a2_step(m, f, loss.item(), grads, before)


def test_graphed_epoch_writes_nothing_after_a_nan_step():
    """A graphed epoch checks the spline's NaN flags only at its end (Algorithm2.train).
    The sticky NaN word stops every step from the failing one on: parameters, Adam state
    and BatchNorm running statistics after an epoch whose 2nd of 4 steps hits a NaN
    discriminant equal those after its 1st step, and the epoch raises the reference's
    error (splines.py:176-183)."""
    from flowstate.normflows.train import GraphedTrainStep
    from test_train_cpu import A2_LR, A2_WD, build_a2

    m, f = build_a2("cuda")
    z0 = torch.from_numpy(f["z0"]).cuda()
    zs = z0.clone()
    m.q0.forward = lambda n: zs[:n].clone()
    step = GraphedTrainStep(m, 256, A2_LR, A2_WD, alpha=1.0)
    x = torch.from_numpy(f["x"]).cuda()
    step.reset_nan()
    loss, flag = step.step(x, check=False)
    torch.cuda.synchronize()
    assert not bool(flag)
    after1 = [t.detach().clone() for t in step._state_tensors] + [b.clone() for b in step.flat_bn.buffers()]
    # step 2: a NaN identity feature makes every conditioner output NaN, so the first
    # layer's inverse splines of the finite transform features see NaN discriminants (a
    # NaN input itself is outside the tail bound: identity, no error, as in the reference)
    bad = z0.clone()
    bad[:, 0] = float("nan")
    flags = []
    for i in range(3):
        zs.copy_(bad if i == 0 else z0)
        _, fl = step.step(x, check=False)
        flags.append(fl)
    # a batch size without a captured graph (an epoch's partial last batch runs eagerly) writes
    # nothing either once the sticky word is set, and hands back the sticky flag
    _, fl = step.step(x[:200], check=False)
    flags.append(fl)
    torch.cuda.synchronize()
    assert bool(flags[0]) and bool(flags[-1]) and bool(step.nan_state())
    now = [t.detach() for t in step._state_tensors] + step.flat_bn.buffers()
    for a, b in zip(now, after1):
        assert torch.equal(a, b)
    # a checked step clears the word first and trains again
    zs.copy_(z0)
    step.step(x)
    assert not bool(step.nan_state())
    assert not torch.equal(step._state_tensors[0], after1[0])


def _pipeline_setup(temperature):
    N, runs = 3, 100
    m = _cycle_model()
    B = float(m.flows[0].tail_bound)
    init = np.array([(initialise_low_left if i % 2 == 0 else initialise_low_right)(N, 0.03, 1.0)[0]
                     for i in range(runs)])
    bmc = BatchedMonteCarlo(None, init, Physics(2 * B, temperature=temperature), [42 + i for i in range(runs)],
                            device="cuda", initial_max_displacement=0.65)
    bmc.local_moves(500, adjust_every=100)
    return bmc, Algorithm2(bmc, m, batch_size=256, alpha=1.0, sampling_frequency=10, update_num_samples=1000)


def test_run_with_speculative_production_matches_cycles():
    """Algorithm2.run (the next cycle's production run beside this cycle's training, from
    a copy of the runs that assumes the refeed rejects every run) against the same number
    of plain cycle() calls from the same start: every snapshot, training set, loss, refeed
    decision and the final runs bit-identical.  At T = 1 refeeds that no run accepts keep
    the speculative production, at T = 50 refeeds with accepts make it run again."""
    cycles = 3
    kept = redone = 0
    for T in (1.0, 50.0):
        res = []
        for piped in (False, True):
            bmc, a = _pipeline_setup(T)
            torch.manual_seed(0)
            out = a.run(cycles) if piped else [a.cycle() for _ in range(cycles)]
            torch.cuda.synchronize()
            res.append((bmc, a, out))
        (b0, a0, o0), (b1, a1, o1) = res
        for (s0, l0, c0, p0), (s1, l1, c1, p1) in zip(o0, o1):
            assert s0.steps == s1.steps and torch.equal(s0.xy, s1.xy) and torch.equal(s0.ew, s1.ew)
            assert torch.equal(s0.is_f32, s1.is_f32)
            assert l0 == l1 and p0 == p1 and torch.equal(c0, c1)
        assert torch.equal(a0.training_data, a1.training_data)
        assert a0.total_mcmc_steps == a1.total_mcmc_steps and a0.p_acc_history == a1.p_acc_history
        for k in ("state", "state_is_f32", "pcg", "pcg_buf", "max_disp", "attempts", "accepted", "E_old", "W_old",
                  "nll_old", "n_accept"):
            assert torch.equal(getattr(b0, k), getattr(b1, k)), (T, k)
        for p in a0.p_acc_history[:-1]:
            kept += p == 0
            redone += p > 0
    assert kept >= 1 and redone >= 1, (kept, redone)
