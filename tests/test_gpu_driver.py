"""The batched Algorithm-1 driver (flowstate.algorithm1) on the GPU against the reference
driver's own run (tests/golden/driver.npz: main_algorithm_1.py's setup, equilibration,
production, testing phase, well statistics and free-energy summary restated with
small sizes around the reference's MonteCarlo objects, N=3, 4 runs, 9 big-move
attempts of 200 local moves each).

Every run is one chain of one BatchedMonteCarlo; each driver loop is one device call.
Checked bit-exactly: training samples, accept matrix, acceptance history, every
sample() tuple (E/N and pressure within 1e-12), the stacked configuration arrays and
their dtypes, well statistics (ΔF within 1 ulp: the log runs on the device), final
states, counters and max_displacement; the free-energy summary within 1e-12.
"""
import os

import numpy as np
import pytest
import torch

from flowstate import algorithm1 as A1
from flowstate.MCMC import BatchedMonteCarlo, Physics, initialise_low_left, initialise_low_right
from flowstate.models import flow_from_state_dict
from oracle import flow as OF

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _close(a, b, rel=1e-12):
    return abs(a - b) <= rel * max(1.0, abs(b))


def test_driver_matches_reference(tmp_path):
    f = np.load(os.path.join(G, "driver.npz"))
    N, RUNS, SEED, EQ, ADJ, SF, PROD, ATT, INT, FSEED = (int(v) for v in f["params"])
    HB = float(f["half_box"])
    init = np.array([(initialise_low_left if i % 2 == 0 else initialise_low_right)(N, 0.03, 1.0)[0]
                     for i in range(RUNS)])
    np.testing.assert_array_equal(init, f["init"])
    phys = Physics(2 * HB, 2 * HB, temperature=1.0, num_wells=2, V0_list=(-10.0, -10.5), r0=1.2, k=15)
    bmc = BatchedMonteCarlo(None, init, phys, [SEED + i for i in range(RUNS)], device="cuda",
                            initial_max_displacement=0.65, target_acceptance=0.5)
    eq = A1.equilibrate(bmc, EQ, ADJ, SF)
    prod, train = A1.production(bmc, PROD, SF)
    np.testing.assert_array_equal(train.cpu().numpy(), f["global_samples_nf"])

    dims = OF.FlowDims(N=N, L=2, H=32, nb=1, K=5, B=HB)
    sd = OF.random_state_dict(dims, seed=FSEED, final_std=0.05)
    bmc.set_model(flow_from_state_dict(sd, N, L=2, H=32, nb=1, K=5, bound=HB))
    total0 = int(f["total_after_production"])
    res = A1.testing_phase(bmc, f["test_configs"], ATT, INT, SF, total_mcmc_steps=total0)
    np.testing.assert_array_equal(res.accepts.cpu().numpy(), f["accepts"])
    hs, hp = A1.reference_history(res, total0)
    np.testing.assert_array_equal(np.array(hs), f["mcmc_steps_history"])
    assert hp == list(f["p_acc_history"])

    for r in range(RUNS):
        k = f"run{r}"
        local = eq.tuples(bmc, r) + prod.tuples(bmc, r) + res.local_sample_tuples(bmc, r)
        ref = f[k + "_local"]
        assert len(local) == len(ref)
        for t, g in zip(local, ref):
            assert t[0] == g[0] and t[2] == g[2] and t[4] == g[4] and t[5] == g[5]
            assert _close(t[1], g[1]) and _close(t[3], g[3])
        cfgs = np.array([t[6] for t in local])
        assert cfgs.dtype == f[k + "_configs"].dtype
        np.testing.assert_array_equal(cfgs, f[k + "_configs"])
        testing = np.array([t[6] for t in res.local_sample_tuples(bmc, r)])
        assert testing.dtype == f[k + "_testing"].dtype
        np.testing.assert_array_equal(testing, f[k + "_testing"])
        final = bmc.particles()[r]
        np.testing.assert_array_equal(final, f[k + "_final"].astype(np.float64))
        assert bool(bmc.state_is_f32[r].item()) == (f[k + "_final"].dtype == np.float32)
        assert [int(bmc.attempts[r]), int(bmc.accepted[r])] == list(f[k + "_counters"])
        assert float(bmc.max_disp[r]) == float(f[k + "_max_disp"])

    avg_x, p_a, p_b, dF = A1.well_statistics(res.testing_configs(), res.testing_is_f32(), HB, 1.2)
    for r in range(RUNS):
        k = f"run{r}"
        np.testing.assert_array_equal(avg_x[r].cpu().numpy(), f[k + "_avg_x"])
        np.testing.assert_array_equal(p_a[r].cpu().numpy(), f[k + "_p_a"])
        np.testing.assert_array_equal(p_b[r].cpu().numpy(), f[k + "_p_b"])
        np.testing.assert_allclose(dF[r].cpu().numpy(), f[k + "_dF"], rtol=4e-16, atol=0)
    mean, sem, fm, fs, fstd = A1.free_energy_curve(dF)
    np.testing.assert_allclose(mean, f["mean_deltaF"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(sem, f["sem_deltaF"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose([fm, fs, fstd], f["final"], rtol=1e-12, atol=1e-15)

    A1.write_outputs(str(tmp_path), bmc, [eq, prod], res, history=(hs, hp), runs=[0, 3])
    for r in (0, 3):
        d = tmp_path / "mc_runs" / f"run_{r + 1:03d}"
        saved = np.load(d / "mc_run_configs.npy")
        assert saved.dtype == f[f"run{r}_configs"].dtype
        np.testing.assert_array_equal(saved, f[f"run{r}_configs"])
        np.testing.assert_array_equal(np.load(d / "mc_run_testing_configs.npy"), f[f"run{r}_testing"])
        rows = (d / "sampled_data.csv").read_text().strip().splitlines()
        assert len(rows) == 1 + len(f[f"run{r}_local"])
    acc_rows = (tmp_path / "acceptance_rate_data.csv").read_text().strip().splitlines()
    assert len(acc_rows) == 1 + len(f["p_acc_history"])


def test_driver_testing_phase_rejects_short_config_list():
    f = np.load(os.path.join(G, "driver.npz"))
    HB = float(f["half_box"])
    phys = Physics(2 * HB)
    bmc = BatchedMonteCarlo(None, f["init"], phys, [42, 43, 44, 45], device="cuda")
    with pytest.raises(IndexError):
        A1.testing_phase(bmc, f["test_configs"][:5], 2, 10, 5)
    with pytest.raises(ValueError):
        A1.testing_phase(bmc, f["test_configs"].astype(np.float64), 1, 10, 5)


def _regime_engine(runs, N, temperature):
    dev = torch.device("cuda", torch.cuda.current_device())
    init = np.array([(initialise_low_left if i % 2 == 0 else initialise_low_right)(N, 0.03, 1.0)[0]
                     for i in range(runs)])
    hb = float(np.sqrt(N) * 1.5)
    bmc = BatchedMonteCarlo(None, init, Physics(2 * hb, temperature=temperature), [42 + i for i in range(runs)],
                            device=dev, initial_max_displacement=0.65)
    A1.equilibrate(bmc, 300, 100, 50)
    dims = OF.FlowDims(N=N, L=2, H=32, nb=1, K=5, B=hb)
    sd = OF.random_state_dict(dims, seed=3, final_std=0.05)
    bmc.set_model(flow_from_state_dict(sd, N, L=2, H=32, nb=1, K=5, bound=hb))
    g = torch.Generator().manual_seed(5)
    return bmc, hb, g


@pytest.mark.parametrize("mode", ["pipeline", "local"])
@pytest.mark.parametrize("runs,N,temperature", [(10, 3, 1.0), (10, 3, 40.0), (64, 12, 1.0), (64, 12, 40.0)])
def test_speculative_testing_phase_is_bit_identical(runs, N, temperature, mode):
    """testing_phase with the attempts overlapped (mode "pipeline": algorithm1._Pipeline,
    the local moves run ahead on a side stream and each stage's density pass on its own
    stream; "local": algorithm1._Speculator, each big move beside the next attempt's local
    moves) against the plain sequence, on two engines from the same start: every accept,
    snapshot, dtype flag, final state, PCG64 state, counter, running energy and
    max_displacement equal.  At T=40 many big moves accept (the speculative stages are
    wrong and run again), at T=1 almost none do (they are kept)."""
    ATT, INT, SF = 12, 120, 25
    out = []
    for spec in (False, mode):
        bmc, hb, g = _regime_engine(runs, N, temperature)
        cfg = ((torch.rand((ATT * runs, N, 2), generator=g, dtype=torch.float64) * 0.8 + 0.1) * 2 * hb).float()
        res = A1.testing_phase(bmc, cfg.numpy(), ATT, INT, SF, speculate=spec)
        torch.cuda.synchronize()
        out.append((bmc, res))
    (b0, r0), (b1, r1) = out
    assert r0.speculated == 0
    dropped = int((r0.accepts[:, :-1].sum(0) > 0).sum())
    if mode == "local":
        assert r1.speculated == ATT - 1 - dropped
    else:
        spec, redo = A1.pipeline_schedule(r0.accepts)
        assert r1.speculated == sum(s and not r for s, r in zip(spec, redo))
        assert r1.speculated <= ATT - 1 - dropped
    if temperature > 1:
        assert dropped >= 1  # the drop-and-rerun path ran
        if mode == "pipeline":
            assert any(redo)  # stages ran again on the main stream, the next ones ahead again
    elif N == 3:
        assert r1.speculated >= 1  # the adopt path ran
    assert torch.equal(r0.accepts, r1.accepts)
    assert len(r0.snapshots) == len(r1.snapshots) == ATT
    for s0, s1 in zip(r0.snapshots, r1.snapshots):
        assert s0.steps == s1.steps
        assert torch.equal(s0.xy, s1.xy) and torch.equal(s0.ew, s1.ew) and torch.equal(s0.is_f32, s1.is_f32)
    for k in ("state", "state_is_f32", "pcg", "pcg_buf", "max_disp", "attempts", "accepted", "E_old", "W_old",
              "nll_old", "n_accept"):
        assert torch.equal(getattr(b0, k), getattr(b1, k)), k
    assert r0.p_acc_history == r1.p_acc_history


@pytest.mark.parametrize("mode", ["pipeline", "local"])
@pytest.mark.parametrize("ATT,INT,SF", [(1, 50, 10), (2, 0, 0), (2, 30, 10), (3, 25, 5), (5, 37, 0), (6, 40, 7)])
def test_speculative_testing_phase_edge_cases(ATT, INT, SF, mode):
    """Speculation on / off agree for one attempt (no speculation), no local moves, two or
    three attempts (the pipeline's shortest schedules), no snapshots and snapshot schedules
    that do not divide the interval."""
    runs, N = 10, 3
    out = []
    for spec in (False, mode):
        bmc, hb, g = _regime_engine(runs, N, 5.0)
        cfg = ((torch.rand((ATT * runs, N, 2), generator=g, dtype=torch.float64) * 0.8 + 0.1) * 2 * hb).float()
        res = A1.testing_phase(bmc, cfg.numpy(), ATT, INT, SF, speculate=spec)
        torch.cuda.synchronize()
        out.append((bmc, res))
    (b0, r0), (b1, r1) = out
    assert torch.equal(r0.accepts, r1.accepts)
    assert len(r0.snapshots) == len(r1.snapshots) == ATT
    for s0, s1 in zip(r0.snapshots, r1.snapshots):
        assert s0.steps == s1.steps
        assert s0.xy.shape == s1.xy.shape and torch.equal(s0.xy, s1.xy) and torch.equal(s0.ew, s1.ew)
        assert torch.equal(s0.is_f32, s1.is_f32)
    for k in ("state", "state_is_f32", "pcg", "pcg_buf", "max_disp", "attempts", "accepted", "E_old", "W_old",
              "nll_old", "n_accept"):
        assert torch.equal(getattr(b0, k), getattr(b1, k)), k
