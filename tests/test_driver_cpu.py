"""Host-side pieces of the batched Algorithm-1 driver (flowstate.algorithm1) against the
reference driver's own run (tests/golden/driver.npz, main_algorithm_1.py restated with
small sizes around the reference's MonteCarlo objects): the low-left / low-right
initial states and the run-major global acceptance history rebuilt from the
per-run accept matrix."""
import os

import numpy as np

from flowstate import algorithm1 as A1
from flowstate.MCMC import initialise_low_left, initialise_low_right

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_low_initialisation_matches_reference():
    f = np.load(os.path.join(G, "driver.npz"))
    N, runs = int(f["params"][0]), int(f["params"][1])
    for i in range(runs):
        init = initialise_low_left if i % 2 == 0 else initialise_low_right
        p, box = init(num_particles=N, rho=0.03, aspect_ratio=1.0)
        np.testing.assert_array_equal(p, f["init"][i])
        assert box.box_size_x == 2 * float(f["half_box"])
    for n in range(1, 13):
        for init in (initialise_low_left, initialise_low_right):
            p, box = init(num_particles=n, rho=0.03, aspect_ratio=1.0)
            assert p.shape == (n, 2) and np.all((p >= 0) & (p < box.box_size_x))


def test_low_initialisation_rejects_large_n():
    import pytest

    with pytest.raises(ValueError):
        initialise_low_left(num_particles=13, rho=0.03)


def test_acceptance_history_matches_reference_loop():
    f = np.load(os.path.join(G, "driver.npz"))
    interval = int(f["params"][8])
    total0 = int(f["total_after_production"])
    p, s, tot, att, nacc = A1.acceptance_history(f["accepts"], interval, total_mcmc_steps=total0)
    res = A1.TestingResult(accepts=None, snapshots=[], p_acc_history=p, mcmc_steps_history=s)
    hs, hp = A1.reference_history(res, total0)
    np.testing.assert_array_equal(np.array(hs), f["mcmc_steps_history"])
    assert hp == list(f["p_acc_history"])
    assert att == f["accepts"].size and nacc == int(f["accepts"].sum())
    assert tot == f["mcmc_steps_history"][-1]


def test_free_energy_curve_matches_reference():
    f = np.load(os.path.join(G, "driver.npz"))
    runs = int(f["params"][1])
    dF = np.stack([f[f"run{r}_dF"] for r in range(runs)])
    mean, sem, fm, fs, fstd = A1.free_energy_curve(dF)
    np.testing.assert_array_equal(mean, f["mean_deltaF"])
    np.testing.assert_array_equal(sem, f["sem_deltaF"])
    assert [fm, fs, fstd] == list(f["final"])
