"""Pin the oracle's Metropolis judge (oracle_metropolis_judge) against the reference's
own judge_normalizing_flow / bulk_judge_normalizing_flow /
metropolis_acceptance_particle_move traces (tests/golden/judge_trace.npz, made by
tests/golden/make_goldens.py from MCMC/monte_carlo.py:191-223, 305-370), including
the nf_big_move that follows a bulk judge (the stale running energy it leaves behind
enters that move's ratio, :243; a reject re-derives the state's energy, :299-301)."""
import os

import numpy as np
import pytest
import torch

from oracle import flow as OF
from oracle import physics as OP

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _close(a, b):
    return (np.isinf(a) and np.isinf(b)) or abs(a - b) <= 1e-12 * max(1.0, abs(b))


@pytest.mark.parametrize("N", [16, 64])
def test_oracle_replays_reference_judge_traces(N):
    f = np.load(os.path.join(G, "judge_trace.npz"))
    dims = OF.FlowDims(N=N, L=2, H=32, nb=1, K=8, B=OF.half_box(N))
    sd = OF.random_state_dict(dims, seed=int(f[f"N{N}_flow_seed"]))
    phys = OP.make_phys(N)
    hw = phys.Lx / 2
    for c in range(int(f[f"N{N}_chains"])):
        k = f"N{N}_c{c}"
        xy = f[k + "_init"].copy()  # the state's values; its reference dtype in xy_dt
        xy_dt = np.float64
        E, W, _ = OP.total_energy(xy, phys)
        pcg = OP.pcg64_seed(42 + c)[None].copy()
        attempts, off = 0, 0
        cfgs = f[k + "_cfgs"]
        for i, (kind, is32, M, a, b) in enumerate(f[k + "_ops"]):
            M = int(M)
            dt = np.float32 if is32 else np.float64
            xs = cfgs[off:off + M].astype(dt)
            off += M
            if kind == 0:  # judge: against the running energy, bookkeeping restored
                En = OP.total_energy(xs[0], phys)[0]
                r = float(OP.metropolis_judge([E], [[En]], pcg)[0, 0])
                attempts += 1
            elif kind == 1:  # metropolis_acceptance_particle_move(a, b)
                r = float(OP.metropolis_judge([a], [[b]], pcg)[0, 0])
            elif kind == 2:  # bulk against ref a; the calculator keeps the last proposal's totals
                ew = [OP.total_energy(x, phys)[:2] for x in xs]
                r = float(OP.metropolis_judge([a], [[e for e, _ in ew]], pcg).sum())
                E, W = ew[-1]
            else:  # nf_big_move with the running (possibly stale) energy
                En, Wn, _ = OP.total_energy(xs[0], phys)
                # monte_carlo.py:251-257: (array - float64 array) -> float64, then torch float32
                old = torch.from_numpy((xy - np.array([hw, hw])).astype(np.float32).reshape(1, -1))
                new = torch.from_numpy((xs[0] - np.array([hw, hw])).astype(np.float32).reshape(1, -1))
                nll_o = -OF.log_prob(sd, old, dims).numpy().astype(np.float64)
                nll_n = -OF.log_prob(sd, new, dims).numpy().astype(np.float64)
                acc, _ = OP.mh_accept([E], [En], nll_o, nll_n, pcg)
                attempts += 1
                r = float(acc[0])
                if acc[0]:
                    xy, xy_dt, E, W = xs[0].astype(np.float64), xs[0].dtype, En, Wn
                else:
                    E, W, _ = OP.total_energy(xy.astype(xy_dt), phys)
            assert r == f[k + "_result"][i], (k, i, kind)
            assert _close(E, f[k + "_E"][i]) and _close(W, f[k + "_W"][i]), (k, i, E, f[k + "_E"][i])
            assert attempts == f[k + "_attempts"][i]
        np.testing.assert_array_equal(pcg[0], f[k + "_pcg_state"])
        np.testing.assert_array_equal(xy, f[k + "_final"])


@pytest.mark.parametrize("tag", ["N16_f32", "N16_f64", "N64_f32", "N64_f64"])
def test_oracle_box_and_particle_energy(tag):
    """oracle min_image / min_image_dist / particle_energy vs the reference's
    SimulationBox and EnergyCalculator.calculate_particle_energy_virial
    (tests/golden/box_trace.npz): bit-exact displacements and distances, energies
    within 1e-12 (both +inf on the hard core)."""
    f = np.load(os.path.join(G, "box_trace.npz"))
    x = f[tag + "_x"]
    N = x.shape[0]
    phys = OP.make_phys(N)
    assert phys.Lx == float(f[tag + "_L"])
    for (i, j), d, r in zip(f[tag + "_ij"], f[tag + "_delta"], f[tag + "_dist"]):
        np.testing.assert_array_equal(OP.min_image(x[i], x[j], phys), d)
        assert OP.min_image_dist(x, int(i), int(j), phys) == r
    for p in range(N):
        E, W = OP.particle_energy(x, p, phys)
        Er, Wr = f[tag + "_particle_ew"][p]
        assert _close(E, Er) and _close(W, Wr), (p, E, Er)
