"""Oracle vs the reference's own local-move traces (tests/golden/local_trace.npz,
made by tests/golden/make_goldens.py:local_case from MCMC/monte_carlo.py:146-223,
375-403): per-move accept flags, running E/W, max_displacement after every
adjust_displacement, the float64 -> float32 state switch at an accepted
nf_big_move, the final particles and the full numpy PCG64 state (including the
buffered 32-bit half used by Generator.integers)."""
import os

import numpy as np
import pytest
import torch

from oracle import flow as OF
from oracle import physics as OP

G = os.path.join(os.path.dirname(__file__), "golden")


def _nll(sd, dims, xy, hw):
    x = torch.tensor((np.asarray(xy) - np.array([hw, hw])).reshape(1, -1), dtype=torch.float)
    return -OF.log_prob(sd, x, dims).item()


def _close(a, b, rel=1e-12):
    return (np.isinf(a) and np.isinf(b)) or abs(a - b) <= rel * max(1.0, abs(b))


@pytest.mark.parametrize("N", [3, 16, 64])
def test_local_trace_matches_reference(N):
    torch.set_num_threads(1)
    f = np.load(os.path.join(G, "local_trace.npz"))
    moves = int(f[f"N{N}_moves"])
    dims = OF.FlowDims(N=N, L=1, H=32, nb=1, K=5, B=OF.half_box(N))
    sd = OF.random_state_dict(dims, seed=int(f[f"N{N}_flow_seed"]))
    phys = OP.make_phys(N)
    hw = phys.Lx / 2
    for c in range(int(f[f"N{N}_chains"])):
        k = f"N{N}_c{c}"
        ch = OP.LocalChain(f[k + "_init"], int(f[k + "_seed"]), phys)
        acc = []
        E, W, md = [], [], []
        for phase in range(3):
            for t in range(moves):
                acc.append(ch.local_moves(1, adjust_every=50, phase=t)[0])
                E.append(ch.E[0])
                W.append(ch.W[0])
                md.append(ch.max_disp[0])
            if phase < 2:
                cfg = f[k + f"_bigcfg{phase}"]
                big = ch.big_move(cfg, _nll(sd, dims, ch.particles, hw), _nll(sd, dims, cfg, hw))
                assert big == bool(f[k + "_big"][phase])
        np.testing.assert_array_equal(np.array(acc, np.int8), f[k + "_accept"])
        for a, b in zip(E, f[k + "_E"]):
            assert _close(a, b)
        for a, b in zip(W, f[k + "_W"]):
            assert _close(a, b)
        np.testing.assert_allclose(md, f[k + "_maxdisp"], rtol=1e-13)
        assert ch.f32 == bool(f[k + "_final_dtype32"])
        np.testing.assert_array_equal(ch.particles, f[k + "_final"])
        assert ch.cnt[0] == f[k + "_attempts"] and ch.cnt[1] == f[k + "_accepted"]
        np.testing.assert_array_equal(ch.pcg, f[k + "_pcg"])


def test_local_moves_in_one_call_match_single_steps():
    """n moves in one call == n calls of one move (the adjust phase bookkeeping)."""
    N = 16
    phys = OP.make_phys(N)
    init = OP.fcc_lattice(N)
    a = OP.LocalChain(init, 7, phys)
    b = OP.LocalChain(init, 7, phys)
    la = a.local_moves(250, adjust_every=50)
    lb = np.concatenate([b.local_moves(1, adjust_every=50, phase=t) for t in range(250)])
    np.testing.assert_array_equal(la, lb)
    np.testing.assert_array_equal(a.xy, b.xy)
    assert a.E[0] == b.E[0] and a.max_disp[0] == b.max_disp[0]
    np.testing.assert_array_equal(a.pcg, b.pcg)


def test_integers_matches_numpy():
    for seed in (0, 42, 12345):
        for n in (1, 2, 3, 16, 64, 1000, 2**31 + 11):
            g = np.random.default_rng(seed)
            s = np.zeros(6, np.uint64)
            s[:4] = OP.pcg64_seed(seed)
            for _ in range(40):
                assert OP.pcg64_integers(s, n) == int(g.integers(n))
                if _ % 7 == 3:   # interleave doubles: they leave the 32-bit buffer alone
                    assert OP.pcg64_random6(s) == g.random()
            st = g.bit_generator.state
            assert int(s[4]) == st["has_uint32"] and int(s[5]) == st["uinteger"]


@pytest.mark.parametrize("N", [3, 16, 64])
def test_numpy_local_chain_matches_reference_trace(N):
    """The numpy per-call restatement (oracle.physics.NumpyLocalChain, the regime's timed
    CPU baseline in bench.py) replays the reference's own traces exactly as the C
    restatement does: accept flags, running E / W, max_displacement, big-move decisions,
    the float32 switch, final particles, counters and numpy's PCG64 state."""
    torch.set_num_threads(1)
    f = np.load(os.path.join(G, "local_trace.npz"))
    moves = int(f[f"N{N}_moves"])
    dims = OF.FlowDims(N=N, L=1, H=32, nb=1, K=5, B=OF.half_box(N))
    sd = OF.random_state_dict(dims, seed=int(f[f"N{N}_flow_seed"]))
    phys = OP.make_phys(N)
    hw = phys.Lx / 2
    for c in range(int(f[f"N{N}_chains"])):
        k = f"N{N}_c{c}"
        ch = OP.NumpyLocalChain(f[k + "_init"], int(f[k + "_seed"]), phys)
        acc, E, W, md = [], [], [], []
        for phase in range(3):
            for t in range(moves):
                acc.append(ch.local_moves(1, adjust_every=50, step0=t)[0])
                E.append(ch.E)
                W.append(ch.W)
                md.append(ch.max_disp)
            if phase < 2:
                cfg = f[k + f"_bigcfg{phase}"]
                big = ch.big_move(cfg, _nll(sd, dims, ch.particles, hw), _nll(sd, dims, cfg, hw))
                assert big == bool(f[k + "_big"][phase])
        np.testing.assert_array_equal(np.array(acc, np.int8), f[k + "_accept"])
        for a, b in zip(E, f[k + "_E"]):
            assert _close(a, b)
        for a, b in zip(W, f[k + "_W"]):
            assert _close(a, b)
        np.testing.assert_allclose(md, f[k + "_maxdisp"], rtol=1e-13)
        assert (ch.particles.dtype == np.float32) == bool(f[k + "_final_dtype32"])
        np.testing.assert_array_equal(ch.particles, f[k + "_final"])
        assert ch.attempts == f[k + "_attempts"] and ch.accepted == f[k + "_accepted"]
        st = ch.rng.bit_generator.state
        assert st["state"]["state"] == (int(f[k + "_pcg"][0]) << 64 | int(f[k + "_pcg"][1]))
