"""GPU parity of the local-move row (fs_local_moves / fs_adjust_displacement and the
FS_MH_HYBRID big move that follows local moves).

1. The reference's own traces (tests/golden/local_trace.npz, MonteCarlo.particle_displacement
   + adjust_displacement + nf_big_move) replayed through the drop-in per-chain
   MonteCarlo and through one batched launch: identical per-move accept flags,
   max_displacement sequence, float64 -> float32 switch, final particles, counters
   and the full PCG64 state (including the buffered 32-bit half); E/W within 1e-12.
   Both big moves are decisive (an overlap reject, a log-ratio > 0.02 accept).
2. Random batches at N = 1, 5, 16, 33, 64 with mixed float32/float64 chains against
   the C oracle (bit-exact accept logs, states, max_displacement, RNG state).
3. Sample snapshots (sample(), monte_carlo.py:416-444) at the driver's schedule.
4. Local moves followed by fused NF-MH steps (hybrid old NLL + energy refresh on
   reject) against the oracle's nf_big_move.
"""
import os

import numpy as np
import pytest
import torch

from flowstate import io
from flowstate.MCMC import BatchedMonteCarlo, MonteCarlo, Physics, SimulationBox
from flowstate.models import flow_from_state_dict
from oracle import flow as OF
from oracle import physics as OP

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TRACE_DIMS = dict(L=1, H=32, nb=1, K=5)


def _close(a, b, rel=1e-12):
    if np.isnan(a) or np.isnan(b):  # an overlapping start state: inf - inf, in the reference too
        return bool(np.isnan(a) and np.isnan(b))
    return (np.isinf(a) and np.isinf(b) and np.sign(a) == np.sign(b)) or abs(a - b) <= rel * max(1.0, abs(b))


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


def _trace_model(N, f):
    dims = OF.FlowDims(N=N, B=OF.half_box(N), **TRACE_DIMS)
    sd = OF.random_state_dict(dims, seed=int(f[f"N{N}_flow_seed"]))
    return flow_from_state_dict(sd, N, bound=dims.B, **TRACE_DIMS)


@pytest.mark.parametrize("N", [3, 16])
def test_reference_local_traces_dropin(N):
    """Per-chain drop-in, one particle_displacement() per call, as the driver does."""
    f = np.load(os.path.join(G, "local_trace.npz"))
    moves = int(f[f"N{N}_moves"])
    model = _trace_model(N, f)
    L = float(np.sqrt(N / 0.03))
    k = f"N{N}_c0"
    mc = MonteCarlo(particles=f[k + "_init"], sim_box=SimulationBox(L, L), temperature=1.0, num_particles=N,
                    num_wells=2, V0_list=[-10.0, -10.5], r0=1.2, k=15, initial_max_displacement=0.65,
                    target_acceptance=0.5, seed=int(f[k + "_seed"]))
    mc.set_nf_model(model)
    acc, E, md = [], [], []
    for phase in range(3):
        for t in range(moves):
            a0 = mc.accepted_displacement
            mc.particle_displacement()
            if (t + 1) % 50 == 0:
                mc.adjust_displacement()
            acc.append(mc.accepted_displacement - a0)
            E.append(mc.energy_calculator.total_energy)
            md.append(mc.max_displacement)
        if phase < 2:
            assert mc.nf_big_move(f[k + f"_bigcfg{phase}"]) == bool(f[k + "_big"][phase])
    np.testing.assert_array_equal(np.array(acc, np.int8), f[k + "_accept"])
    assert all(_close(a, b) for a, b in zip(E, f[k + "_E"]))
    np.testing.assert_array_equal(np.array(md), f[k + "_maxdisp"])
    assert (mc.particles.dtype == np.float32) == bool(f[k + "_final_dtype32"])
    np.testing.assert_array_equal(mc.particles, f[k + "_final"])
    assert mc.attempts_displacement == f[k + "_attempts"] and mc.accepted_displacement == f[k + "_accepted"]
    st = mc.rng_state
    ref = f[k + "_pcg"]
    assert st["state"]["state"] == (int(ref[0]) << 64) | int(ref[1])
    assert st["has_uint32"] == int(ref[4]) and st["uinteger"] == int(ref[5])


@pytest.mark.parametrize("N", [3, 16, 64])
def test_reference_local_traces_batched(N):
    """All chains of a case in one launch per phase, per-move E/W from sample_every=1."""
    f = np.load(os.path.join(G, "local_trace.npz"))
    moves, C = int(f[f"N{N}_moves"]), int(f[f"N{N}_chains"])
    model = _trace_model(N, f)
    L = float(np.sqrt(N / 0.03))
    keys = [f"N{N}_c{c}" for c in range(C)]
    init = np.stack([f[k + "_init"] for k in keys])
    seeds = np.array([int(f[k + "_seed"]) for k in keys], np.uint64)
    b = BatchedMonteCarlo(None, init, Physics(L, L), seeds, initial_max_displacement=0.65)
    logs, ews, tuples = [], [], [[] for _ in keys]
    for phase in range(3):
        sxy, sew, log = b.local_moves(moves, adjust_every=50, sample_every=1, log_accepts=True)
        logs.append(log.cpu().numpy())
        ews.append(sew.cpu().numpy())
        # the driver's sample() every 75 steps, from the per-step snapshots
        for c in range(C):
            for tup in io.sample_tuples(b, sxy, sew, c, 0, 1, moves):
                if tup[0] % 75 == 0:
                    tuples[c].append(tup)
        if phase == 0:
            b.set_model(model)
        if phase < 2:
            acc = b.nf_big_move(torch.from_numpy(np.stack([f[k + f"_bigcfg{phase}"] for k in keys])))
            np.testing.assert_array_equal(acc.cpu().numpy().astype(bool), [bool(f[k + "_big"][phase]) for k in keys])
    log = np.concatenate(logs, axis=1)
    ew = np.concatenate(ews, axis=1)
    for c, k in enumerate(keys):
        np.testing.assert_array_equal(log[c].astype(np.int8), f[k + "_accept"])
        assert all(_close(a, r) for a, r in zip(ew[c, :, 0], f[k + "_E"]))
        assert all(_close(a, r) for a, r in zip(ew[c, :, 1], f[k + "_W"]))
        np.testing.assert_array_equal(b.state[c].cpu().numpy(), np.asarray(f[k + "_final"], np.float64))
        assert bool(b.state_is_f32[c].item()) == bool(f[k + "_final_dtype32"])
        assert b.max_disp[c].item() == f[k + "_maxdisp"][-1]
        assert b.attempts[c].item() == f[k + "_attempts"] and b.accepted[c].item() == f[k + "_accepted"]
        np.testing.assert_array_equal(_u64(b.pcg[c]), f[k + "_pcg"][:4])
        np.testing.assert_array_equal(_u64(b.pcg_buf[c]), f[k + "_pcg"][4:])
        ref = f[k + "_samples"]
        assert len(tuples[c]) == len(ref)
        for tup, r in zip(tuples[c], ref):
            assert tup[0] == r[0] and tup[2] == r[2] and tup[4] == r[4] and tup[5] == r[5]
            assert _close(tup[1], r[1]) and _close(tup[3], r[3])


def test_writers_round_trip(tmp_path):
    """sampled_data.csv / configs .npy in the driver's format (main_algorithm_1.py:499-547)."""
    import ast
    import csv

    N, C = 16, 4
    L, init, _ = _random_batch(N, C, seed=2, spread=0.2)
    b = BatchedMonteCarlo(None, init, Physics(L, L), np.arange(C, dtype=np.uint64), initial_max_displacement=0.65)
    sxy, sew, _ = b.local_moves(600, sample_every=150)
    tup = io.sample_tuples(b, sxy, sew, 1, 0, 150, 600)
    io.write_run_dir(str(tmp_path / "run_002"), tup, [t[6] for t in tup[:2]])
    rows = list(csv.reader(open(tmp_path / "run_002" / "sampled_data.csv")))
    assert rows[0][0] == "cycle_number" and len(rows) == 5
    for row, t in zip(rows[1:], tup):
        assert int(row[0]) == t[0] and float(row[1]) == t[1] and float(row[3]) == t[3]
        np.testing.assert_array_equal(np.array(ast.literal_eval(row[6])), t[6].ravel())
    cf = np.load(tmp_path / "run_002" / "mc_run_configs.npy")
    assert cf.shape == (4, N, 2)
    np.testing.assert_array_equal(cf[-1], b.state[1].cpu().numpy())


def _random_batch(N, C, seed, spread):
    L = float(np.sqrt(N / 0.03))
    rng = np.random.default_rng(seed)
    base = OP.fcc_lattice(N) if N > 1 else np.array([[L / 3, L / 2]])
    init = np.mod(base[None] + rng.normal(0, spread, (C, N, 2)), L)
    f32 = rng.random(C) < 0.5
    return L, init, f32


@pytest.mark.parametrize("N,C,moves", [(1, 64, 50), (3, 10, 1000), (5, 256, 300), (16, 256, 300), (24, 128, 200),
                                     (33, 128, 200), (64, 256, 200)])
def test_local_moves_match_oracle(N, C, moves):
    L, init, f32 = _random_batch(N, C, seed=N, spread=0.3)
    state = np.where(f32[:, None, None], init.astype(np.float32).astype(np.float64), init)
    seeds = np.arange(1000, 1000 + C, dtype=np.uint64)
    b = BatchedMonteCarlo(None, state, Physics(L, L), seeds, initial_max_displacement=0.65)
    b.state_is_f32.copy_(torch.from_numpy(f32.astype(np.uint8)))
    b.E_old, b.W_old = b._energy_of_state()
    E0, W0 = b.E_old.cpu().numpy().copy(), b.W_old.cpu().numpy().copy()
    _, _, log = b.local_moves(moves, adjust_every=50, log_accepts=True)
    log = log.cpu().numpy()
    phys = OP.make_phys(N)
    for c in range(C):
        pc = state[c].astype(np.float32) if f32[c] else state[c]
        ch = OP.LocalChain(pc, int(seeds[c]), phys, E=E0[c], W=W0[c], max_disp=0.65)
        ref = ch.local_moves(moves, adjust_every=50)
        np.testing.assert_array_equal(log[c], ref.astype(np.uint8), err_msg=f"chain {c}")
        np.testing.assert_array_equal(b.state[c].cpu().numpy(), ch.xy)
        assert _close(b.E_old[c].item(), ch.E[0], 1e-10) and _close(b.W_old[c].item(), ch.W[0], 1e-10)
        assert b.max_disp[c].item() == ch.max_disp[0]
        np.testing.assert_array_equal(_u64(b.pcg[c]), ch.pcg[:4])
        np.testing.assert_array_equal(_u64(b.pcg_buf[c]), ch.pcg[4:])
        assert b.attempts[c].item() == ch.cnt[0] and b.accepted[c].item() == ch.cnt[1]


LAYOUTS = [(8, 1), (8, 2), (8, 4), (8, 8), (64, 1), (16, 4), (4, 16), (4, 8), (4, 4), (1, 4), (1, 8), (2, 4), (4, 1)]


@pytest.mark.parametrize("N", [3, 7, 16, 30, 64])
def test_every_local_layout_gives_the_same_chains(N, monkeypatch):
    """Every instantiated lanes-per-chain x particles-per-lane layout (FS_LOCAL_LAYOUT) runs
    the same chains bit for bit (the default layout is the one the oracle test covers)."""
    C, moves = 96, 150
    L, init, f32 = _random_batch(N, C, seed=11 + N, spread=0.3)
    state = np.where(f32[:, None, None], init.astype(np.float32).astype(np.float64), init)
    seeds = np.arange(500, 500 + C, dtype=np.uint64)
    ref = None
    for lpc, ppl in LAYOUTS:
        if lpc * ppl < N:
            continue
        monkeypatch.setenv("FS_LOCAL_LAYOUT", f"{lpc}x{ppl}")
        b = BatchedMonteCarlo(None, state, Physics(L, L), seeds, initial_max_displacement=0.65)
        b.state_is_f32.copy_(torch.from_numpy(f32.astype(np.uint8)))
        b.E_old, b.W_old = b._energy_of_state()
        xy, ew, log = b.local_moves(moves, adjust_every=40, sample_every=50, log_accepts=True)
        got = [t.cpu().numpy() for t in (b.state, b.E_old, b.W_old, b.max_disp, b.pcg, b.pcg_buf, xy, ew, log)]
        if ref is None:
            ref = got
        else:
            for a, r in zip(got, ref):
                np.testing.assert_array_equal(a, r, err_msg=f"layout {lpc}x{ppl}")
    assert ref is not None


@pytest.mark.parametrize("N,C", [(3, 10), (3, 64), (16, 40), (64, 32)])
def test_dtype_sorted_workgroups_give_the_same_chains(N, C, monkeypatch):
    """Small launches pack each workgroup's float64 and float32 chains into separate waves
    (FS_LOCAL_SORT, the default at <= 8 workgroups): on a mixed batch the chains, samples
    and accept logs equal an unsorted launch's bit for bit."""
    L, init, f32 = _random_batch(N, C, seed=70 + N, spread=0.3)
    f32[:2] = [True, False]  # both dtypes present
    state = np.where(f32[:, None, None], init.astype(np.float32).astype(np.float64), init)
    seeds = np.arange(900, 900 + C, dtype=np.uint64)
    out = []
    for mode in ("0", "1"):
        monkeypatch.setenv("FS_LOCAL_SORT", mode)
        b = BatchedMonteCarlo(None, state, Physics(L, L), seeds, initial_max_displacement=0.65)
        b.state_is_f32.copy_(torch.from_numpy(f32.astype(np.uint8)))
        b.E_old, b.W_old = b._energy_of_state()
        xy, ew, log = b.local_moves(200, adjust_every=40, sample_every=50, log_accepts=True)
        out.append([t.cpu().numpy() for t in (b.state, b.E_old, b.W_old, b.max_disp, b.pcg, b.pcg_buf, b.attempts,
                                              b.accepted, xy, ew, log)])
    for a, r in zip(*out):
        np.testing.assert_array_equal(a, r)


def test_local_moves_split_calls_and_samples():
    """n moves in one launch == the same moves over several launches (step0 carries the
    driver's counter); sample() snapshots land at steps divisible by sample_every."""
    N, C = 16, 64
    L, init, _ = _random_batch(N, C, seed=3, spread=0.2)
    seeds = np.arange(7, 7 + C, dtype=np.uint64)
    a = BatchedMonteCarlo(None, init, Physics(L, L), seeds, initial_max_displacement=0.65)
    b = BatchedMonteCarlo(None, init, Physics(L, L), seeds, initial_max_displacement=0.65)
    sxy, sew, _ = a.local_moves(450, adjust_every=100, sample_every=150)
    assert sxy.shape == (C, 3, N, 2)
    parts = []
    for s0, n in ((0, 100), (100, 220), (320, 130)):
        xy, ew, _ = b.local_moves(n, adjust_every=100, sample_every=150, step0=s0)
        if xy is not None:
            parts.append((xy, ew))
    np.testing.assert_array_equal(a.state.cpu().numpy(), b.state.cpu().numpy())
    np.testing.assert_array_equal(a.max_disp.cpu().numpy(), b.max_disp.cpu().numpy())
    np.testing.assert_array_equal(sxy.cpu().numpy(), torch.cat([p[0] for p in parts], 1).cpu().numpy())
    np.testing.assert_array_equal(sew.cpu().numpy(), torch.cat([p[1] for p in parts], 1).cpu().numpy())
    # snapshot k == oracle state after move 150*(k+1)
    phys = OP.make_phys(N)
    for c in range(0, C, 9):
        ch = OP.LocalChain(init[c], int(seeds[c]), phys, max_disp=0.65)
        done = 0
        for k in range(3):
            ch.local_moves(150, adjust_every=100, phase=done)
            done += 150
            np.testing.assert_array_equal(sxy[c, k].cpu().numpy(), ch.xy)
            assert _close(sew[c, k, 0].item(), ch.E[0], 1e-10)


def test_hybrid_big_moves_after_local_moves():
    """Algorithm-1 interleaving: local moves, then a fused NF-MH step that must use the
    old NLL of the moved state and recompute the energy on reject."""
    N, C = 16, 256
    dims_kw = dict(L=2, H=64, nb=1, K=8)
    dims = OF.FlowDims(N=N, B=OF.half_box(N), **dims_kw)
    sd = OF.random_state_dict(dims, seed=4)
    model = flow_from_state_dict(sd, N, bound=dims.B, **dims_kw)
    L, init, _ = _random_batch(N, C, seed=9, spread=0.1)
    seeds = np.arange(42, 42 + C, dtype=np.uint64)
    b = BatchedMonteCarlo(model, init, Physics(L, L), seeds, initial_max_displacement=0.65)
    phys = OP.make_phys(N)
    chains = [OP.LocalChain(init[c], int(seeds[c]), phys, max_disp=0.65) for c in range(C)]
    flips = 0
    for rnd in range(3):
        b.local_moves(200)
        for ch in chains:
            ch.local_moves(200)
        b.step()
        D = 2 * N
        cfg = b.last_proposals().cpu().numpy()
        acc = b.accept.cpu().numpy().astype(bool)
        x_old = torch.from_numpy(np.stack([(ch.particles - L / 2).reshape(-1) for ch in chains]).astype(np.float32))
        x_new = torch.from_numpy((cfg.astype(np.float64) - L / 2).astype(np.float32).reshape(C, -1))
        nll_old = -OF.log_prob(sd, x_old, dims).numpy().astype(np.float64)
        nll_new = -OF.log_prob(sd, x_new, dims).numpy().astype(np.float64)
        for c, ch in enumerate(chains):
            pcg_before = ch.pcg.copy()
            a = ch.big_move(cfg[c], nll_old[c], nll_new[c])
            if a != acc[c]:  # borderline float32 log_prob: follow the GPU, count the flip
                flips += 1
                ch.pcg[:] = pcg_before
                ch.cnt[0] -= 1
                ch.big_move(cfg[c], 1e30 if acc[c] else -1e30, 0.0)
                ch.pcg[:4] = _u64(b.pcg[c])
        np.testing.assert_array_equal(b.state.cpu().numpy(), np.stack([ch.xy for ch in chains]))
        E = b.E_old.cpu().numpy()
        for c, ch in enumerate(chains):
            assert _close(E[c], ch.E[0], 1e-10), (rnd, c)
            assert bool(b.state_is_f32[c].item()) == ch.f32
        assert b.accepted.cpu().numpy().tolist() == [int(ch.cnt[1]) for ch in chains]
    assert flips <= 2, flips
