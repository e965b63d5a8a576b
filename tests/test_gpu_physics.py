"""GPU parity of the energy kernel, the PCG64 stream and the acceptance rule.

Energies: within 1e-12 relative of the C oracle (which is within 1e-12 of the
reference, tests/test_oracle_golden.py) — far inside the north star's 1e-5;
overlap flags and r <= 2.5 neighbour masks bit-exact; PCG64 states and draws
bit-exact; acceptance masks bit-exact on identical (E, NLL, u) inputs."""
import os

import numpy as np
import pytest
import torch

from flowstate import _lib
from flowstate.MCMC.energy_calculator import make_phys, total_energy
from oracle import physics as OP

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def gphys(N):
    L = float(np.sqrt(N / 0.03))
    return make_phys(L, L)


def test_energy_matches_reference_golden():
    f = np.load(os.path.join(G, "energy.npz"))
    for i in range(int(f["count"])):
        pos = f[f"c{i}_pos"]
        N = int(f[f"c{i}_N"])
        E, W, ov, nbr = total_energy(torch.from_numpy(pos[None]).cuda(), gphys(N), with_neighbours=True)
        E, W, ov = E.item(), W.item(), int(ov.item())
        Eref = float(f[f"c{i}_E"])
        if np.isinf(Eref):
            assert ov == 1 and np.isinf(E) and np.isinf(W)
        else:
            assert ov == 0
            assert abs(E - Eref) <= 1e-12 * max(1.0, abs(Eref)), (i, E, Eref)
            assert abs(W - float(f[f"c{i}_W"])) <= 1e-12 * max(1.0, abs(float(f[f"c{i}_W"])))
        want = np.unpackbits(f[f"c{i}_nbr"], bitorder="little")[: N * N].astype(bool).reshape(N, N)
        words = nbr[0].cpu().numpy().view(np.uint64)
        got = ((words[:, None] >> np.arange(N, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("N", [3, 16, 64])
def test_energy_matches_oracle_random(dtype, N):
    rng = np.random.default_rng(N)
    L = float(np.sqrt(N / 0.03))
    C = 2000
    base = OP.fcc_lattice(N) if N > 3 else np.array([[2.0, 5.0], [4.0, 5.0], [3.0, 7.0]])
    pos = np.mod(base[None] + rng.normal(0, 0.35, (C, N, 2)), L)
    pos[::7] = rng.random((len(pos[::7]), N, 2)) * L  # uniform configs: mostly hard-core overlaps
    pos = pos.astype(dtype)
    Eo, Wo, ovo = OP.total_energy_batch(pos, OP.make_phys(N))
    E, W, ov = total_energy(torch.from_numpy(pos).cuda(), gphys(N))
    E, W, ov = E.cpu().numpy(), W.cpu().numpy(), ov.cpu().numpy()
    np.testing.assert_array_equal(ov, ovo)
    fin = np.isfinite(Eo)
    assert np.array_equal(np.isfinite(E), fin)
    np.testing.assert_allclose(E[fin], Eo[fin], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(W[fin], Wo[fin], rtol=1e-12, atol=1e-12)
    assert 0 < fin.sum() < C


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("N", [16, 64])
def test_energy_clustered_states(dtype, N):
    """Dense clusters (lattice spacing 0.7-0.9 < r_cut, > r_core): every particle has tens
    of pairs inside the cutoff, so the kernel's queue of in-cutoff pair terms fills and
    drains several times per row; energies, virials and neighbour masks against the oracle."""
    rng = np.random.default_rng(100 + N)
    L = float(np.sqrt(N / 0.03))
    C = 512
    side = int(np.ceil(np.sqrt(N)))
    g = np.stack(np.meshgrid(np.arange(side), np.arange(side), indexing="ij"), -1).reshape(-1, 2)[:N].astype(float)
    sp = rng.uniform(0.7, 0.9, (C, 1, 1))
    pos = g[None] * sp + rng.uniform(0, L, (C, 1, 2)) + rng.normal(0, 0.02, (C, N, 2))
    pos = np.mod(pos, L).astype(dtype)
    Eo, Wo, ovo = OP.total_energy_batch(pos, OP.make_phys(N))
    E, W, ov, nbr = total_energy(torch.from_numpy(pos).cuda(), gphys(N), with_neighbours=True)
    E, W, ov = E.cpu().numpy(), W.cpu().numpy(), ov.cpu().numpy()
    np.testing.assert_array_equal(ov, ovo)
    assert (ov == 0).all()
    np.testing.assert_allclose(E, Eo, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(W, Wo, rtol=1e-12, atol=1e-12)
    words = nbr.cpu().numpy().view(np.uint64)
    for c in range(0, C, 64):
        _, _, _, cut = OP.total_energy(pos[c], OP.make_phys(N), with_cutoff=True)
        got = ((words[c][:, None] >> np.arange(N, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)
        np.testing.assert_array_equal(got, np.triu(cut, 1))
        assert got.sum() > 4 * N  # dense: many in-cutoff pairs per row


def test_pcg64_seed_and_draws_bit_exact():
    f = np.load(os.path.join(G, "pcg64.npz"))
    seeds = torch.from_numpy(f["seeds"].astype(np.uint64).view(np.int64)).cuda()
    st = torch.empty((len(seeds), 4), dtype=torch.int64, device="cuda")
    L = _lib.load()
    _lib.check(L.fs_pcg64_seed(_lib.ptr(seeds), len(seeds), _lib.ptr(st), _lib.stream_ptr()))
    np.testing.assert_array_equal(st.cpu().numpy().view(np.uint64), f["state"])
    out = torch.empty(len(seeds), dtype=torch.float64, device="cuda")
    for k in range(8):
        _lib.check(L.fs_pcg64_random(_lib.ptr(st), len(seeds), _lib.ptr(out), _lib.stream_ptr()))
        np.testing.assert_array_equal(out.cpu().numpy(), f["draws"][:, k])


def test_pcg64_seed_many_matches_oracle():
    seeds = np.concatenate([np.arange(0, 300), [2**32 - 1, 2**32, 2**40 + 3, 2**63 + 11]]).astype(np.uint64)
    t = torch.from_numpy(seeds.view(np.int64)).cuda()
    st = torch.empty((len(seeds), 4), dtype=torch.int64, device="cuda")
    _lib.check(_lib.load().fs_pcg64_seed(_lib.ptr(t), len(seeds), _lib.ptr(st), _lib.stream_ptr()))
    np.testing.assert_array_equal(st.cpu().numpy().view(np.uint64), OP.pcg64_seed_many(seeds))


@pytest.mark.parametrize("correct_sign", [False, True])
def test_accept_mask_bit_exact(correct_sign):
    C = 5000
    rng = np.random.default_rng(9)
    E_old = rng.normal(-50, 5, C)
    E_new = E_old + rng.normal(0, 2, C)
    E_new[::17] = np.inf  # hard-core proposals: draw + reject
    E_old[::23] = np.inf  # overlapping old state: accept without a draw (or NaN with inf new)
    nll_old = rng.normal(490, 3, C).astype(np.float32).astype(np.float64)
    lq_new = (-rng.normal(490, 3, C)).astype(np.float32)
    lq_new[::29] = -np.inf  # proposal outside the base support
    E_new[5] = E_old[5]
    lq_new[5] = -nll_old[5]  # ratio exactly 1: accept without a draw
    seeds = np.arange(42, 42 + C, dtype=np.uint64)
    pcg_o = OP.pcg64_seed_many(seeds)
    acc_o, _ = OP.mh_accept(E_old, E_new, nll_old, -lq_new.astype(np.float64), pcg_o, correct_sign=correct_sign)

    d = lambda a, dt=torch.float64: torch.from_numpy(np.ascontiguousarray(a)).to(dt).cuda()
    Eo, Wo, No = d(E_old), d(np.zeros(C)), d(nll_old)
    pcg = torch.empty((C, 4), dtype=torch.int64, device="cuda")
    L = _lib.load()
    seeds_t = d(seeds.view(np.int64), torch.int64)
    _lib.check(L.fs_pcg64_seed(_lib.ptr(seeds_t), C, _lib.ptr(pcg), _lib.stream_ptr()))
    acc = torch.empty(C, dtype=torch.uint8, device="cuda")
    att = torch.zeros(C, dtype=torch.int64, device="cuda")
    accd = torch.zeros(C, dtype=torch.int64, device="cuda")
    nacc = torch.zeros(1, dtype=torch.int64, device="cuda")
    En, lq, Wn = d(E_new), d(lq_new, torch.float32), d(np.zeros(C))
    _lib.check(L.fs_mh_accept(make_phys(10.0, 10.0), C, 16, _lib.ptr(Eo), _lib.ptr(Wo), _lib.ptr(No), _lib.ptr(En),
                              _lib.ptr(Wn), _lib.ptr(lq), _lib.ptr(pcg), None, None, None, _lib.ptr(acc),
                              _lib.ptr(att), _lib.ptr(accd), _lib.ptr(nacc), int(correct_sign), _lib.stream_ptr()),
               "fs_mh_accept")
    got = acc.cpu().numpy()
    np.testing.assert_array_equal(got, acc_o)
    assert int(nacc.item()) == int(acc_o.sum())
    np.testing.assert_array_equal(pcg.cpu().numpy().view(np.uint64), pcg_o)  # same number of draws per chain
    assert att.sum().item() == C and accd.sum().item() == acc_o.sum()
    newE = np.where(acc_o == 1, E_new, E_old)
    np.testing.assert_array_equal(Eo.cpu().numpy(), newE)
    assert 0.05 < acc_o.mean() < 0.95


def test_hist2d_and_well_stats():
    from flowstate.MCMC.batched import Physics
    N, C = 16, 300
    L = float(np.sqrt(N / 0.03))
    B = L / 2
    rng = np.random.default_rng(1)
    pos = rng.random((C, N, 2)) * L
    pos[0, :, 0] = L / 4 + rng.normal(0, 0.1, N)  # all in well A
    pos[0, :, 1] = L / 2 + rng.normal(0, 0.1, N)
    pos[1, :, 0] = 3 * L / 4 + rng.normal(0, 0.1, N)  # all in well B
    pos[1, :, 1] = L / 2 + rng.normal(0, 0.1, N)
    pos[2, 0, 0] = L  # exactly on the right edge after centring (right-inclusive last bin)
    edges = np.linspace(-B, B, 100)
    want, _, _ = np.histogram2d((pos - B).reshape(-1, 2)[:, 0], (pos - B).reshape(-1, 2)[:, 1], bins=[edges, edges])
    tpos = torch.from_numpy(pos).cuda()
    hist = torch.zeros(99 * 99, dtype=torch.int64, device="cuda")
    tedges = torch.from_numpy(edges).cuda()
    _lib.check(_lib.load().fs_hist2d(_lib.ptr(tpos), C, N, B, _lib.ptr(tedges), 99,
                                     _lib.ptr(hist), _lib.stream_ptr()))
    np.testing.assert_array_equal(hist.cpu().numpy().reshape(99, 99), want.astype(np.int64))
    counts = torch.zeros((C, 3), dtype=torch.int64, device="cuda")
    _lib.check(_lib.load().fs_well_stats(_lib.ptr(tpos), None, C, N, B, 1.2, _lib.ptr(counts), _lib.stream_ptr()))
    c = counts.cpu().numpy()
    assert c[0].tolist() == [1, 0, 1] and c[1].tolist() == [0, 1, 1] and c[2:, :2].sum() == 0


@pytest.mark.parametrize("nedges", [100, 151])
def test_hist2d_clustered_large(nedges):
    """fs_hist2d on 16384 chains x 64 particles crowded into few bins (lattice + jitter,
    many chains per bin): the LDS-privatised kernel (nb <= 120) and the global-atomic one
    (nb = 150) against np.histogram2d."""
    N, C = 64, 16384
    L = float(np.sqrt(N / 0.03))
    B = L / 2
    rng = np.random.default_rng(5)
    pos = np.mod(OP.fcc_lattice(N)[None] + rng.normal(0, 0.3, (C, N, 2)), L)
    pos[:64, 0] = [L, L]  # on the right / top edge after centring: the last bin is right-inclusive
    pos[64:128, 0] = [L + 1.0, 0.5]  # outside the edges: dropped
    edges = np.linspace(-B, B, nedges)
    want, _, _ = np.histogram2d((pos - B).reshape(-1, 2)[:, 0], (pos - B).reshape(-1, 2)[:, 1], bins=[edges, edges])
    hist = torch.zeros((nedges - 1) ** 2, dtype=torch.int64, device="cuda")
    _lib.check(_lib.load().fs_hist2d(_lib.ptr(torch.from_numpy(pos).cuda()), C, N, B,
                                     _lib.ptr(torch.from_numpy(edges).cuda()), nedges - 1, _lib.ptr(hist),
                                     _lib.stream_ptr()))
    np.testing.assert_array_equal(hist.cpu().numpy().reshape(nedges - 1, nedges - 1), want.astype(np.int64))


@pytest.mark.gpu
@pytest.mark.parametrize("half_box_scale", [1.0, 0.8])
def test_well_stats_matches_classify_particles(half_box_scale):
    """fs_well_stats = calculate_well_statistics' all-in-A / all-in-B (utils.py:61-141)
    with box = 2*half_box on both axes and each chain in its own dtype: checked against
    the oracle's classify (pinned to the reference in test_oracle_analysis.py), also for
    a half_box that is not box_x / 2 (the driver passes HALF_BOX explicitly)."""
    from oracle import analysis as OA
    N, C = 16, 512
    L = float(np.sqrt(N / 0.03))
    hb = L / 2 * half_box_scale
    rng = np.random.default_rng(7)
    box = 2 * hb
    # most chains packed near one well, a spread around the radius
    centre = np.where(rng.random(C)[:, None] < 0.5, box / 4, 3 * box / 4)
    pos = np.empty((C, N, 2))
    pos[..., 0] = centre + rng.normal(0, 0.6, (C, N))
    pos[..., 1] = box / 2 + rng.normal(0, 0.6, (C, N))
    is_f32 = (rng.random(C) < 0.5).astype(np.uint8)
    pos[is_f32 == 1] = pos[is_f32 == 1].astype(np.float32)
    counts = torch.zeros((C, 3), dtype=torch.int64, device="cuda")
    tpos, tf32 = torch.from_numpy(pos).cuda(), torch.from_numpy(is_f32).cuda()  # alive across the launch
    _lib.check(_lib.load().fs_well_stats(_lib.ptr(tpos), _lib.ptr(tf32), C, N, hb, 1.2,
                                         _lib.ptr(counts), _lib.stream_ptr()))
    got = counts.cpu().numpy()
    want = np.zeros((C, 3), np.int64)
    for dt, sel in ((np.float32, is_f32 == 1), (np.float64, is_f32 == 0)):
        _, st, _ = OA.classify(pos[sel].astype(dt), hb, 1.2)
        want[sel, 0] = st == 1
        want[sel, 1] = st == 2
    want[:, 2] = 1
    np.testing.assert_array_equal(got, want)
    assert 0 < want[:, 0].sum() < C and 0 < want[:, 1].sum() < C
