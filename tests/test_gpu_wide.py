"""The wide path of the flow passes (small batches, csrc/flow_kernels.hip "Wide path"):
the same pass phase by phase over the whole chip.  It must be bit-identical to the
fused kernel (flow_pass_kernel) in every mode: density (log_prob / inverse), sampling
(forward) and propose (in-kernel base draws -> config / centered), including ragged
batch sizes, the K <= 16 feature-pair kernels (A2), the K = 32 kernels (A1), and the
fused NF-MH step built on them."""
import numpy as np
import pytest
import torch

from flowstate import _lib
from flowstate.MCMC import BatchedMonteCarlo, Physics
from flowstate.models import A1, A2, flow_from_state_dict, half_box
from oracle import flow as OF
from oracle import physics as OP

pytestmark = pytest.mark.gpu


class wide_rows:
    """Set the wide-path row limit for a block (0 = always the fused kernel)."""

    def __init__(self, rows):
        self.rows = rows

    def __enter__(self):
        self.prev = _lib.load().fs_set_wide_rows(self.rows)

    def __exit__(self, *exc):
        _lib.load().fs_set_wide_rows(self.prev)


def _model(N, kw, seed=21):
    dims = OF.FlowDims(N=N, B=half_box(N), **kw)
    sd = OF.random_state_dict(dims, seed=seed)
    return dims, sd, flow_from_state_dict(sd, N, bound=dims.B, **kw)


def _both(fn):
    with wide_rows(0):
        a = fn()
        torch.cuda.synchronize()
    with wide_rows(16384):
        b = fn()
        torch.cuda.synchronize()
    return a, b


CASES = [(16, dict(L=3, H=64, nb=2, K=8)), (64, A2), (16, A1), (3, dict(L=2, H=32, nb=2, K=5))]


@pytest.mark.parametrize("N,kw", CASES, ids=["n16-h64", "a2-n64", "a1-n16", "n3-h32"])
@pytest.mark.parametrize("B", [1, 63, 100, 257])
def test_density_and_sampling_bit_identical(N, kw, B):
    dims, sd, m = _model(N, kw)
    g = torch.Generator().manual_seed(B)
    x = ((torch.rand((B, dims.D), generator=g) * 2 - 1) * dims.B * 1.001).cuda()  # a few rows outside the bound
    (lq_f, z_f), (lq_w, z_w) = _both(lambda: (m.log_prob(x).clone(), m.inverse(x).clone()))
    assert torch.equal(lq_f, lq_w) and torch.equal(z_f, z_w)
    zb = ((torch.rand((B, dims.D), generator=g) * 2 - 1) * dims.B).cuda()
    (xf, lf), (xw, lw) = _both(lambda: tuple(t.clone() for t in m.forward_and_log_det(zb)))
    assert torch.equal(xf, xw) and torch.equal(lf, lw)
    # the wide pass replays a cached graph: a second call with new inputs of the same
    # shape must see them (input / output launches updated per call)
    x2 = ((torch.rand((B, dims.D), generator=g) * 2 - 1) * dims.B).cuda()
    with wide_rows(16384):
        a1 = m.log_prob(x).clone()
        a2 = m.log_prob(x2).clone()
    with wide_rows(0):
        b2 = m.log_prob(x2).clone()
    assert torch.equal(a1, lq_w) and torch.equal(a2, b2)


@pytest.mark.parametrize("N,kw", CASES[:3], ids=["n16-h64", "a2-n64", "a1-n16"])
def test_propose_bit_identical(N, kw):
    dims, sd, m = _model(N, kw)
    L = _lib.load()
    C = 300

    def run():
        cfg = torch.empty((C, dims.D), device="cuda")
        cen = torch.empty_like(cfg)
        lq = torch.empty(C, device="cuda")
        err = torch.zeros(1, dtype=torch.int32, device="cuda")
        _lib.check(L.fs_flow_propose_lq(m.dims(), _lib.ptr(m.packed()), C, 99, 7, 1000, 2 * dims.B / 2, _lib.ptr(cfg),
                                        _lib.ptr(cen), None, _lib.ptr(lq), _lib.ptr(err), _lib.stream_ptr()))
        return cfg, cen, lq

    (a, b, c), (d, e, f) = _both(run)
    assert torch.equal(a, d) and torch.equal(b, e) and torch.equal(c, f)
    assert not torch.equal(a[0], a[1])  # rows draw different proposals


def test_a1_oracle_parity_on_wide_path():
    """The wide path against the oracle at A1 (N=16, 96 rows), as the fused kernel's test."""
    dims, sd, m = _model(16, A1, seed=7)
    g = torch.Generator().manual_seed(3)
    x = (torch.rand((96, dims.D), generator=g) * 2 - 1) * dims.B
    with wide_rows(16384):
        got = m.log_prob(x.cuda()).cpu().numpy()
    want = OF.log_prob(sd, x.clone(), dims).numpy()
    assert np.all(np.abs(got - want) <= 1e-5 * np.abs(want) + 1e-4)


@pytest.mark.parametrize("N,kw,C", [(16, A1, 512), (64, A2, 100)], ids=["a1-n16", "a2-n64-refeed"])
def test_fused_steps_bit_identical(N, kw, C):
    """Whole NF-MH steps (pure, then hybrid after local moves) on the two paths: states,
    energies, NLLs, PCG64 states and counters identical."""
    dims, sd, m = _model(N, kw, seed=5)
    Lb = float(np.sqrt(N / 0.03))
    init = np.mod(OP.fcc_lattice(N)[None] + np.random.default_rng(1).normal(0, 0.05, (C, N, 2)), Lb)
    seeds = np.arange(42, 42 + C, dtype=np.uint64)

    def run():
        bmc = BatchedMonteCarlo(m, init, Physics(Lb), seeds)
        bmc.MAX_STEPS_PER_LAUNCH = 1
        bmc.step()
        bmc.step()
        bmc.local_moves(20)
        bmc.step()
        torch.cuda.synchronize()
        return [t.clone() for t in (bmc.state, bmc.E_old, bmc.nll_old, bmc.pcg, bmc.accepted, bmc.attempts)]

    a, b = _both(run)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


class trunk16:
    """The wide path's trunk for a block: by batch size (5, the default: 4 for small batches,
    else 3), each 16-row tile's columns split over several workgroups with in-launch hand-offs
    (4, where the tiles fit half the chip, else 3), 16-row tiles with the layer's start merged
    in and two waves per 32-column tile (3), the same with one wave per tile (2), 16-row tiles
    after a start launch (1) or 32-row tiles (0)."""

    def __init__(self, on):
        self.on = on

    def __enter__(self):
        self.prev = _lib.load().fs_set_wide_trunk16(self.on)

    def __exit__(self, *exc):
        _lib.load().fs_set_wide_trunk16(self.prev)


@pytest.mark.parametrize("N,kw,B", [(64, A1, 1000), (16, A1, 4096), (64, A2, 200), (3, dict(L=2, H=32, nb=2, K=5), 77),
                                    (16, dict(L=3, H=64, nb=2, K=8), 130)],
                         ids=["a1-n64-1000", "a1-n16-4096", "a2-n64-200", "n3-h32-77", "n16-h64-130"])
def test_trunk16_bit_identical_to_trunk32(N, kw, B):
    """The 16-row trunk (v_mfma_f32_16x16x4_f32 fed the 32x32x2 k order), with the start
    merged in (one or two waves per column tile) and without, against the 32-row one,
    density and sampling, and all against the fused kernel."""
    dims, sd, m = _model(N, kw, seed=11)
    g = torch.Generator().manual_seed(B)
    x = ((torch.rand((B, dims.D), generator=g) * 2 - 1) * dims.B).cuda()
    zb = ((torch.rand((B, dims.D), generator=g) * 2 - 1) * dims.B).cuda()
    outs = []
    with wide_rows(16384):
        for on in (5, 4, 3, 2, 1, 0):
            with trunk16(on):
                outs.append([m.log_prob(x).clone()] + [t.clone() for t in m.forward_and_log_det(zb)])
    with wide_rows(0):
        outs.append([m.log_prob(x).clone()] + [t.clone() for t in m.forward_and_log_det(zb)])
    torch.cuda.synchronize()
    for t in zip(*outs):
        assert all(torch.equal(t[0], u) for u in t[1:])


class final32:
    """The wide path's final phase on 16- or 32-row blocks (2), 32-row at most (1) or 64-row
    blocks (0), for small batches."""

    def __init__(self, on):
        self.on = on

    def __enter__(self):
        self.prev = _lib.load().fs_set_wide_final32(self.on)

    def __exit__(self, *exc):
        _lib.load().fs_set_wide_final32(self.prev)


@pytest.mark.parametrize("N,kw,B", [(64, A2, 200), (64, A2, 1000), (3, dict(L=2, H=32, nb=2, K=5), 77),
                                    (16, dict(L=3, H=64, nb=1, K=8), 333), (16, dict(L=2, H=256, nb=2, K=15), 150),
                                    (16, dict(L=2, H=256, nb=2, K=32), 150), (3, dict(L=3, H=128, nb=1, K=32), 77),
                                    (16, dict(L=2, H=256, nb=2, K=32), 4096)],
                         ids=["a2-n64-200", "a2-n64-1000", "n3-h32-77", "n16-h64-333", "n16-h256-k15-150",
                              "n16-h256-k32-150", "n3-h128-k32-77", "n16-h256-k32-4096"])
def test_final32_bit_identical_to_final64(N, kw, B):
    """The final phase on 16-row blocks (K <= 16: v_mfma_f32_16x16x4_f32 fed the 32x32x2 k
    order, one lane per chain and feature for the splines) and 32-row blocks (one row tile per
    wave, each chain's spline in both lane halves; K = 32 too, A1's final phase) against
    64-row blocks and the fused kernel, density and sampling, with a few out-of-bound inputs
    among the rows."""
    dims, sd, m = _model(N, kw, seed=12)
    g = torch.Generator().manual_seed(B + 1)
    x = ((torch.rand((B, dims.D), generator=g) * 2 - 1) * dims.B * 1.001).cuda()  # a few rows outside the bound
    zb = ((torch.rand((B, dims.D), generator=g) * 2 - 1) * dims.B).cuda()
    outs = []
    with wide_rows(16384):
        for on in (2, 1, 0):
            with final32(on):
                outs.append([m.log_prob(x).clone()] + [t.clone() for t in m.forward_and_log_det(zb)])
    with wide_rows(0):
        outs.append([m.log_prob(x).clone()] + [t.clone() for t in m.forward_and_log_det(zb)])
    torch.cuda.synchronize()
    for a, b, c, d in zip(*outs):
        assert torch.equal(a, b) and torch.equal(a, c) and torch.equal(a, d)


@pytest.mark.parametrize("N,kw,B", [(16, A1, 100), (3, dict(L=3, H=128, nb=2, K=32), 10), (64, A2, 500)],
                         ids=["a1-n16-100", "n3-h128-10", "a2-n64-500"])
def test_column_split_trunk_hand_offs_complete(N, kw, B):
    """The column-split trunk (4): every in-launch hand-off completes (err word 0, no bounded
    poll gave up) across density and propose passes replayed back to back (the counters are
    reset per pass and per launch parity), and the results equal the half-tile trunk's (3)."""
    dims, sd, m = _model(N, kw, seed=9)
    L = _lib.load()
    g = torch.Generator().manual_seed(B)
    x = ((torch.rand((B, dims.D), generator=g) * 2 - 1) * dims.B).cuda()

    def run():
        err = torch.zeros(1, dtype=torch.int32, device="cuda")
        lq = torch.empty(B, device="cuda")
        cfg = torch.empty((B, dims.D), device="cuda")
        cen = torch.empty_like(cfg)
        lq2 = torch.empty(B, device="cuda")
        outs = []
        for rep in range(3):
            _lib.check(L.fs_flow_log_prob(m.dims(), _lib.ptr(m.packed()), _lib.ptr(x), B, _lib.ptr(lq), None,
                                          _lib.ptr(err), _lib.stream_ptr()))
            _lib.check(L.fs_flow_propose_lq(m.dims(), _lib.ptr(m.packed()), B, 99, rep, 0, dims.B, _lib.ptr(cfg),
                                            _lib.ptr(cen), None, _lib.ptr(lq2), _lib.ptr(err), _lib.stream_ptr()))
            outs += [lq.clone(), cfg.clone(), lq2.clone()]
        torch.cuda.synchronize()
        return int(err.item()), outs

    with wide_rows(16384):
        with trunk16(4):
            e4, o4 = run()
        with trunk16(3):
            e3, o3 = run()
    assert e4 == 0 and e3 == 0
    assert all(torch.equal(a, b) for a, b in zip(o4, o3))


def test_column_split_hand_offs_under_uneven_load():
    """The column-split trunk's hand-offs while a large fused pass (A1, N=64, 32768 rows,
    ~40 ms) runs on another stream, so the tile's workgroups start and run at uneven times
    (the guide's advice: test hand-offs under uneven load): every hand-off completes (err 0)
    and the results equal the half-tile trunk's, over repeated small passes."""
    dims, sd, m = _model(16, A1, seed=13)
    dbig, sdb, mb = _model(64, A1, seed=14)
    L = _lib.load()
    B = 48
    g = torch.Generator().manual_seed(5)
    x = ((torch.rand((B, dims.D), generator=g) * 2 - 1) * dims.B).cuda()
    xb = ((torch.rand((32768, dbig.D), generator=g) * 2 - 1) * dbig.B).cuda()
    err = torch.zeros(1, dtype=torch.int32, device="cuda")

    def small(mode, reps):
        out = []
        with trunk16(mode):
            for _ in range(reps):
                lq = torch.empty(B, device="cuda")
                _lib.check(L.fs_flow_log_prob(m.dims(), _lib.ptr(m.packed()), _lib.ptr(x), B, _lib.ptr(lq), None,
                                              _lib.ptr(err), _lib.stream_ptr()))
                out.append(lq)
        return out

    with wide_rows(16384):
        ref = small(3, 1)[0].clone()
        side = torch.cuda.Stream()
        mb.packed()
        torch.cuda.synchronize()
        with torch.cuda.stream(side):
            for _ in range(2):
                mb.log_prob(xb)
        got = small(4, 12)
        torch.cuda.synchronize()
    assert int(err.item()) == 0
    assert all(torch.equal(t, ref) for t in got)


class handoff_spins:
    """The column-split trunk's poll budget for a block (0: every hand-off wait gives up at
    once, the timeout hook)."""

    def __init__(self, spins):
        self.spins = spins

    def __enter__(self):
        self.prev = _lib.load().fs_set_wide_handoff_spins(self.spins)

    def __exit__(self, *exc):
        _lib.load().fs_set_wide_handoff_spins(self.prev)


def test_column_split_timeout_reported_and_recovered():
    """A column-split hand-off that gives up waiting (forced: fs_set_wide_handoff_spins(0))
    leaves wrong outputs and err |= 4.  It can never pass unnoticed: the public
    passes (log_prob, inverse, forward) see the bit and re-run on the half-tile trunk, so
    they return the correct values; the MCMC engine's passes report it in its sticky err
    word, so check_errors() raises; and a pass given no err word never takes the
    column-split trunk at all."""
    N, B = 16, 100
    dims, sd, m = _model(N, A1, seed=9)
    L = _lib.load()
    g = torch.Generator().manual_seed(2)
    x = ((torch.rand((B, dims.D), generator=g) * 2 - 1) * dims.B).cuda()
    zb = ((torch.rand((B, dims.D), generator=g) * 2 - 1) * dims.B).cuda()
    with wide_rows(16384):
        with trunk16(3):
            want = [m.log_prob(x).clone(), m.inverse(x).clone()] + [t.clone() for t in m.forward_and_log_det(zb)]
        with trunk16(4), handoff_spins(0):
            # the hook fires: the raw pass reports the timeout
            err = torch.zeros(1, dtype=torch.int32, device="cuda")
            lq = torch.empty(B, device="cuda")
            _lib.check(L.fs_flow_log_prob(m.dims(), _lib.ptr(m.packed()), _lib.ptr(x), B, _lib.ptr(lq), None,
                                          _lib.ptr(err), _lib.stream_ptr()))
            assert int(err.item()) & 4
            # no err word: the half-tile trunk, correct values
            lq0 = torch.empty(B, device="cuda")
            _lib.check(L.fs_flow_log_prob(m.dims(), _lib.ptr(m.packed()), _lib.ptr(x), B, _lib.ptr(lq0), None,
                                          None, _lib.stream_ptr()))
            assert torch.equal(lq0, want[0])
            # the public passes recover
            got = [m.log_prob(x).clone(), m.inverse(x).clone()] + [t.clone() for t in m.forward_and_log_det(zb)]
            for a, b in zip(got, want):
                assert torch.equal(a, b)
            # the engine's sticky word: a density pass of its own (stale NLL) and the fused step
            Lb = float(np.sqrt(N / 0.03))
            init = np.mod(OP.fcc_lattice(N)[None] + np.random.default_rng(1).normal(0, 0.05, (64, N, 2)), Lb)
            bmc = BatchedMonteCarlo(m, init, Physics(Lb), np.arange(42, 42 + 64, dtype=np.uint64))
            bmc.check_errors()  # construction's NLL pass went through the public path
            bmc.invalidate_nll()
            bmc.nf_big_move(torch.from_numpy(init.astype(np.float32)).cuda())
            with pytest.raises(_lib.FlowStateError, match="hand-off"):
                bmc.check_errors()
            bmc2 = BatchedMonteCarlo(m, init, Physics(Lb), np.arange(42, 42 + 64, dtype=np.uint64))
            bmc2.MAX_STEPS_PER_LAUNCH = 1
            bmc2.step()
            with pytest.raises(_lib.FlowStateError, match="hand-off"):
                bmc2.check_errors()
    assert L.fs_set_wide_handoff_spins(-1) == 1 << 20
