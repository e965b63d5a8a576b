"""GPU parity of the split-bf16 conditioner GEMMs (NormalizingFlow.set_precision:
"bf16x6" = fs_flow_dims.precision 1, "bf16x3" = 2; flow_split_kernels.hip) against the
reference goldens and the oracle, with the f32 path's own bounds (north star: log_prob
within 1e-5 relative; test_gpu_flow.close).  bf16x6 carries every f32 operand as three
bf16 planes and drops only plane products below 2^-24 relative; bf16x3 keeps 16
significant bits per operand.  The f32 path is the default and the headline; these
modes are opt-in."""
import numpy as np
import pytest
import torch

from flowstate.models import A1, A2, build_flow, flow_from_state_dict, half_box
from oracle import flow as OF
from test_gpu_flow import close, golden_model
from test_gpu_mh import _fused_vs_oracle

pytestmark = pytest.mark.gpu
PRECS = ["bf16x6", "bf16x3"]


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("name", ["tiny", "n16", "n64"])
def test_split_log_prob_matches_reference_golden(prec, name):
    f, dims, sd, m = golden_model(name)
    m.set_precision(prec)
    lp = m.log_prob(torch.from_numpy(f["x"]).cuda()).cpu().numpy()
    close(lp, f["log_prob"])
    z = m.inverse(torch.from_numpy(f["x"]).cuda()).cpu().numpy()
    np.testing.assert_allclose(z, f["z_layers"][-1], rtol=0, atol=2e-4 * dims.B)


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("name", ["tiny", "n16", "n64"])
def test_split_sample_direction_matches_reference_golden(prec, name):
    f, dims, sd, m = golden_model(name)
    m.set_precision(prec)
    x, ld = m.forward_and_log_det(torch.from_numpy(f["z_base"]).cuda())
    np.testing.assert_allclose(x.cpu().numpy(), f["x_sample"], rtol=0, atol=5e-4 * dims.B)
    close(ld.cpu().numpy(), f["logdet_sample"], rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("hp,N", [(A1, 16), (A1, 64), (A2, 64)])
def test_split_log_prob_matches_oracle(prec, hp, N):
    """Algorithm-1 (L=15, H=256, 32 blocks, K=32) and Algorithm-2 (L=23, H=128, 2 blocks,
    K=15) hyper-parameters."""
    dims = OF.FlowDims(N=N, B=half_box(N), **hp)
    sd = OF.random_state_dict(dims, seed=7)
    m = flow_from_state_dict(sd, N, bound=dims.B, **hp).set_precision(prec)
    g = torch.Generator().manual_seed(3)
    x = (torch.rand((96, dims.D), generator=g) * 2 - 1) * dims.B
    want = OF.log_prob(sd, x.clone(), dims).numpy()
    got = m.log_prob(x.cuda()).cpu().numpy()
    close(got, want)


def test_split_modes_track_f32_kernel_full_batch():
    """At the benchmark shape (A1, N=64, 4096 chains): each mode within the log_prob bound
    of the exact-f32 kernel on the same inputs; switching back restores the f32 results
    bit for bit; ragged batches give the same per-chain values."""
    N = 64
    m = build_flow(N, device="cuda", **A1).eval()
    with torch.no_grad():
        g = torch.Generator().manual_seed(0)
        for p in m.parameters():
            if p.dim() == 2 and p.shape[0] == N * 97:
                p.copy_(torch.randn(p.shape, generator=g) * 0.01)
    B = half_box(N)
    x = ((torch.rand((4096, 2 * N), generator=torch.Generator().manual_seed(1)) * 2 - 1) * B).cuda()
    ref = m.log_prob(x)
    for prec in PRECS:
        got = m.set_precision(prec).log_prob(x)
        close(got.cpu().numpy(), ref.cpu().numpy())
        for n in (1, 63, 65):
            assert torch.equal(m.log_prob(x[:n]), got[:n])
    assert torch.equal(m.set_precision("f32").log_prob(x), ref)


@pytest.mark.parametrize("prec", PRECS)
def test_split_forward_inverse_roundtrip(prec):
    N = 64
    m = build_flow(N, device="cuda", **A1).eval().set_precision(prec)
    with torch.no_grad():
        g = torch.Generator().manual_seed(0)
        for p in m.parameters():
            if p.dim() == 2 and p.shape[0] == N * 97:
                p.copy_(torch.randn(p.shape, generator=g) * 0.01)
    B = half_box(N)
    z = ((torch.rand((1024, 2 * N), device="cuda") * 2 - 1) * B).contiguous()
    x, ld_f = m.forward_and_log_det(z)
    z2, ld_i = m.inverse_and_log_det(x)
    assert torch.isfinite(x).all() and torch.isfinite(ld_f).all()
    assert (z2 - z).abs().max().item() < 5e-3 * B
    assert (ld_f + ld_i).abs().max().item() < 5e-2


@pytest.mark.parametrize("prec", PRECS)
def test_split_fused_step_matches_oracle_a1_n64(prec):
    """The fused NF-MH step with the split conditioner: the oracle's rule on the step's own
    inputs gives its decision on every chain, the oracle's own values at most one borderline
    flip, and log q within 1e-5 of the exact value on every row (test_gpu_mh._fused_vs_oracle)."""
    flips, rule, acc, n = _fused_vs_oracle(64, A1, C=128, steps=2, precision=prec)
    assert rule == 0
    assert flips <= 1, (flips, n)


def test_precision_rejects_unknown():
    m = build_flow(4, L=1, H=32, nb=1, K=5)
    with pytest.raises(ValueError):
        m.set_precision("fp8")


@pytest.mark.parametrize("prec", PRECS)
def test_split_single_pass_log_q(prec):
    """FS_MH_SINGLE_PASS on the split images: the propose launch's own log q against the
    density pass of the same image on fl32(config - half_width)."""
    from flowstate import _lib

    N, C = 16, 1024
    kw = dict(L=3, H=64, nb=2, K=8)
    dims = OF.FlowDims(N=N, B=half_box(N), **kw)
    m = flow_from_state_dict(OF.random_state_dict(dims, seed=13), N, bound=dims.B, **kw).set_precision(prec)
    lib, p = _lib.load(), _lib.ptr
    cfg = torch.empty((C, 2 * N), device="cuda")
    cen = torch.empty_like(cfg)
    lq1 = torch.empty(C, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    _lib.check(lib.fs_flow_propose_lq(m.dims(), p(m.packed()), C, 3, 0, 0, float(dims.B), p(cfg), p(cen), None,
                                      p(lq1), p(err), _lib.stream_ptr()))
    lq2 = m.log_prob(cen)
    rel = ((lq1.double() - lq2.double()).abs() / lq2.double().abs()).cpu().numpy()
    assert np.median(rel) < 1e-5 and rel.max() < 1e-3, (np.median(rel), rel.max())


def test_bf16x6_headline_flow_matches_reference_golden():
    """The bf16x6 image on the headline flow (A1, N=64, the bench's weights) against the
    REFERENCE's log_prob (tests/golden/flow_a1.npz), with test_gpu_flow's f32 bound written
    out: every row within 1e-5 relative of the exact (float64) value, and each row within
    1e-5 of the reference's float32 value or no further from the exact value than it."""
    from test_gpu_flow import a1_golden_model

    f, m = a1_golden_model()
    m.set_precision("bf16x6")
    got = m.log_prob(torch.from_numpy(f["x"]).cuda()).double().cpu().numpy()
    ref = f["log_prob"].astype(np.float64)
    exact = f["log_prob_f64"]
    r_ref = np.abs(got - ref) / np.abs(ref)
    e_gpu = np.abs(got - exact) / np.abs(exact)
    e_ref = np.abs(ref - exact) / np.abs(exact)
    assert e_gpu.max() <= 1e-5, e_gpu.max()
    ok = (r_ref <= 1e-5) | (e_gpu <= e_ref)
    assert ok.all(), (np.flatnonzero(~ok), r_ref[~ok], e_gpu[~ok], e_ref[~ok])


def test_bf16x6_acceptance_match_at_headline_flow():
    """The metric's qualifier for the bf16x6 image: the bench's own
    acceptance-rate replay (bench.acceptance_match) on the headline flow and synthetic
    states, both flow passes on the bf16x6 image: 2048 chains x 10 steps = 20480
    decisions re-derived by the oracle's restatement of the reference (float32 energies,
    log q and PCG64 draws from the same proposals).  Bound: no decision differs on
    identical inputs; log q of the last 4 steps' proposals (8192 rows) against the exact
    (float64) value within the f32 kernel's own bounds (test_gpu_flow): p99.9 within 1e-5,
    max within 1.25e-5, closer than the reference's float32 op order at the maximum."""
    import bench
    from flowstate.MCMC import BatchedMonteCarlo, Physics

    N, C = 64, 4096
    dev = torch.device("cuda")
    model = bench.synthetic_model(N, dev).set_precision("bf16x6")
    init, L = bench.synthetic_states(N, C, 0)
    bmc = BatchedMonteCarlo(model, init, Physics(L, L), np.arange(42, 42 + C, dtype=np.uint64), device=dev)
    bench.decorrelate(bmc)
    st = bench.Stepper(bmc)
    for _ in range(2):
        st.step(timed=False)
    am = bench.acceptance_match(bmc, st, n_chains=2048, steps=10)
    print({k: am[k] for k in ("gpu_accepts", "oracle_accepts", "mismatched_decisions",
                              "mismatched_on_identical_inputs")}, am["log_q_vs_f64"])
    assert am["gpu_accepts"] > 0
    assert am["mismatched_on_identical_inputs"] == 0, am["per_step"]
    g, r = am["log_q_vs_f64"]["gpu_f32"], am["log_q_vs_f64"]["reference_order_f32"]
    assert g["rows"] >= 8000
    assert g["p999_rel"] <= 1e-5 and g["max_rel"] <= 1.25e-5, g
    assert g["max_rel"] < r["max_rel"], (g, r)
