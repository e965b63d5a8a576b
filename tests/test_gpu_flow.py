"""GPU parity of the HIP coupling-flow passes against the oracle and the
reference goldens.  Tolerance (north star): log_prob within 1e-5 relative.
The reference itself is float32; its own float32-vs-float64 log_prob error
reaches ~1e-5 relative on outliers, so the bound is checked as
|gpu - ref32| <= 1e-5*|ref32| + 1e-4 (absolute floor for values near 0)."""
import os

import numpy as np
import pytest
import torch

from flowstate.models import A1, build_flow, flow_from_state_dict, half_box
from oracle import flow as OF

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
RTOL, ATOL = 1e-5, 1e-4


def close(a, b, rtol=RTOL, atol=ATOL):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    fin = np.isfinite(b)
    assert np.array_equal(np.isfinite(a), fin) and np.array_equal(a[~fin], b[~fin])
    err = np.abs(a[fin] - b[fin])
    bound = rtol * np.abs(b[fin]) + atol
    bad = err > bound
    assert not bad.any(), f"{bad.sum()} / {bad.size} out of tolerance; worst rel {np.max(err / (np.abs(b[fin]) + 1e-30))}"


def golden_model(name):
    f = np.load(os.path.join(G, f"flow_{name}.npz"))
    dims = OF.FlowDims(N=int(f["N"]), L=int(f["L"]), H=int(f["H"]), nb=int(f["nb"]), K=int(f["K"]), B=float(f["B"]))
    sd = OF.random_state_dict(dims, seed=int(f["seed"]))
    m = flow_from_state_dict(sd, dims.N, dims.L, dims.H, dims.nb, dims.K, bound=dims.B)
    return f, dims, sd, m


@pytest.mark.parametrize("name", ["tiny", "n16", "n64"])
def test_log_prob_matches_reference_golden(name):
    f, dims, sd, m = golden_model(name)
    lp = m.log_prob(torch.from_numpy(f["x"]).cuda()).cpu().numpy()
    close(lp, f["log_prob"])
    z = m.inverse(torch.from_numpy(f["x"]).cuda()).cpu().numpy()
    np.testing.assert_allclose(z, f["z_layers"][-1], rtol=0, atol=2e-4 * dims.B)


@pytest.mark.parametrize("name", ["tiny", "n16", "n64"])
def test_sample_direction_matches_reference_golden(name):
    f, dims, sd, m = golden_model(name)
    x, ld = m.forward_and_log_det(torch.from_numpy(f["z_base"]).cuda())
    # the sampling direction's root solve is ill-conditioned: abs tolerance in box units
    np.testing.assert_allclose(x.cpu().numpy(), f["x_sample"], rtol=0, atol=5e-4 * dims.B)
    close(ld.cpu().numpy(), f["logdet_sample"], rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("N", [16, 64])
def test_a1_log_prob_matches_oracle(N):
    """Algorithm-1 hyper-parameters (L=15, H=256, 32 blocks, K=32) at N=16 and N=64."""
    dims = OF.FlowDims(N=N, B=half_box(N), **A1)
    sd = OF.random_state_dict(dims, seed=7)
    m = flow_from_state_dict(sd, N, bound=dims.B, **A1)
    g = torch.Generator().manual_seed(3)
    x = (torch.rand((96, dims.D), generator=g) * 2 - 1) * dims.B
    want = OF.log_prob(sd, x.clone(), dims).numpy()
    got = m.log_prob(x.cuda()).cpu().numpy()
    close(got, want)


@pytest.mark.parametrize("N", [15, 64])
def test_a2_log_prob_and_sample_match_oracle(N):
    """Algorithm-2 hyper-parameters (L=23, H=128, 2 blocks, K=15): the K <= 16 kernels
    compute two transform features per widths / heights tile (columns 0-15, 16-31).  Odd
    N=15 leaves the last pair with one feature.  log_prob and the sampling direction
    against the oracle."""
    from flowstate.models import A2

    dims = OF.FlowDims(N=N, B=half_box(N), **A2)
    sd = OF.random_state_dict(dims, seed=11)
    m = flow_from_state_dict(sd, N, bound=dims.B, **A2)
    g = torch.Generator().manual_seed(4)
    x = (torch.rand((96, dims.D), generator=g) * 2 - 1) * dims.B
    close(m.log_prob(x.cuda()).cpu().numpy(), OF.log_prob(sd, x.clone(), dims).numpy())
    z = (torch.rand((96, dims.D), generator=g) * 2 - 1) * dims.B
    xs = m.forward(z.cuda()).cpu().numpy()
    want = OF.sample_from(sd, z.clone(), dims).numpy()
    np.testing.assert_allclose(xs, want, rtol=0, atol=5e-4 * dims.B)


def test_a1_log_prob_on_flow_samples_within_reference_f32_envelope():
    """The bench's inputs: proposals drawn by the flow itself (sampling pass), A1, N=64.
    There the reference's own float32 log_prob is up to ~2e-5 relative from the exact
    value (float64 restatement), so "within 1e-5 of the reference" is below float32
    noise there.  The bound checked is against the exact value: the HIP pass (spline
    knots normalised in double, flow_device.h knots_from_logits) is within 1e-5 of it
    everywhere, and closer to it than the reference's float32 arithmetic, at the worst
    chain and at the median (measured: ~3x closer)."""
    N = 64
    dims = OF.FlowDims(N=N, B=half_box(N), **A1)
    sd = OF.random_state_dict(dims, seed=7)
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    m = flow_from_state_dict(sd, N, bound=dims.B, **A1)
    g = torch.Generator().manual_seed(5)
    z = (torch.rand((256, dims.D), generator=g) * 2 - 1) * dims.B
    x = m.forward(z.cuda())
    got = m.log_prob(x).double().cpu().numpy()
    xc = x.cpu()
    ref32 = OF.log_prob(sd, xc.clone(), dims).double().numpy()
    exact = OF.log_prob(sd64, xc.double(), dims).numpy()
    assert np.isfinite(exact).all()
    e_gpu = np.abs(got - exact) / np.abs(exact)
    e_ref = np.abs(ref32 - exact) / np.abs(exact)
    assert e_gpu.max() <= 1e-5, e_gpu.max()
    assert e_gpu.max() <= e_ref.max(), (e_gpu.max(), e_ref.max())
    assert np.median(e_gpu) <= 0.5 * np.median(e_ref), (np.median(e_gpu), np.median(e_ref))


def a1_golden_model():
    """bench.synthetic_model (the headline's flow) rebuilt here; its checksum must be the
    one the reference fixture was made with (tests/golden/make_goldens.py a1_case)."""
    import bench
    from test_oracle_golden import _sd_checksum

    f = np.load(os.path.join(G, "flow_a1.npz"))
    m = bench.synthetic_model(int(f["N"]), "cpu")
    assert _sd_checksum(m.state_dict()) == f["checksum"].tobytes(), "synthetic A1 weights drifted"
    return f, m.cuda().eval()


def test_a1_headline_flow_matches_reference_golden():
    """The headline flow (A1, N=64, the bench's own weights) against the REFERENCE's
    log_prob (tests/golden/flow_a1.npz: reference float32, and the reference model in
    float64).  Tolerance, written out: every row within 1e-5 relative of the exact value
    (float64), and each row either within 1e-5 relative of the reference's float32 value
    or no further from the exact value than the reference's own float32 evaluation is
    (its ~1e-5 float32 drift on flow samples, SURVEY §7, is not a target to reproduce).
    The uniform rows must meet the plain 1e-5 bound against the reference."""
    f, m = a1_golden_model()
    got = m.log_prob(torch.from_numpy(f["x"]).cuda()).double().cpu().numpy()
    ref = f["log_prob"].astype(np.float64)
    exact = f["log_prob_f64"]
    assert np.isfinite(exact).all()
    r_ref = np.abs(got - ref) / np.abs(ref)
    e_gpu = np.abs(got - exact) / np.abs(exact)
    e_ref = np.abs(ref - exact) / np.abs(exact)
    assert e_gpu.max() <= 1e-5, e_gpu.max()
    ok = (r_ref <= 1e-5) | (e_gpu <= e_ref)
    assert ok.all(), (np.flatnonzero(~ok), r_ref[~ok], e_gpu[~ok], e_ref[~ok])
    nu = int(f["n_uniform"])
    assert r_ref[:nu].max() <= 1e-5, r_ref[:nu].max()


def test_a1_flow_samples_closer_to_float64_than_reference_f32():
    """The evidence behind the headline tolerance (test above), on 8192 flow samples
    prepared exactly as the bench prepares them: the bench's synthetic flow and states
    (bench.synthetic_model / synthetic_states / decorrelate), the fused step's own
    proposals (in-kernel base draws, fl32(x + HALF_BOX), fl32(config - half_width);
    main_algorithm_1.py:340-343, monte_carlo.py:251-262).  Against the exact value (the
    oracle's float64 evaluation of the same weights and inputs):
      * every row's relative error is within the north star's 1e-5 (measured at r05 on
        this deterministic sample: max 9.8e-6, p99.9 7.6e-6, p99 4.6e-6; the bound is the
        north star's, not fitted to the data);
      * the GPU is closer to the exact value than the reference's own float32 op order
        at p99.9 and at the maximum.
    The GPU's error is float32 latent rounding carried through the layers
    (tools/logq_error_split.py, profiles/r05/r05a_logq_split.json: the per-layer log-det
    arithmetic and its summation contribute < 4e-7 relative; each layer's latents are
    within ~1.3 ulp of the float64 layer on the same input), i.e. the precision of the
    reference's own float32 arithmetic, which a float32 drop-in cannot go below."""
    import bench
    from flowstate.MCMC import BatchedMonteCarlo, Physics

    N, C = 64, 8192
    dev = torch.device("cuda")
    model = bench.synthetic_model(N, dev)
    init, L = bench.synthetic_states(N, C, 0)
    bmc = BatchedMonteCarlo(model, init, Physics(L, L), np.arange(42, 42 + C, dtype=np.uint64), device=dev)
    bench.decorrelate(bmc)
    st = bench.Stepper(bmc)
    for _ in range(3):
        st.step(timed=False)
    torch.cuda.synchronize()
    centered = st.centered.cpu()
    got = st.log_q.double().cpu().numpy()  # the density launch of the step itself
    assert np.array_equal(got, model.log_prob(st.centered).double().cpu().numpy())
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    dims = OF.FlowDims(N=N, B=half_box(N), **A1)
    ref32 = OF.log_prob(sd, centered.clone(), dims).double().numpy()
    exact = OF.log_prob(sd64, centered.double(), dims).numpy()
    fin = np.isfinite(exact)
    assert fin.sum() >= C - 8
    e_gpu = np.abs(got[fin] - exact[fin]) / np.abs(exact[fin])
    e_ref = np.abs(ref32[fin] - exact[fin]) / np.abs(exact[fin])
    q = lambda e, p: float(np.percentile(e, p))  # noqa: E731
    print(f"vs float64 on {fin.sum()} rows: gpu max {e_gpu.max():.3e} p99.9 {q(e_gpu, 99.9):.3e} "
          f"p99 {q(e_gpu, 99):.3e} beyond 1e-5 {(e_gpu > 1e-5).sum()}; reference-order f32 max {e_ref.max():.3e} "
          f"p99.9 {q(e_ref, 99.9):.3e} beyond 1e-5 {(e_ref > 1e-5).sum()}")
    assert e_gpu.max() <= 1e-5, e_gpu.max()
    assert q(e_gpu, 99.9) < q(e_ref, 99.9) and e_gpu.max() < e_ref.max()


def test_a1_headline_flow_samples_roundtrip_golden_rows():
    """The flow-sample rows of the A1 golden map back through the sampling direction:
    forward(inverse(x)) == x on the headline flow."""
    f, m = a1_golden_model()
    nu = int(f["n_uniform"])
    x = torch.from_numpy(f["x"][nu:]).cuda()
    z = m.inverse(x)
    x2 = m.forward(z)
    assert (x2 - x).abs().max().item() < 5e-3 * float(f["B"])


def test_a1_forward_inverse_roundtrip_full_batch():
    """Size-independent property at the benchmark shape: inverse(forward(z)) == z and
    log-dets cancel (FlowTest.checkForwardInverse, flows/flow_test.py:40-47)."""
    N = 64
    m = build_flow(N, device="cuda", **A1).eval()
    with torch.no_grad():
        g = torch.Generator().manual_seed(0)
        for p in m.parameters():
            if p.dim() == 2 and p.shape[0] == N * 97:
                p.copy_(torch.randn(p.shape, generator=g) * 0.01)
    B = half_box(N)
    z = ((torch.rand((4096, 2 * N), device="cuda") * 2 - 1) * B).contiguous()
    x, ld_f = m.forward_and_log_det(z)
    z2, ld_i = m.inverse_and_log_det(x)
    assert torch.isfinite(x).all() and torch.isfinite(ld_f).all()
    err = (z2 - z).abs().max().item()
    assert err < 5e-3 * B, err
    assert (ld_f + ld_i).abs().max().item() < 5e-2


def test_per_layer_api_matches_stack():
    f, dims, sd, m = golden_model("n16")
    x = torch.from_numpy(f["x"]).cuda()
    z, ld = x, torch.zeros(x.shape[0], device="cuda")
    for i in range(dims.L - 1, -1, -1):
        z, l = m.flows[i].inverse(z)
        ld = ld + l
    z2, ld2 = m.inverse_and_log_det(x)
    torch.testing.assert_close(z, z2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(ld, ld2, rtol=1e-5, atol=1e-4)


def test_outside_bound_is_identity_and_minus_inf():
    f, dims, sd, m = golden_model("n16")
    x = torch.from_numpy(f["x"][:4]).cuda()
    lp = m.log_prob(x).cpu().numpy()
    assert np.isneginf(lp[2]) and np.isfinite(lp[[0, 1, 3]]).all()


def test_ragged_batches():
    f, dims, sd, m = golden_model("tiny")
    x = torch.from_numpy(f["x"]).cuda()
    full = m.log_prob(x).cpu().numpy()
    for n in (1, 3, 63, 64):
        part = m.log_prob(x[:n]).cpu().numpy()
        np.testing.assert_array_equal(part, full[:n])
    assert m.log_prob(x[:0]).numel() == 0


def test_pack_tracks_weight_updates():
    f, dims, sd, m = golden_model("tiny")
    x = torch.from_numpy(f["x"]).cuda()
    a = m.log_prob(x)
    with torch.no_grad():
        m.flows[0].prqct.transform_net.final_layer.weight.mul_(2.0)
    b = m.log_prob(x)
    assert not torch.equal(a, b)
    sd2 = {k: v.clone() for k, v in sd.items()}
    sd2["flows.0.prqct.transform_net.final_layer.weight"] *= 2.0
    close(b.cpu().numpy(), OF.log_prob(sd2, torch.from_numpy(f["x"]), dims).numpy())


@pytest.mark.parametrize("N", [1, 3])
def test_layer_forward_inverse_like_reference_flowtest(N):
    """The reference's own FlowTest.checkForwardInverse (flows/flow_test.py, used by
    neural_spline/wrapper_test.py::test_circular_nsf) on the drop-in layer, in the
    configuration the hot path uses (all coordinates circular, no context): dtype and
    shape kept, inverse(forward(x)) == x, log-dets cancel."""
    from flowstate.normflows.flows import CircularCoupledRationalQuadraticSpline

    torch.manual_seed(N)
    D, B = 2 * N, 5.0
    flow = CircularCoupledRationalQuadraticSpline(D, 2, 32, range(D), num_bins=8, tail_bound=B).cuda().eval()
    with torch.no_grad():  # leave the identity initialisation (wrapper.py:181-185)
        for p in flow.parameters():
            p.add_(0.1 * torch.randn_like(p))
    inputs = 6 * torch.rand((3, D), device="cuda") - 3
    out, ld = flow(inputs)
    assert out.dtype == inputs.dtype and out.shape == inputs.shape and ld.shape == (3,)
    back, ld_inv = flow.inverse(out)
    assert back.dtype == inputs.dtype and back.shape == inputs.shape
    torch.testing.assert_close(back, inputs, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(ld + ld_inv, torch.zeros_like(ld), atol=1e-3, rtol=1e-3)
