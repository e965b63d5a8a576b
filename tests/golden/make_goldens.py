"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Container-only: imports /root/reference (read-only) through the recipe of
SURVEY.md §8(c) and never ships it anywhere; only the produced vectors
(inputs + outputs, *.npz) are committed.  Re-run with

    python tests/golden/make_goldens.py

Fixtures:
  flow_<case>.npz   reference NormalizingFlow.log_prob / sampling-direction
                    outputs (+ per-layer z, spline bins) for seeded weights
                    from oracle.flow.random_state_dict (weights stored for the
                    small cases, seed + checksum for the N=64 case)
  spline.npz        reference unconstrained_rational_quadratic_spline I/O
  energy.npz        reference EnergyCalculator totals, overlap flags and
                    r<=2.5 neighbour masks (float32 and float64 states,
                    N = 3, 16, 64, with overlap / exact-cutoff / PBC-straddling pairs)
  mh_trace.npz      reference MonteCarlo.nf_big_move traces (accept mask,
                    energies, NLLs, final PCG64 state) for given proposals
  pcg64.npz         numpy default_rng(seed) states and first draws, seeds 42..105
  judge_trace.npz   reference judge_normalizing_flow / bulk_judge_normalizing_flow /
                    metropolis_acceptance_particle_move on a scripted op sequence
                    (with nf_big_move after a bulk judge), results + energies + PCG64
  target_energy.npz reference DoubleWellLJ._energy and its gradient wrt the samples
                    (N = 4, 16, 64; uniform, lattice, linear-core and near-origin rows)
  flow_a1.npz       reference log_prob (float32, and the same model in float64) at the
                    headline flow A1, N=64, with bench.synthetic_model's weights (checksum
                    only), on uniform rows and flow samples prepared as nf_big_move does
  box_trace.npz     reference SimulationBox.minimum_image / compute_distance(s) and
                    EnergyCalculator.calculate_particle_energy_virial outputs
  train_a2.npz      one Algorithm-2 training step at config 5's own size (A2 flow L=23,
                    H=128, 2 blocks, K=15, N=64, batch 256, ALPHA=1; weights by seed +
                    checksum): losses, every parameter gradient's norm plus a few whole
                    gradients, the BatchNorm running statistics after the step, and the
                    Adam update (per-tensor norms plus a few whole tensors)
"""
import contextlib
import hashlib
import io
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

REF = "/root/reference"
LINK = "/tmp/oracle_ref/flow_state"  # get_project_root() needs a dir named flow_state


def import_reference():
    os.makedirs(os.path.dirname(LINK), exist_ok=True)
    if not os.path.islink(LINK):
        os.symlink(REF, LINK)
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.dont_write_bytecode = True
    for p in (LINK, os.path.join(LINK, "MCMC"), os.path.join(LINK, "NF")):
        sys.path.insert(0, p)
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        import normflows as NF  # noqa
        import MCMC as MC  # noqa
        import energy_calculator  # noqa  (module-level names used by MonteCarlo)
        from simulation_box import SimulationBox  # noqa
    return NF, MC, SimulationBox


def sd_checksum(sd):
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(sd[k].detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


def build_ref_model(NF, dims):
    layers = []
    with contextlib.redirect_stdout(io.StringIO()):
        for _ in range(dims.L):
            layers.append(NF.flows.CircularCoupledRationalQuadraticSpline(
                dims.D, dims.nb, dims.H, range(dims.D), num_bins=dims.K, tail_bound=dims.B))
    base = NF.Energy.UniformParticle(dims.N, 2, dims.B)
    return NF.NormalizingFlow(base, layers)


def flow_case(NF, name, dims, seed, nbatch, store_weights):
    from oracle import flow as OF
    sd = OF.random_state_dict(dims, seed=seed)
    model = build_ref_model(NF, dims)
    model.load_state_dict(sd, strict=True)  # pins the reference key set
    model.eval()
    g = torch.Generator().manual_seed(seed + 100)
    B = dims.B
    # density-direction inputs: uniform in the box, plus exact edges and outside points
    x = (torch.rand((nbatch, dims.D), generator=g) * 2 - 1) * B
    x[0, :] = B
    x[1, :] = -B
    x[2, 0] = B * 1.0001  # outside the tail bound -> identity tail, base -inf
    with torch.no_grad():
        lp = model.log_prob(x.clone())
        zs = []
        z = x.clone()
        for i in range(dims.L - 1, -1, -1):
            z, _ = model.flows[i].inverse(z)
            zs.append(z.clone())
        # sampling direction from supplied base draws (NormalizingFlow.sample body, core.py:192-193)
        zb = (torch.rand((nbatch, dims.D), generator=g) * 2 - 1) * B
        xs = zb.clone()
        ld_s = torch.zeros(nbatch)
        for f in model.flows:
            xs, ld = f(xs)
            ld_s += ld
    out = dict(N=dims.N, L=dims.L, H=dims.H, nb=dims.nb, K=dims.K, B=B, seed=seed,
               checksum=np.frombuffer(bytes.fromhex(sd_checksum(sd)), dtype=np.uint8),
               x=x.numpy(), log_prob=lp.numpy(), z_layers=np.stack([t.numpy() for t in zs]),
               z_base=zb.numpy(), x_sample=xs.numpy(), logdet_sample=ld_s.numpy())
    if store_weights:
        for k, v in sd.items():
            out["sd/" + k] = v.numpy()
    np.savez_compressed(os.path.join(HERE, f"flow_{name}.npz"), **out)
    print(f"flow_{name}: log_prob[:4]={lp[:4].tolist()}")


def spline_case():
    from normflows.utils import splines as S  # reference module
    rng = np.random.default_rng(7)
    rows = {}
    for K in (5, 8, 32):
        n = 257
        B = 11.547005383792516
        x = ((rng.random(n) * 2 - 1) * B * 1.02).astype(np.float32)
        x[0], x[1] = np.float32(B), np.float32(-B)
        uw = (rng.standard_normal((n, K)) * 0.7).astype(np.float32)
        uh = (rng.standard_normal((n, K)) * 0.7).astype(np.float32)
        ud = (rng.standard_normal((n, K + 1)) * 0.9 + 0.54).astype(np.float32)
        for inv in (False, True):
            o, l = S.unconstrained_rational_quadratic_spline(
                torch.from_numpy(x), torch.from_numpy(uw), torch.from_numpy(uh), torch.from_numpy(ud),
                inverse=inv, tails=["circular"] * n, tail_bound=B)
            rows[f"K{K}_{'inv' if inv else 'fwd'}_out"] = o.numpy()
            rows[f"K{K}_{'inv' if inv else 'fwd'}_lad"] = l.numpy()
        rows[f"K{K}_x"], rows[f"K{K}_uw"], rows[f"K{K}_uh"], rows[f"K{K}_ud"] = x, uw, uh, ud
        rows[f"K{K}_B"] = np.float64(B)
    np.savez_compressed(os.path.join(HERE, "spline.npz"), **rows)
    print("spline: ok")


def energy_case(MC, SimulationBox):
    from energy_calculator import EnergyCalculator
    from oracle.physics import fcc_lattice
    rng = np.random.default_rng(11)
    out = {}
    idx = 0
    for N in (3, 16, 64):
        L = float(np.sqrt(N / 0.03))
        box = SimulationBox(np.sqrt(N / 0.03 * 1.0), np.sqrt(N / 0.03 / 1.0))
        confs = []
        base = fcc_lattice(N) if N > 3 else np.array([[2.0, 5.0], [4.0, 5.0], [3.0, 7.0]])
        confs.append(base.copy())
        for t in range(6):
            confs.append(base + rng.normal(0, 0.3, base.shape))
        for t in range(3):
            confs.append(rng.random((N, 2)) * L)  # uniform: often overlapping
        c = base.copy()
        c[1] = c[0] + np.array([2.5, 0.0])  # exact cutoff pair (r == 2.5)
        confs.append(c)
        c = base.copy()
        c[0] = np.array([0.1, 3.0])
        c[1] = np.array([L - 0.9, 3.0])  # PBC-straddling pair at r ~ 1.0
        confs.append(c)
        c = base.copy()
        c[-1] = c[0] + np.array([0.3, 0.2])  # hard-core overlap late in the row loop
        confs.append(c)
        for ci, conf in enumerate(confs):
            conf = np.mod(conf, L)
            for dt in (np.float64, np.float32):
                pos = conf.astype(dt)
                with contextlib.redirect_stdout(io.StringIO()):
                    ec = EnergyCalculator(N, pos, box, num_wells=2, V0_list=[-10.0, -10.5], r0=1.2,
                                          k=15, timing=False, checking=False)
                E, W = ec.total_energy, ec.total_virial
                # neighbour mask: r <= 2.5 over i<j from the reference's own distance routine
                nb = np.zeros((N, N), bool)
                for i in range(N - 1):
                    r = box.compute_distances(pos[i], pos[i + 1:])
                    nb[i, i + 1:] = r <= 2.5
                out[f"c{idx}_pos"] = pos
                out[f"c{idx}_E"] = np.float64(E)
                out[f"c{idx}_W"] = np.float64(W)
                out[f"c{idx}_nbr"] = np.packbits(nb, bitorder="little")
                out[f"c{idx}_N"] = np.int64(N)
                idx += 1
    out["count"] = np.int64(idx)
    np.savez_compressed(os.path.join(HERE, "energy.npz"), **out)
    print(f"energy: {idx} configs")


def mh_trace_case(NF, MC, SimulationBox):
    from oracle import flow as OF
    from oracle.physics import fcc_lattice
    out = {}
    for N, chains, steps in ((16, 4, 40), (64, 2, 20)):
        dims = OF.FlowDims(N=N, L=2, H=32, nb=1, K=8, B=OF.half_box(N))
        sd = OF.random_state_dict(dims, seed=5 + N)
        model = build_ref_model(NF, dims)
        model.load_state_dict(sd, strict=True)
        model.eval()
        HB = OF.half_box(N)
        rng = np.random.default_rng(123 + N)
        for c in range(chains):
            particles, box = None, None
            with contextlib.redirect_stdout(io.StringIO()):
                particles, box = MC.initialise_fcc(num_particles=N, rho=0.03, aspect_ratio=1.0)
                mc = MC.MonteCarlo(particles=particles, sim_box=box, temperature=1.0, num_particles=N,
                                   num_wells=2, V0_list=[-10.0, -10.5], r0=1.2, k=15,
                                   initial_max_displacement=0.65, target_acceptance=0.5,
                                   timing=False, checking=False, logger=None, seed=42 + c,
                                   device=torch.device("cpu"))
                mc.set_nf_model(model)
            props, acc, E, nll_o, nll_n = [], [], [], [], []
            for t in range(steps):
                if t % 3 == 0:
                    # flow proposal exactly as main_algorithm_1.py:340-343 (float32 + HALF_BOX)
                    z = (torch.rand((1, dims.D), generator=torch.Generator().manual_seed(1000 * c + t)) * 2 - 1) * HB
                    with torch.no_grad():
                        for f in model.flows:
                            z, _ = f(z)
                    cfg = z.reshape(N, 2).numpy() + HB
                else:
                    # local perturbation of the current state so acceptances happen
                    cfg = (np.asarray(mc.particles, np.float64) + rng.normal(0, 0.05, (N, 2)))
                    cfg = np.mod(cfg, 2 * HB).astype(np.float32)
                cfg = np.asarray(cfg, np.float32)
                old = mc.particles - np.array([mc.half_width, mc.half_width])
                old_nll = -model.log_prob(torch.tensor(old.reshape(1, -1), dtype=torch.float)).item()
                new_c = cfg - np.array([mc.half_width, mc.half_width])
                new_nll = -model.log_prob(torch.tensor(new_c.reshape(1, -1), dtype=torch.float)).item()
                with contextlib.redirect_stdout(io.StringIO()):
                    a = mc.nf_big_move(cfg)
                props.append(cfg)
                acc.append(bool(a))
                E.append(mc.energy_calculator.total_energy)
                nll_o.append(old_nll)
                nll_n.append(new_nll)
            st = mc.rng.bit_generator.state["state"]
            key = f"N{N}_c{c}"
            out[key + "_init"] = np.asarray(particles, np.float64)
            out[key + "_props"] = np.stack(props)
            out[key + "_accept"] = np.array(acc)
            out[key + "_E"] = np.array(E)
            out[key + "_nll_old"] = np.array(nll_o)
            out[key + "_nll_new"] = np.array(nll_n)
            out[key + "_final"] = np.asarray(mc.particles)
            out[key + "_pcg_state"] = np.array([st["state"] >> 64, st["state"] & (2**64 - 1),
                                                st["inc"] >> 64, st["inc"] & (2**64 - 1)], np.uint64)
            out[key + "_seed"] = np.int64(42 + c)
            print(f"mh {key}: accepts {sum(acc)}/{steps}")
        out[f"N{N}_flow_seed"] = np.int64(5 + N)
        out[f"N{N}_checksum"] = np.frombuffer(bytes.fromhex(sd_checksum(sd)), dtype=np.uint8)
        out[f"N{N}_chains"] = np.int64(chains)
    np.savez_compressed(os.path.join(HERE, "mh_trace.npz"), **out)


def a1_case(NF, nrows=32):
    """The headline flow (A1: L=15, H=256, 32 blocks, K=32; main_algorithm_1.py:59-67,
    281-283) at N=64, with the bench's own synthetic weights (bench.synthetic_model:
    reference init order under torch.manual_seed(0), perturbed final layers and
    unconditional splines), loaded into the REFERENCE NormalizingFlow.  353 MB of
    weights are not committed: the fixture holds their checksum, and the test rebuilds
    them with the same recipe.  Rows: half uniform in the box, half flow samples (the
    class the bench's proposals belong to), the latter prepared as the MH step feeds
    them to the flow: config = fl32(x + HALF_BOX) (main_algorithm_1.py:340-343), then
    fl32(config - half_width) (monte_carlo.py:251-258).  Outputs: the reference's
    float32 log_prob, and the same reference model in float64 (the exact value the two
    float32 evaluations are measured against)."""
    import bench
    N = 64
    B = bench.half_box(N)
    sd = bench.synthetic_model(N, "cpu").state_dict()
    from oracle import flow as OF
    dims = OF.FlowDims(N=N, B=B, **bench.A1)
    model = build_ref_model(NF, dims)
    model.load_state_dict(sd, strict=True)
    model.eval()
    g = torch.Generator().manual_seed(2024)
    half = nrows // 2
    hw = float(np.sqrt(N / 0.03)) / 2  # MonteCarlo.half_width = box_x / 2 (monte_carlo.py:66)
    with torch.no_grad():
        xu = (torch.rand((half, dims.D), generator=g) * 2 - 1) * B
        z = (torch.rand((half, dims.D), generator=g) * 2 - 1) * B
        xs = z.clone()
        for f in model.flows:
            xs, _ = f(xs)
        cfg = xs.numpy() + B                              # float32 array + Python float -> float32
        cen = (cfg.astype(np.float64) - np.float64(hw)).astype(np.float32)
        x = torch.cat([xu, torch.from_numpy(cen)])
        lp = model.log_prob(x.clone())
        m64 = build_ref_model(NF, dims)
        m64.load_state_dict(sd, strict=True)
        m64 = m64.double().eval()
        lp64 = m64.log_prob(x.clone().double())
    out = dict(N=N, B=B, checksum=np.frombuffer(bytes.fromhex(sd_checksum(sd)), dtype=np.uint8),
               x=x.numpy(), n_uniform=half, log_prob=lp.numpy(), log_prob_f64=lp64.numpy())
    np.savez_compressed(os.path.join(HERE, "flow_a1.npz"), **out)
    rel = (lp.double() - lp64).abs() / lp64.abs()
    print(f"flow_a1: log_prob[:2]={lp[:2].tolist()} ref f32 vs f64 max rel {float(rel.max()):.3g}")


def target_energy_case(NF):
    """DoubleWellLJ._energy (NF/normflows/Energy/SimpleLJ.py:15-39, 63-128) and its
    gradient with respect to the samples (torch.autograd.grad of the energy sum), by the
    reference module on CPU (its hard-coded device='cuda' zero row routed to the CPU).
    N = 4, 16, 64 with the drivers' constants (bound = HALF_BOX, T = 1, V0 = -10, -10.5,
    r0 = 1.2, k = 15): uniform rows (some outside the box, so the wrap acts), lattice rows,
    rows with a pair inside the linear core, one particle near the origin particle."""
    from oracle import flow as OF
    from oracle.physics import fcc_lattice
    real_zeros = torch.zeros

    def zeros_cpu(*a, **k):
        if k.get("device") == "cuda":
            k["device"] = "cpu"
        return real_zeros(*a, **k)

    out = {}
    g = torch.Generator().manual_seed(99)
    torch.zeros = zeros_cpu
    try:
        for N in (4, 16, 64):
            B = OF.half_box(N)
            mod = NF.Energy.DoubleWellLJ(2 * N, N, 1.0, B, V0_list=[-10.0, -10.5], r0=1.2, k=15)
            rows = [(torch.rand((6, 2 * N), generator=g) * 2 - 1) * B * 1.1]
            lat = torch.from_numpy(fcc_lattice(N) - B).float().reshape(1, -1)
            rows.append(lat + torch.randn((4, 2 * N), generator=g) * 0.05)
            core = lat.repeat(3, 1)
            core[0, 2:4] = core[0, 0:2] + torch.tensor([0.5, 0.1])     # pair at r ~ 0.51
            core[1, 2:4] = core[1, 0:2] + torch.tensor([0.0, 0.8])     # just inside 0.82
            core[2, 0:2] = torch.tensor([0.3, -0.2])                   # near the origin particle
            rows.append(core)
            x = torch.cat(rows).contiguous()
            xr = x.clone().requires_grad_(True)
            E = mod._energy(xr)
            (gx,) = torch.autograd.grad(E.sum(), xr)
            out[f"N{N}_x"], out[f"N{N}_E"], out[f"N{N}_grad"] = x.numpy(), E.detach().numpy(), gx.numpy()
            out[f"N{N}_B"] = np.float64(B)
    finally:
        torch.zeros = real_zeros
    np.savez_compressed(os.path.join(HERE, "target_energy.npz"), **out)
    print("target_energy: ok", out["N64_E"][:3])


def init_case(NF):
    """Reference module-construction RNG order: state_dict right after
    torch.manual_seed(seed) + construction (wrapper.py:98-275, resnet.py:53-104)."""
    from oracle import flow as OF
    dims = OF.FlowDims(N=4, L=2, H=32, nb=1, K=5, B=OF.half_box(4))
    torch.manual_seed(123)
    model = build_ref_model(NF, dims)
    out = dict(seed=123, N=dims.N, L=dims.L, H=dims.H, nb=dims.nb, K=dims.K)
    for k, v in model.state_dict().items():
        out["sd/" + k] = v.numpy()
    np.savez_compressed(os.path.join(HERE, "init.npz"), **out)
    print("init: ok")


def local_case(NF, MC):
    """Reference local-move traces (monte_carlo.py:146-223, 375-403) in three phases
    of local moves with adjust_displacement every 50 moves, separated by two
    nf_big_move calls (which count in the displacement counters, monte_carlo.py:240):
      A) a proposal with a hard-core overlap: E = inf, ratio 0, one draw, rejected
         (the running energy is replaced by a recomputed total, :299-301);
      B) a jittered copy of the current state chosen (with the pinned oracle) so
         that log ratio > 0.02: accepted without a draw, state -> float32.
    Both decisions are far from the ratio = 1 boundary, so a float32 log_prob that
    is not bit-identical to torch's cannot change the random stream."""
    from oracle import flow as OF
    from oracle import physics as OP
    out = {}
    for N, chains, moves in ((3, 2, 200), (16, 3, 200), (64, 2, 150)):
        dims = OF.FlowDims(N=N, L=1, H=32, nb=1, K=5, B=OF.half_box(N))
        sd = OF.random_state_dict(dims, seed=77)
        model = build_ref_model(NF, dims)
        model.load_state_dict(sd, strict=True)
        model.eval()
        phys = OP.make_phys(N)
        for c in range(chains):
            with contextlib.redirect_stdout(io.StringIO()):
                if N > 12:
                    particles, box = MC.initialise_fcc(num_particles=N, rho=0.03, aspect_ratio=1.0)
                else:
                    particles, box = MC.initialise_low_left(num_particles=N, rho=0.03, aspect_ratio=1.0,
                                                            visualise=False, checking=False)
                mc = MC.MonteCarlo(particles=particles, sim_box=box, temperature=1.0, num_particles=N,
                                   num_wells=2, V0_list=[-10.0, -10.5], r0=1.2, k=15,
                                   initial_max_displacement=0.65, target_acceptance=0.5, timing=False,
                                   checking=False, logger=None, seed=42 + c, device=torch.device("cpu"))
                mc.set_nf_model(model)
            hw = box.box_size_x / 2
            key = f"N{N}_c{c}"
            out[key + "_init"] = np.asarray(particles, np.float64)
            acc, E, W, mdisp, big, samp = [], [], [], [], [], []
            for phase in range(3):
                for t in range(moves):
                    a0 = mc.accepted_displacement
                    with contextlib.redirect_stdout(io.StringIO()):
                        mc.particle_displacement()
                        if (t + 1) % 50 == 0:
                            mc.adjust_displacement()
                        if (t + 1) % 75 == 0:  # sample() tuples (monte_carlo.py:416-444)
                            s_ = mc.sample(t + 1)
                            samp.append([float(v) for v in s_[:6]])
                    acc.append(mc.accepted_displacement - a0)
                    E.append(mc.energy_calculator.total_energy)
                    W.append(mc.energy_calculator.total_virial)
                    mdisp.append(mc.max_displacement)
                if phase == 2:
                    break
                cur = np.asarray(mc.particles, np.float64)
                if phase == 0:  # A: particle 1 on top of particle 0
                    cfg = cur.astype(np.float32)
                    cfg[1] = cfg[0] + np.float32(0.1)
                else:           # B: decisive accept
                    def nll(x):
                        t = torch.tensor((np.asarray(x, np.float64) - hw).reshape(1, -1), dtype=torch.float)
                        return -OF.log_prob(sd, t, dims).item()
                    E_old, nll_old = mc.energy_calculator.total_energy, nll(cur)
                    cfg = None
                    for sigma in (0.02, 0.01, 0.005, 0.002, 0.001):
                        for s in range(400):
                            cand = np.mod(cur + np.random.default_rng(s).normal(0, sigma, cur.shape),
                                          box.box_size_x).astype(np.float32)
                            lr = -(OP.total_energy(cand, phys)[0] - E_old) - (nll(cand) - nll_old)
                            if lr > 0.02:
                                cfg = cand
                                break
                        if cfg is not None:
                            break
                    assert cfg is not None, key
                with contextlib.redirect_stdout(io.StringIO()):
                    big.append(bool(mc.nf_big_move(cfg)))
                out[key + f"_bigcfg{phase}"] = cfg
            st = mc.rng.bit_generator.state
            out[key + "_accept"] = np.array(acc, np.int8)
            out[key + "_E"] = np.array(E)
            out[key + "_W"] = np.array(W)
            out[key + "_maxdisp"] = np.array(mdisp)
            out[key + "_samples"] = np.array(samp)
            out[key + "_big"] = np.array(big)
            out[key + "_final"] = np.asarray(mc.particles)
            out[key + "_final_dtype32"] = np.int8(np.asarray(mc.particles).dtype == np.float32)
            out[key + "_attempts"] = np.int64(mc.attempts_displacement)
            out[key + "_accepted"] = np.int64(mc.accepted_displacement)
            s_ = st["state"]
            out[key + "_pcg"] = np.array([s_["state"] >> 64, s_["state"] & (2**64 - 1), s_["inc"] >> 64,
                                          s_["inc"] & (2**64 - 1), st["has_uint32"], st["uinteger"]], np.uint64)
            out[key + "_seed"] = np.int64(42 + c)
            print(f"local {key}: accepted {sum(acc)}/{3 * moves}, big {big}, maxdisp {mc.max_displacement:.4f}")
        out[f"N{N}_chains"] = np.int64(chains)
        out[f"N{N}_moves"] = np.int64(moves)
        out[f"N{N}_flow_seed"] = np.int64(77)
    np.savez_compressed(os.path.join(HERE, "local_trace.npz"), **out)


def analysis_case():
    """classify_particles / calculate_well_statistics / calculate_pair_correlation of
    hybrid_NF_MCMC/utils.py (loaded by path: the name `utils` is taken by MCMC/utils.py)
    on float64 and float32 configuration sets, including all-in-A / all-in-B
    configurations, particles across the periodic edges and on the well radius."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("hyb_utils", os.path.join(LINK, "hybrid_NF_MCMC", "utils.py"))
    U = importlib.util.module_from_spec(spec)
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        spec.loader.exec_module(U)
    out = {}
    N, M = 16, 240
    hb = ((N / 0.03) ** (1 / 2)) / 2  # HALF_BOX, main_algorithm_1.py:50
    L = 2 * hb
    rng = np.random.default_rng(123)
    cfg = rng.random((M, N, 2)) * L
    for m in range(0, M, 3):  # all in well A
        cfg[m, :, 0] = L / 4 + rng.normal(0, 0.35, N)
        cfg[m, :, 1] = L / 2 + rng.normal(0, 0.35, N)
    for m in range(1, M, 5):  # all in well B
        cfg[m, :, 0] = 3 * L / 4 + rng.normal(0, 0.35, N)
        cfg[m, :, 1] = L / 2 + rng.normal(0, 0.35, N)
    cfg[2, :, 0] = rng.choice([1e-9, L - 1e-9, 0.0], N)  # across the periodic edge
    rad = 1.2 * 1.1
    ang = rng.random(N) * 2 * np.pi
    cfg[4, :, 0] = L / 4 + rad * np.cos(ang)  # on the well radius (both dtypes)
    cfg[4, :, 1] = L / 2 + rad * np.sin(ang)
    for name, arr in (("f64", cfg), ("f32", cfg.astype(np.float32))):
        cls = U.classify_particles(arr, hb, 1.2)
        ax, pa, pb, dF, runs = U.calculate_well_statistics(arr, 3, hb, 1.2)
        out[f"{name}_cfg"] = arr
        out[f"{name}_cls"] = cls.astype("U7")
        out[f"{name}_avg_x"] = np.array(ax)
        out[f"{name}_avg_x_dtype32"] = np.int8(np.asarray(ax).dtype == np.float32)
        out[f"{name}_p_a"] = np.array(pa)
        out[f"{name}_p_b"] = np.array(pb)
        out[f"{name}_dF"] = np.array(dF, np.float64)
        out[f"{name}_runs"] = np.array(runs)
    out["half_box"] = np.float64(hb)
    # pair correlation of centred float32 samples (as main_algorithm_1.py:354 passes a_ - HALF_BOX)
    samp = (rng.random((150, N, 2)) * L).astype(np.float32)
    samp[0, 1] = samp[0, 0]  # a coincident pair (distance 0 is dropped)
    cen = samp - hb
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        r, g = U.calculate_pair_correlation(cen, N, hb, dr=hb / 50)
        r2, g2 = U.calculate_pair_correlation(cen.astype(np.float64)[:40], N, hb, dr=hb / 30)
    out["rdf_samples"] = cen
    out["rdf_r"] = r
    out["rdf_g"] = np.asarray(g, np.float64)
    out["rdf64_r"] = r2
    out["rdf64_g"] = np.asarray(g2, np.float64)
    np.savez_compressed(os.path.join(HERE, "analysis.npz"), **out)
    print("analysis: ok", np.bincount([{"A": 0, "B": 1, "Outside": 2}[c] for c in out["f64_cls"].ravel()]))


def driver_case(NF, MC):
    """The Algorithm-1 driver's phases (main_algorithm_1.py:138-186 setup, 202-210
    equilibration, 240-253 production, 375-424 testing, 443-455 well statistics, 467-471
    free energy) restated with small sizes around the reference's own MonteCarlo
    objects and hybrid utils: N=3, 4 runs (even runs start left, odd right), a seeded
    flow.  Test configurations alternate between flow samples (+HALF_BOX, float32;
    mostly rejected) and float32 jitters of the run's current state chosen so that the
    MH decision is far from both ratio = 1 and the uniform draw (accepted or rejected
    decisively), so a float32 log_prob that is not bit-identical cannot flip it."""
    import copy
    import importlib.util
    import tempfile

    from oracle import flow as OF

    spec = importlib.util.spec_from_file_location("hyb_utils", os.path.join(LINK, "hybrid_NF_MCMC", "utils.py"))
    U = importlib.util.module_from_spec(spec)
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        spec.loader.exec_module(U)
    N, RUNS, SEED = 3, 4, 42
    EQ, ADJ, SF = 600, 200, 50
    PROD, ATTEMPTS, INTERVAL = 300, 9, 200
    HB = ((N / 0.03) ** (1 / 2)) / 2
    dims = OF.FlowDims(N=N, L=2, H=32, nb=1, K=5, B=HB)
    flow_seed = 91
    sd = OF.random_state_dict(dims, seed=flow_seed, final_std=0.05)
    model = build_ref_model(NF, dims)
    model.load_state_dict(sd, strict=True)
    model.eval()
    runs = []
    with contextlib.redirect_stdout(io.StringIO()):
        for i in range(RUNS):
            np.random.seed(i + SEED)
            init = MC.initialise_low_left if i % 2 == 0 else MC.initialise_low_right
            particles, box = init(num_particles=N, rho=0.03, aspect_ratio=1.0, visualise=False, checking=False)
            runs.append(MC.MonteCarlo(particles=particles, sim_box=box, temperature=1.0, num_particles=N,
                                      num_wells=2, V0_list=[-10.0, -10.5], r0=1.2, k=15,
                                      initial_max_displacement=0.65, target_acceptance=0.5, timing=False,
                                      checking=False, logger=None, seed=i + SEED, device=torch.device("cpu")))
    out = {"init": np.array([np.asarray(m.particles, np.float64) for m in runs])}
    for m in runs:
        m.local_samples, m.testing_samples = [], []
    with contextlib.redirect_stdout(io.StringIO()):
        for m in runs:  # equilibration
            for step in range(1, EQ + 1):
                m.particle_displacement()
                if step % ADJ == 0:
                    m.adjust_displacement()
                if step % SF == 0:
                    m.local_samples.append(m.sample(step))
    total = 0
    p_hist, s_hist = [0.0], [0]
    gmc = []
    with contextlib.redirect_stdout(io.StringIO()):
        for m in runs:  # production
            for step in range(1, PROD + 1):
                m.particle_displacement()
                total += 1
                if step % SF == 0:
                    s_ = m.sample(step)
                    m.local_samples.append(s_)
                    gmc.append(s_[6])
    out["global_samples_nf"] = np.array([np.array([p - np.array([HB, HB]) for p in c]) for c in gmc])
    out["total_after_production"] = np.int64(total)
    p_hist.append(0.0)
    s_hist.append(total)
    for m in runs:
        m.set_nf_model(model)
    torch.manual_seed(5)
    with torch.no_grad():
        flow_cfgs = (model.sample(ATTEMPTS * RUNS).reshape(-1, N, 2).numpy() + HB)
    test_cfgs = np.zeros((ATTEMPTS * RUNS, N, 2), np.float32)

    def log_ratio_and_u(m, cfg):
        E = m.energy_calculator
        keep = (E.total_energy, E.total_virial)
        enn, _ = E.calculate_total_energy_virial(cfg)
        E.total_energy, E.total_virial = keep
        nll = lambda x: -OF.log_prob(sd, torch.tensor((np.asarray(x, np.float64) - m.half_width).reshape(1, -1),
                                                      dtype=torch.float), dims).item()
        lr = -m.beta * (enn - keep[0]) - (nll(cfg) - nll(m.particles))
        return lr, copy.deepcopy(m.rng).random()

    big_attempts = big_accepts = 0
    acc = np.zeros((RUNS, ATTEMPTS), np.int8)
    with contextlib.redirect_stdout(io.StringIO()):
        for r, m in enumerate(runs):  # testing phase (run-major, as the reference)
            for a in range(ATTEMPTS):
                for step in range(1, INTERVAL + 1):
                    m.particle_displacement()
                    total += 1
                    if step % SF == 0:
                        s_ = m.sample(step)
                        m.local_samples.append(s_)
                        m.testing_samples.append(s_[6])
                if a % 3 == 0:
                    cfg = flow_cfgs[a * RUNS + r].astype(np.float32)
                else:  # a jitter of the state (a % 3 == 1) or of its mirror image in the other well
                    cur = np.asarray(m.particles, np.float64)
                    if a % 3 == 2:
                        cur = cur + np.array([m.sim_box.box_size_x / 2, 0.0])
                    cfg = None
                    for sigma in (0.05, 0.02, 0.01, 0.005):
                        for s in range(200):
                            cand = np.mod(cur + np.random.default_rng(1000 * r + 10 * a + s).normal(0, sigma, cur.shape),
                                          m.sim_box.box_size_x).astype(np.float32)
                            lr, u = log_ratio_and_u(m, cand)
                            if abs(lr) > 0.02 and (lr > 0 or abs(np.exp(lr) - u) > 0.02):
                                cfg = cand
                                break
                        if cfg is not None:
                            break
                    assert cfg is not None
                test_cfgs[a * RUNS + r] = cfg
                ok = m.nf_big_move(test_cfgs[a * RUNS + r])
                big_attempts += 1
                big_accepts += int(ok)
                acc[r, a] = int(ok)
                p_hist.append(big_accepts / big_attempts)
                s_hist.append(total)
    out["test_configs"] = test_cfgs
    out["accepts"] = acc
    out["p_acc_history"] = np.array(p_hist)
    out["mcmc_steps_history"] = np.array(s_hist)
    dF_all = []
    for r, m in enumerate(runs):
        k = f"run{r}"
        out[k + "_local"] = np.array([[float(v) for v in s_[:6]] for s_ in m.local_samples])
        cfgs = np.array([s_[6] for s_ in m.local_samples])
        out[k + "_configs"] = cfgs
        tc = np.array(m.testing_samples)
        out[k + "_testing"] = tc
        ax, pa, pb, dF, _ = U.calculate_well_statistics(tc, 0, HB, 1.2)
        out[k + "_avg_x"] = np.array(ax, np.float64)
        out[k + "_p_a"] = np.array(pa)
        out[k + "_p_b"] = np.array(pb)
        out[k + "_dF"] = np.array(dF, np.float64)
        out[k + "_final"] = np.asarray(m.particles)
        out[k + "_counters"] = np.array([m.attempts_displacement, m.accepted_displacement])
        out[k + "_max_disp"] = np.float64(m.max_displacement)
        dF_all.append(dF)
    with tempfile.TemporaryDirectory() as td, contextlib.redirect_stdout(io.StringIO()):
        _, _, fm, fs, fstd = U.plot_avg_free_energy(dF_all, td, color="C2")
        import json
        d = json.load(open(os.path.join(td, "avg_free_energy_data.json")))
    out["mean_deltaF"] = np.array(d["mean_deltaF"])
    out["sem_deltaF"] = np.array(d["sem_deltaF"])
    out["final"] = np.array([fm, fs, fstd])
    out["params"] = np.array([N, RUNS, SEED, EQ, ADJ, SF, PROD, ATTEMPTS, INTERVAL, flow_seed])
    out["half_box"] = np.float64(HB)
    np.savez_compressed(os.path.join(HERE, "driver.npz"), **out)
    print("driver: ok accepts", acc.sum(), "of", acc.size, "dtypes", [out[f"run{r}_testing"].dtype for r in range(RUNS)])


def train_case(NF):
    """Algorithm-2 training pieces (main_algorithm_2.py:314-331) on a small flow in
    train mode: forward_kld / reverse_kld losses, their parameter gradients, the
    BatchNorm running statistics they update, and one Adam step of
    loss = ALPHA*forward_kld + (1-ALPHA)*reverse_kld with ALPHA = 1.  reverse_kld's
    base draw is supplied (q0 patched) so a GPU run can replay it; SimpleLJ._energy's
    hard-coded device='cuda' zero row is routed to the CPU by a local torch.zeros
    wrapper."""
    from oracle import flow as OF
    dims = OF.FlowDims(N=4, L=2, H=32, nb=2, K=5, B=OF.half_box(4))
    sd = OF.random_state_dict(dims, seed=5, final_std=0.05)
    g = torch.Generator().manual_seed(11)
    x = (torch.rand((64, dims.D), generator=g) * 2 - 1) * dims.B * 0.9
    z0 = (torch.rand((64, dims.D), generator=g) * 2 - 1) * dims.B
    real_zeros = torch.zeros

    def zeros_cpu(*a, **k):
        if k.get("device") == "cuda":
            k["device"] = "cpu"
        return real_zeros(*a, **k)

    def fresh():
        model = build_ref_model(NF, dims)
        model.load_state_dict(sd, strict=True)
        model.p = NF.Energy.DoubleWellLJ(dims.D, dims.N, 1.0, dims.B, V0_list=[-10.0, -10.5], r0=1.2, k=15)
        model.q0.forward = lambda n: z0[:n].clone()
        model.train()
        return model

    out = {"x": x.numpy(), "z0": z0.numpy()}
    names = [n for n, _ in fresh().named_parameters()]
    torch.zeros = zeros_cpu
    try:
        m = fresh()
        lf = m.forward_kld(x)
        gf = torch.autograd.grad(lf, list(m.parameters()), allow_unused=True)
        out["fkld"] = lf.detach().numpy()
        for n, gr in zip(names, gf):
            out["gf/" + n] = (gr if gr is not None else torch.zeros(0)).numpy()
        for k, v in m.state_dict().items():
            if "running" in k:
                out["bn_after_f/" + k] = v.numpy()
        m = fresh()
        lr_, zr = m.reverse_kld(64)
        gr_ = torch.autograd.grad(lr_, list(m.parameters()), allow_unused=True)
        out["rkld"] = lr_.detach().numpy()
        out["rkld_z"] = zr.detach().numpy()
        out["energy"] = m.p._energy(zr.detach()).numpy()
        for n, gr in zip(names, gr_):
            out["gr/" + n] = (gr if gr is not None else torch.zeros(0)).numpy()
        m = fresh()
        opt = torch.optim.Adam(m.parameters(), lr=0.000543510751759681, weight_decay=9.5857178422352e-05)
        opt.zero_grad()
        energy_loss, _ = m.reverse_kld(64)
        sample_loss = m.forward_kld(x)
        loss = 1.0 * sample_loss + (1 - 1.0) * energy_loss
        out["step_loss"] = loss.detach().numpy()
        if ~(torch.isnan(loss) | torch.isinf(loss)):
            loss.backward()
            opt.step()
        for k, v in m.state_dict().items():
            out["after_step/" + k] = v.numpy()
    finally:
        torch.zeros = real_zeros
    out["names"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "train.npz"), **out)
    print("train: ok", float(out["fkld"]), float(out["rkld"]), float(out["step_loss"]))


def train_cycle_case(NF):
    """One Algorithm-2 training epoch as main_algorithm_2.py:430-452 runs it: the
    reference's get_dataloader (utils.py:49-59, shuffle=True, batch 256, a partial last
    batch), a fresh Adam, loss = ALPHA * forward_kld + (1 - ALPHA) * reverse_kld(256)
    with the base draws taken from the default generator, cycle_loss / len(dataloader).
    ALPHA = 1 and 0.5, torch.manual_seed(23) before the epoch; N=3, L=2, H=32, nb=2, K=15."""
    import importlib.util

    from oracle import flow as OF
    spec = importlib.util.spec_from_file_location("hyb_utils", os.path.join(LINK, "hybrid_NF_MCMC", "utils.py"))
    U = importlib.util.module_from_spec(spec)
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        spec.loader.exec_module(U)
    dims = OF.FlowDims(N=3, L=2, H=32, nb=2, K=15, B=OF.half_box(3))
    sd = OF.random_state_dict(dims, seed=17, final_std=0.05)
    rng = np.random.default_rng(3)
    data = (rng.random((600, dims.N, 2)) * 2 - 1) * dims.B * 0.9  # centred float64 configurations
    real_zeros = torch.zeros

    def zeros_cpu(*a, **k):
        if k.get("device") == "cuda":
            k["device"] = "cpu"
        return real_zeros(*a, **k)

    out = {"data": data}
    torch.zeros = zeros_cpu
    try:
        for alpha in (1.0, 0.5):
            model = build_ref_model(NF, dims)
            model.load_state_dict(sd, strict=True)
            model.p = NF.Energy.DoubleWellLJ(dims.D, dims.N, 1.0, dims.B, V0_list=[-10.0, -10.5], r0=1.2, k=15)
            model.train()
            torch.manual_seed(23)
            with contextlib.redirect_stdout(io.StringIO()):
                dl = U.get_dataloader(data, dims.N, 2, torch.device("cpu"), batch_size=256, shuffle=True)
            opt = torch.optim.Adam(model.parameters(), lr=0.000543510751759681, weight_decay=9.5857178422352e-05)
            cycle_loss, losses = 0.0, []
            for batch in dl:
                opt.zero_grad()
                energy_loss, z = model.reverse_kld(256)
                sample_loss = model.forward_kld(batch[0])
                loss = alpha * sample_loss + (1 - alpha) * energy_loss
                if ~(torch.isnan(loss) | torch.isinf(loss)):
                    loss.backward()
                    opt.step()
                cycle_loss += loss.item()
                losses.append(loss.item())
            tag = f"a{int(alpha * 10)}"
            out[tag + "_losses"] = np.array(losses)
            out[tag + "_avg"] = np.float64(cycle_loss / len(dl))
            for k, v in model.state_dict().items():
                out[tag + "/" + k] = v.numpy()
    finally:
        torch.zeros = real_zeros
    np.savez_compressed(os.path.join(HERE, "train_cycle.npz"), **out)
    print("train_cycle: ok", out["a10_losses"], out["a5_losses"])


TRAIN_A2_FULL = ("flows.0.prqct.transform_net.initial_layer.weight",
                 "flows.0.prqct.transform_net.final_layer.bias",
                 "flows.0.prqct.unconditional_transform.unnormalized_heights",
                 "flows.11.prqct.transform_net.blocks.0.batch_norm_layers.1.weight",
                 "flows.11.prqct.transform_net.blocks.1.linear_layers.0.weight",
                 "flows.22.prqct.transform_net.blocks.1.linear_layers.1.bias",
                 "flows.22.prqct.transform_net.initial_layer.bias")


def train_a2_case(NF):
    """One step of the Algorithm-2 training loop (main_algorithm_2.py:437-452) at config
    5's own size: the A2 flow (L=23, H=128, nb=2, K=15; main_algorithm_2.py:43-51,287-294)
    at N=64 in train mode, seeded weights (oracle.flow.random_state_dict, seed 41, final
    layers N(0, 0.05); only the checksum is stored), a fresh Adam (LR / WEIGHT_DECAY of
    main_algorithm_2.py), one batch of 256 training rows, reverse_kld(256) with supplied
    base draws (q0 patched, so the GPU replays the same z), loss = ALPHA * forward_kld +
    (1 - ALPHA) * reverse_kld at ALPHA = 1 (core.py:88-142).  Stored: both losses, each
    parameter gradient's norm (and a few whole gradients), every BatchNorm running
    statistic after the step (both passes updated them, reverse_kld first), and the Adam
    update p_after - p_before (norms, and the same few tensors whole).  The same step's
    gradients by the reference model in float64 give the exact values the float32
    gradients are measured against: per tensor |g32 - g64|, and g64 of the few tensors."""
    from oracle import flow as OF
    from oracle import physics as OP
    N = 64
    dims = OF.FlowDims(N=N, L=23, H=128, nb=2, K=15, B=OF.half_box(N))
    sd = OF.random_state_dict(dims, seed=41, final_std=0.05)
    B, bs = dims.B, 256
    rng = np.random.default_rng(43)
    # training rows as the driver feeds them (sampled box configurations - HALF_BOX): an
    # FCC lattice with thermal jitter for half the batch, uniform rows for the other half
    lat = OP.fcc_lattice(N)[None] + rng.normal(0, 0.35, (bs // 2, N, 2))
    lat = np.mod(lat, 2 * B) - B
    uni = (rng.random((bs - bs // 2, N, 2)) * 2 - 1) * B * 0.95
    x = torch.from_numpy(np.concatenate([lat, uni]).reshape(bs, -1).astype(np.float32))
    z0 = (torch.rand((bs, dims.D), generator=torch.Generator().manual_seed(44)) * 2 - 1) * B
    real_zeros = torch.zeros

    def zeros_cpu(*a, **k):
        if k.get("device") == "cuda":
            k["device"] = "cpu"
        return real_zeros(*a, **k)

    model = build_ref_model(NF, dims)
    model.load_state_dict(sd, strict=True)
    model.p = NF.Energy.DoubleWellLJ(dims.D, dims.N, 1.0, dims.B, V0_list=[-10.0, -10.5], r0=1.2, k=15)
    model.q0.forward = lambda n: z0[:n].clone()
    model.train()
    names = [n for n, _ in model.named_parameters()]
    before = {n: p.detach().clone() for n, p in model.named_parameters()}
    out = {"x": x.numpy(), "z0": z0.numpy(), "seed": np.int64(41), "names": np.array(names),
           "checksum": np.frombuffer(bytes.fromhex(sd_checksum(sd)), dtype=np.uint8)}
    torch.zeros = zeros_cpu
    try:
        opt = torch.optim.Adam(model.parameters(), lr=0.000543510751759681, weight_decay=9.5857178422352e-05)
        opt.zero_grad()
        energy_loss, _ = model.reverse_kld(bs)
        sample_loss = model.forward_kld(x)
        loss = 1.0 * sample_loss + (1 - 1.0) * energy_loss
        out["rkld"] = energy_loss.detach().numpy()
        out["fkld"] = sample_loss.detach().numpy()
        out["step_loss"] = loss.detach().numpy()
        assert bool(~(torch.isnan(loss) | torch.isinf(loss)))
        loss.backward()
        gnorm, dnorm = [], []
        for n, p in model.named_parameters():
            g = p.grad
            gnorm.append(float(g.double().norm()) if g is not None else -1.0)
            if n in TRAIN_A2_FULL:
                out["grad/" + n] = g.numpy().copy()
        opt.step()
        for n, p in model.named_parameters():
            d = (p.detach() - before[n]).double()
            dnorm.append(float(d.norm()))
            if n in TRAIN_A2_FULL:
                out["update/" + n] = (p.detach() - before[n]).numpy()
        out["grad_norm"] = np.array(gnorm)
        out["update_norm"] = np.array(dnorm)
        for k, v in model.state_dict().items():
            if "running" in k or "num_batches" in k:
                out["bn/" + k] = v.numpy()
        # the reference's own float32 error: the same step's gradients in float64
        g32 = {n: p.grad.detach().double().clone() for n, p in model.named_parameters() if p.grad is not None}
        m64 = build_ref_model(NF, dims)
        m64.load_state_dict(sd, strict=True)
        m64 = m64.double()
        m64.p = NF.Energy.DoubleWellLJ(dims.D, dims.N, 1.0, dims.B, V0_list=[-10.0, -10.5], r0=1.2, k=15)
        z64 = z0.double()
        m64.q0.forward = lambda n: z64[:n].clone()
        m64.train()
        m64.reverse_kld(bs)  # its BatchNorm updates, as the float32 step (values unused)
        l64 = m64.forward_kld(x.double())
        l64.backward()
        err = []
        for n, p in m64.named_parameters():
            if n in g32:
                err.append(float((g32[n] - p.grad.detach()).norm()))
                if n in TRAIN_A2_FULL:
                    out["grad64/" + n] = p.grad.detach().numpy().copy()
            else:
                err.append(-1.0)
        out["grad_err32_norm"] = np.array(err)
        out["fkld64"] = l64.detach().numpy()
    finally:
        torch.zeros = real_zeros
    np.savez_compressed(os.path.join(HERE, "train_a2.npz"), **out)
    print("train_a2: ok", float(out["fkld"]), float(out["rkld"]), float(out["step_loss"]))


def judge_case(NF, MC):
    """Reference judge_normalizing_flow / bulk_judge_normalizing_flow /
    metropolis_acceptance_particle_move (monte_carlo.py:191-223, 305-370) on a scripted
    sequence per chain, with an nf_big_move after a bulk judge (the stale running energy
    it leaves behind enters that move's ratio, :243).  Per op: the verdict (bool, or the
    accepted count for bulk), the calculator's total energy / virial and the attempt
    counter afterwards; per chain the final particles and PCG64 state."""
    from oracle import flow as OF
    out = {}
    for N, chains in ((16, 3), (64, 2)):
        dims = OF.FlowDims(N=N, L=2, H=32, nb=1, K=8, B=OF.half_box(N))
        sd = OF.random_state_dict(dims, seed=7 + N)
        model = build_ref_model(NF, dims)
        model.load_state_dict(sd, strict=True)
        model.eval()
        for c in range(chains):
            rng = np.random.default_rng(500 + 10 * N + c)
            with contextlib.redirect_stdout(io.StringIO()):
                particles, box = MC.initialise_fcc(num_particles=N, rho=0.03, aspect_ratio=1.0)
                mc = MC.MonteCarlo(particles=particles, sim_box=box, temperature=1.0, num_particles=N,
                                   num_wells=2, V0_list=[-10.0, -10.5], r0=1.2, k=15,
                                   initial_max_displacement=0.65, target_acceptance=0.5,
                                   timing=False, checking=False, logger=None, seed=42 + c,
                                   device=torch.device("cpu"))
                mc.set_nf_model(model)
            L = box.box_size_x

            def near(scale, dt):
                x = np.mod(np.asarray(mc.particles, np.float64) + rng.normal(0, scale, (N, 2)), L)
                return x.astype(dt)

            def overlap(dt):
                x = near(0.02, dt)
                x[1] = x[0]
                return x

            ops, cfgs, res, Es, Ws, att = [], [], [], [], [], []
            script = [("judge", np.float32, 0.05), ("judge", np.float64, 0.6), ("judge_ov", np.float32, 0),
                      ("metro", -5.0, -4.0), ("metro", -4.0, -5.0), ("metro", 1.0, np.inf),
                      ("metro", np.inf, np.inf), ("metro", 2.0, np.nan), ("metro", -3.0, -2.999),
                      ("bulk", np.float32, 6), ("big", np.float32, 0.05), ("judge", np.float32, 0.4),
                      ("bulk", np.float64, 5), ("judge", np.float64, 0.05), ("big", np.float32, 0.02)]
            for op in script:
                kind = op[0]
                with contextlib.redirect_stdout(io.StringIO()):
                    if kind in ("judge", "judge_ov"):
                        x = overlap(op[1]) if kind == "judge_ov" else near(op[2], op[1])
                        r = float(mc.judge_normalizing_flow(x))
                        cfgs.append(x.astype(np.float64)[None]); ops.append((0, int(op[1] == np.float32), 1, 0.0, 0.0))
                    elif kind == "metro":
                        r = float(mc.metropolis_acceptance_particle_move(op[1], op[2]))
                        cfgs.append(np.zeros((0, N, 2))); ops.append((1, 0, 0, op[1], op[2]))
                    elif kind == "bulk":
                        M = op[2]
                        xs = [near(0.03 * (m + 1), op[1]) for m in range(M - 1)] + [overlap(op[1])]
                        xs = xs[:2] + [xs[-1]] + xs[2:-1]  # an overlapping one in the middle
                        ref = mc.energy_calculator.total_energy - 0.3
                        a, t = mc.bulk_judge_normalizing_flow(xs, ref)
                        assert t == M
                        r = float(a)
                        cfgs.append(np.stack(xs).astype(np.float64)); ops.append((2, int(op[1] == np.float32), M, ref, 0.0))
                    else:  # big
                        x = near(op[2], op[1])
                        r = float(mc.nf_big_move(x))
                        cfgs.append(x.astype(np.float64)[None]); ops.append((3, 1, 1, 0.0, 0.0))
                res.append(r)
                Es.append(mc.energy_calculator.total_energy)
                Ws.append(mc.energy_calculator.total_virial)
                att.append(mc.attempts_displacement)
            key = f"N{N}_c{c}"
            st = mc.rng.bit_generator.state["state"]
            out[key + "_init"] = np.asarray(particles, np.float64)
            out[key + "_ops"] = np.array(ops, np.float64)  # kind, is_f32, M, a, b
            out[key + "_cfgs"] = np.concatenate(cfgs)
            out[key + "_result"] = np.array(res)
            out[key + "_E"] = np.array(Es)
            out[key + "_W"] = np.array(Ws)
            out[key + "_attempts"] = np.array(att, np.int64)
            out[key + "_final"] = np.asarray(mc.particles, np.float64)
            out[key + "_final_f32"] = np.bool_(np.asarray(mc.particles).dtype == np.float32)
            out[key + "_pcg_state"] = np.array([st["state"] >> 64, st["state"] & (2**64 - 1),
                                                st["inc"] >> 64, st["inc"] & (2**64 - 1)], np.uint64)
            print(f"judge {key}: results {res}")
        out[f"N{N}_flow_seed"] = np.int64(7 + N)
        out[f"N{N}_chains"] = np.int64(chains)
    np.savez_compressed(os.path.join(HERE, "judge_trace.npz"), **out)


def box_case(MC):
    """Reference SimulationBox.minimum_image / compute_distance / compute_distances
    (simulation_box.py:31-65) and EnergyCalculator.calculate_particle_energy_virial
    (energy_calculator.py:48-108) on float32 and float64 configurations with
    boundary-straddling pairs, exact half-box separations and a hard-core overlap."""
    from energy_calculator import EnergyCalculator
    out = {}
    for N in (16, 64):
        with contextlib.redirect_stdout(io.StringIO()):
            base, box = MC.initialise_fcc(num_particles=N, rho=0.03, aspect_ratio=1.0)
        L = box.box_size_x
        rng = np.random.default_rng(77 + N)
        for dt in (np.float32, np.float64):
            tag = f"N{N}_{'f32' if dt == np.float32 else 'f64'}"
            x = np.mod(np.asarray(base, np.float64) + rng.normal(0, 0.6, (N, 2)), L)
            x[1] = [0.05, x[1, 1]]
            x[2] = [L - 0.05, x[1, 1]]  # straddles x = 0 with particle 1
            x[3] = [x[4, 0] + L / 2, x[4, 1]]  # exact half-box separation (round half to even)
            x[5] = [x[6, 0] + 0.3, x[6, 1]]  # hard-core overlap (r < 0.5)
            x = np.mod(x, L).astype(dt)
            ii = rng.integers(0, N, 64)
            jj = rng.integers(0, N, 64)
            ii[:4], jj[:4] = [1, 3, 5, 2], [2, 4, 6, 1]
            deltas = np.stack([box.minimum_image(x[i], x[j]) for i, j in zip(ii, jj)])
            dist = np.array([box.compute_distance(x[i], x[j]) for i, j in zip(ii, jj)])
            rows = np.stack([box.compute_distances(x[i], np.delete(x, i, axis=0)) for i in range(N)])
            with contextlib.redirect_stdout(io.StringIO()):
                ec = EnergyCalculator(num_particles=N, initial_particles=x, simulation_box=box, num_wells=2,
                                      V0_list=[-10.0, -10.5], r0=1.2, k=15, timing=False, checking=False)
            pe = np.array([ec.calculate_particle_energy_virial(x, p) for p in range(N)], np.float64)
            out[tag + "_x"] = x
            out[tag + "_ij"] = np.stack([ii, jj], 1)
            out[tag + "_delta"] = deltas
            out[tag + "_delta_dtype_f32"] = np.bool_(deltas.dtype == np.float32)
            out[tag + "_dist"] = np.asarray(dist)
            out[tag + "_dist_dtype_f32"] = np.bool_(np.asarray(dist).dtype == np.float32)
            out[tag + "_rows"] = rows
            out[tag + "_particle_ew"] = pe
            out[tag + "_L"] = np.float64(L)
            print(f"box {tag}: inf rows {int(np.isinf(pe[:, 0]).sum())}, dtypes {deltas.dtype}/{np.asarray(dist).dtype}")
    np.savez_compressed(os.path.join(HERE, "box_trace.npz"), **out)


def pcg_case():
    seeds = np.arange(42, 42 + 64)
    st = np.zeros((64, 4), np.uint64)
    draws = np.zeros((64, 8))
    for i, s in enumerate(seeds):
        g = np.random.default_rng(int(s))
        d = g.bit_generator.state["state"]
        st[i] = [d["state"] >> 64, d["state"] & (2**64 - 1), d["inc"] >> 64, d["inc"] & (2**64 - 1)]
        draws[i] = g.random(8)
    np.savez_compressed(os.path.join(HERE, "pcg64.npz"), seeds=seeds, state=st, draws=draws)
    print("pcg64: ok")


def main(only=None):
    NF, MC, SimulationBox = import_reference()
    from oracle import flow as OF
    torch.set_num_threads(1)
    if only == "local":
        local_case(NF, MC)
        return
    if only == "analysis":
        analysis_case()
        return
    if only == "train":
        train_case(NF)
        return
    if only == "driver":
        driver_case(NF, MC)
        return
    if only == "train_cycle":
        train_cycle_case(NF)
        return
    if only == "judge":
        judge_case(NF, MC)
        return
    if only == "box":
        box_case(MC)
        return
    if only == "target":
        target_energy_case(NF)
        return
    if only == "a1":
        torch.set_num_threads(8)
        a1_case(NF)
        return
    if only == "train_a2":
        torch.set_num_threads(8)
        train_a2_case(NF)
        return
    flow_case(NF, "tiny", OF.FlowDims(N=4, L=2, H=32, nb=1, K=5, B=OF.half_box(4)), 1, 64, True)
    flow_case(NF, "n16", OF.FlowDims(N=16, L=3, H=64, nb=2, K=8, B=OF.half_box(16)), 2, 48, False)
    flow_case(NF, "n64", OF.FlowDims(N=64, L=2, H=128, nb=2, K=32, B=OF.half_box(64)), 3, 16, False)
    spline_case()
    energy_case(MC, SimulationBox)
    mh_trace_case(NF, MC, SimulationBox)
    pcg_case()
    init_case(NF)
    local_case(NF, MC)
    analysis_case()
    train_case(NF)
    driver_case(NF, MC)
    train_cycle_case(NF)
    judge_case(NF, MC)
    box_case(MC)
    target_energy_case(NF)
    torch.set_num_threads(8)
    a1_case(NF)
    train_a2_case(NF)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
