"""Benchmark: NF-proposed MH steps/sec, N=64 2D LJ, 65536 chains per GPU (BASELINE.json).

One "step" = one fused NF-MH step of every chain (Algorithm-1 flow, A1
hyper-parameters L=15, H=256, 32 residual blocks, K=32 bins, N=64 particles):
  proposal sampling pass (in-kernel U(-B,B) base draws -> 15 sampling-direction
  couplings -> box coordinates) -> log q(x') density pass (15 couplings + base)
  -> LJ + double-well energy of x' -> reference-sign MH accept with per-chain
  PCG64 streams -> state / energy / NLL update.
The kernel sequence is exactly fs_nf_mh_step's; the pieces are launched through
the C ABI one by one so HIP events on the launch stream time each kernel over the
timed region.  Multi-GPU: one process per GPU (torchrun), chains sharded (global
chain index -> PCG64 seed 42+g and proposal-stream row), no per-step collective;
the final density histogram and well-occupancy counters are all-reduced (RCCL).

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "flow-state_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from flowstate import _lib  # noqa: E402
from flowstate.MCMC import BatchedMonteCarlo, Physics, initialise_fcc  # noqa: E402
from flowstate import parallel  # noqa: E402
from flowstate.models import A1, build_flow, half_box  # noqa: E402

PEAK_F32_TFLOPS = 157.3  # MI355X dense FP32 (MFMA = vector rate), MI355X_MICROARCH.md
PEAK_F64_TFLOPS = 78.6   # MI355X FP64 vector
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense BF16 MFMA (spec, no sparsity), MI355X_MICROARCH.md
SPLIT_PRODUCTS = {"bf16x6": 6, "bf16x3": 3}  # bf16 MFMAs per f32-equivalent product
ENERGY_BYTES = lambda N: 4 * 2 * N + 16  # noqa: E731  float32 proposal in, E and W out
ENERGY_FLOP = lambda N: 30 * N * (N - 1) // 2 + 40 * N  # noqa: E731


def flops_per_pass(N, L, H, nb, K):
    """Conditioner GEMM FLOP per chain per pass."""
    return 2 * L * (2 * N * H + 2 * nb * H * H + H * N * (3 * K + 1))


def mfma_flops_per_pass(N, L, H, nb, K):
    """FLOP per chain per pass the f32 kernel actually issues to the matrix cores: the
    initial layer (2N inputs padded to k-groups of 8), the ResNet GEMMs, and per transform
    feature the widths and heights tiles (32 columns each).  The derivative logits are not
    a GEMM: a chain's spline reads only d_bin and d_bin+1 (splines.py:157-158), which the
    kernel takes as two per-lane dot products (VALU, 4*H FLOP per feature)."""
    kin = (2 * N + 7) // 8 * 8
    return 2 * L * (kin * H + 2 * nb * H * H + N * 2 * 32 * H)


def synthetic_model(N, device):
    """Random-init A1 flow (no checkpoint exists offline): reference init order under
    torch.manual_seed(0), then final layers N(0, 0.01) and unconditional spline
    logits N(0, 0.3) so log q is not the identity-init constant."""
    torch.manual_seed(0)
    m = build_flow(N, **A1)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for f in m.flows:
            f.prqct.transform_net.final_layer.weight.copy_(
                torch.randn(f.prqct.transform_net.final_layer.weight.shape, generator=g) * 0.01)
            u = f.prqct.unconditional_transform
            u.unnormalized_widths.copy_(torch.randn(u.unnormalized_widths.shape, generator=g) * 0.3)
            u.unnormalized_heights.copy_(torch.randn(u.unnormalized_heights.shape, generator=g) * 0.3)
    return m.to(device).eval()


def synthetic_states(N, C, c0, seed=7, block=1024):
    """FCC lattice (initialise.py:8-116) + small per-chain jitter, float64 box coords.
    Global chain g's jitter comes from block g // `block` of a generator keyed by
    (seed, block), so a chain's start state does not depend on how the chains are
    sharded over ranks (a 1-rank run over world*C chains holds the same states)."""
    base, box = initialise_fcc(num_particles=N, rho=0.03, aspect_ratio=1.0)
    L = float(box.box_size_x)
    jit = np.empty((C, N, 2))
    g = c0
    while g < c0 + C:
        b = g // block
        rows = np.random.default_rng([seed, b]).normal(0, 0.05, (block, N, 2))
        n = min(c0 + C, (b + 1) * block) - g
        jit[g - c0:g - c0 + n] = rows[g - b * block:g - b * block + n]
        g += n
    return np.mod(base[None] + jit, L), L


def alt_precisions(bmc, stepper, steps=3):
    """The opt-in split-bf16 conditioner modes (NormalizingFlow.set_precision) on the same
    chains right after the headline run: steps/s of the same fused step, the flow kernels'
    f32-equivalent TFLOP/s against the emulated-f32 peak (bf16 dense peak / plane
    products), and the largest relative log q difference to the f32 kernel on the same
    4096 proposals.  Reported beside the headline, never as `value`."""
    model, C, N = bmc.model, bmc.C, bmc.N
    base = model.precision
    x = stepper.centered[:4096].clone()
    ref = model.log_prob(x).double()
    fpp = flops_per_pass(N, **A1)
    out = {}
    for prec, nprod in SPLIT_PRODUCTS.items():
        model.set_precision(prec)
        lq = model.log_prob(x).double()
        fin = torch.isfinite(ref)
        rel = float(((lq - ref).abs() / ref.abs())[fin].max().item()) if bool(fin.any()) else 0.0
        st = Stepper(bmc)
        st.step(timed=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            st.step(timed=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        st.harvest()
        t_prop, t_lp, t_en, t_acc = st.t / steps
        ach = 2 * fpp * C / ((t_prop + t_lp) * 1e-3) / 1e12
        peak = PEAK_BF16_TFLOPS / nprod
        out[prec] = {"value": C * steps / dt, "unit": "steps/s", "steps": steps, "ms_per_step": dt / steps * 1e3,
                     "kernel_ms": {"flow_propose": t_prop, "flow_log_prob": t_lp, "energy": t_en, "mh_accept": t_acc},
                     "max_rel_log_q_vs_f32": rel,
                     "roofline": {"bound": "mfma", "achieved": ach, "peak": peak,
                                  "unit": "TFLOP/s (f32-equivalent)", "frac": ach / peak,
                                  "kernel": f"flow_split_kernel<256,32,*,{3 if nprod == 6 else 2}>"}}
    # proposals drawn through the bf16x6 image, log q (the parity-relevant value) by the
    # f32 kernel: the proposal pass only produces the draws, whose stream differs from the
    # reference's anyway (in-kernel Philox vs torch's generator)
    model.set_precision("bf16x6")
    img = (model.dims(), model.packed())
    model.set_precision("f32")
    st = Stepper(bmc, propose_image=img)
    st.step(timed=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        st.step(timed=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st.harvest()
    t_prop, t_lp, t_en, t_acc = st.t / steps
    out["propose_bf16x6_log_prob_f32"] = {
        "value": C * steps / dt, "unit": "steps/s", "steps": steps, "ms_per_step": dt / steps * 1e3,
        "kernel_ms": {"flow_propose": t_prop, "flow_log_prob": t_lp, "energy": t_en, "mh_accept": t_acc},
        "what": "proposal pass on the bf16x6 image, density pass (log q) on the f32 kernel"}
    # the fastest opt-in combination: bf16x3 image and single-pass log q (one flow pass per
    # step, FS_MH_SINGLE_PASS); neither is the reference's arithmetic or semantics
    model.set_precision("bf16x3")
    bmc.single_pass_log_q = True
    try:
        bmc.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            bmc.step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    finally:
        bmc.single_pass_log_q = False
        model.set_precision(base)
    out["bf16x3_single_pass"] = {"value": C * steps / dt, "unit": "steps/s", "steps": steps,
                                 "ms_per_step": dt / steps * 1e3,
                                 "what": "bf16x3 split conditioner + single-pass log q: one bf16x3 flow pass per step"}
    return out


def given_proposal(bmc, stepper, steps=3):
    """SURVEY §8(d) secondary: the nf_big_move equivalent, i.e. proposals supplied as
    box-coordinate float32 configs (pre-generated as main_algorithm_1.py:340-343 does,
    outside the timed region), then per step: their energy, log q by the density pass,
    and the MH accept (BatchedMonteCarlo.nf_big_move).  The old NLL and energy are the
    cached values (pure NF chains).  Reported beside the headline, never as `value`."""
    C = bmc.C
    batches = []
    for _ in range(2):
        stepper.step(timed=False)  # a fused step leaves its proposals in stepper.config
        batches.append(stepper.config.clone().view(C, bmc.N, 2))
    bmc.nf_big_move(batches[0])
    torch.cuda.synchronize()
    acc0 = int(bmc.n_accept.item())
    t0 = time.perf_counter()
    for i in range(steps):
        bmc.nf_big_move(batches[i % 2])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"value": C * steps / dt, "unit": "steps/s", "steps": steps, "ms_per_step": dt / steps * 1e3,
            "acceptance_rate": (int(bmc.n_accept.item()) - acc0) / (C * steps),
            "what": "energy + density pass + accept of supplied float32 proposals (proposal generation excluded)"}


def single_pass(bmc, stepper, steps=3, n_chains=2048):
    """SURVEY §7 option (i), opt-in (FS_MH_SINGLE_PASS), never the headline: the
    proposals' log q taken from the sampling pass's own log-dets (log q0(z) - sum of
    log|dx/dz|, core.py:178-196 with the log-dets kept) instead of the reference's
    second, density-direction pass over fl32(config - half_width) (monte_carlo.py:
    251-262), so one flow pass per step.  Reports: the deviation from the density-pass
    value on one full batch of proposals (all chains), fused single-pass steps/s on the
    same chains, and one step's decisions on the first n_chains chains against the
    oracle's restatement of the reference (which evaluates log q with the second pass)."""
    from oracle import flow as OF
    from oracle import physics as OP

    L, p, st = _lib.load(), _lib.ptr, _lib.stream_ptr()
    C, N, hw = bmc.C, bmc.N, bmc.phys.half_width
    lq1 = torch.empty(C, dtype=torch.float32, device=bmc.device)
    _lib.check(L.fs_flow_propose_lq(stepper.dims, p(stepper.packed), C, bmc.proposal_seed, bmc.step_count + 10 ** 6,
                                    bmc.chain_offset, hw, p(stepper.config), p(stepper.centered), None, p(lq1),
                                    p(bmc.err), st))
    _lib.check(L.fs_flow_log_prob(stepper.dims, p(stepper.packed), p(stepper.centered), C, p(stepper.log_q), None,
                                  p(bmc.err), st))
    a, b = lq1.double(), stepper.log_q.double()
    fin = torch.isfinite(b) & torch.isfinite(a)
    rel = ((a - b).abs() / b.abs())[fin]
    acc_rel = {"rows": int(fin.sum().item()), "max_rel": float(rel.max().item()),
               "median_rel": float(rel.median().item()), "frac_beyond_1e-5": float((rel > 1e-5).double().mean().item())}
    bmc.single_pass_log_q = True
    try:
        bmc.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            bmc.step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        S = min(n_chains, C)
        state0 = bmc.state[:S].cpu().numpy()
        f32 = bmc.state_is_f32[:S].cpu().numpy().astype(bool)
        pcg = bmc.pcg[:S].cpu().numpy().view(np.uint64).copy()
        bmc.step()
        torch.cuda.synchronize()
        cfg = bmc.last_proposals()[:S].cpu().numpy()
        acc = bmc.accept[:S].cpu().numpy().astype(bool)
    finally:
        bmc.single_pass_log_q = False
    bmc.check_errors()
    sd = {k: v.detach().cpu() for k, v in bmc.model.state_dict().items()}
    dims = OF.FlowDims(N=N, B=half_box(N), **A1)
    phys = OP.make_phys(N)
    E = np.where(f32, OP.total_energy_batch(state0.astype(np.float32), phys)[0], OP.total_energy_batch(state0, phys)[0])
    nll = -OF.log_prob(sd, torch.from_numpy((state0 - hw).astype(np.float32).reshape(S, -1)), dims).numpy() \
        .astype(np.float64)
    lq = OF.log_prob(sd, torch.from_numpy((cfg.astype(np.float64) - hw).astype(np.float32).reshape(S, -1)),
                     dims).numpy().astype(np.float64)
    acc_o, _ = OP.mh_accept(E, OP.total_energy_batch(cfg, phys)[0], nll, -lq, pcg)
    acc_o = acc_o.astype(bool)
    return {"value": C * steps / dt, "unit": "steps/s", "steps": steps, "ms_per_step": dt / steps * 1e3,
            "log_q_vs_density_pass": acc_rel,
            "decisions_vs_oracle": {"chains": S, "gpu_accepts": int(acc.sum()), "oracle_accepts": int(acc_o.sum()),
                                    "mismatched": int((acc != acc_o).sum())},
            "what": "opt-in FS_MH_SINGLE_PASS: log q(x') from the sampling pass (one flow pass per step); "
                    "not the reference's semantics"}


def decorrelate(bmc):
    """SURVEY §8(d) synthetic states: 10 N local moves per chain on its PCG64 stream
    (default_rng(42 + i)) away from the lattice, then one big move, which re-derives the
    old NLL and energy of the moved states (FS_MH_HYBRID); untimed setup."""
    bmc.local_moves(10 * bmc.N)
    bmc.step()


def config2(steps=16, C=4096, N=16):
    """BASELINE config 2 (Algorithm 1, N=16, 4096 chains, A1 flow, f32) as a secondary
    line: fused NF-MH steps/s with the same synthetic flow and states.  4096 chains are
    64 workgroups of the flow kernel, a quarter of the CUs, so BatchedMonteCarlo.step(n)
    runs the proposal passes of several consecutive steps in one launch
    (fs_nf_mh_steps: the same draws and results as one launch per step,
    tests/test_gpu_mh.py::test_multi_step_launch_matches_single_steps); one step per
    launch is reported beside it.  Never the headline `value`."""
    model = synthetic_model(N, torch.device("cuda"))
    init, L = synthetic_states(N, C, 0)
    phys = Physics(L, L, temperature=1.0, num_wells=2, V0_list=(-10.0, -10.5), r0=1.2, k=15)
    bmc = BatchedMonteCarlo(model, init, phys, np.arange(42, 42 + C, dtype=np.uint64))
    decorrelate(bmc)
    S = bmc.steps_per_launch()

    def run(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        bmc.step(n)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    run(S)  # warm-up
    a0 = int(bmc.n_accept.item())
    dt = run(steps)
    rate = (int(bmc.n_accept.item()) - a0) / (C * steps)
    # a loop of step(1) calls (the per-call pattern of the reference's driver loop): the
    # proposal bank serves them from S-step launches (fs_nf_mh_bank / fs_nf_mh_step_banked)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        bmc.step(1)
    torch.cuda.synchronize()
    dt_call = time.perf_counter() - t0
    bmc.MAX_STEPS_PER_LAUNCH = 1
    run(1)
    dt1 = run(steps)
    return {"workload": "config 2: Algorithm 1, N=16, 4096 chains, A1 flow", "value": C * steps / dt,
            "unit": "steps/s", "steps": steps, "ms_per_step": dt / steps * 1e3, "steps_per_launch": S,
            "step1_calls": {"value": C * steps / dt_call, "ms_per_step": dt_call / steps * 1e3},
            "one_step_per_launch": {"value": C * steps / dt1, "ms_per_step": dt1 / steps * 1e3},
            "acceptance_rate": rate}


def algorithm1_regime(attempts=1000, runs=10, N=3, interval=1000, sampling=150, equilibration=5000, speculate=None):
    """The reference's own Algorithm-1 regime (main_algorithm_1.py:33-35, 40-71, 136-210,
    340-343, 375-424) end to end on one MI355X, as a secondary line (VERDICT r04 missing #4):
    NUM_PARTICLES = 3, NUM_MC_RUNS = 10 runs started low-left / low-right alternately with
    seeds 42 + i, EQUILIBRATION_STEPS = 5000 local moves (adjust every 5000, sample() every
    150; untimed), then the testing phase, timed: BIG_MOVE_ATTEMPTS = 1000 attempts, each
    BIG_MOVE_INTERVAL = 1000 particle_displacement calls per run with sample() every 150 and
    one nf_big_move per run with its own flow proposal (generate_samples + HALF_BOX, float32;
    A1 flow L=15 H=256 32 blocks K=32 at N=3, random-init as synthetic_model).  Reports
    big-move attempts/s and local moves/s over the whole phase (flowstate.algorithm1)."""
    from flowstate import algorithm1 as A1D
    from flowstate.analysis import generate_samples
    from flowstate.MCMC import initialise_low_left, initialise_low_right

    dev = torch.device("cuda", torch.cuda.current_device())
    model = synthetic_model(N, dev)
    B = half_box(N)
    init = np.array([(initialise_low_left if i % 2 == 0 else initialise_low_right)(N, 0.03, 1.0)[0]
                     for i in range(runs)])
    bmc = BatchedMonteCarlo(model, init, Physics(2 * B), [42 + i for i in range(runs)], device=dev,
                            initial_max_displacement=0.65)
    A1D.equilibrate(bmc, equilibration, 5000, sampling)
    n = attempts * runs
    cfg = (generate_samples(model, N, 2, n_iterations=n // 5000 + 1, samples_per_iteration=5000,
                            device_output=True) + B).to(torch.float32)
    A1D.testing_phase(bmc, cfg, 2, interval, sampling, speculate=speculate)  # warm-up: graphs, code objects
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = A1D.testing_phase(bmc, cfg, attempts, interval, sampling, speculate=speculate)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    acc = int(res.accepts.sum().item())
    return {"workload": f"Algorithm-1 testing phase as the reference runs it: N={N}, {runs} runs, {attempts} attempts "
                        f"x ({interval} local moves + 1 NF big move) per run, sample() every {sampling}, A1 flow",
            "value": n / dt, "unit": "big-move attempts/s", "local_moves_per_s": n * interval / dt,
            "seconds": dt, "big_move_acceptance": acc / n, "speculated_attempts": res.speculated,
            "what": "main_algorithm_1.py's testing phase on the device (flowstate.algorithm1.testing_phase: the "
                    "local moves back to back on a side stream, each attempt's density pass on its own stream, the "
                    "big moves on the main stream; stages after an accept run again, bit-identical); "
                    "equilibration and proposal generation untimed"}


def algorithm1_regime_cpu(N=3, interval=1000, budget_s=8.0, sample_every=150):
    """A bounded CPU sample of algorithm1_regime's testing phase, timed as the reference
    runs it (oracle/, test infrastructure): one run (low-left start, seed 42) at a time, as
    the reference's driver runs them (main_algorithm_1.py:378-395), each attempt `interval`
    particle_displacement calls in the reference's per-call numpy form
    (oracle.physics.NumpyLocalChain: monte_carlo.py:146-223 over
    energy_calculator.py:48-119, a Python loop of minimum_image + np.linalg.norm per pair,
    numpy's own Generator; bit-identical to the reference's local-move traces,
    tests/test_oracle_local.py) with sample() every `sample_every` moves, then nf_big_move
    (monte_carlo.py:235-303): batch-1 float32 log_prob of the current and the proposed
    configuration in torch-CPU (the reference's op sequence), the proposal's energy by the
    reference's pair loop and the accept.  Proposals generated beforehand, untimed, as on
    the GPU."""
    from oracle import flow as OF
    from oracle import physics as OP
    from flowstate.MCMC import initialise_low_left

    dims = OF.FlowDims(N=N, B=half_box(N), **A1)
    sd = {k: v.detach().cpu() for k, v in synthetic_model(N, "cpu").state_dict().items()}
    hw = np.float32(dims.B)
    g = torch.Generator().manual_seed(77)
    z = (torch.rand((64, dims.D), generator=g) * 2 - 1) * dims.B
    props = (OF.sample_from(sd, z, dims).numpy() + hw).astype(np.float32).reshape(-1, N, 2)
    ch = OP.NumpyLocalChain(initialise_low_left(N, 0.03, 1.0)[0], 42, OP.make_phys(N), max_disp=0.65)
    hw2 = np.array([ch.Lx / 2, ch.Lx / 2])
    threads = torch.get_num_threads()
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < budget_s or n == 0:
        ch.local_moves(interval, sample_every=sample_every)
        cfg = props[n % len(props)]
        old = torch.tensor((ch.particles - hw2).reshape(1, -1), dtype=torch.float)
        new = torch.tensor((cfg - hw2).reshape(1, -1), dtype=torch.float)
        ch.big_move(cfg, -OF.log_prob(sd, old, dims).item(), -OF.log_prob(sd, new, dims).item())
        n += 1
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "big-move attempts/s", "kind": "port", "cores": threads,
            "sample": f"{n} attempts of one run ({interval} local moves + 1 NF big move each, sample() every "
                      f"{sample_every}, A1 flow, N={N}), {dt:.1f} s wall; local moves in the reference's per-call "
                      f"numpy form (oracle.physics.NumpyLocalChain: per-pair minimum_image + np.linalg.norm loop, "
                      f"numpy's Generator; bit-identical to the reference's traces), log_prob by the reference's "
                      f"torch-CPU float32 op sequence at batch 1 on {threads} threads"}


def config5(cycles=10, train_steps=100):
    """BASELINE config 5 (Algorithm 2 on-the-fly retrain + sample, N=64, A2 flow) on one
    GPU as a secondary line, at the reference's sizes (main_algorithm_2.py:33-52): 100
    runs, UPDATE_NUM_SAMPLES=1000 (100 local moves per run, sample() every 10), one
    epoch of batch 256 (graph-captured forward_kld + reverse_kld + Adam, ALPHA=1), then
    the refeed (one fused NF-MH step per run).  Reports cycles/s of the driver's loop
    (Algorithm2.run), the same cycles with the phases called and timed one at a time
    (the phase split), graphed training steps/s on a full batch, and the training step's achieved
    TFLOP/s: 4 A2 passes per sample (forward_kld forward + its backward at 2x, and
    reverse_kld's sampling pass) x 256 samples x SURVEY §8(d)'s F_pass, against the
    dense f32 peak.  Never the headline `value`."""
    from flowstate.algorithm2 import Algorithm2
    from flowstate.models import A2
    from flowstate.normflows.Energy import DoubleWellLJ

    N, runs, bs = 64, 100, 256
    dev = torch.device("cuda", torch.cuda.current_device())
    torch.manual_seed(0)
    B = half_box(N)
    m = build_flow(N, bound=B, device="cpu", **A2)
    m.p = DoubleWellLJ(2 * N, N, 1.0, B, V0_list=[-10.0, -10.5], r0=1.2, k=15)
    m = m.to(dev)
    m.q0.device = dev
    base, box = initialise_fcc(num_particles=N, rho=0.03, aspect_ratio=1.0)
    bmc = BatchedMonteCarlo(None, np.repeat(base[None], runs, 0), Physics(box.box_size_x, box.box_size_y),
                            [42 + i for i in range(runs)], device=dev, initial_max_displacement=0.65)
    bmc.local_moves(10 * N, adjust_every=5 * N)
    algo = Algorithm2(bmc, m, batch_size=bs, alpha=1.0, sampling_frequency=10, update_num_samples=1000)
    t = np.zeros(3)

    def cycle(timed):
        ts = [time.perf_counter()]
        algo.production()
        torch.cuda.synchronize()
        ts.append(time.perf_counter())
        algo.train()
        torch.cuda.synchronize()
        ts.append(time.perf_counter())
        algo.refeed()
        torch.cuda.synchronize()
        ts.append(time.perf_counter())
        if timed:
            t[:] += np.diff(ts)

    cycle(False)
    t0 = time.perf_counter()
    for _ in range(cycles):
        cycle(True)
    dt_phases = time.perf_counter() - t0
    bmc.check_errors()
    # the driver's own loop (Algorithm2.run: main_algorithm_2.py's cycle loop, each next
    # production beside the current training, bit-identical to cycle() calls)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    runs_out = algo.run(cycles)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    bmc.check_errors()
    kept = sum(1 for o in runs_out[:-1] if o[3] == 0)
    # graphed training steps on one full batch of the last training set
    step = algo._step
    x = algo.training_data[:bs].to(dev)
    step.step(x)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(train_steps):
        step.step(x)
    torch.cuda.synchronize()
    sps = train_steps / (time.perf_counter() - t1)
    # the same steps back to back, as an epoch replays them (Algorithm2.train: no host
    # synchronisation per step, every step's NaN flag checked once at the end)
    step.reset_nan()
    flags = []
    t1 = time.perf_counter()
    for _ in range(train_steps):
        flags.append(step.step(x, check=False)[1])
    torch.cuda.synchronize()
    sps_epoch = train_steps / (time.perf_counter() - t1)
    if bool(torch.stack(flags).any()):
        raise ValueError("Discriminant computation resulted in NaN.")
    fpp = flops_per_pass(N, **A2)
    ach = 4 * fpp * bs * sps / 1e12
    return {"workload": "config 5: Algorithm 2 cycle, A2 flow (L=23 H=128 blocks=2 K=15), N=64, 100 runs, "
                        "UPDATE_NUM_SAMPLES=1000, batch 256, 1 GPU",
            "value": cycles / dt, "unit": "cycles/s", "cycles": cycles, "ms_per_cycle": dt / cycles * 1e3,
            "what": "Algorithm2.run(cycles): the next cycle's production runs beside this cycle's training "
                    "(kept when the refeed accepts no run, else run again; bit-identical to cycle() calls)",
            "speculated_productions_kept": kept,
            "phases_timed_separately": {"value": cycles / dt_phases, "ms_per_cycle": dt_phases / cycles * 1e3,
                                        "what": "production / training / refeed called one at a time, a device "
                                                "synchronisation after each (phase_ms)"},
            "phase_ms": {"production": t[0] / cycles * 1e3, "training": t[1] / cycles * 1e3,
                         "refeed": t[2] / cycles * 1e3},
            "train_steps_per_s": sps,
            "train_steps_per_s_epoch": sps_epoch,
            "train_roofline": {"bound": "mfma", "achieved": ach, "peak": PEAK_F32_TFLOPS, "unit": "TFLOP/s",
                               "frac": ach / PEAK_F32_TFLOPS,
                               "flop_per_step": 4 * fpp * bs,
                               "what": "4 A2 passes per sample (forward_kld fwd + bwd, reverse_kld sampling) x 256"},
            "last_loss": algo.loss_history[-1], "last_p_acc": algo.p_acc_history[-1]}


class Stepper:
    """The fs_nf_mh_step kernel sequence, launched piecewise with HIP events."""

    def __init__(self, bmc, propose_image=None):
        self.b = bmc
        self.L = _lib.load()
        self.dims = bmc.model.dims()
        self.packed = bmc.model.packed()
        # (dims, packed) of another precision's image for the proposal pass only
        self.pdims, self.ppacked = propose_image if propose_image else (self.dims, self.packed)
        C, D = bmc.C, 2 * bmc.N
        dev = bmc.device
        self.config = torch.empty((C, D), dtype=torch.float32, device=dev)
        self.centered = torch.empty_like(self.config)
        self.log_q = torch.empty(C, dtype=torch.float32, device=dev)
        self.E_new = torch.empty(C, dtype=torch.float64, device=dev)
        self.W_new = torch.empty_like(self.E_new)
        self.events = []
        self.t = np.zeros(4)  # propose, log_prob, energy, accept (ms, summed over timed steps)

    def step(self, timed):
        b, L, st = self.b, self.L, _lib.stream_ptr()
        p = _lib.ptr
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)] if timed else None
        if timed:
            self.events.append(ev)
            ev[0].record()
        _lib.check(L.fs_flow_propose(self.pdims, p(self.ppacked), b.C, b.proposal_seed, b.step_count, b.chain_offset,
                                     b.phys.half_width, p(self.config), p(self.centered), None, p(b.err), st))
        if timed:
            ev[1].record()
        _lib.check(L.fs_flow_log_prob(self.dims, p(self.packed), p(self.centered), b.C, p(self.log_q), None,
                                      p(b.err), st))
        if timed:
            ev[2].record()
        _lib.check(L.fs_energy_lj_dw(b.phys.c, p(self.config), 1, b.C, b.N, p(self.E_new), p(self.W_new), None, None,
                                     st))
        if timed:
            ev[3].record()
        _lib.check(L.fs_mh_accept(b.phys.c, b.C, b.N, p(b.E_old), p(b.W_old), p(b.nll_old), p(self.E_new),
                                  p(self.W_new), p(self.log_q), p(b.pcg), p(b.state), p(b.state_is_f32),
                                  p(self.config), p(b.accept), p(b.attempts), p(b.accepted), p(b.n_accept), b.flags,
                                  st))
        if timed:
            ev[4].record()
        b.step_count += 1

    def harvest(self):
        for ev in self.events:
            for i in range(4):
                self.t[i] += ev[i].elapsed_time(ev[i + 1])
        self.events = []


def final_reduction(bmc):
    """End-of-run reduction: flowstate.parallel.final_reduction."""
    return parallel.final_reduction(bmc)


FLOW_SOURCES = ("flow-state_amd/csrc/flow_kernels.hip", "flow-state_amd/csrc/flow_device.h",
                "flow-state_amd/csrc/flow_layout.h", "flow-state_amd/csrc/fs_internal.h",
                "flow-state_amd/csrc/Makefile")


def flow_source_sha16():
    """Fingerprint of the sources the f32 flow kernel is built from: a PMC traffic profile
    (profiles/traffic.json, tools/pmc_traffic.py) carries the fingerprint of the sources it
    was collected on, so the bench can say whether its `traffic` is that of THIS kernel."""
    import hashlib

    h = hashlib.sha256()
    for rel in FLOW_SOURCES:
        with open(os.path.join(REPO, rel), "rb") as f:
            h.update(rel.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def _pmc_traffic(C):
    """HBM bytes per flow-pass launch of THIS bench's shape (C rows: grid C/64*512) from
    the committed rocprofv3 PMC passes (profiles/traffic.json, tools/pmc_traffic.py:
    FETCH_SIZE x2 per the gfx950 calibration + WRITE_SIZE): the mean of the propose
    (<256,32,2>) and density (<256,32,0>) launches at that grid.  (None, None) if no
    profile of that shape was recorded."""
    path = os.path.join(REPO, "profiles", "traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, None
    grid = str((C + 63) // 64 * 512)
    vals = [v[grid][0] for k, v in t.get("kernels", {}).items()
            if k.startswith(("void fs::flow_pass_kernel<256, 32, 0>", "void fs::flow_pass_kernel<256, 32, 2>"))
            and isinstance(v, dict) and grid in v]
    if not vals:
        return None, None
    src = t.get("flow_src_sha16")
    return sum(vals) / len(vals), {"profile": "profiles/traffic.json", "head": t.get("head"), "grid": int(grid),
                                   "launch_kinds": len(vals), "flow_src_sha16": src,
                                   "matches_flow_sources": src == flow_source_sha16()}


def flow_algorithmic_bytes(model, C, N):
    """Algorithmic HBM bytes of one flow-pass launch (mean of the propose and density
    launches): the flow's parameters read once, plus the launch's own rows: propose
    writes config + centered (2 x C x 2N float32), density reads C x 2N float32 and
    writes C float32 log q."""
    w = sum(p.numel() * p.element_size() for p in model.parameters())
    D = 2 * N
    return w + (2 * C * D * 4 + (C * D * 4 + C * 4)) / 2


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(N, budget_s=15.0):
    """The reference CPU path restated (oracle/, test infrastructure), per chain, on the
    host cores: proposals generated in a batch (as main_algorithm_1.py:340-343 does),
    then per chain nf_big_move semantics (monte_carlo.py:235-303): the proposal's total
    energy by the reference's numpy pair loop (oracle.physics.total_energy_pairloop,
    bit-identical to energy_calculator.py:121-203), batch-1 float32 log_prob of old AND
    new in torch-CPU (the reference's op sequence), the PCG64 accept, and the energy
    recomputed on reject.  Threads: every CPU this process may run on, capped by
    OMP_NUM_THREADS when the host sets it (the GPU box allots a 16-CPU share of its
    256 visible CPUs that way); both numbers and the CPU model are reported."""
    from oracle import flow as OF
    from oracle import physics as OP

    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    threads = min(avail, int(cap)) if cap and cap.isdigit() and int(cap) > 0 else avail
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    dims = OF.FlowDims(N=N, B=half_box(N), **A1)
    sd = {k: v.detach().cpu() for k, v in synthetic_model(N, "cpu").state_dict().items()}
    init, L = synthetic_states(N, 4, 0)
    phys = OP.make_phys(N)
    hw = L / 2
    chains = [dict(state=init[c].copy(), pcg=OP.pcg64_seed(42 + c)[None].copy()) for c in range(4)]
    for ch in chains:
        ch["E"] = OP.total_energy_pairloop(ch["state"], phys)[0]
    t0 = time.perf_counter()
    g = torch.Generator().manual_seed(1234)
    z = (torch.rand((16, dims.D), generator=g) * 2 - 1) * dims.B
    props = (OF.sample_from(sd, z, dims).numpy() + np.float32(dims.B)).astype(np.float32)
    steps = 0
    k = 0
    while time.perf_counter() - t0 < budget_s or steps == 0:
        ch = chains[steps % len(chains)]
        cfg = props[k % len(props)].reshape(N, 2)
        k += 1
        E_new = OP.total_energy_pairloop(cfg, phys)[0]
        old = torch.tensor((ch["state"] - np.array([hw, hw])).reshape(1, -1), dtype=torch.float)
        new = torch.tensor((cfg - np.array([hw, hw])).reshape(1, -1), dtype=torch.float)
        nll_o = -OF.log_prob(sd, old, dims).item()
        nll_n = -OF.log_prob(sd, new, dims).item()
        acc, _ = OP.mh_accept([ch["E"]], [E_new], [nll_o], [nll_n], ch["pcg"])
        if acc[0]:
            ch["state"], ch["E"] = cfg, E_new
        else:
            ch["E"] = OP.total_energy_pairloop(ch["state"], phys)[0]
        steps += 1
    dt = time.perf_counter() - t0
    torch.set_num_threads(prev)
    return {"value": steps / dt, "unit": "steps/s", "cores": threads, "kind": "port",
            "nproc": os.cpu_count(), "cpus_available": avail, "omp_num_threads": cap, "cpu_model": _cpu_model(),
            "sample": f"{steps} nf_big_move steps (A1 flow, N={N}) over 4 chains incl. batched generation of "
                      f"16 proposals, {dt:.1f} s wall on {threads} host threads ({avail} CPUs available to the "
                      f"process, {os.cpu_count()} visible, OMP_NUM_THREADS={cap}); energy by the reference's numpy "
                      f"pair loop, log_prob by its torch-CPU float32 op sequence at batch 1"}


def acceptance_match(bmc, stepper, n_chains=2048, steps=10, f64_steps=4):
    """Checker of the metric's "acceptance-rate match" (oracle/, test infrastructure):
    `steps` more fused steps of all chains, untimed, then the oracle's restatement of
    the reference replays the first n_chains chains through the same steps on its own:
    the old state's energy and NLL recomputed from the state (monte_carlo.py:243-262),
    then per step the kernel's proposals (both sides see the same float32 configs),
    their energy and log q by the reference's float32 arithmetic, and each chain's own
    PCG64 stream (draw only when ratio < 1, :284-287).  Reported: both acceptance
    counts per step, the decisions that differ (a flip makes that chain's later inputs
    differ: `chains_diverged`), and log q against the reference-order float32 value
    (max, median, fraction beyond the north star's 1e-5) and both float32 evaluations
    (the GPU's and the reference-order one) against the exact value (the oracle in
    float64), on the last
    f64_steps steps' proposals (n_chains x f64_steps rows): max, p99.9, p99, median and the
    rows beyond 1e-5 for each."""
    from oracle import flow as OF
    from oracle import physics as OP

    N, S = bmc.N, min(n_chains, bmc.C)
    dims = OF.FlowDims(N=N, B=half_box(N), **A1)
    hw = bmc.phys.half_width
    phys = OP.make_phys(N)
    torch.cuda.synchronize()
    state0 = bmc.state[:S].cpu().numpy()
    f32 = bmc.state_is_f32[:S].cpu().numpy().astype(bool)
    pcg = bmc.pcg[:S].cpu().numpy().view(np.uint64).copy()
    rec = []
    for _ in range(steps):
        stepper.step(timed=False)
        torch.cuda.synchronize()
        rec.append((stepper.config[:S].cpu().numpy().reshape(S, N, 2), stepper.centered[:S].cpu().clone(),
                    stepper.log_q[:S].cpu().numpy().astype(np.float64), bmc.accept[:S].cpu().numpy().astype(bool)))
    t0 = time.perf_counter()
    sd = {k: v.detach().cpu() for k, v in bmc.model.state_dict().items()}
    # the chain's running energy / NLL as the reference holds them: E of the state in its
    # dtype (float32 after an accepted big move), -log q of fl32(state - half_width)
    E = np.where(f32, OP.total_energy_batch(state0.astype(np.float32), phys)[0],
                 OP.total_energy_batch(state0, phys)[0])
    nll = -OF.log_prob(sd, torch.from_numpy((state0 - hw).astype(np.float32).reshape(S, -1)), dims).numpy() \
        .astype(np.float64)
    diverged = np.zeros(S, bool)
    per_step, rels, tail = [], [], []
    for si, (cfg, cen, lq_gpu, acc) in enumerate(rec):
        E_new = OP.total_energy_batch(cfg, phys)[0]
        lq = OF.log_prob(sd, cen.clone(), dims).numpy().astype(np.float64)
        acc_o, _ = OP.mh_accept(E, E_new, nll, -lq, pcg)
        acc_o = acc_o.astype(bool)
        flips = acc != acc_o
        per_step.append({"gpu_accepts": int(acc.sum()), "oracle_accepts": int(acc_o.sum()),
                         "mismatched": int(flips.sum()), "mismatched_on_identical_inputs": int((flips & ~diverged).sum())})
        diverged |= flips
        E = np.where(acc_o, E_new, E)
        nll = np.where(acc_o, -lq, nll)
        fin = np.isfinite(lq)
        rels.append(np.abs(lq_gpu[fin] - lq[fin]) / np.abs(lq[fin]))
        if si >= len(rec) - f64_steps:
            tail.append((cen, lq_gpu, lq))
    rel = np.concatenate(rels)
    # both float32 evaluations against the exact value (the oracle in float64) on the last
    # f64_steps steps' proposals of every replayed chain (S x f64_steps rows)
    cen = torch.cat([t[0] for t in tail])
    lq_gpu = np.concatenate([t[1] for t in tail])
    lq = np.concatenate([t[2] for t in tail])
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    t64 = time.perf_counter()
    lq64 = OF.log_prob(sd64, cen.double(), dims).numpy()
    t64 = time.perf_counter() - t64

    def vs64(a, b):
        fin = np.isfinite(b) & np.isfinite(a)
        r = np.abs(a[fin] - b[fin]) / np.abs(b[fin])
        if not r.size:
            return {"rows": 0}
        return {"rows": int(r.size), "max_rel": float(r.max()), "p999_rel": float(np.percentile(r, 99.9)),
                "p99_rel": float(np.percentile(r, 99)), "median_rel": float(np.median(r)),
                "frac_beyond_1e-5": float((r > 1e-5).mean()), "beyond_1e-5": int((r > 1e-5).sum())}

    n = S * steps
    ga = sum(p["gpu_accepts"] for p in per_step)
    oa = sum(p["oracle_accepts"] for p in per_step)
    return {"chains": S, "steps": steps, "decisions": n,
            "gpu_acceptance_rate": ga / n, "oracle_acceptance_rate": oa / n,
            "gpu_accepts": ga, "oracle_accepts": oa,
            "mismatched_decisions": sum(p["mismatched"] for p in per_step),
            "mismatched_on_identical_inputs": sum(p["mismatched_on_identical_inputs"] for p in per_step),
            "chains_diverged": int(diverged.sum()), "per_step": per_step,
            "log_q_vs_oracle_f32": {"rows": int(rel.size), "max_rel": float(rel.max()) if rel.size else 0.0,
                                    "median_rel": float(np.median(rel)) if rel.size else 0.0,
                                    "frac_beyond_1e-5": float((rel > 1e-5).mean()) if rel.size else 0.0},
            "max_rel_log_q_gpu_vs_oracle_f32": float(rel.max()) if rel.size else 0.0,
            # which float32 evaluation is closer to the exact value, on all S rows
            "log_q_vs_f64": {"what": f"the last {len(tail)} steps' proposals of every replayed chain; relative to "
                                     "the oracle's float64 evaluation of the same weights and inputs",
                             "gpu_f32": vs64(lq_gpu, lq64), "reference_order_f32": vs64(lq, lq64),
                             "f64_s": t64},
            "oracle_s": time.perf_counter() - t0}


def _launch_ranks(n):
    """python -m torch.distributed.run --nproc-per-node n bench.py <same args>, on
    127.0.0.1 and a free port; returns its exit code (rank 0 prints the JSON line)."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)  # 10 warm-up, 100 timed steps
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--chains", type=int, default=65536, help="chains per GPU")
    ap.add_argument("--particles", type=int, default=64)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    ap.add_argument("--precision", default="f32", choices=["f32", "bf16x6", "bf16x3"],
                    help="conditioner GEMM arithmetic of the headline run (f32 = the reference's)")
    ap.add_argument("--no-alt-precision", action="store_true",
                    help="skip the secondary measurement of the split-bf16 modes")
    ap.add_argument("--no-given-proposal", action="store_true",
                    help="skip the secondary nf_big_move-equivalent measurement (supplied proposals)")
    ap.add_argument("--no-config2", action="store_true",
                    help="skip the secondary BASELINE config-2 line (N=16, 4096 chains)")
    ap.add_argument("--no-single-pass", action="store_true",
                    help="skip the secondary measurement of the opt-in single-pass log q mode")
    ap.add_argument("--no-config5", action="store_true",
                    help="skip the secondary BASELINE config-5 line (Algorithm 2 cycle, A2 flow, N=64)")
    ap.add_argument("--no-algorithm1-regime", action="store_true",
                    help="skip the secondary line of the reference's own Algorithm-1 regime (N=3, 10 runs)")
    ap.add_argument("--dump", default=None,
                    help="write each rank's final per-chain state to DUMP.rank<r>.npz (rehearsals: a sharded "
                         "run must hold the chains a 1-rank run over the same global chains holds)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `bench.py --gpus N` outside a launcher: start the N rank processes here, as fresh
        # children (nothing in this process has touched the GPU), and exit with their code
        sys.exit(_launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()  # counts devices without initialising them
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    if args.backend == "nccl" and world > ndev:
        print(f"bench.py: {world} ranks need {world} GPUs, {ndev} visible", file=sys.stderr)
        sys.exit(2)
    local = local % max(1, ndev)  # rehearsal with more ranks than GPUs (gloo) shares devices
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)

    N, C = args.particles, args.chains
    c0, seeds = parallel.shard(C, rank)
    model = synthetic_model(N, dev).set_precision(args.precision)
    init, L = synthetic_states(N, C, c0)
    phys = Physics(L, L, temperature=1.0, num_wells=2, V0_list=(-10.0, -10.5), r0=1.2, k=15)
    bmc = BatchedMonteCarlo(model, init, phys, seeds, device=dev, chain_offset=c0)
    decorrelate(bmc)
    stepper = Stepper(bmc)
    for _ in range(args.warmup):
        stepper.step(timed=False)
    if args.warmup:
        final_reduction(bmc)  # first use loads the reduction's kernels (lazy code-object loading)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    acc0 = int(bmc.n_accept.item())
    t0 = time.perf_counter()
    for _ in range(args.steps):
        stepper.step(timed=True)
    torch.cuda.synchronize()  # this rank's steps done: the rest is the end reduction
    t_steps = time.perf_counter() - t0
    hist, wells, table = final_reduction(bmc)
    torch.cuda.synchronize()
    t_red = time.perf_counter() - t0 - t_steps
    stepper.harvest()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    bmc.check_errors()
    if args.dump:
        np.savez(f"{args.dump}.rank{rank}.npz", chain_offset=c0, state=bmc.state.cpu().numpy(),
                 state_is_f32=bmc.state_is_f32.cpu().numpy(), E_old=bmc.E_old.cpu().numpy(),
                 nll_old=bmc.nll_old.cpu().numpy(), accepted=bmc.accepted.cpu().numpy(),
                 attempts=bmc.attempts.cpu().numpy(), pcg=bmc.pcg.cpu().numpy())
    n_acc =torch.tensor([int(bmc.n_accept.item()) - acc0], dtype=torch.int64, device=dev)
    t_max = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    # per-rank attribution of the timed region (gathered to rank 0): its own wall time,
    # its steps alone, the end reduction's RCCL calls (which also absorb the wait for the
    # slowest rank) and its kernels' HIP-event times
    mine = torch.tensor([elapsed, t_steps, t_red] + list(stepper.t / args.steps), dtype=torch.float64,
                        device=dev if args.backend == "nccl" else "cpu")
    per_rank = [mine]
    if dist:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        dist.all_reduce(n_acc)
        per_rank = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(per_rank, mine)
    elapsed = float(t_max.item())
    per_rank = [r.cpu().tolist() for r in per_rank]
    ranks = [{"rank": i, "elapsed_s": r[0], "steps_s": r[1], "final_reduction_ms": r[2] * 1e3,
              "kernel_ms": {"flow_propose": r[3], "flow_log_prob": r[4], "energy": r[5], "mh_accept": r[6]}}
             for i, r in enumerate(per_rank)]

    total_steps = C * world * args.steps
    value = total_steps / elapsed
    fpp = flops_per_pass(N, **A1)
    t_prop, t_lp, t_en, t_acc = (stepper.t / args.steps)  # ms per launch
    achieved = 2 * fpp * C / ((t_prop + t_lp) * 1e-3) / 1e12  # both flow passes (same kernel template)
    mfpp = mfma_flops_per_pass(N, **A1)
    mfma_ach = 2 * mfpp * C / ((t_prop + t_lp) * 1e-3) / 1e12
    peak = PEAK_F32_TFLOPS if args.precision == "f32" else PEAK_BF16_TFLOPS / SPLIT_PRODUCTS[args.precision]
    traffic, traffic_src = _pmc_traffic(C) if args.precision == "f32" else (None, None)
    alg_bytes = flow_algorithmic_bytes(model, C, N)
    out = {
        "metric": "NF-proposed MH steps/sec, N=64 2D LJ, 65536 chains; acceptance-rate match",
        "value": value,
        "unit": "steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if args.precision == "f32" else f"f32 operands, {args.precision} split on bf16 MFMA",
        "data": "synthetic (FCC lattice + jitter + 10N local moves per chain, random-init A1 flow with perturbed final layers)",
        "config": {"workload": f"Algorithm-1 NF-proposed MH step, N={N}, {C} chains per GPU",
                   "particles": N, "chains_per_gpu": C, "flow": "A1: L=15 H=256 blocks=32 K=32",
                   "parallelism": f"dp{world} (chains sharded; RCCL all-reduce of the final histogram, all-gather of per-chain counters)"},
        "acceptance_rate": n_acc.item() / total_steps,
        "final_stats": {"hist_total": int(hist.sum().item()), "all_in_A": int(wells[0].item()),
                        "all_in_B": int(wells[1].item()), "chains": int(wells[2].item()),
                        "gathered_chain_rows": int(table.shape[0]),
                        "deltaF_mean_sem": parallel.free_energy_stats(table)[:2]},
        "kernel_ms": {"flow_propose": t_prop, "flow_log_prob": t_lp, "energy": t_en, "mh_accept": t_acc},
        # where a multi-GPU run loses time: each rank's timed region, its steps alone, the
        # end reduction (RCCL all-reduce + all-gather), and the spread over ranks
        "ranks": ranks,
        "timed_region_skew_ms": (max(r["elapsed_s"] for r in ranks) - min(r["elapsed_s"] for r in ranks)) * 1e3,
        "steps_skew_ms": (max(r["steps_s"] for r in ranks) - min(r["steps_s"] for r in ranks)) * 1e3,
        "final_reduction_ms_max": max(r["final_reduction_ms"] for r in ranks),
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                     "frac": achieved / peak, "traffic": traffic,
                     "traffic_source": traffic_src, "algorithmic_bytes_per_launch": alg_bytes,
                     "traffic_over_algorithmic": traffic / alg_bytes if traffic else None,
                     "kernel": "flow_pass_kernel<256,32,*> (propose + log_prob)",
                     "algorithmic_flop_per_launch": fpp * C,
                     # what the matrix cores actually execute (the derivative logits are
                     # two per-lane dot products instead of a 33-column GEMM)
                     "executed_mfma": {"flop_per_launch": mfpp * C, "achieved": mfma_ach,
                                       "frac": mfma_ach / peak} if args.precision == "f32" else None},
        # the LJ + double-well kernel the north star asks about: HBM rate of its algorithmic
        # bytes (float32 proposal in, E / W out) and fp64 rate (~30 FLOP per
        # pair + ~40 per particle), against the fp64 vector peak that bounds it
        "energy_kernel": {"ms": t_en, "bytes_per_chain": ENERGY_BYTES(N), "flop_per_chain": ENERGY_FLOP(N),
                          "achieved_gbs": ENERGY_BYTES(N) * C / (t_en * 1e-3) / 1e9,
                          "achieved_fp64_tflops": ENERGY_FLOP(N) * C / (t_en * 1e-3) / 1e12,
                          "peak_fp64_tflops": PEAK_F64_TFLOPS,
                          "frac": ENERGY_FLOP(N) * C / (t_en * 1e-3) / 1e12 / PEAK_F64_TFLOPS},
    }
    def leg(name, fn, *a):
        # a secondary measurement that fails is reported in the line (never silently
        # dropped) without costing the headline; its kernels' own errors still raise there
        try:
            out[name] = fn(*a)
        except Exception as e:  # noqa: BLE001
            out[name] = {"error": f"{type(e).__name__}: {e}"}
            print(f"bench.py: {name} failed: {e!r}", file=sys.stderr, flush=True)

    out["parity_checked"] = None  # the acceptance-rate match runs on rank 0 at N=1 only
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        leg("acceptance_match", acceptance_match, bmc, stepper)
        am = out["acceptance_match"]
        # the metric's qualifier: true only when the replay ran and matched every decision
        # made on identical inputs (an errored check is false, never a clean run)
        out["parity_checked"] = "error" not in am and am["mismatched_on_identical_inputs"] == 0
    if world == 1 and not args.no_alt_precision and args.precision == "f32":
        leg("alt_precision", alt_precisions, bmc, stepper)
    if world == 1 and not args.no_single_pass and args.precision == "f32":
        leg("single_pass", single_pass, bmc, stepper)
    if world == 1 and not args.no_given_proposal:
        leg("given_proposal", given_proposal, bmc, stepper)
    if world == 1 and not args.no_config2:
        leg("config2", config2)
    if world == 1 and not args.no_config5:
        leg("config5", config5)
    if world == 1 and not args.no_algorithm1_regime:
        leg("algorithm1_regime", algorithm1_regime)
        if not args.no_cpu_baseline and "error" not in out["algorithm1_regime"]:
            reg = out["algorithm1_regime"]
            try:
                reg["cpu_baseline"] = algorithm1_regime_cpu()
                reg["vs_cpu_baseline"] = reg["value"] / reg["cpu_baseline"]["value"]
            except Exception as e:  # noqa: BLE001
                reg["cpu_baseline"] = {"error": f"{type(e).__name__}: {e}"}
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        leg("cpu_baseline", cpu_baseline, N, args.cpu_budget)
        # vs_baseline stays null: BASELINE.md has no published number for this metric
        if "value" in out["cpu_baseline"]:
            out["vs_cpu_baseline"] = value / out["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
