"""BatchedMonteCarlo — C independent chains, one NF-proposed MH step per call.

The reference runs chains in a Python loop, one ``MonteCarlo.nf_big_move``
per chain (main_algorithm_1.py:381-395, monte_carlo.py:235-303).  Here all C
chains live on the device:

  state        (C, N, 2) float64  box coordinates (holds the reference's float64
                                   initial state and the float32 values it
                                   switches to after an accepted big move)
  state_is_f32 (C,) u8            the reference dtype of each chain's state
  E_old, W_old (C,) float64       cached total energy / virial (energy_calculator.py:46)
  nll_old      (C,) float64       cached -log q(state) (float32 value, exact on replay)
  pcg          (C, 4) u64         numpy PCG64 state, seeded like default_rng(seed_c)
  pcg_buf      (C, 2) u64         its buffered 32-bit half (has_uint32, uinteger)
  attempts, accepted (C,) int64   monte_carlo.py:80-81 counters (shared by local
                                   and big moves, as in the reference)
  max_disp     (C,) float64       max_displacement
  prev_counts  (C, 2) int64       previous_{attempts,accepted}_displacement

``local_moves(n)`` = fs_local_moves: n particle_displacement calls per chain
(with adjust_displacement / sample() on the driver's step schedule).
``step()`` = fs_nf_mh_step: proposal sampling pass (base draws in-kernel) ->
density pass on the proposals -> energies -> accept/update.  ``nf_big_move``
takes externally supplied proposals (the reference's pre-generated configs).
After local moves the next big move re-derives the old NLL from the current
state and recomputes the energy on reject, as nf_big_move does on every call
(monte_carlo.py:243-261, 299-301); without local moves in between the cached
values are exactly those numbers.  The flow model is optional until the first
big move (the reference equilibrates before set_nf_model).
"""
import functools
import warnings
import weakref

import numpy as np
import torch

from .. import _lib
from .energy_calculator import make_phys, total_energy


def _on_own_device(fn):
    """Run a method with the engine's device current: the library launches on the
    current device's stream (flowstate._lib.require_device)."""

    @functools.wraps(fn)
    def wrapped(self, *args, **kwargs):
        with _lib.on_device(self.device):
            return fn(self, *args, **kwargs)

    return wrapped


class Physics:
    """Physics constants of the driver (main_algorithm_1.py:40-53)."""

    def __init__(self, box_x, box_y=None, temperature=1.0, num_wells=2, V0_list=(-10.0, -10.5), r0=1.2, k=15):
        self.box_x = float(box_x)
        self.box_y = float(box_x if box_y is None else box_y)
        self.beta = 1.0 / temperature
        self.num_wells, self.V0_list, self.r0, self.k = num_wells, tuple(V0_list), r0, k
        self.c = make_phys(self.box_x, self.box_y, num_wells, V0_list, r0, k, self.beta)

    @property
    def half_width(self):
        return self.box_x / 2  # MonteCarlo.half_width (monte_carlo.py:66)


def _splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return x ^ (x >> 31)


def default_proposal_seed(seeds, chain_offset=0):
    """Seed of the in-kernel proposal stream when none is given.

    The stream is keyed (proposal_seed, step, global chain = chain_offset + c), so two
    engines share proposals exactly when they share this seed and chain indices.  The
    default derives it from the chains' own PCG64 seeds: the base seed
    seeds[0] - chain_offset (the driver's MASTER_SEED under seed = i + MASTER_SEED,
    main_algorithm_1.py:139) mixed by splitmix64.  Ranks of one job (same base seed,
    disjoint chain_offset) therefore draw one consistent global stream, independent of
    the number of ranks, while jobs with different master seeds draw independent ones.
    Engines that reuse the same seeds for the same global chains draw the same
    proposals, as the same chains should."""
    base = (int(np.asarray(seeds, dtype=np.uint64).reshape(-1)[0]) - int(chain_offset)) & 0xFFFFFFFFFFFFFFFF
    return _splitmix64(base ^ 0x70726F706F736531) & 0x7FFFFFFFFFFFFFFF


class BatchedMonteCarlo:
    def __init__(self, model, particles, physics, seeds, device=None, proposal_seed=None,
                 correct_sign=False, state_is_f32=None, chain_offset=0, initial_max_displacement=0.5,
                 target_acceptance=0.5, single_pass_log_q=False):
        """single_pass_log_q: opt-in, not the reference's semantics (FS_MH_SINGLE_PASS):
        step() takes the proposals' log q from the sampling pass's own log-dets instead of
        the reference's second (density) pass over fl32(config - half_width), one flow
        pass per step instead of two, always one fused step per launch."""
        self.model = None
        self.single_pass_log_q = bool(single_pass_log_q)
        self.phys = physics
        if device is None:
            device = next(model.parameters()).device if model is not None else "cuda"
        dev = torch.device(device)
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else dev
        self.device = dev
        with _lib.on_device(dev):
            _lib.require_device(torch.empty(0, device=dev))
            self._init_state(model, particles, seeds, proposal_seed, correct_sign, state_is_f32, chain_offset,
                             initial_max_displacement, target_acceptance)

    def _init_state(self, model, particles, seeds, proposal_seed, correct_sign, state_is_f32, chain_offset,
                    initial_max_displacement, target_acceptance):
        dev = self.device
        p = torch.as_tensor(np.asarray(particles) if not torch.is_tensor(particles) else particles)
        if p.dim() == 2:
            p = p[None]
        self.C, self.N = int(p.shape[0]), int(p.shape[1])
        if state_is_f32 is None:
            state_is_f32 = p.dtype == torch.float32
        self.state = p.to(device=dev, dtype=torch.float64).contiguous()
        self.state_is_f32 = torch.full((self.C,), int(bool(state_is_f32)), dtype=torch.uint8, device=dev)
        self.correct_sign = bool(correct_sign)
        self.flags = _lib.FS_MH_CORRECT_SIGN if correct_sign else 0
        self.chain_offset = int(chain_offset)
        self.step_count = 0
        seeds_np = np.asarray(seeds, dtype=np.uint64).reshape(-1)
        if seeds_np.size != self.C:
            raise ValueError("one seed per chain")
        if proposal_seed is None and self.chain_offset > 0 and self.C > 1 and not np.array_equal(
                seeds_np, seeds_np[0] + np.arange(self.C, dtype=np.uint64)):
            # the default stream assumes seed = MASTER_SEED + global chain index on every rank
            # (main_algorithm_1.py:139); with other seeds each rank would derive its own stream
            warnings.warn("BatchedMonteCarlo: chain_offset > 0 with seeds that are not seeds[0] + arange(C): the "
                          "default proposal stream is then not one global stream across ranks; pass proposal_seed",
                          stacklevel=3)
        self.proposal_seed = default_proposal_seed(seeds_np, self.chain_offset) if proposal_seed is None \
            else int(proposal_seed)
        seeds = torch.as_tensor(seeds_np.view(np.int64), device=dev)
        self.pcg = torch.empty((self.C, 4), dtype=torch.int64, device=dev)
        L = _lib.load()
        _lib.check(L.fs_pcg64_seed(_lib.ptr(seeds), self.C, _lib.ptr(self.pcg), _lib.stream_ptr()), "fs_pcg64_seed")
        self.attempts = torch.zeros(self.C, dtype=torch.int64, device=dev)
        self.accepted = torch.zeros(self.C, dtype=torch.int64, device=dev)
        self.n_accept = torch.zeros(1, dtype=torch.int64, device=dev)
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        self.accept = torch.zeros(self.C, dtype=torch.uint8, device=dev)
        self.pcg_buf = torch.zeros((self.C, 2), dtype=torch.int64, device=dev)
        self.max_disp = torch.full((self.C,), float(initial_max_displacement), dtype=torch.float64, device=dev)
        self.prev_counts = torch.zeros((self.C, 2), dtype=torch.int64, device=dev)
        self.target_acceptance = float(target_acceptance)
        self.E_old, self.W_old = self._energy_of_state()
        self.nll_old = torch.zeros(self.C, dtype=torch.float64, device=dev)
        self._moved = False  # local moves since E_old / nll_old were exact
        self._ws = None
        if model is not None:
            self.set_model(model)

    @_on_own_device
    def set_model(self, model):
        """MonteCarlo.set_nf_model (monte_carlo.py:229-233)."""
        if 2 * self.N != model.flows[0].num_input_channels:
            raise ValueError("particles do not match the flow dimension")
        self.model = model
        self._ws = None
        self.nll_old = -(model.log_prob(self._centered_f32(self.state)).to(torch.float64))

    # ------------------------------------------------------------------
    def _centered_f32(self, pos, is_f32_mask=None):
        """fl32(pos - half_width) as nf_big_move feeds the flow (monte_carlo.py:251-258)."""
        return (pos - self.phys.half_width).to(torch.float32).reshape(pos.shape[0], -1).contiguous()

    @_on_own_device
    def _energy_of_state(self):
        """Total energy / virial in the reference dtype of each chain's state
        (EnergyCalculator.__init__, energy_calculator.py:46)."""
        E = torch.empty(self.C, dtype=torch.float64, device=self.device)
        W = torch.empty_like(E)
        # one launch over the float64 states with the per-chain dtype flags (no host round
        # trip to split the chains, which cost each Algorithm-1 attempt a synchronisation)
        _lib.check(_lib.load().fs_energy_state(self.phys.c, _lib.ptr(self.state), _lib.ptr(self.state_is_f32),
                                               self.C, self.N, _lib.ptr(E), _lib.ptr(W), _lib.stream_ptr()),
                   "fs_energy_state")
        return E, W

    def _need_model(self):
        if self.model is None:
            raise RuntimeError("no flow model: set_model() / set_nf_model() first")

    def _workspace(self):
        if self._ws is None:
            n = _lib.load().fs_nf_mh_step_ws_bytes(self.model.dims(), self.C)
            _lib.check(0 if n >= 0 else -1, "fs_nf_mh_step_ws_bytes")
            self._ws = torch.empty((n + 255) // 256 * 64, dtype=torch.float32, device=self.device)
        return self._ws

    # ------------------------------------------------------------------
    @_on_own_device
    def step(self, n=1):
        """n fused NF-MH steps for all chains (stream-ordered, no host sync)."""
        self._need_model()
        L = _lib.load()
        packed = self.model.packed()
        dims = self.model.dims()
        st = _lib.stream_ptr()
        done = 0
        while done < n:
            fill = 1 if self.single_pass_log_q else self.steps_per_launch()
            same_flow = self._last_packed is not None and self._last_packed() is packed
            if fill > 1 and (self._bank_covers(packed) or (same_flow and (self._moved or n - done == 1))):
                # a small batch stepped one step at a time with the flow unchanged since
                # the last step (Algorithm 1's cycle: local moves between big moves, or a
                # loop of step(1) calls): this step's proposal, log q and energy come from
                # a bank of `fill` steps made in one launch per pass; after local moves
                # only the current states' density pass and energy run per step.  A step
                # after new weights (Algorithm 2's refeed) stays one fused step: its bank
                # would not be reused.
                bank, s = self._bank_for(packed, dims, fill)
                _lib.check(L.fs_nf_mh_step_banked(dims, _lib.ptr(packed), self.phys.c, self.C, self._bank["S"], s,
                                                  _lib.ptr(bank), _lib.ptr(self.E_old), _lib.ptr(self.W_old),
                                                  _lib.ptr(self.nll_old), _lib.ptr(self.pcg), _lib.ptr(self.state),
                                                  _lib.ptr(self.state_is_f32), _lib.ptr(self.accept),
                                                  _lib.ptr(self.attempts), _lib.ptr(self.accepted),
                                                  _lib.ptr(self.n_accept), _lib.ptr(self.err),
                                                  self.flags | (_lib.FS_MH_HYBRID if self._moved else 0),
                                                  _lib.ptr(self._workspace_banked()), st), "fs_nf_mh_step_banked")
                self._last_src = (bank, self._bank["S"] * self.C, s)
                self.step_count += 1
                done += 1
                self._moved = False
                continue
            S = 1 if self._moved else min(n - done, fill)
            if S == 1:
                _lib.check(L.fs_nf_mh_step(dims, _lib.ptr(packed), self.phys.c, self.C, self.proposal_seed,
                                           self.step_count, self.chain_offset, _lib.ptr(self.E_old),
                                           _lib.ptr(self.W_old), _lib.ptr(self.nll_old), _lib.ptr(self.pcg),
                                           _lib.ptr(self.state), _lib.ptr(self.state_is_f32), _lib.ptr(self.accept),
                                           _lib.ptr(self.attempts), _lib.ptr(self.accepted), _lib.ptr(self.n_accept),
                                           _lib.ptr(self.err), self.flags | (_lib.FS_MH_HYBRID if self._moved else 0)
                                           | (_lib.FS_MH_SINGLE_PASS if self.single_pass_log_q else 0),
                                           _lib.ptr(self._workspace()), st), "fs_nf_mh_step")
                self._last_src = (self._ws, self.C, 0)
            else:
                _lib.check(L.fs_nf_mh_steps(dims, _lib.ptr(packed), self.phys.c, self.C, S, self.proposal_seed,
                                            self.step_count, self.chain_offset, _lib.ptr(self.E_old),
                                            _lib.ptr(self.W_old), _lib.ptr(self.nll_old), _lib.ptr(self.pcg),
                                            _lib.ptr(self.state), _lib.ptr(self.state_is_f32), _lib.ptr(self.accept),
                                            _lib.ptr(self.attempts), _lib.ptr(self.accepted),
                                            _lib.ptr(self.n_accept), _lib.ptr(self.err), self.flags,
                                            _lib.ptr(self._workspace_steps(S)), st), "fs_nf_mh_steps")
                self._last_src = (self._ws_steps, S * self.C, S - 1)
            self.step_count += S
            done += S
            self._moved = False
        self._last_packed = weakref.ref(packed)  # not kept alive past a repack
        return self.accept

    # proposal rows per launch that fill the chip: 2 resident 64-chain workgroups on each
    # of the 256 CUs (a batch that already fills it keeps one step per launch)
    FILL_ROWS = 2 * 256 * 64
    MAX_STEPS_PER_LAUNCH = 16

    def steps_per_launch(self):
        """Consecutive steps whose proposal passes share one launch (fs_nf_mh_steps)."""
        return max(1, min(self.MAX_STEPS_PER_LAUNCH, self.FILL_ROWS // max(1, self.C)))

    def _workspace_steps(self, S):
        """Workspace of fs_nf_mh_steps for S steps (grown on demand, kept)."""
        n = _lib.load().fs_nf_mh_steps_ws_bytes(self.model.dims(), self.C, S)
        _lib.check(0 if n >= 0 else -1, "fs_nf_mh_steps_ws_bytes")
        ws = getattr(self, "_ws_steps", None)
        if ws is None or ws.numel() * 8 < n:
            self._ws_steps = torch.empty((n + 7) // 8, dtype=torch.float64, device=self.device)
        return self._ws_steps

    _bank = None
    _last_packed = None
    _last_src = None

    def last_proposals(self, centered=False):
        """The float32 proposals (C, N, 2) box coordinates of the last step() (or, with
        centered, the flow's input fl32(config - half_width), (C, 2N)), read from the
        buffer that step used: the fused step's workspace, the multi-step launch's or the
        proposal bank's rows of that step.  Valid until the next step()."""
        if self._last_src is None:
            raise RuntimeError("no step() has run")
        buf, R, s = self._last_src
        D = 2 * self.N
        off = ((R * D * 4 + 255) // 256 * 256 if centered else 0) + s * self.C * D * 4
        rows = buf.view(torch.uint8)[off:off + self.C * D * 4].view(torch.float32)
        return rows.reshape(self.C, D) if centered else rows.reshape(self.C, self.N, 2)

    def _bank_key(self, packed):
        # what a bank's rows depend on: the flow image (a new tensor on every repack),
        # the proposal stream and the chains' global indices
        return (id(packed), self.proposal_seed, self.chain_offset, self.C)

    def _bank_covers(self, packed):
        b = self._bank
        return (b is not None and b["packed"]() is packed and b["key"] == self._bank_key(packed)
                and b["step0"] <= self.step_count < b["step0"] + b["S"])

    def _bank_for(self, packed, dims, S):
        """(bank buffer, row block) of step step_count: the open bank when it covers the
        step, else a new bank of steps step_count .. step_count+S-1 (fs_nf_mh_bank)."""
        if not self._bank_covers(packed):
            n = _lib.load().fs_nf_mh_steps_ws_bytes(dims, self.C, S)
            _lib.check(0 if n >= 0 else -1, "fs_nf_mh_steps_ws_bytes")
            buf = self._bank["buf"] if self._bank is not None else None
            if buf is None or buf.numel() * 8 < n:
                buf = torch.empty((n + 7) // 8, dtype=torch.float64, device=self.device)
            self._bank = None  # a failed fill leaves no bank behind
            _lib.check(_lib.load().fs_nf_mh_bank(dims, _lib.ptr(packed), self.phys.c, self.C, S, self.proposal_seed,
                                                 self.step_count, self.chain_offset, _lib.ptr(self.err),
                                                 _lib.ptr(buf), _lib.stream_ptr()), "fs_nf_mh_bank")
            self._bank = {"packed": weakref.ref(packed), "key": self._bank_key(packed), "step0": self.step_count, "S": S,
                          "buf": buf}
        return self._bank["buf"], self.step_count - self._bank["step0"]

    def _workspace_banked(self):
        ws = getattr(self, "_ws_banked", None)
        if ws is None:
            n = _lib.load().fs_nf_mh_banked_ws_bytes(self.model.dims(), self.C)
            _lib.check(0 if n >= 0 else -1, "fs_nf_mh_banked_ws_bytes")
            ws = self._ws_banked = torch.empty((n + 7) // 8, dtype=torch.float64, device=self.device)
        return ws

    @_on_own_device
    def local_moves(self, n, adjust_every=0, sample_every=0, step0=0, log_accepts=False):
        """n MonteCarlo.particle_displacement calls per chain (monte_carlo.py:146-223),
        numbered step0+1 .. step0+n like the driver's loop counter
        (main_algorithm_1.py:204-210): adjust_displacement after each step divisible
        by adjust_every, a sample() snapshot after each step divisible by
        sample_every.  Returns (samples_xy (C,S,N,2) f64, samples_ew (C,S,2) f64,
        accept_log (C,n) u8) — the unused ones None."""
        L = _lib.load()
        n, step0 = int(n), int(step0)
        S = L.fs_local_samples_per_chain(step0, n, int(sample_every))
        sxy = sew = log = None
        if S > 0:
            sxy = torch.empty((self.C, S, self.N, 2), dtype=torch.float64, device=self.device)
            sew = torch.empty((self.C, S, 2), dtype=torch.float64, device=self.device)
        if log_accepts:
            log = torch.empty((self.C, n), dtype=torch.uint8, device=self.device)
        _lib.check(L.fs_local_moves(self.phys.c, self.C, self.N, _lib.ptr(self.state), _lib.ptr(self.state_is_f32),
                                    _lib.ptr(self.E_old), _lib.ptr(self.W_old), _lib.ptr(self.pcg),
                                    _lib.ptr(self.pcg_buf), _lib.ptr(self.max_disp), _lib.ptr(self.attempts),
                                    _lib.ptr(self.accepted), _lib.ptr(self.prev_counts), n, step0, int(adjust_every),
                                    self.target_acceptance, int(sample_every), _lib.ptr(sxy), _lib.ptr(sew),
                                    _lib.ptr(log), None, _lib.stream_ptr()), "fs_local_moves")
        if n > 0:
            self._moved = True
        return sxy, sew, log

    def invalidate_nll(self):
        """The cached old NLL is stale (the flow's weights changed): the next big move
        re-derives it from the current state, as nf_big_move does on every call
        (monte_carlo.py:251-261), and recomputes the energy a reject writes back (:299-301)."""
        self._moved = True

    @_on_own_device
    def adjust_displacement(self):
        """MonteCarlo.adjust_displacement (monte_carlo.py:375-403) for every chain."""
        _lib.check(_lib.load().fs_adjust_displacement(self.C, _lib.ptr(self.max_disp), _lib.ptr(self.attempts),
                                                      _lib.ptr(self.accepted), _lib.ptr(self.prev_counts),
                                                      self.target_acceptance, _lib.stream_ptr()),
                   "fs_adjust_displacement")

    def check_errors(self):
        """Raise the reference's ValueError if any flow pass since construction met a NaN
        discriminant (splines.py:176-183).  Passes that make several steps' proposals at once
        (step(n), the proposal bank) report a NaN in any of those proposals when they are
        made, as the reference raises when it pre-generates its proposals in batches
        (main_algorithm_1.py:340-343, utils.py:422-450), even if a later weight change
        retires the bank before those steps run."""
        v = int(self.err.item())
        if v & 4:  # (not the reference's: a wide-path column hand-off gave up waiting)
            raise _lib.FlowStateError("a wide-path trunk hand-off timed out")
        if v & 1:
            raise ValueError("Discriminant computation resulted in NaN.")  # splines.py:176-183

    # ------------------------------------------------------------------ judging
    @_on_own_device
    def metropolis_judge(self, E_ref, E_new):
        """metropolis_acceptance_particle_move (monte_carlo.py:191-223) for M energies per
        chain against one reference energy each, judged in order on the chain's own PCG64
        stream: E_new <= E_ref accepts and an infinite E_new rejects without a draw, else
        Generator.random() < exp(-beta (E_new - E_ref)).  E_ref (C,), E_new (C, M) float64.
        Returns accept (C, M) uint8; nothing else changes but the PCG64 states."""
        E_ref = torch.as_tensor(E_ref, dtype=torch.float64, device=self.device).reshape(-1).contiguous()
        E_new = torch.as_tensor(E_new, dtype=torch.float64, device=self.device).contiguous()
        if E_ref.numel() != self.C or E_new.dim() != 2 or E_new.shape[0] != self.C:
            raise ValueError(f"E_ref must be ({self.C},) and E_new ({self.C}, M)")
        M = int(E_new.shape[1])
        acc = torch.empty((self.C, M), dtype=torch.uint8, device=self.device)
        _lib.check(_lib.load().fs_metropolis_judge(float(self.phys.c.beta), self.C, M, _lib.ptr(E_ref),
                                                   _lib.ptr(E_new), _lib.ptr(self.pcg), _lib.ptr(acc), None,
                                                   _lib.stream_ptr()), "fs_metropolis_judge")
        return acc

    def _proposal_energies(self, configs, M):
        """Total energy / virial of C x M supplied configurations, each in its own dtype
        (float32 or float64, as calculate_total_energy_virial computes it): (C, M) each."""
        cfg = torch.as_tensor(configs, device=self.device)
        if cfg.dtype not in (torch.float32, torch.float64):
            raise ValueError(f"proposals must be float32 or float64, got {cfg.dtype}")
        if cfg.numel() != self.C * M * self.N * 2:
            raise ValueError(f"expected {self.C} x {M} configurations of ({self.N}, 2)")
        E, W, _ = total_energy(cfg.reshape(self.C * M, self.N, 2).contiguous(), self.phys.c)
        return E.reshape(self.C, M), W.reshape(self.C, M)

    @_on_own_device
    def judge_normalizing_flow(self, configs):
        """MonteCarlo.judge_normalizing_flow (monte_carlo.py:305-329), batched: the
        energy-only Metropolis verdict on one supplied proposal per chain (C, N, 2) against
        the chain's current total energy (:313), without accepting it.  As the reference:
        attempts_displacement += 1 (:309), the energy bookkeeping is restored (:327-328),
        the state is untouched, and the PCG64 stream advances when a draw is taken.
        Returns accept (C,) uint8."""
        E_new, _ = self._proposal_energies(configs, 1)
        acc = self.metropolis_judge(self.E_old, E_new)[:, 0]
        self.attempts += 1
        return acc

    @_on_own_device
    def bulk_judge_normalizing_flow(self, configs, ref_energy):
        """MonteCarlo.bulk_judge_normalizing_flow (monte_carlo.py:331-370), batched: M
        supplied proposals per chain, configs (C, M, N, 2), each judged in order against
        ref_energy (scalar or (C,)) on the chain's PCG64 stream.  Returns (accepted (C,)
        int64, M).  Kept from the reference: every calculate_total_energy_virial call there
        overwrites the calculator's running totals (energy_calculator.py:121-203) and this
        method does not restore them, so afterwards a chain's running energy / virial are
        those of its last proposal (the next big move's ratio uses that value, :243, and a
        reject re-derives the energy of the state, :299-301, as after local moves)."""
        cfg = torch.as_tensor(configs, device=self.device)
        M = int(cfg.numel() // (self.C * self.N * 2)) if cfg.numel() else 0
        ref = torch.as_tensor(ref_energy, dtype=torch.float64, device=self.device).reshape(-1)
        ref = ref.expand(self.C).contiguous() if ref.numel() == 1 else ref
        if M == 0:
            return torch.zeros(self.C, dtype=torch.int64, device=self.device), 0
        E_new, W_new = self._proposal_energies(cfg, M)
        acc = self.metropolis_judge(ref, E_new)
        self.E_old, self.W_old = E_new[:, -1].contiguous(), W_new[:, -1].contiguous()
        self._moved = True
        return acc.sum(dim=1, dtype=torch.int64), M

    @_on_own_device
    def proposal_terms(self, configs):
        """(E_new, W_new, log_q) of R supplied proposals (R, N, 2) box coords, each exactly
        as nf_big_move derives it (monte_carlo.py:247, 251-262): energy and virial in the
        config's dtype, log q of fl32(config - half_width).  They do not depend on the chain
        states, so the proposals of many attempts (the drivers pre-generate them,
        main_algorithm_1.py:340-343) share one launch per pass; pass each attempt's rows to
        nf_big_move(configs, terms=...).  The kernels are row-independent: the values are
        bit-identical to nf_big_move's own."""
        cfg = torch.as_tensor(configs, device=self.device)
        if cfg.dtype not in (torch.float32, torch.float64):
            raise ValueError(f"proposals must be float32 or float64, got {cfg.dtype}")
        cfg = cfg.reshape(-1, self.N, 2).contiguous()
        self._need_model()
        E, W, _ = total_energy(cfg, self.phys.c)
        lq = self.model._log_prob(self._centered_f32(cfg.to(torch.float64)), self.err)
        return E, W, lq

    def state_nll(self, state=None, log_prob=None):
        """-log q of the states (C, N, 2) f64 as nf_big_move re-derives the old NLL after
        local moves (monte_carlo.py:251-261): the density pass over fl32(state - half_width),
        widened to float64.  Runs on the current stream; a pass that meets a NaN or a
        hand-off timeout reports it in the engine's sticky err word.  log_prob: optional
        model.frozen_log_prob() function (the same pass without its per-call checks)."""
        self._need_model()
        x = self._centered_f32(self.state if state is None else state)
        lq = self.model._log_prob(x, self.err) if log_prob is None else log_prob(x, self.err)
        return -(lq.to(torch.float64))

    @_on_own_device
    def nf_big_move(self, configs, terms=None, nll=None):
        """Batched nf_big_move with supplied proposals (C, N, 2) box coords.

        The proposals keep their dtype, as in the reference (monte_carlo.py:245-296):
        float32 (the drivers' proposals, main_algorithm_1.py:340-343) or float64.  The
        energy is computed in that dtype, the flow sees fl32(config - half_width)
        either way (:251-258), and an accepted chain's state takes the config's dtype.
        terms: optional (E_new, W_new, log_q), each (C,), of these configs from
        proposal_terms().  nll: optional (C,) f64 state_nll() of the current states,
        computed ahead (the Algorithm-1 pipeline); used only after local moves, where the
        move would re-derive it, and it becomes the engine's nll_old (updated in place)."""
        cfg = torch.as_tensor(configs, device=self.device)
        if cfg.dtype not in (torch.float32, torch.float64):
            raise ValueError(f"proposals must be float32 or float64, got {cfg.dtype}")
        cfg = cfg.reshape(self.C, self.N, 2).contiguous()
        cfg64 = None
        if cfg.dtype == torch.float64:
            cfg64, cfg = cfg, cfg.to(torch.float32)
        self._need_model()
        stale = self._moved
        if stale:  # old NLL of the current state (monte_carlo.py:251-261); energy for a reject (:299-301)
            if nll is not None and (not torch.is_tensor(nll) or nll.dtype != torch.float64 or nll.shape != (self.C,)
                                    or nll.device != self.device):
                raise ValueError(f"nll must be a ({self.C},) float64 tensor on {self.device}")
            self.nll_old = self.state_nll() if nll is None else nll
            E_cur, W_cur = self._energy_of_state()
        if terms is None:
            E_new, W_new, _ = total_energy(cfg if cfg64 is None else cfg64, self.phys.c)
            lq = self.model._log_prob(self._centered_f32(cfg.to(torch.float64) if cfg64 is None else cfg64), self.err)
        else:
            E_new, W_new, lq = terms
            for t, dt in ((E_new, torch.float64), (W_new, torch.float64), (lq, torch.float32)):
                if not torch.is_tensor(t) or t.dtype != dt or t.shape != (self.C,) or t.device != self.device:
                    raise ValueError(f"terms must be proposal_terms() rows for {self.C} chains on {self.device}")
            E_new, W_new, lq = E_new.contiguous(), W_new.contiguous(), lq.contiguous()
        L = _lib.load()
        _lib.check(L.fs_mh_accept(self.phys.c, self.C, self.N, _lib.ptr(self.E_old), _lib.ptr(self.W_old),
                                  _lib.ptr(self.nll_old), _lib.ptr(E_new), _lib.ptr(W_new), _lib.ptr(lq),
                                  _lib.ptr(self.pcg), _lib.ptr(self.state), _lib.ptr(self.state_is_f32),
                                  _lib.ptr(cfg), _lib.ptr(self.accept), _lib.ptr(self.attempts),
                                  _lib.ptr(self.accepted), _lib.ptr(self.n_accept), self.flags,
                                  _lib.stream_ptr()), "fs_mh_accept")
        if cfg64 is not None:  # the kernel stored the float32 copy: accepted chains take the float64 config
            acc = (self.accept != 0)
            self.state.copy_(torch.where(acc[:, None, None], cfg64, self.state))
            self.state_is_f32.copy_(torch.where(acc, torch.zeros_like(self.state_is_f32), self.state_is_f32))
        if stale:
            rej = self.accept == 0
            self.E_old = torch.where(rej, E_cur, self.E_old)
            self.W_old = torch.where(rej, W_cur, self.W_old)
            self._moved = False
        return self.accept

    # ------------------------------------------------------------------
    def particles(self):
        """State in each chain's reference dtype, host numpy (C, N, 2)."""
        return self.state.cpu().numpy()

    def acceptance_rate(self):
        a = self.attempts.sum().item()
        return self.accepted.sum().item() / a if a else 0.0

    @_on_own_device
    def histogram2d(self, bins=100):
        """Density histogram of the current states (utils.py:488-495): counts (bins-1, bins-1)."""
        B = self.phys.half_width
        edges = torch.as_tensor(np.linspace(-B, B, bins), device=self.device)
        hist = torch.zeros((bins - 1) * (bins - 1), dtype=torch.int64, device=self.device)
        _lib.check(_lib.load().fs_hist2d(_lib.ptr(self.state), self.C, self.N, B, _lib.ptr(edges), bins - 1,
                                         _lib.ptr(hist), _lib.stream_ptr()), "fs_hist2d")
        return hist.reshape(bins - 1, bins - 1)

    @_on_own_device
    def well_counts(self, counts=None, half_box=None, r0=None):
        """(C, 3) int64: all-in-A, all-in-B, samples (utils.py:61-141) accumulated into counts.
        half_box is the driver's HALF_BOX (default box_x / 2), r0 the well radius parameter
        (default the physics' r0); each chain is classified in its state's dtype."""
        if counts is None:
            counts = torch.zeros((self.C, 3), dtype=torch.int64, device=self.device)
        _lib.check(_lib.load().fs_well_stats(_lib.ptr(self.state), _lib.ptr(self.state_is_f32), self.C, self.N,
                                             float(half_box if half_box is not None else self.phys.half_width),
                                             float(self.phys.r0 if r0 is None else r0), _lib.ptr(counts),
                                             _lib.stream_ptr()), "fs_well_stats")
        return counts
