"""The phases of the Algorithm-1 driver (hybrid_NF_MCMC/main_algorithm_1.py) with every
run ("MC run" = chain) batched on the device.

The reference drives NUM_MC_RUNS MonteCarlo objects one after the other in Python
loops.  Runs never interact, so each loop below is one device call over all runs;
the bookkeeping that depends on the reference's run-major loop order (the global
acceptance history, total_mcmc_steps, the order of the training samples) is
rebuilt from the per-run device results afterwards:

  equilibrate        main_algorithm_1.py:202-210  (particle_displacement, adjust_displacement, sample)
  production         main_algorithm_1.py:240-251  (training samples, run-major)
  testing_phase      main_algorithm_1.py:375-424  (BIG_MOVE_INTERVAL local moves + one nf_big_move per attempt)
  well_statistics    main_algorithm_1.py:443-455 -> utils.py:61-101 (calculate_well_statistics per run)
  free_energy_curve  utils.py:738-763 (plot_avg_free_energy's mean / sem / std, no plotting)
  write_outputs      main_algorithm_1.py:434-440, 499-547 (acceptance CSV, per-run CSV / npy)

Snapshots stay on the device as (runs, samples, N, 2) float64 tensors together with
the reference dtype each snapshot had (a run's state turns float32 after its first
accepted big move, monte_carlo.py:289-292); tuples and files are produced only when
asked for.
"""
import copy
import ctypes
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib, analysis, io
from .MCMC.batched import BatchedMonteCarlo


@dataclass
class Snapshots:
    """sample() snapshots of one batched local-move call: cycle numbers `steps`,
    configurations xy (C, S, N, 2) f64, (E, W) (C, S, 2) f64, and the reference dtype
    of every run's state during the call (C,) bool (True = float32)."""
    steps: list
    xy: torch.Tensor
    ew: torch.Tensor
    is_f32: torch.Tensor

    def configs(self):
        return self.xy

    def tuples(self, bmc, run):
        """The reference's sample() tuples of one run (monte_carlo.py:416-444)."""
        if not self.steps:
            return []
        xy = self.xy[run].cpu().numpy()
        ew = self.ew[run].cpu().numpy()
        f32 = bool(self.is_f32[run].item())
        bx, by = np.float64(bmc.phys.box_x), np.float64(bmc.phys.box_y)
        return [io.sample_tuple(s, np.float64(ew[k, 0]), np.float64(ew[k, 1]), bmc.N, bx, by, bmc.phys.beta,
                                xy[k].astype(np.float32) if f32 else xy[k])
                for k, s in enumerate(self.steps)]


def _local(bmc, n, adjust_every, sample_every):
    is_f32 = bmc.state_is_f32.bool().clone()
    xy, ew, _ = bmc.local_moves(n, adjust_every=adjust_every, sample_every=sample_every, step0=0)
    steps = [s for s in range(1, n + 1) if sample_every and s % sample_every == 0]
    if xy is None:
        xy = torch.empty((bmc.C, 0, bmc.N, 2), dtype=torch.float64, device=bmc.device)
        ew = torch.empty((bmc.C, 0, 2), dtype=torch.float64, device=bmc.device)
    return Snapshots(steps, xy, ew, is_f32)


def equilibrate(bmc: BatchedMonteCarlo, steps, adjusting_frequency, sampling_frequency):
    """main_algorithm_1.py:202-210: `steps` particle_displacement calls per run,
    adjust_displacement after every step divisible by adjusting_frequency, a sample()
    after every step divisible by sampling_frequency."""
    return _local(bmc, int(steps), int(adjusting_frequency), int(sampling_frequency))


def production(bmc: BatchedMonteCarlo, steps, sampling_frequency, half_box=None):
    """main_algorithm_1.py:240-253: local moves with sampling (no adjustment).  Returns
    (snapshots, global_samples_nf): the training set in the reference's order (run 0's
    samples first) shifted by -HALF_BOX, float64 on the device, as the reference's
    np.array(... particle - [HALF_BOX, HALF_BOX] ...) builds it."""
    snap = _local(bmc, int(steps), 0, int(sampling_frequency))
    hb = bmc.phys.half_width if half_box is None else float(half_box)
    samples = snap.xy.reshape(-1, bmc.N, 2) - hb
    return snap, samples


@dataclass
class TestingResult:
    """Outputs of the testing phase, per run (C) and attempt (A)."""
    accepts: torch.Tensor                  # (C, A) u8 nf_big_move decisions
    snapshots: list                        # A Snapshots (one per attempt)
    p_acc_history: list = field(default_factory=list)
    mcmc_steps_history: list = field(default_factory=list)
    total_mcmc_steps: int = 0
    big_move_attempts: int = 0
    big_move_accepts: int = 0
    speculated: int = 0                    # attempts whose successor kept the speculative local moves

    def testing_configs(self):
        """(C, A*S, N, 2) f64: every run's mc_run.testing_samples in order."""
        return torch.cat([s.xy for s in self.snapshots], 1)

    def testing_is_f32(self):
        """(C,) bool: np.array(mc_run.testing_samples) is float32 only if every
        snapshot of the run was taken from a float32 state."""
        m = torch.ones_like(self.snapshots[0].is_f32)
        for s in self.snapshots:
            m &= s.is_f32
        return m

    def local_sample_tuples(self, bmc, run):
        out = []
        for s in self.snapshots:
            out += s.tuples(bmc, run)
        return out

    def test_moves(self):
        """Per-run (test_moves_attempted, test_moves_accepted) (main_algorithm_1.py:401-408)."""
        a = self.accepts.to(torch.int64)
        return torch.full((a.shape[0],), a.shape[1], dtype=torch.int64, device=a.device), a.sum(1)


def acceptance_history(accepts, interval, total_mcmc_steps=0, big_move_attempts=0, big_move_accepts=0):
    """The global acceptance history of the reference's run-major testing loop
    (main_algorithm_1.py:381-419) from the (C, A) accept matrix: for run r, attempt a,
    total_mcmc_steps grows by `interval`, then the cumulative global acceptance is
    appended.  Returns (p_acc_history, mcmc_steps_history, total_mcmc_steps,
    big_move_attempts, big_move_accepts) — the appended entries and the new counters."""
    acc = np.asarray(torch.as_tensor(accepts).cpu().numpy(), dtype=np.int64).reshape(-1)  # run-major
    n = acc.size
    cum = big_move_accepts + np.cumsum(acc)
    att = big_move_attempts + np.arange(1, n + 1)
    steps = total_mcmc_steps + interval * np.arange(1, n + 1)
    p = [int(c) / int(t) for c, t in zip(cum, att)]  # Python int / int, as the reference
    return (p, [int(s) for s in steps], total_mcmc_steps + interval * n, big_move_attempts + n,
            big_move_accepts + int(acc.sum()))


_PIPE_STREAMS = {}


def _priority_streams(device):
    """Three high-priority streams of torch's pool, made once per process (FS_PIPE_STREAMS=
    priority).  The runtime deals a process's streams over a few hardware queues
    (GPU_MAX_HW_QUEUES), and two streams that share one run their kernels one after the
    other, so the pipeline's overlap depends on which pool streams it gets: with fresh
    normal-priority streams (the default) the same code measured 2137-3546 attempts/s
    depending on the streams the process had taken before (profiles/r06/r06f5_regime_ab.log;
    3522-3545 in the bench's own sequence, r06f1, r06f8), with these 3228-3363 in every process
    measured (r06f7, r06f8)."""
    key = torch.device(device).index
    if key not in _PIPE_STREAMS:
        _PIPE_STREAMS[key] = [torch.cuda.Stream(device=device, priority=-1) for _ in range(3)]
    return _PIPE_STREAMS[key]


class _Speculator:
    """The next attempt's local moves, run ahead on a side stream while the big move runs.

    A big move that no chain accepts leaves every chain as it was except for what the
    reject itself does (mh_accept_kernel / nf_big_move, monte_carlo.py:264-303): one
    Generator.random() draw (a reject always draws: ratio < 1 or NaN), attempts += 1,
    and the running energy / virial set to those of the current state (:299-301).  So the
    next `interval` local moves can start, before the big move is decided, from a shadow
    copy of the chains with exactly those changes made (begin).  After the big move
    (finish), a device byte says whether any chain accepted; only then do
    fs_chains_copy_if / fs_local_moves_if redo the local moves from the real chains, and
    the shadow becomes the real chains either way: the same kernels on the same inputs,
    so the results are bit-identical, and no step waits for the host.  The gain is in the
    attempts that follow a big move no chain accepted (0.2-0.3 % acceptance in the bench's
    regime: nearly all of them); there the local moves and the big move, which each fill
    only a few CUs at this batch size, run side by side."""

    FIELDS = ("state", "state_is_f32", "pcg", "pcg_buf", "max_disp", "attempts", "accepted", "prev_counts",
              "E_old", "W_old")

    def __init__(self, bmc):
        self.bmc = bmc
        self.main = torch.cuda.current_stream(bmc.device)
        self.side = torch.cuda.Stream(device=bmc.device)
        self.shadow = copy.copy(bmc)  # shares the physics and the flow; own chain buffers
        for k in self.FIELDS:
            setattr(self.shadow, k, torch.empty_like(getattr(bmc, k)))
        self.draw = torch.empty(bmc.C, dtype=torch.float64, device=bmc.device)
        self.one = torch.ones(1, dtype=torch.uint8, device=bmc.device)  # an always-open gate: one copy launch
        self.L = _lib.load()

    @staticmethod
    def _chains(m):
        return _lib.LocalChains(*(getattr(m, k).data_ptr() for k in (
            "state", "state_is_f32", "E_old", "W_old", "pcg", "pcg_buf", "max_disp", "attempts", "accepted",
            "prev_counts")))

    def _moves(self, m, n, sf, gate=None):
        args = (m.phys.c, m.C, m.N, _lib.ptr(m.state), _lib.ptr(m.state_is_f32), _lib.ptr(m.E_old),
                _lib.ptr(m.W_old), _lib.ptr(m.pcg), _lib.ptr(m.pcg_buf), _lib.ptr(m.max_disp), _lib.ptr(m.attempts),
                _lib.ptr(m.accepted), _lib.ptr(m.prev_counts), n, 0, 0, m.target_acceptance, sf, _lib.ptr(self.xy),
                _lib.ptr(self.ew), None, None, _lib.stream_ptr())
        if gate is None:
            _lib.check(self.L.fs_local_moves(*args), "fs_local_moves")
        else:
            _lib.check(self.L.fs_local_moves_if(_lib.ptr(gate), *args), "fs_local_moves_if")

    def begin(self, n, sf):
        """Before the big move: copy the chains (main stream, ahead of the big move's
        writes), then on the side stream the local moves that follow a reject."""
        b, sh, L = self.bmc, self.shadow, self.L
        _lib.check(L.fs_chains_copy_if(_lib.ptr(self.one), b.C, b.N, ctypes.byref(self._chains(b)),
                                       ctypes.byref(self._chains(sh)), _lib.stream_ptr()), "fs_chains_copy_if")
        self.n0 = b.n_accept.clone()
        S = L.fs_local_samples_per_chain(0, n, sf)
        self.steps = [s for s in range(1, n + 1) if sf and s % sf == 0]
        self.xy = torch.empty((b.C, S, b.N, 2), dtype=torch.float64, device=b.device)
        self.ew = torch.empty((b.C, S, 2), dtype=torch.float64, device=b.device)
        self.side.wait_stream(self.main)
        with torch.cuda.stream(self.side):
            st = _lib.stream_ptr()
            _lib.check(L.fs_pcg64_random(_lib.ptr(sh.pcg), b.C, _lib.ptr(self.draw), st), "fs_pcg64_random")
            sh.attempts += 1
            _lib.check(L.fs_energy_state(b.phys.c, _lib.ptr(sh.state), _lib.ptr(sh.state_is_f32), b.C, b.N,
                                         _lib.ptr(sh.E_old), _lib.ptr(sh.W_old), st), "fs_energy_state")
            self._moves(sh, n, sf)

    def finish(self, n, sf):
        """After the big move: redo the local moves from the real chains if any chain
        accepted (decided on the device), then swap the shadow in.  Returns the Snapshots."""
        b, sh = self.bmc, self.shadow
        gate = b.n_accept != self.n0
        self.main.wait_stream(self.side)
        _lib.check(self.L.fs_chains_copy_if(_lib.ptr(gate), b.C, b.N, ctypes.byref(self._chains(b)),
                                            ctypes.byref(self._chains(sh)), _lib.stream_ptr()), "fs_chains_copy_if")
        self._moves(sh, n, sf, gate)
        for k in self.FIELDS:
            bk, sk = getattr(b, k), getattr(sh, k)
            setattr(b, k, sk)
            setattr(sh, k, bk)
        b._moved = True
        return Snapshots(self.steps, self.xy, self.ew, b.state_is_f32.bool())  # (a new tensor: uint8 -> bool)

    def close(self):
        self.main.wait_stream(self.side)


def pipeline_schedule(accepts):
    """The stage schedule _Pipeline follows for a (C, A) accept matrix: (spec, redo), two
    lists of A bools.  Stage k = the local moves before big move k.  spec[k]: the stage ran
    ahead, from stage k-1's state as a rejected big move k-1 leaves it (every stage but the
    first).  redo[k]: big move k-1 accepted on some chain, so the main stream ran stage k
    again from the finished state, and stage k+1 was run ahead again from that redone stage
    (its first version started from the wrong one): each stage's last version starts from the
    right state, and only an accept in the big move just before it sends it back."""
    acc = torch.as_tensor(accepts)
    A = int(acc.shape[1]) if acc.dim() == 2 else 0
    spec = [k >= 1 for k in range(A)]
    redo = [k >= 1 and bool(acc[:, k - 1].any()) for k in range(A)]
    return spec, redo


class _Pipeline:
    """The testing phase as a three-stream pipeline: the local moves run back to back on a
    side stream, each stage started from the previous stage's state as a rejected big move
    leaves it (_Speculator's reject transform), and each stage's density pass (the big
    move's old NLL, state_nll) runs on one of two density streams as soon as its local
    moves end; the main stream runs only the big moves' energy and accept, each when its
    density pass is done.  A stage is the truth as long as no big move it assumed rejected
    accepted on any chain; the host learns each big move's outcome one attempt behind
    (a pinned copy of the accept flags, read while the GPU runs the queued stages), runs a
    wrong stage again on the main stream from the finished state (copy, local moves,
    density pass: the same kernels on the same inputs, so every result is bit-identical to
    the plain sequence) and runs the next stage ahead again on the side stream as soon as
    the redone local moves end.

    With the chains' rare accepts (0.2-0.3 % per big move in the reference's regime), the
    attempt time is the local moves' (the density pass, 1.3x as long, overlaps two
    attempts), where _Speculator's is the density pass plus the big move: 2.50 ms per stage
    against 3.55 ms (r06, timing events: tools/regime_gpu_timeline.py), the regime 2780 ->
    3737-3777 attempts/s with the stages after its accepts run again.  The density passes
    use model.frozen_log_prob() (the flow is fixed in the testing phase): the per-pass
    checks cost ~0.9 ms of host time, which paced the pipeline.  The schedule of stages is
    pipeline_schedule(accepts)."""

    R = 4  # ring of chain-state slots: a stage's slot is free once the big move after the next is done

    def __init__(self, bmc, n, sf):
        self.bmc, self.n, self.sf = bmc, n, sf
        self.L = _lib.load()
        dev = bmc.device
        self.main = torch.cuda.current_stream(dev)
        # two density streams: a pass (~3.6 ms at 10 rows) outlasts a stage's local moves
        # (~2.4 ms), so consecutive passes overlap (4 streams measured slower, r06zh)
        if os.environ.get("FS_PIPE_STREAMS") == "priority":
            self.side, *self.dens = _priority_streams(dev)
        else:
            self.side, *self.dens = [torch.cuda.Stream(device=dev) for _ in range(3)]
        # the flow is fixed during the testing phase: its density pass without the per-call
        # checks, over the image packed now (before another stream reads it)
        self.log_prob = bmc.model.frozen_log_prob()
        self.slots = []
        for r in range(self.R):
            s = copy.copy(bmc)  # shares the physics, the flow, accept / n_accept / err
            if r > 0:
                for k in _Speculator.FIELDS:
                    setattr(s, k, torch.empty_like(getattr(bmc, k)))
            self.slots.append(s)
        self.nll = [torch.empty(bmc.C, dtype=torch.float64, device=dev) for _ in range(self.R)]
        self.acc_host = [torch.empty(bmc.C, dtype=torch.uint8, pin_memory=True) for _ in range(self.R)]
        self.draw = torch.empty(bmc.C, dtype=torch.float64, device=dev)
        self.one = torch.ones(1, dtype=torch.uint8, device=dev)
        self.S = self.L.fs_local_samples_per_chain(0, n, sf)
        self.steps = [s for s in range(1, n + 1) if sf and s % sf == 0]
        self.spec, self.redo, self.acc = {0: False}, {0: False}, {}
        self.ev_L, self.ev_copy, self.ev_D, self.ev_main, self.ev_redo = {}, {}, {}, {}, {}
        self.xy, self.ew = {}, {}
        self.kept = 0
        for s in [self.side] + self.dens:
            s.wait_stream(self.main)  # stage 0's local moves, the flow image, the slots
        self.ev_L[0] = self.main.record_event()
        self._density(0)

    def slot(self, k):
        return self.slots[k % self.R]

    def _moves(self, m, k):
        _lib.check(self.L.fs_local_moves(
            m.phys.c, m.C, m.N, _lib.ptr(m.state), _lib.ptr(m.state_is_f32), _lib.ptr(m.E_old), _lib.ptr(m.W_old),
            _lib.ptr(m.pcg), _lib.ptr(m.pcg_buf), _lib.ptr(m.max_disp), _lib.ptr(m.attempts), _lib.ptr(m.accepted),
            _lib.ptr(m.prev_counts), self.n, 0, 0, m.target_acceptance, self.sf, _lib.ptr(self.xy[k]),
            _lib.ptr(self.ew[k]), None, None, _lib.stream_ptr()), "fs_local_moves")

    def _copy(self, k):
        """slot k := slot k-1 (every chain array), on the current stream."""
        _lib.check(self.L.fs_chains_copy_if(_lib.ptr(self.one), self.bmc.C, self.bmc.N,
                                            ctypes.byref(_Speculator._chains(self.slot(k - 1))),
                                            ctypes.byref(_Speculator._chains(self.slot(k))), _lib.stream_ptr()),
                   "fs_chains_copy_if")

    def _density(self, k):
        ds = self.dens[k % len(self.dens)]
        with torch.cuda.stream(ds):
            ds.wait_event(self.ev_L[k])
            self.nll[k % self.R].copy_(self.bmc.state_nll(self.slot(k).state, self.log_prob))
            self.ev_D[k] = ds.record_event()

    def stage(self, k, after_redo=False):
        """Queue stage k (k >= 1) on the side stream and its density pass: from stage k-1's
        state as big move k-1 leaves it on a reject — the side stream's stage k-1, or, with
        after_redo, stage k-1 as the main stream ran it again (queued after that redo's
        local moves; this version of stage k replaces the one queued before)."""
        b, sl = self.bmc, self.slot(k)
        self.spec[k] = True
        if k not in self.xy:  # (a stage run again writes the same snapshot tensors, in stream order)
            self.xy[k] = torch.empty((b.C, self.S, b.N, 2), dtype=torch.float64, device=b.device)
            self.ew[k] = torch.empty((b.C, self.S, 2), dtype=torch.float64, device=b.device)
        with torch.cuda.stream(self.side):
            if k - self.R + 1 >= 0:  # the slot's previous stage: its big move and the next one's redo are done
                self.side.wait_event(self.ev_main[k - self.R + 1])
            if k == 1:
                self.side.wait_event(self.ev_L[0])
            if after_redo:
                self.side.wait_event(self.ev_redo[k - 1])
            self._copy(k)  # before big move k-1 writes slot k-1 (it waits for this event)
            self.ev_copy[k] = self.side.record_event()
            st = _lib.stream_ptr()
            _lib.check(self.L.fs_pcg64_random(_lib.ptr(sl.pcg), b.C, _lib.ptr(self.draw), st), "fs_pcg64_random")
            sl.attempts += 1
            _lib.check(self.L.fs_energy_state(b.phys.c, _lib.ptr(sl.state), _lib.ptr(sl.state_is_f32), b.C, b.N,
                                              _lib.ptr(sl.E_old), _lib.ptr(sl.W_old), st), "fs_energy_state")
            self._moves(sl, k)
            self.ev_L[k] = self.side.record_event()
        self._density(k)

    def learn(self, k):
        """Wait for big move k; stage k+1 runs again if it accepted on some chain."""
        self.ev_main[k].synchronize()
        self.acc[k] = bool(self.acc_host[k % self.R].any())
        self.redo[k + 1] = self.acc[k]

    def redo_moves(self, k):
        """When stage k was wrong: its local moves again on the main stream, from the
        finished state after big move k-1 (the event marks their end for stage k+1)."""
        if self.redo[k]:
            self.main.wait_event(self.ev_D[k])  # (the wrong pass read slot k and writes its NLL)
            # (the first version of stage k+1 copied slot k after its local moves, before that
            # pass started; were it later, only that version, which is replaced, would differ)
            self._copy(k)
            self._moves(self.slot(k), k)
            self.ev_redo[k] = self.main.record_event()

    def attempt(self, k, configs, terms):
        """Queue big move k on the main stream (after the rest of stage k's redo if it was
        wrong).  Returns (the Snapshots of stage k, or None for stage 0; the accept flags)."""
        b, sl = self.bmc, self.slot(k)
        self.main.wait_event(self.ev_D[k])
        if self.redo[k]:
            self.nll[k % self.R].copy_(b.state_nll(sl.state, self.log_prob))
        elif self.spec[k]:
            self.kept += 1
        if self.spec.get(k + 1):  # stage k+1 copied slot k before this big move writes it
            self.main.wait_event(self.ev_copy[k + 1])
        snap = Snapshots(self.steps, self.xy[k], self.ew[k], sl.state_is_f32.bool()) if k > 0 else None
        sl._moved = True
        acc = sl.nf_big_move(configs, terms=terms, nll=self.nll[k % self.R]).clone()
        self.acc_host[k % self.R].copy_(acc, non_blocking=True)
        self.ev_main[k] = self.main.record_event()
        return snap, acc

    def close(self, last):
        """Join the streams; the engine takes the chain arrays of the last attempt's slot."""
        for s in [self.side] + self.dens:
            self.main.wait_stream(s)
        if last is not None:
            b, sl = self.bmc, self.slot(last)
            for k in _Speculator.FIELDS + ("nll_old",):
                setattr(b, k, getattr(sl, k))
            b._moved = False


def _run_pipeline(bmc, cfg, A, n, sf, terms_of, snaps, acc):
    """testing_phase's attempts through _Pipeline on the current stream (its main stream)."""
    C = bmc.C
    last = None
    pipe = _Pipeline(bmc, n, sf)
    try:
        pipe.stage(1)
        for a in range(A):
            if a >= 1:
                pipe.learn(a - 1)
            if a + 2 < A and not pipe.redo[a]:  # the side stream's next stage first: it sets the pace
                pipe.stage(a + 2)
            pipe.redo_moves(a)
            if pipe.redo[a]:  # stage a+1 ran ahead from the wrong stage a: again, from the redone one
                if a + 1 < A:
                    pipe.stage(a + 1, after_redo=True)
                if a + 2 < A:
                    pipe.stage(a + 2)
            snap, ac = pipe.attempt(a, cfg[a * C:(a + 1) * C], terms_of(a))
            last = a
            acc.append(ac)
            if snap is not None:
                snaps.append(snap)
    finally:
        pipe.close(last if last == A - 1 else None)
    return pipe


def testing_phase(bmc: BatchedMonteCarlo, test_configs, attempts, interval, sampling_frequency,
                  total_mcmc_steps=0, big_move_attempts=0, big_move_accepts=0, speculate=None):
    """main_algorithm_1.py:375-424 for all runs: per attempt, `interval` local moves with
    sampling, then nf_big_move with test_configs[attempt * C + run] (float32 box
    coordinates, (>= attempts*C, N, 2), numpy or device).  speculate: how the attempts
    overlap on a device engine with a flow and local moves between the big moves (the
    results are the same every way): "pipeline" (the default, also True / None: _Pipeline,
    the local moves back to back on a side stream, each stage's density pass on its own
    stream, the big moves on the main stream), "local" (_Speculator: each big move beside
    the next attempt's local moves) or False (one phase after the other).  The engine's
    chain buffers (bmc.state, bmc.pcg, ...) may afterwards be other tensors of the same
    shape: read them from bmc after the call, not through references taken before it."""
    C = bmc.C
    cfg = torch.as_tensor(test_configs)
    if cfg.dtype != torch.float32:
        raise ValueError("test configurations are float32 (main_algorithm_1.py:340-343)")
    if cfg.shape[0] < attempts * C:
        raise IndexError(f"index {attempts * C - 1} is out of bounds for axis 0 with size {cfg.shape[0]}")
    if speculate not in (None, True, False, "pipeline", "local"):
        raise ValueError(f"speculate must be 'pipeline', 'local', True, False or None, got {speculate!r}")
    cfg = cfg.to(bmc.device)
    A, n, sf = int(attempts), int(interval), int(sampling_frequency)
    # (speculation needs a device engine with a flow, and local moves between the big moves:
    # the reject transform assumes a big move after local moves, which re-derives the running
    # energy, monte_carlo.py:299-301)
    mode = None
    if speculate is not False and bmc.device.type == "cuda" and bmc.model is not None and n > 0 and A > 1:
        mode = "local" if speculate == "local" else "pipeline"
    snaps, acc = [], []
    # the test configurations' energies and log q do not depend on the chain states: one
    # launch per pass over a block of attempts (bit-identical rows), so each attempt's big
    # move runs only the current states' density pass and energy
    block = max(1, BatchedMonteCarlo.FILL_ROWS // max(1, C))
    terms, a0 = None, 0
    spec = pipe = None

    def terms_of(a):
        nonlocal terms, a0
        if bmc.model is None:
            return None
        if a % block == 0:
            a0, a1 = a, min(A, a + block)
            terms = bmc.proposal_terms(cfg[a0 * C:a1 * C])
        o = (a - a0) * C
        return tuple(x[o:o + C] for x in terms)

    with _lib.on_device(bmc.device):
        if A > 0:
            snaps.append(_local(bmc, n, 0, sf))
        if mode == "pipeline":
            pipe = _run_pipeline(bmc, cfg, A, n, sf, terms_of, snaps, acc)
        else:
            if mode == "local":
                spec = _Speculator(bmc)
            try:
                for a in range(A):
                    if spec is not None and a + 1 < A:
                        spec.begin(n, sf)
                    t = terms_of(a)
                    acc.append(bmc.nf_big_move(cfg[a * C:(a + 1) * C], terms=t).clone())
                    if a + 1 < A:
                        snaps.append(spec.finish(n, sf) if spec is not None else _local(bmc, n, 0, sf))
            finally:
                if spec is not None:
                    spec.close()
    accepts = torch.stack(acc, 1) if acc else torch.zeros((C, 0), dtype=torch.uint8, device=bmc.device)
    # attempts whose successor's local moves were the speculative ones, kept
    if pipe is not None:
        adopted = pipe.kept
    else:
        adopted = int((accepts[:, :-1].sum(0) == 0).sum()) if spec is not None else 0
    bmc.check_errors()  # a NaN discriminant or a wide-path hand-off timeout in any pass raises
    p, s, tot, att, nacc = acceptance_history(accepts, n, total_mcmc_steps, big_move_attempts, big_move_accepts)
    return TestingResult(accepts, snaps, p, s, tot, att, nacc, adopted)


def well_statistics(configs, is_f32, half_box, r0=1.2):
    """calculate_well_statistics(configs[run], 0, half_box, r0) for every run at once
    (utils.py:61-101).  configs (C, M, N, 2) f64 device tensor, is_f32 (C,) bool (the
    dtype np.array gives the run's snapshots).  Returns device tensors avg_x (C, M) f64
    (np.mean of the x column, in the run's dtype, widened), p_a, p_b (C, M) f64 and
    deltaF (C, M) f64 (log on the device: within 1 ulp of numpy's)."""
    C, M, N, _ = configs.shape
    dev = configs.device
    state = torch.zeros((C, M), dtype=torch.uint8, device=dev)
    avg_x = torch.zeros((C, M), dtype=torch.float64, device=dev)
    f32 = torch.as_tensor(is_f32, device=dev).bool()
    for mask, dt in ((f32, torch.float32), (~f32, torch.float64)):
        idx = mask.nonzero().flatten()
        if idx.numel() == 0 or M == 0:
            continue
        _, st, ax = analysis.classify_wells(configs[idx].to(dt).reshape(-1, N, 2), half_box, r0)
        state[idx] = st.reshape(-1, M)
        avg_x[idx] = ax.reshape(-1, M)
    i = torch.arange(1, M + 1, dtype=torch.float64, device=dev)
    p_a = torch.cumsum((state == 1).to(torch.int64), 1).to(torch.float64) / i
    p_b = torch.cumsum((state == 2).to(torch.int64), 1).to(torch.float64) / i
    both = (p_a > 0) & (p_b > 0)
    dF = torch.where(both, torch.log(torch.where(both, p_b / p_a, torch.ones_like(p_a))), torch.zeros_like(p_a))
    return avg_x, p_a, p_b, dF


def free_energy_curve(deltaF):
    """plot_avg_free_energy's statistics (utils.py:738-763) over runs: mean_deltaF,
    sem_deltaF (per sample index, numpy arrays), final_mean, final_sem, final_std."""
    d = np.asarray(torch.as_tensor(deltaF).cpu().numpy(), dtype=np.float64)
    mean = np.nanmean(d, axis=0)
    sem = np.nanstd(d, axis=0) / np.sqrt(d.shape[0])
    final_mean, final_sem = float(mean[-1]), float(sem[-1])
    return mean, sem, final_mean, final_sem, final_sem * np.sqrt(d.shape[0])


def reference_history(result, production_steps=0):
    """The full acceptance history main_algorithm_1.py writes: the initial (0, 0.0)
    (:234-235), the (total_mcmc_steps, 0.0) point appended after training (:362-363),
    then the testing-phase entries."""
    return [0, production_steps] + result.mcmc_steps_history, [0.0, 0.0] + result.p_acc_history


def write_outputs(directory, bmc, local_snapshots, result=None, history=None, runs=None):
    """acceptance_rate_data.csv (main_algorithm_1.py:434-440, written when `history` =
    (mcmc_steps_history, p_acc_history) is given) and, per run,
    mc_runs/run_XXX/{sampled_data.csv, mc_run_configs.npy, mc_run_testing_configs.npy}
    (:499-547).  local_snapshots: the Snapshots of every phase whose samples went to
    mc_run.local_samples, in order (equilibration, production); the testing phase's
    snapshots are appended from `result`."""
    import os

    os.makedirs(directory, exist_ok=True)
    if history is not None:
        io.write_acceptance_rate(os.path.join(directory, "acceptance_rate_data.csv"), history[0], history[1])
    runs = range(bmc.C) if runs is None else runs
    for r in runs:
        local = []
        for s in local_snapshots:
            local += s.tuples(bmc, r)
        testing = []
        if result is not None:
            t = result.local_sample_tuples(bmc, r)
            local += t
            testing = [x[6] for x in t]
        io.write_run_dir(os.path.join(directory, "mc_runs", f"run_{r + 1:03d}"), local, testing)
