"""One update cycle of the Algorithm-2 driver (hybrid_NF_MCMC/main_algorithm_2.py:393-570)
over batched runs, optionally sharded over ranks.

A cycle is
  production   UPDATE_NUM_SAMPLES / (NUM_MC_RUNS / SAMPLING_FREQUENCY) local moves per
               run with sample() every SAMPLING_FREQUENCY steps; the sampled
               configurations (run-major, minus HALF_BOX) are the training set
               (:399-417, cumulative or not :420-425);
  training     one epoch over the set: DataLoader(batch_size, shuffle=True) batches, a
               fresh Adam, loss = ALPHA * forward_kld(batch) + (1 - ALPHA) *
               reverse_kld(BATCH_SIZE), skipped when not finite (:433-452);
  refeeding    model.eval(); one flow proposal per run (model.sample(NUM_MC_RUNS) +
               HALF_BOX) offered through nf_big_move (:476-540).

Device mapping: production and refeeding are one batched call each over all runs (the
refeed is the fused fs_nf_mh_step: in-kernel base draws -> sampling pass -> density
pass -> energies -> accept); training runs through PyTorch-ROCm autograd with the
fused spline kernels, the full-size batches and the partial last batch replaying captured HIP graphs
(train.GraphedTrainStep, one per batch size, sharing one Adam state).

Several ranks: each owns a contiguous block of runs (global run order = rank order, so
the gathered training set is in the reference's run-major order).  The training set
is all-gathered and every rank trains the same replicated model with the same data
order; rank 0's weights are then broadcast (42.9 MB at A2 / N=64) so that the replicas
cannot drift.  The reference trains on one device (main_algorithm_2.py:437-452); this
keeps its batch and BatchNorm semantics exactly (no per-rank batch statistics).
"""
import torch

from . import algorithm1 as A1
from . import parallel
from .normflows.train import step_loss


class _Indices(torch.utils.data.Dataset):
    """Dataset of the sample indices 0..n-1, fetched a batch at a time."""

    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return i

    def __getitems__(self, idx):
        return torch.tensor(idx, dtype=torch.int64)


def _first(batch):
    return batch


class Algorithm2:
    def __init__(self, bmc, model, batch_size=256, lr=0.000543510751759681, weight_decay=9.5857178422352e-05,
                 alpha=1.0, sampling_frequency=10, update_num_samples=1000, num_mc_runs=None, cumulative=False,
                 graphed=True, group=None):
        """bmc: this rank's BatchedMonteCarlo (its runs); model: the flow (the same
        initial weights on every rank); num_mc_runs: NUM_MC_RUNS over all ranks
        (default: bmc.C x world size).  Defaults are main_algorithm_2.py:32-64."""
        self.bmc, self.model = bmc, model
        self.batch_size, self.lr, self.wd, self.alpha = int(batch_size), float(lr), float(weight_decay), float(alpha)
        self.sf = int(sampling_frequency)
        self.group = group
        self.world = parallel.world_size(group)
        runs = bmc.C * self.world if num_mc_runs is None else int(num_mc_runs)
        self.production_runs = int(update_num_samples / (runs / self.sf))  # :402
        self.cumulative = bool(cumulative)
        self.training_data = None
        self.total_mcmc_steps = 0
        self.loss_history = []
        self.p_acc_history = []
        self.mcmc_steps_history = []
        self.graphed = bool(graphed) and next(model.parameters()).is_cuda
        self._step = None
        self._mods = None  # (model, its modules) for the mode switches (_set_training)

    # ------------------------------------------------------------------
    def production(self):
        """:399-417 — returns this rank's Snapshots; sets the (gathered) training set."""
        snap, _ = A1.production(self.bmc, self.production_runs, self.sf)
        return self._take(snap)

    def _take(self, snap):
        """The training set of a production phase's snapshots (A1.production's samples)."""
        local = snap.xy.reshape(-1, self.bmc.N, 2) - self.bmc.phys.half_width
        self.total_mcmc_steps += self.production_runs * self.bmc.C * self.world
        data = parallel.all_gather_configs(local.contiguous(), group=self.group)
        data = data.to(torch.float32).reshape(data.shape[0], -1)  # get_dataloader: float32 (M, N*dim)
        if self.cumulative and self.training_data is not None:
            self.training_data = torch.cat([self.training_data, data], 0)
        else:
            self.training_data = data
        return snap

    def _batches(self, n):
        """The index batches DataLoader(TensorDataset(data), batch_size, shuffle=True)
        yields (same sampler, same draws from the default generator), fetched as whole
        index batches (Dataset.__getitems__) instead of item by item and collated: 0.6
        instead of 7.4 ms per epoch of 1000 samples on the host."""
        from torch.utils.data import DataLoader

        return list(DataLoader(_Indices(n), batch_size=self.batch_size, shuffle=True, collate_fn=_first))

    def _set_training(self, mode):
        """model.train(mode) as a flag write per module: nn.Module.train walks the ~500
        modules of an A2 flow through Module.__setattr__ (~2 ms per call on the host, twice
        per cycle while the GPU waits); the same flags are set when no module overrides
        train(), else model.train(mode) itself."""
        m = self.model
        if self._mods is None or self._mods[0] is not m:
            mods = list(m.modules())
            self._mods = (m, mods if all(type(x).train is torch.nn.Module.train for x in mods) else None)
        mods = self._mods[1]
        if mods is None:
            m.train(mode)
        else:
            for x in mods:
                x.__dict__["training"] = mode

    def train(self):
        """:430-452 — one epoch with a fresh Adam; returns the mean loss (reference:
        cycle_loss / len(dataloader), NaN / inf losses included)."""
        m = self.model
        self._set_training(True)
        data = self.training_data.to(next(m.parameters()).device)
        batches = self._batches(data.shape[0])
        losses = []
        if self.graphed:
            if self._step is None:
                from .normflows.train import GraphedTrainStep

                tail = data.shape[0] % self.batch_size  # the partial last batch gets its own graph
                self._step = GraphedTrainStep(m, self.batch_size, self.lr, self.wd, alpha=self.alpha,
                                              extra_batch_sizes=(tail,) if tail else ())
            tail = data.shape[0] % self.batch_size
            if tail:
                self._step.add_batch_size(tail)  # cumulative training sets change the tail
            self._step.reset_optimizer()
            self._step.reset_nan()
            # the epoch's batches gathered once (one index upload, one gather) and the
            # steps replayed back to back: no host synchronisation until the epoch's end,
            # where the spline NaN flags of all steps are checked together (the reference
            # raises inside the failing step; here the later steps have replayed by then,
            # but the sticky NaN word kept them from writing: parameters, Adam state and
            # BatchNorm statistics are those after the last good step, train.py)
            shuffled = data[torch.cat(batches).to(data.device)] if batches else data[:0]
            flags, off = [], 0
            for b in batches:
                loss, flag = self._step.step(shuffled[off:off + b.numel()], check=False)
                off += b.numel()
                losses.append(loss.detach().reshape(()))
                flags.append(flag.reshape(()))
            if flags and bool(torch.stack(flags).any()):
                raise ValueError("Discriminant computation resulted in NaN.")  # splines.py:176-183
        else:
            opt = torch.optim.Adam(m.parameters(), lr=self.lr, weight_decay=self.wd)
            for b in batches:
                x = data[b.to(data.device)]
                opt.zero_grad()
                loss = step_loss(m, x, self.batch_size, self.alpha)
                if bool(~(torch.isnan(loss) | torch.isinf(loss))):
                    loss.backward()
                    opt.step()
                losses.append(loss.detach().reshape(()))
            m.invalidate_packed()
        if self.world > 1:
            parallel.broadcast_state(m, src=0, group=self.group)
            m.invalidate_packed()
        total = 0.0
        for v in torch.stack(losses).tolist() if losses else []:
            total += v  # cycle_loss += loss.item(), in batch order
        avg = total / len(batches) if batches else float("nan")
        self.loss_history.append(avg)
        return avg

    def refeed(self):
        """:476-540 — model.eval(), one NF-proposed MH step per run (fused HIP step);
        returns (accepted runs on this rank (C,) u8, global acceptance p_acc_update)."""
        self._set_training(False)  # model.eval()
        if self.bmc.model is not self.model:
            self.bmc.set_model(self.model)
        self.bmc.invalidate_nll()  # nf_big_move re-derives the old NLL with the current weights (:251-261)
        acc = self.bmc.step().clone()
        n = acc.to(torch.int64).sum().reshape(1)
        if self.world > 1:
            import torch.distributed as dist

            dist.all_reduce(n, group=self.group)
        p = int(n.item()) / (self.bmc.C * self.world)
        self.bmc.check_errors()
        self.p_acc_history.append(p)
        self.mcmc_steps_history.append(self.total_mcmc_steps)
        return acc, p

    def cycle(self):
        """One update cycle: production -> training -> refeeding."""
        snap = self.production()
        loss = self.train()
        acc, p = self.refeed()
        return snap, loss, acc, p

    def run(self, cycles, speculate=None):
        """`cycles` update cycles in the reference's loop (main_algorithm_2.py:393-570),
        returning each cycle's (snapshots, loss, accepted, p_acc) as cycle() does.
        speculate (default: on for a device engine): the next cycle's production runs on a
        second stream during this cycle's training, from a copy of the runs with what a
        refeed that every run rejects does to them (one Generator.random() draw, attempts +
        1, the running energy re-derived; algorithm1._Speculator); after the refeed a device
        byte says whether any run accepted, and only then does the production run again
        from the real runs.  The results are those of `cycles` calls of cycle()."""
        from . import _lib

        bmc, n, sf = self.bmc, self.production_runs, self.sf
        cycles = int(cycles)
        spec = None
        if (speculate is None or bool(speculate)) and bmc.device.type == "cuda" and n > 0 and cycles > 1:
            spec = A1._Speculator(bmc)
        out, ahead = [], None
        with _lib.on_device(bmc.device):
            try:
                for c in range(cycles):
                    snap = self.production() if ahead is None else self._take(ahead)
                    more = spec is not None and c + 1 < cycles
                    if more:
                        spec.begin(n, sf)
                    loss = self.train()
                    acc, p = self.refeed()
                    out.append((snap, loss, acc, p))
                    ahead = spec.finish(n, sf) if more else None
            finally:
                if spec is not None:
                    spec.close()
        return out
