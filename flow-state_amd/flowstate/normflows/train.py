"""Algorithm-2 training step captured in a HIP graph (hybrid_NF_MCMC/main_algorithm_2.py:314-331).

One step of the reference loop is

    optimizer.zero_grad()
    energy_loss, z = model.reverse_kld(BATCH_SIZE)
    sample_loss = model.forward_kld(batch)
    loss = ALPHA * sample_loss + (1 - ALPHA) * energy_loss
    if ~(torch.isnan(loss) | torch.isinf(loss)):
        loss.backward(); optimizer.step()

With eager PyTorch that is ~7 k small kernel launches per step at A2 / batch 256, so the
step is launch-bound.  `GraphedTrainStep` records the whole step once with
torch.cuda.graph (fused spline kernels and HIP GEMMs included) and replays it:

  * the batch is copied into a static input buffer before each replay;
  * the base draws of reverse_kld come from the default generator inside the graph
    (fresh draws every replay, as the reference's q0 sampling);
  * Adam is one fused HIP pass over the flat parameter / gradient / moment buffers
    (fs_adam_step, csrc/optim_kernels.hip: torch's capturable Adam arithmetic, ~16
    launches in torch), and the reference's "skip the step when the loss is NaN / inf"
    happens inside it: the kernel reads the loss and writes nothing when it is not
    finite.  Options it does not cover (amsgrad, maximize, tensor lr) keep torch's
    capturable Adam with a device-side snapshot / restore around it;
  * the spline's NaN-discriminant flags are reduced inside the graph and checked after
    the replay (the reference raises ValueError; here it is raised after the step).  They
    are also ORed into a sticky device word that Adam and the BatchNorm running-statistics
    update skip on, so when an epoch replays its steps back to back and checks the flags
    only at its end (Algorithm2.train), the failing step and every later one write no
    parameters, moments or running statistics: the state is the one after the last good
    step.  (The reference stops inside the failing step's sampling pass, after that pass
    has updated the running statistics of the layers up to the failing one; here that
    step's updates are dropped as a whole.)
"""
import inspect

import torch

from . import autograd_flow as AF


def step_loss(model, x, n_reverse, alpha, flat_bn=None):
    """loss = ALPHA * forward_kld(x) + (1 - ALPHA) * reverse_kld(n_reverse)
    (main_algorithm_2.py:316-318).  With ALPHA = 1 (the reference's setting) the
    reverse term only contributes its value (0 * e: NaN / inf when e is, so the skip
    rule sees it) and its BatchNorm statistics, so it runs without autograd: its
    gradient 0 * de/dtheta is exactly zero whenever the loss is finite.  Likewise the
    forward term when ALPHA = 0.  With ALPHA = 1 and the model's BatchNorm buffers flat
    (flat_bn, autograd_flow.FlatBatchNorm) the two passes share their launches
    (autograd_flow.paired_kld): same values, same running statistics, half the launches
    of the forward half of the step."""
    if alpha == 1.0:
        if flat_bn is not None:
            dev = next(model.parameters()).device
            z = model.q0(n_reverse).to(dev)  # reverse_kld's base draws, first as in the reference
            if AF.paired_ok(model, x, z, flat_bn):
                log_q, zs, lqs = AF.paired_kld(model, x, z, flat_bn, reduce=False)
                with torch.no_grad():
                    energy = model.p._energy(zs)
                return AF.kld_loss(log_q, energy, lqs)  # -mean(log_q) + 0 * (mean(E) + mean(lqs))
            with torch.no_grad():
                energy_loss, _ = model._reverse_kld_from(z)
            return model.forward_kld(x) + 0.0 * energy_loss
        with torch.no_grad():
            energy_loss, _ = model.reverse_kld(n_reverse)
        return model.forward_kld(x) + 0.0 * energy_loss
    if alpha == 0.0:
        energy_loss, _ = model.reverse_kld(n_reverse)
        with torch.no_grad():
            sample_loss = model.forward_kld(x)
        return 0.0 * sample_loss + energy_loss
    energy_loss, _ = model.reverse_kld(n_reverse)
    sample_loss = model.forward_kld(x)
    return alpha * sample_loss + (1 - alpha) * energy_loss


class _Captured:
    """One captured step for one batch size: its static input, loss and NaN flag, and every
    tensor allocated outside the graph's pool that its replays read or write (`keep`): a
    replay writes into them, so they must live as long as the graph.  (r05 / r06: the
    BatchNorm snapshot buffers were locals of _capture; freed after capture, their memory went
    to later allocations, e.g. another model's Adam state, which every replay then overwrote:
    the NaN discriminant of tests/test_gpu_train_graph.py at alpha = 0.7, DESIGN_HISTORY r06.)"""

    def __init__(self, graph, x, loss, nan_flag, keep=()):
        self.graph, self.x, self.loss, self.nan_flag = graph, x, loss, nan_flag
        self.keep = list(keep)


class GraphedTrainStep:
    def __init__(self, model, batch_size, lr, weight_decay=0.0, alpha=1.0, warmup=3, example=None,
                 extra_batch_sizes=(), paired=True):
        """Captures the step for `batch_size` (reverse_kld always draws `batch_size`
        samples, as the reference's reverse_kld(BATCH_SIZE)) and for every size in
        extra_batch_sizes (e.g. the epoch's partial last batch); all graphs share the
        parameters, gradients and one Adam state."""
        dev = next(model.parameters()).device
        if dev.type != "cuda":
            raise ValueError("GraphedTrainStep needs the model on the GPU")
        self.model = model
        if hasattr(model.q0, "device") and torch.device(model.q0.device) != dev:
            # UniformParticle keeps its construction device (Uniform.py:5-18) when the
            # model is moved; host draws cannot be captured, so draw on the GPU
            model.q0.device = dev
        self.batch_size = int(batch_size)
        self.alpha = float(alpha)
        self.D = model.flows[0].num_input_channels
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.opt = torch.optim.Adam(self.params, lr=lr, weight_decay=weight_decay, capturable=True)
        # BatchNorm running buffers re-homed flat: the step's two passes share launches
        # (step_loss, autograd_flow.paired_kld); None keeps them separate
        self.flat_bn = AF.FlatBatchNorm.try_build(model) if paired else None
        # sticky spline-NaN word of the replays since the last reset_nan() (see the module doc)
        self._sticky = torch.zeros(1, dtype=torch.int32, device=dev)
        self._one = torch.ones((), device=dev)  # the captured backward's seed gradient
        model.train()
        self.graphs = {}
        for bs in [self.batch_size] + [int(b) for b in extra_batch_sizes if int(b) != self.batch_size]:
            ex = example if (example is not None and example.shape[0] == bs) else None
            self.graphs[bs] = self._capture(bs, ex, warmup, dev)
        main = self.graphs[self.batch_size]
        self.x, self.graph, self.loss, self.nan_flag = main.x, main.graph, main.loss, main.nan_flag

    def _capture(self, bs, example, warmup, dev):
        model = self.model
        x = torch.zeros((bs, self.D), device=dev) if example is None else example.clone().to(dev)
        # warm up on a side stream (allocator, hipBLASLt heuristics, Adam state), then put
        # the parameters, BatchNorm buffers and optimizer state back: capturing must not
        # change the model
        saved = [t.detach().clone() for t in list(model.parameters()) + list(model.buffers())]
        saved_opt = [v.detach().clone() for v in self._opt_tensors()] if self.opt.state else None
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        AF._last_paired = False
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._eager_step(x)
        torch.cuda.current_stream().wait_stream(s)
        # the shared-launch passes skip their deferred running-statistics update on the
        # sticky word themselves; any other path updates the BatchNorm buffers inside the
        # forward, so the graph snapshots them and puts them back after a NaN step
        paired = AF._last_paired and warmup > 0
        bn_bufs = [] if paired else self._bn_buffers()
        bn_backup = [b.detach().clone() for b in bn_bufs]
        with torch.no_grad():
            for t, v in zip(list(model.parameters()) + list(model.buffers()), saved):
                t.copy_(v)
            for j, v in enumerate(self._opt_tensors()):
                v.copy_(saved_opt[j]) if saved_opt else v.zero_()
        # snapshots of everything the optimizer step mutates: parameters and Adam state
        # live in a few flat buffers, so the skip-on-non-finite snapshot / restore is 4
        # copies + 4 selects instead of ~4 per parameter tensor (~8k graph nodes at A2)
        if not hasattr(self, "_state_tensors"):
            # parameters the step never reaches (the fork's unused preprocessing weights)
            # keep grad None and are skipped by Adam, as in the reference: leave them out
            used = [p for p in self.params if p.grad is not None]
            self.opt.param_groups[0]["params"] = used
            self.params = used
            self._state_tensors = self._flatten()
            # the snapshot buffers of torch's Adam path only (fs_adam_step skips by itself)
            self._backup = None if self._fused_adam_ok() else [t.detach().clone() for t in self._state_tensors]
        graph = torch.cuda.CUDAGraph()
        self._zero_grad()
        AF._defer_nan = True
        AF._sticky_nan = self._sticky
        try:
            with torch.cuda.graph(graph):  # own pool: graphs replay in any order
                with torch.no_grad():
                    for b, t in zip(bn_backup, bn_bufs):
                        b.copy_(t)
                self._zero_grad()
                loss = step_loss(model, x, self.batch_size, self.alpha, self.flat_bn)
                loss.backward(self._one)  # a constant seed gradient: no fill launch
                self._gather_grads()
                nan_flag, only_sticky = AF.reduce_nan_flags(dev)
                if not only_sticky:  # (the shared-launch passes wrote their flags into it)
                    with torch.no_grad():
                        self._sticky.bitwise_or_(nan_flag.to(torch.int32))
                if self._fused_adam_ok():
                    # skips itself on a non-finite loss or a set sticky word
                    self._adam_step(loss.detach(), skip=self._sticky)
                else:
                    keep = ~(torch.isnan(loss) | torch.isinf(loss)) & (self._sticky[0] == 0)
                    for b, t in zip(self._backup, self._state_tensors):
                        b.copy_(t.detach())
                    self.opt.step()
                    with torch.no_grad():
                        for b, t in zip(self._backup, self._state_tensors):
                            t.copy_(torch.where(keep, t, b))
                if bn_bufs:
                    with torch.no_grad():
                        failed = self._sticky[0] != 0
                        for b, t in zip(bn_backup, bn_bufs):
                            t.copy_(torch.where(failed, b, t))
        finally:
            AF._defer_nan = False
            AF._sticky_nan = None
        # keep no autograd graph alive; keep the snapshot buffers the replays write
        return _Captured(graph, x, loss.detach(), nan_flag, keep=bn_backup)

    def _bn_buffers(self):
        """The running-statistics buffers a training step updates."""
        if self.flat_bn is not None and self.flat_bn.intact():
            return self.flat_bn.buffers()
        return [t for m in self.model.modules() if isinstance(m, torch.nn.BatchNorm1d)
                for t in (m.running_mean, m.running_var, m.num_batches_tracked) if t is not None]

    def reset_nan(self):
        """Clear the sticky spline-NaN word (an epoch starts with it clear)."""
        self._sticky.zero_()

    def nan_state(self):
        """The sticky word as a device bool: some replay since reset_nan() hit a NaN."""
        return self._sticky[0] != 0

    def _fused_adam_ok(self):
        """fs_adam_step covers the reference's Adam: flat buffers, float lr, L2 weight decay,
        no amsgrad / maximize / differentiable, a float32 step count on the device."""
        if getattr(self, "_flat_grad", None) is None:
            return False
        g = self.opt.param_groups[0]
        st = self.opt.state.get(self._flat_param, {})
        step = st.get("step")
        if (g.get("amsgrad") or g.get("maximize") or g.get("differentiable") or g.get("decoupled_weight_decay")
                or torch.is_tensor(g["lr"]) or any(torch.is_tensor(b) for b in g["betas"])):
            return False
        # fs_adam_step's preconditions (capi.cpp); lr = 0 etc. keep torch's Adam
        b1, b2 = g["betas"]
        if not (g["lr"] > 0 and 0 <= b1 < 1 and 0 <= b2 < 1 and g["eps"] >= 0 and g["weight_decay"] >= 0):
            return False
        return (torch.is_tensor(step) and step.is_cuda and step.dtype == torch.float32 and "exp_avg" in st
                and "exp_avg_sq" in st)

    def _adam_step(self, loss=None, skip=None):
        """One Adam step over the flat buffers (fs_adam_step); loss (device scalar,
        nullable): nothing is written when it is NaN / inf; skip (int32 [1], nullable):
        nothing is written when it is non-zero."""
        from .. import _lib

        g = self.opt.param_groups[0]
        st = self.opt.state[self._flat_param]
        p = _lib.ptr
        b1, b2 = g["betas"]
        if loss is not None:
            loss = loss.reshape(1).to(torch.float32).contiguous()
        _lib.check(_lib.load().fs_adam_step(p(self._flat_param), p(self._flat_grad), p(st["exp_avg"]),
                                            p(st["exp_avg_sq"]), self._flat_param.numel(), p(st["step"]),
                                            p(loss), p(skip), float(g["lr"]), float(b1), float(b2), float(g["eps"]),
                                            float(g["weight_decay"]), _lib.stream_ptr()), "fs_adam_step")

    def _opt_tensors(self):
        return [v for st in self.opt.state.values() for v in st.values() if torch.is_tensor(v)]

    def _zero_grad(self):
        if getattr(self, "_flat_grad", None) is not None:
            for p in self.params:  # autograd hands each parameter its gradient buffer as is
                p.grad = None
        else:
            self.opt.zero_grad(set_to_none=False)

    def _gather_grads(self):
        """The parameters' gradients into the flat buffer Adam reads.  The backward kernels
        write them there directly (autograd_flow.register_grad_home: each p.grad is then a
        view of its own slice), so nothing is copied; otherwise one concatenation instead
        of one accumulate-add per parameter tensor."""
        if getattr(self, "_flat_grad", None) is None:
            return
        base = self._flat_grad.data_ptr()
        home = [p.grad is not None and p.grad.data_ptr() == base + 4 * o for p, o in zip(self.params, self._goffs)]
        if all(home):
            return
        if not any(home):
            gs = [p.grad.reshape(-1) if p.grad is not None else torch.zeros(p.numel(), device=p.device)
                  for p in self.params]
            torch.cat(gs, out=self._flat_grad)
            return
        # some gradients are their home slices already (torch.cat may not read its output):
        # copy only the others
        for p, o, h in zip(self.params, self._goffs, home):
            if h:
                continue
            dst = self._flat_grad[o:o + p.numel()]
            if p.grad is None:
                dst.zero_()
            else:
                dst.copy_(p.grad.reshape(-1))

    @torch.no_grad()
    def _flatten(self):
        """Re-home the parameters and the optimizer's state tensors as views of one flat
        buffer each (values unchanged); returns the buffers."""
        ps = self.params
        sizes = [p.numel() for p in ps]
        offs = [0]
        for n in sizes:
            offs.append(offs[-1] + n)
        flat = torch.cat([p.detach().reshape(-1) for p in ps])
        for p, o, n in zip(ps, offs, sizes):
            p.data = flat[o:o + n].view_as(p)
        # gradients: written into one flat buffer by the backward kernels, or gathered
        # there after each backward (_gather_grads)
        self._flat_grad = torch.zeros_like(flat)
        self._goffs = offs[:-1]
        AF.register_grad_home(flat, self._flat_grad)
        # Adam is elementwise, so one optimizer over the flat buffer is the same update as one
        # per parameter, in a handful of launches instead of a per-tensor fallback of
        # ~2 x (number of parameters) kernels: its state is the per-parameter state
        # concatenated (every used parameter has taken the same number of steps)
        state = {}
        for k, v0 in list(self.opt.state[ps[0]].items()):
            if not torch.is_tensor(v0):
                state[k] = v0
            elif v0.dim() == 0:  # capturable Adam's step count
                state[k] = v0.detach().clone()
            else:
                state[k] = torch.cat([self.opt.state[p][k].reshape(-1) for p in ps])
        self._flat_param = torch.nn.Parameter(flat)
        self._flat_param.grad = self._flat_grad
        known = inspect.signature(torch.optim.Adam.__init__).parameters
        group = {k: v for k, v in self.opt.param_groups[0].items() if k != "params" and k in known}
        self.opt = torch.optim.Adam([self._flat_param], **group)
        self.opt.state[self._flat_param] = state
        self.model.invalidate_packed()
        return [flat] + [v for v in state.values() if torch.is_tensor(v)]

    def add_batch_size(self, bs, warmup=3):
        """Capture one more batch size (warm-up steps are undone, as at construction)."""
        bs = int(bs)
        if bs not in self.graphs:
            self.graphs[bs] = self._capture(bs, None, warmup, next(self.model.parameters()).device)

    def reset_optimizer(self):
        """A fresh Adam (main_algorithm_2.py:437 builds one per cycle): moments and step
        counts zeroed in place, so the captured graph keeps its buffers."""
        with torch.no_grad():
            for b in self._state_tensors[1:]:
                b.zero_()

    def eager_step(self, batch):
        """One step on a batch of another size (the epoch's last, partial batch) with the
        same optimizer state, outside the graph; returns the loss tensor."""
        loss = self._eager_step(batch)
        self.model.invalidate_packed()
        return loss

    def _eager_step(self, x):
        self._zero_grad()
        loss = step_loss(self.model, x, self.batch_size, self.alpha, self.flat_bn)
        if bool(~(torch.isnan(loss) | torch.isinf(loss))):
            loss.backward()
            self._gather_grads()
            if self._fused_adam_ok():
                self._adam_step()
            else:
                self.opt.step()
        return loss.detach()

    def step(self, batch, check=True):
        """One training step on `batch` (B, D); returns the loss tensor (device scalar).
        A batch size without a captured graph runs eagerly with the same optimizer.
        check=False: no host synchronisation for the spline's NaN flag on a graphed batch
        size; the step returns (loss, nan_flag) instead, both device tensors owned by the
        caller, and the caller raises (an epoch checks all its steps' flags at once,
        Algorithm2.train).  The sticky word is not cleared then: after a NaN step every
        later replay writes nothing until reset_nan().  An ungraphed (eager) batch size
        synchronises either way: the eager step tests the loss on the host (the reference's
        skip of a non-finite loss) and reads the sticky word before it runs."""
        c = self.graphs.get(int(batch.shape[0]))
        if c is None:
            if not check and bool(self.nan_state()):
                # an earlier replay of this epoch hit a NaN: write nothing (the state stays
                # that of the last good step) and hand back the sticky flag
                return torch.full((), float("nan"), device=self._sticky.device), self.nan_state()
            loss = self.eager_step(batch)
            return loss if check else (loss, self.nan_state())
        if check:
            self.reset_nan()  # a NaN of an earlier checked step has raised already
        c.x.copy_(batch)
        c.graph.replay()
        self.model.invalidate_packed()  # replayed writes do not bump tensor versions
        if not check:
            return c.loss.clone(), c.nan_flag.clone()
        if bool(c.nan_flag):
            raise ValueError("Discriminant computation resulted in NaN.")  # splines.py:176-183
        return c.loss
