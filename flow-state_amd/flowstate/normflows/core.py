"""NormalizingFlow drop-in (reference: NF/normflows/core.py:10-230).

Same constructor and method names/semantics as the reference fork:
``forward`` / ``forward_and_log_det`` (sampling direction), ``inverse`` /
``inverse_and_log_det`` (density direction), ``log_prob`` (density direction +
UniformParticle base term), ``sample(n)`` returning the tensor only (the fork's
change, core.py:178-196), ``save`` / ``load``.  Every pass runs as ONE
libflowstate launch over the whole coupling stack (fs_flow_*), reading a packed
copy of the parameters that is rebuilt on the device whenever a parameter or
BatchNorm buffer changes (eval-mode BatchNorm is folded at pack time).

Training (forward_kld / reverse_kld, Algorithm 2) runs the same layers through
PyTorch autograd (autograd_flow.py) with train-mode BatchNorm, as the reference
does; the inference kernels then see the updated parameters.
"""
import torch
import torch.nn as nn

from .. import _lib
from .Energy import UniformParticle
from .flows import PRECISIONS


def _tensor_key(ts):
    # every in-place update bumps _version; .to() / .data = ... move data_ptr (UVA: pointers
    # of different devices never coincide)
    return tuple([t._version for t in ts]), tuple([t.data_ptr() for t in ts])


# Module-structure generation: bumped whenever any module registers (or re-assigns) a
# parameter, buffer or submodule, so the per-stack tensor list below is re-derived only
# then (walking the A1 stack's ~5.9k tensors costs milliseconds of host time per pass).
_STRUCT_GEN = [0]


def _bump_struct_gen(*_args):
    _STRUCT_GEN[0] += 1


nn.modules.module.register_module_parameter_registration_hook(_bump_struct_gen)
nn.modules.module.register_module_buffer_registration_hook(_bump_struct_gen)
nn.modules.module.register_module_module_registration_hook(_bump_struct_gen)


class _PackCache:
    """Device-resident packed parameter image of a list of identical-shape layers."""

    def __init__(self):
        self.key = None
        self.packed = None
        self.raw = None
        self._tensors = None
        self._struct = None

    def _tensor_list(self, layers):
        struct = (_STRUCT_GEN[0], tuple(map(id, layers)))
        if self._tensors is None or struct != self._struct:
            self._tensors = [t for layer in layers for t in layer.raw_param_tensors()]
            self._struct = struct
        return self._tensors

    def get(self, layers):
        tensors = self._tensor_list(layers)
        dims = layers[0].dims(L=len(layers))
        key = (_tensor_key(tensors), int(dims.precision))
        if key == self.key:
            return self.packed
        dev = tensors[0].device
        with _lib.on_device(dev):
            return self._pack(tensors, dims, key, dev)

    _CHUNK = 8192

    def _gather(self, tensors, ptrs, nraw, dev):
        """The raw image in one fs_gather_chunks launch, its chunk table rebuilt only when a
        tensor moved (ptrs: the key's data pointers); None (torch.cat instead) unless every
        tensor is contiguous float32 and they add up to nraw."""
        if getattr(self, "_tab_ptrs", None) != ptrs:
            self._tab, self._tab_ptrs = None, ptrs
            if all(t.dtype == torch.float32 and t.is_contiguous() for t in tensors) and \
                    sum(t.numel() for t in tensors) == nraw:
                rows, off = [], 0
                for t in tensors:
                    n, a = t.numel(), t.data_ptr()
                    for s in range(0, n, self._CHUNK):
                        rows.append((a + 4 * s, off + s, min(self._CHUNK, n - s)))
                    off += n
                self._tab = torch.tensor(rows, dtype=torch.int64).to(dev)
        if self._tab is None:
            return None
        raw = torch.empty(nraw, dtype=torch.float32, device=dev)
        L = _lib.load()
        _lib.check(L.fs_gather_chunks(_lib.ptr(self._tab), self._tab.shape[0], _lib.ptr(raw), _lib.stream_ptr()),
                   "fs_gather_chunks")
        return raw

    def _pack(self, tensors, dims, key, dev):
        _lib.require_device(*tensors)
        L = _lib.load()
        nraw = L.fs_flow_raw_floats(dims)
        nbytes = L.fs_flow_packed_bytes(dims)
        if nraw < 0 or nbytes < 0:
            _lib.check(-1, "flow dims")
        raw = self._gather(tensors, key[0][1], nraw, dev)
        if raw is None:
            with torch.no_grad():
                raw = torch.cat([t.detach().reshape(-1).to(torch.float32) for t in tensors])
        if raw.numel() != nraw:
            raise _lib.FlowStateError(f"raw parameter count {raw.numel()} != expected {nraw}")
        packed = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=dev)
        _lib.check(L.fs_flow_pack(dims, _lib.ptr(raw), _lib.ptr(packed), _lib.stream_ptr()), "fs_flow_pack")
        self.raw, self.packed, self.key = raw, packed, key
        return packed


def _check_stack(layers):
    if not layers:
        raise ValueError("empty flow stack")
    for l in layers[1:]:
        if not layers[0].same_shape(l):
            raise _lib.FlowStateError("all coupling layers of a stack must share hyper-parameters")
    for l in layers:
        if l.training and any(m.training for m in l.modules() if isinstance(m, nn.BatchNorm1d)):
            raise _lib.FlowStateError(
                "flowstate runs the flow in eval mode (BatchNorm running statistics, as the reference's "
                "hot path does after model.eval(), main_algorithm_1.py:331); call .eval() first")


def _prepare_input(x, D):
    _lib.require_device(x)
    if x.dim() != 2 or x.shape[1] != D:
        raise ValueError(f"Expected input of shape (B, {D}), got {tuple(x.shape)}")
    return x.detach().to(torch.float32).contiguous()


def _raise_on_nan(err):
    if int(err.item()) & 1:
        raise ValueError("Discriminant computation resulted in NaN.")  # splines.py:176-183


# A pass of at most this many rows may run its A1 trunk on the column-split kernel, whose
# in-launch hand-offs report a wait that gave up as err |= 4 (fs_set_wide_trunk16).
_GSPLIT_MAX_ROWS = 512


def _run_stack(layers, x, direction, cache=None, base_log_prob=None, err=None):
    """Run the coupling stack in one launch.  direction: 'forward' (sampling,
    layers 0..L-1) or 'inverse' (density, layers L-1..0).  Returns (out, log_det).
    Runs on x's device (its current stream); the parameters must live there too.
    err: the caller's sticky device int32 error word (density direction only), checked by
    the caller later (BatchedMonteCarlo.check_errors); without it the pass checks its own."""
    with _lib.on_device(x):
        return _run_stack_here(layers, x, direction, cache, base_log_prob, err)


def _launch_stack(L, dims, packed, x, B, out, ld, err, direction, base_log_prob):
    st = _lib.stream_ptr()
    e = None if err is None else _lib.ptr(err)
    if direction == "forward":
        _lib.check(L.fs_flow_forward(dims, _lib.ptr(packed), _lib.ptr(x), B, _lib.ptr(out), _lib.ptr(ld), e, st),
                   "fs_flow_forward")
    elif base_log_prob:
        _lib.check(L.fs_flow_log_prob(dims, _lib.ptr(packed), _lib.ptr(x), B, _lib.ptr(ld), _lib.ptr(out), e, st),
                   "fs_flow_log_prob")
    else:
        _lib.check(L.fs_flow_inverse(dims, _lib.ptr(packed), _lib.ptr(x), B, _lib.ptr(out), _lib.ptr(ld), e, st),
                   "fs_flow_inverse")


def _run_stack_here(layers, x, direction, cache, base_log_prob, err=None):
    _check_stack(layers)
    cache = cache or getattr(layers[0], "_fs_cache", None)
    if cache is None:
        cache = _PackCache()
        layers[0]._fs_cache = cache
    D = layers[0].num_input_channels
    x = _prepare_input(x, D)
    packed = cache.get(layers)
    _lib.require_device(packed)
    dims = layers[0].dims(L=len(layers))
    B = x.shape[0]
    out = torch.empty_like(x)
    ld = torch.empty(B, dtype=torch.float32, device=x.device)
    L = _lib.load()
    if err is not None:
        if direction == "forward":
            raise ValueError("a sticky err word is for the density direction")
        _launch_stack(L, dims, packed, x, B, out, ld, err, direction, base_log_prob)
        return out, ld
    own = torch.zeros(1, dtype=torch.int32, device=x.device)
    _launch_stack(L, dims, packed, x, B, out, ld, own, direction, base_log_prob)
    if direction == "forward":
        if int(own.item()) & 4:  # a column-split hand-off gave up: the same pass on trunk 3
            # (fs_set_wide_trunk16 is process-wide: a pass another thread launches meanwhile
            # may take trunk 3 too, with the same results; every trunk is bit-identical)
            own.zero_()
            prev = L.fs_set_wide_trunk16(3)
            try:
                _launch_stack(L, dims, packed, x, B, out, ld, own, direction, base_log_prob)
            finally:
                L.fs_set_wide_trunk16(prev)
        _raise_on_nan(own)
    elif B <= _GSPLIT_MAX_ROWS and int(own.item()) & 4:
        # (no NaN check in this direction: the density pass solves no root) a column-split
        # hand-off gave up waiting, so these outputs are wrong: re-run without an err word,
        # which never takes the column-split trunk (bit-identical results)
        _launch_stack(L, dims, packed, x, B, out, ld, None, direction, base_log_prob)
    return out, ld


class NormalizingFlow(nn.Module):
    """Normalizing flow (core.py:10-230) over CircularCoupledRationalQuadraticSpline layers."""

    def __init__(self, q0, flows, p=None):
        super().__init__()
        self.q0 = q0
        self.flows = nn.ModuleList(flows)
        self.p = p
        self._cache = _PackCache()

    def _layers(self):
        return list(self.flows)

    def _base_check(self):
        if not isinstance(self.q0, UniformParticle):
            raise NotImplementedError("the fused base density is UniformParticle (main_algorithm_1.py:277)")
        b = float(self.q0.bound)
        if any(abs(f.tail_bound - b) > 0 for f in self.flows):
            raise NotImplementedError("q0.bound must equal the layers' tail_bound (main_algorithm_1.py:276-283)")

    def set_precision(self, precision="f32"):
        """Arithmetic of the conditioner GEMMs in the fused passes (flows.PRECISIONS):
        "f32" (default: the reference's float32, exact-f32 MFMA products), "bf16x6" or
        "bf16x3" (f32 operands split into bf16 planes on the bf16 matrix cores, DESIGN.md
        'Precision modes').  The spline, base density and everything outside the
        conditioner GEMMs are unchanged.  Returns self."""
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(PRECISIONS)}, got {precision!r}")
        for f in self.flows:
            f._fs_precision = precision
            if getattr(f, "_fs_cache", None) is not None:
                f._fs_cache.key = None
        self.invalidate_packed()
        return self

    @property
    def precision(self):
        return getattr(self.flows[0], "_fs_precision", "f32")

    def packed(self):
        """Device packed parameter image (rebuilt when parameters/buffers change)."""
        return self._cache.get(self._layers())

    def invalidate_packed(self):
        """Force a repack on the next pass: for writes that bypass the tensor version
        counters (HIP-graph replays of a training step, train.GraphedTrainStep)."""
        self._cache.key = None

    def dims(self):
        return self.flows[0].dims(L=len(self.flows))

    @torch.no_grad()
    def forward(self, z):
        """core.py:28-39: latent z -> x (sampling direction)."""
        return _run_stack(self._layers(), z, "forward", self._cache)[0]

    @torch.no_grad()
    def forward_and_log_det(self, z):
        """core.py:41-56."""
        return _run_stack(self._layers(), z, "forward", self._cache)

    @torch.no_grad()
    def inverse(self, x):
        """core.py:58-69: x -> latent z (density direction)."""
        return _run_stack(self._layers(), x, "inverse", self._cache)[0]

    @torch.no_grad()
    def inverse_and_log_det(self, x):
        """core.py:71-86."""
        return _run_stack(self._layers(), x, "inverse", self._cache)

    @torch.no_grad()
    def log_prob(self, x):
        """core.py:198-214: sum of layer log-dets + UniformParticle.log_prob, in x.dtype."""
        return self._log_prob(x)

    @torch.no_grad()
    def _log_prob(self, x, err=None):
        """log_prob; err: the caller's sticky device int32 error word (a column-split
        hand-off timeout is then reported there, |= 4, instead of re-run here)."""
        self._base_check()
        _, lq = _run_stack(self._layers(), x, "inverse", self._cache, base_log_prob=True, err=err)
        return lq.to(x.dtype)

    def frozen_log_prob(self):
        """log_prob over the flow as it is now, for a caller that holds the weights fixed over
        many passes (the Algorithm-1 testing phase's density passes): the structure, eval-mode
        and parameter-version checks a pass makes (~1 ms of host time per pass on the A1 flow,
        thousands of tensors and modules) run once here, and the returned function
        run(x, err) launches the same density pass over the packed image taken now
        (bit-identical to _log_prob(x, err)).  err: the caller's sticky device int32 error
        word, required (a column-split hand-off timeout is reported there)."""
        self._base_check()
        layers = self._layers()
        _check_stack(layers)
        packed = self._cache.get(layers)
        _lib.require_device(packed)
        dims = layers[0].dims(L=len(layers))
        D = layers[0].num_input_channels
        L = _lib.load()

        @torch.no_grad()
        def run(x, err):
            if err is None:
                raise ValueError("frozen_log_prob: err is required")
            xin = _prepare_input(x, D)
            B = xin.shape[0]
            out = torch.empty_like(xin)
            ld = torch.empty(B, dtype=torch.float32, device=xin.device)
            with _lib.on_device(xin):
                _launch_stack(L, dims, packed, xin, B, out, ld, err, "inverse", True)
            return ld.to(x.dtype)

        return run

    @torch.no_grad()
    def sample(self, num_samples=1):
        """core.py:178-196 (fork): returns the samples only."""
        z = self.q0(num_samples)
        dev = next(self.parameters()).device
        return self.forward(z.to(dev))

    def forward_kld(self, x):
        """core.py:88-103 (fork: no base term): -mean of the summed density-direction
        log-dets, differentiable, BatchNorm in the module's current mode."""
        from . import autograd_flow as AF

        log_q = None  # zeros (core.py:96); the first fused layer starts from 0
        z = x
        with _lib.on_device(x):  # the HIP kernels launch on the current device's stream
            for i in range(len(self.flows) - 1, -1, -1):
                if AF.fused_coupling_ok(self.flows[i], z):
                    z, log_q = AF.density_step(self.flows[i], z, log_q)
                else:
                    if log_q is None:
                        log_q = torch.zeros(len(x), device=x.device)
                    z, log_det = AF.coupling_density(self.flows[i], z)
                    log_q = log_q + log_det
        AF.check_nan_flags()
        if log_q is None:
            log_q = torch.zeros(len(x), device=x.device)
        return -torch.mean(log_q)

    def reverse_kld(self, num_samples=1, beta=1.0, score_fn=True):
        """core.py:105-142 (fork): base draws -> sampling direction -> mean(target
        energy) + mean(log q); returns (loss, samples)."""
        z = self.q0(num_samples).to(next(self.parameters()).device)
        return self._reverse_kld_from(z, score_fn)

    def _reverse_kld_from(self, z, score_fn=True):
        from . import autograd_flow as AF

        log_q = None  # zeros (core.py:118); the first fused layer starts from 0
        grads = torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
        nan_flag = None
        with _lib.on_device(z):
            for flow in self.flows:
                if not grads and AF.fused_coupling_ok(flow, z):
                    if nan_flag is None:
                        nan_flag = torch.zeros(1, dtype=torch.int32, device=z.device)
                    z, log_q = AF.sample_step(flow, z, log_q, nan_flag)
                else:
                    if log_q is None:
                        log_q = torch.zeros(len(z), device=z.device)
                    z, log_det = AF.coupling_sample(flow, z)
                    log_q = log_q - log_det
        if nan_flag is not None:
            AF._nan_flags.append(nan_flag[0] != 0)
        if log_q is None:
            log_q = torch.zeros(len(z), device=z.device)
        if not score_fn:
            z_ = z
            log_q = torch.zeros(len(z_), device=z_.device)
            req = [p.requires_grad for p in self.parameters()]
            for p in self.parameters():
                p.requires_grad_(False)
            for i in range(len(self.flows) - 1, -1, -1):
                z_, log_det = AF.coupling_density(self.flows[i], z_)
                log_q += log_det
            log_q += self.q0.log_prob(z_)
            for p, r in zip(self.parameters(), req):
                p.requires_grad_(r)
        AF.check_nan_flags()
        energy = self.p._energy(z)
        return torch.mean(energy) + torch.mean(log_q), z

    def save(self, path):
        torch.save(self.state_dict(), path)

    def load(self, path):
        self.load_state_dict(torch.load(path, weights_only=True))
