"""ctypes binding of libflowstate.so (include/flowstate.h).

This is the product's only route to compute: there is no CPU fallback.  If the
HIP library is missing (not built) or no HIP device is present, calls raise.
"""
import contextlib
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# FLOWSTATE_LIB: an alternative build of the same library (A/B kernel measurements)
LIB_PATH = os.environ.get("FLOWSTATE_LIB") or os.path.join(_HERE, "lib", "libflowstate.so")
_lib = None

FS_MH_CORRECT_SIGN = 1
FS_MH_HYBRID = 2
FS_MH_SINGLE_PASS = 4
FS_EUNSUPPORTED = -2  # include/flowstate.h


class FlowDims(ctypes.Structure):
    _fields_ = [("N", ctypes.c_int32), ("L", ctypes.c_int32), ("H", ctypes.c_int32), ("nb", ctypes.c_int32),
                ("K", ctypes.c_int32), ("precision", ctypes.c_int32), ("tail_bound", ctypes.c_double)]


class Phys(ctypes.Structure):
    _fields_ = [("Lx", ctypes.c_double), ("Ly", ctypes.c_double), ("V0", ctypes.c_double * 2),
                ("r0", ctypes.c_double), ("k", ctypes.c_double), ("num_wells", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("r_cut", ctypes.c_double), ("r_core", ctypes.c_double),
                ("beta", ctypes.c_double)]


class Coupling(ctypes.Structure):
    """fs_coupling (include/flowstate.h)."""
    _fields_ = [("rows", ctypes.c_int64), ("D", ctypes.c_int32), ("K", ctypes.c_int32), ("hidden", ctypes.c_int32),
                ("identity_features", ctypes.c_void_p), ("transform_features", ctypes.c_void_p),
                ("tail_bound", ctypes.c_double)]


class GemmF32(ctypes.Structure):
    """fs_gemm_f32 (include/flowstate.h): one fs_linear_f32 product."""
    _fields_ = [("M", ctypes.c_int64), ("N", ctypes.c_int64), ("K", ctypes.c_int64), ("A", ctypes.c_void_p),
                ("sam", ctypes.c_int64), ("sak", ctypes.c_int64), ("B", ctypes.c_void_p), ("sbk", ctypes.c_int64),
                ("sbn", ctypes.c_int64), ("bias", ctypes.c_void_p), ("R", ctypes.c_void_p), ("ldr", ctypes.c_int64),
                ("C", ctypes.c_void_p), ("ldc", ctypes.c_int64), ("rowsum_a", ctypes.c_void_p)]


class LocalChains(ctypes.Structure):
    """fs_local_chains (include/flowstate.h): the per-chain arrays of fs_local_moves."""
    _fields_ = [(k, ctypes.c_void_p) for k in ("state", "state_is_f32", "E", "W", "pcg", "pcg_buf", "max_disp",
                                               "attempts", "accepted", "prev_counts")]


class BnIn(ctypes.Structure):
    """fs_bn_in (include/flowstate.h): BatchNorm1d (train) + ReLU on fs_linear_f32_ex's A."""
    _fields_ = [("stats", ctypes.c_void_p), ("tiles", ctypes.c_int64), ("rows", ctypes.c_int64),
                ("gamma", ctypes.c_void_p), ("beta", ctypes.c_void_p), ("eps", ctypes.c_float),
                ("momentum", ctypes.c_float), ("running_mean", ctypes.c_void_p), ("running_var", ctypes.c_void_p),
                ("num_batches", ctypes.c_void_p), ("mean_out", ctypes.c_void_p), ("invstd_out", ctypes.c_void_p),
                ("a_out", ctypes.c_void_p), ("var_out", ctypes.c_void_p)]


class BnFold(ctypes.Structure):
    """fs_bn_fold (include/flowstate.h): a BatchNorm + ReLU backward folded into the
    backward pairs around it (fs_linear_f32_pair_bn)."""
    _fields_ = [("gu", ctypes.c_void_p), ("u", ctypes.c_void_p), ("y", ctypes.c_void_p), ("mean", ctypes.c_void_p),
                ("invstd", ctypes.c_void_p), ("gamma", ctypes.c_void_p), ("part", ctypes.c_void_p),
                ("dgamma", ctypes.c_void_p), ("dbeta", ctypes.c_void_p), ("dx_add", ctypes.c_void_p),
                ("a_out", ctypes.c_void_p), ("B", ctypes.c_int64), ("H", ctypes.c_int32)]


class FlowStateError(RuntimeError):
    pass


_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_CP = ctypes.POINTER(Coupling)
_D = ctypes.POINTER(FlowDims)
_PH = ctypes.POINTER(Phys)
_SIGS = {
    "fs_last_error": (ctypes.c_char_p, []),
    "fs_version": (ctypes.c_int, []),
    "fs_flow_raw_floats": (_I64, [_D]),
    "fs_gather_chunks": (ctypes.c_int, [_P, _I64, _P, _P]),
    "fs_flow_packed_bytes": (_I64, [_D]),
    "fs_flow_pack": (ctypes.c_int, [_D, _P, _P, _P]),
    "fs_flow_log_prob": (ctypes.c_int, [_D, _P, _P, _I64, _P, _P, _P, _P]),
    "fs_flow_inverse": (ctypes.c_int, [_D, _P, _P, _I64, _P, _P, _P, _P]),
    "fs_flow_forward": (ctypes.c_int, [_D, _P, _P, _I64, _P, _P, _P, _P]),
    "fs_flow_propose": (ctypes.c_int, [_D, _P, _I64, ctypes.c_uint64, ctypes.c_uint64, _I64, ctypes.c_double,
                                       _P, _P, _P, _P, _P]),
    "fs_flow_propose_lq": (ctypes.c_int, [_D, _P, _I64, ctypes.c_uint64, ctypes.c_uint64, _I64, ctypes.c_double]
                           + [_P] * 5 + [_P]),
    "fs_energy_lj_dw": (ctypes.c_int, [_PH, _P, ctypes.c_int, _I64, ctypes.c_int32, _P, _P, _P, _P, _P]),
    "fs_energy_state": (ctypes.c_int, [_PH, _P, _P, _I64, ctypes.c_int32, _P, _P, _P]),
    "fs_pcg64_seed": (ctypes.c_int, [_P, _I64, _P, _P]),
    "fs_pcg64_random": (ctypes.c_int, [_P, _I64, _P, _P]),
    "fs_min_image": (ctypes.c_int, [_PH, _P, _I64, _P, ctypes.c_int, _I64, _P, _P, _P]),
    "fs_particle_energy": (ctypes.c_int, [_PH, _P, ctypes.c_int, _I64, ctypes.c_int32, _P, _P, _P, _P]),
    "fs_metropolis_judge": (ctypes.c_int, [ctypes.c_double, _I64, _I64] + [_P] * 5 + [_P]),
    "fs_mh_accept": (ctypes.c_int, [_PH, _I64, ctypes.c_int32] + [_P] * 14 + [ctypes.c_int, _P]),
    "fs_nf_mh_step_ws_bytes": (_I64, [_D, _I64]),
    "fs_nf_mh_step": (ctypes.c_int, [_D, _P, _PH, _I64, ctypes.c_uint64, ctypes.c_uint64, _I64] + [_P] * 11
                      + [ctypes.c_int, _P, _P]),
    "fs_nf_mh_steps_ws_bytes": (_I64, [_D, _I64, _I64]),
    "fs_nf_mh_steps": (ctypes.c_int, [_D, _P, _PH, _I64, _I64, ctypes.c_uint64, ctypes.c_uint64, _I64] + [_P] * 11
                       + [ctypes.c_int, _P, _P]),
    "fs_nf_mh_bank": (ctypes.c_int, [_D, _P, _PH, _I64, _I64, ctypes.c_uint64, ctypes.c_uint64, _I64, _P, _P, _P]),
    "fs_nf_mh_banked_ws_bytes": (_I64, [_D, _I64]),
    "fs_nf_mh_step_banked": (ctypes.c_int, [_D, _P, _PH, _I64, _I64, _I64] + [_P] * 12 + [ctypes.c_int, _P, _P]),
    "fs_local_moves": (ctypes.c_int, [_PH, _I64, ctypes.c_int32] + [_P] * 10
                       + [_I64, _I64, ctypes.c_int32, ctypes.c_double, ctypes.c_int32] + [_P] * 5),
    "fs_local_moves_if": (ctypes.c_int, [_P, _PH, _I64, ctypes.c_int32] + [_P] * 10
                          + [_I64, _I64, ctypes.c_int32, ctypes.c_double, ctypes.c_int32] + [_P] * 5),
    "fs_chains_copy_if": (ctypes.c_int, [_P, _I64, ctypes.c_int32, ctypes.POINTER(LocalChains),
                                         ctypes.POINTER(LocalChains), _P]),
    "fs_local_samples_per_chain": (_I64, [_I64, _I64, ctypes.c_int32]),
    "fs_adjust_displacement": (ctypes.c_int, [_I64, _P, _P, _P, _P, ctypes.c_double, _P]),
    "fs_rqs_forward": (ctypes.c_int, [_I64, ctypes.c_int32, ctypes.c_int32] + [_P] * 4 + [ctypes.c_double]
                       + [_P] * 4),
    "fs_rqs_backward": (ctypes.c_int, [_I64, ctypes.c_int32, ctypes.c_int32] + [_P] * 4 + [ctypes.c_double]
                        + [_P] * 7),
    "fs_linear_f32": (ctypes.c_int, [_I64, _I64, _I64, _P, _I64, _I64, _P, _I64, _I64, _P, _P, _I64, _P, _I64,
                                     _P, _P]),
    "fs_linear_f32_pair": (ctypes.c_int, [ctypes.POINTER(GemmF32), ctypes.POINTER(GemmF32), _P]),
    "fs_linear_f32_pair_bn": (ctypes.c_int, [ctypes.POINTER(GemmF32), ctypes.POINTER(GemmF32),
                                             ctypes.POINTER(BnFold), ctypes.POINTER(BnFold), _P]),
    "fs_linear_f32_splitk_floats": (_I64, [ctypes.POINTER(GemmF32)]),
    "fs_linear_f32_splitk": (ctypes.c_int, [ctypes.POINTER(GemmF32), _P, _I64, _P]),
    "fs_linear_f32_ex": (ctypes.c_int, [ctypes.POINTER(GemmF32), ctypes.POINTER(BnIn), _P, _P]),
    "fs_linear_f32_ex2": (ctypes.c_int, [ctypes.POINTER(GemmF32), ctypes.POINTER(BnIn), _P, ctypes.POINTER(GemmF32),
                                         ctypes.POINTER(BnIn), _P, _P]),
    "fs_linear_f32_group": (ctypes.c_int, [ctypes.POINTER(ctypes.POINTER(GemmF32)), ctypes.c_int32, _P, _I64, _P]),
    "fs_bn_running_update": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, _P, _P, _P, _P, ctypes.c_int32, _I64, _I64,
                                            ctypes.c_double, _P, _P]),
    "fs_bn_relu_train_fwd": (ctypes.c_int, [_I64, ctypes.c_int32] + [_P] * 6 + [ctypes.c_double, ctypes.c_double]
                             + [_P] * 4),
    "fs_bn_relu_train_bwd": (ctypes.c_int, [_I64, ctypes.c_int32] + [_P] * 11),
    "fs_coupling_features_fwd": (ctypes.c_int, [_CP] + [_P] * 3),
    "fs_coupling_density_fwd": (ctypes.c_int, [_CP] + [_P] * 9),
    "fs_coupling_density_bwd": (ctypes.c_int, [_CP] + [_P] * 11),
    "fs_coupling_features_bwd": (ctypes.c_int, [_CP] + [_P] * 5),
    "fs_coupling_sample_pre": (ctypes.c_int, [_CP] + [_P] * 9),
    "fs_coupling_sample_post": (ctypes.c_int, [_CP] + [_P] * 7),
    "fs_coupling_pair_pre": (ctypes.c_int, [_CP] + [_P] * 8 + [_CP, _P, _P, _P]),
    "fs_coupling_bwd_step": (ctypes.c_int, [_CP] + [_P] * 4 + [_CP] + [_P] * 9 + [_P]),
    "fs_coupling_pair_step": (ctypes.c_int, [_CP] + [_P] * 6 + [_CP] + [_P] * 6 + [_CP] + [_P] * 8 + [_CP, _P, _P]),
    "fs_coupling_pair_post": (ctypes.c_int, [_CP] + [_P] * 6 + [_CP] + [_P] * 9),
    "fs_set_wide_rows": (_I64, [_I64]),
    "fs_set_wide_trunk16": (ctypes.c_int32, [ctypes.c_int32]),
    "fs_set_wide_final32": (ctypes.c_int32, [ctypes.c_int32]),
    "fs_set_wide_handoff_spins": (_I64, [_I64]),
    "fs_set_coupling_waves": (ctypes.c_int32, [ctypes.c_int32]),
    "fs_set_lean_gemm": (ctypes.c_int32, [ctypes.c_int32]),
    "fs_kld_loss": (ctypes.c_int, [_P, _I64, _P, _P, _I64, _P, _P, _P, _P]),
    "fs_kld_loss_backward": (ctypes.c_int, [_P, _I64, _P, _P]),
    "fs_linear_f32_pair_bn_sk": (ctypes.c_int, [ctypes.POINTER(GemmF32), ctypes.POINTER(GemmF32),
                                                 ctypes.POINTER(BnFold), ctypes.POINTER(BnFold), ctypes.c_int32, _I64,
                                                 ctypes.c_int32, _I64, _P]),
    "fs_linear_f32_group_partial": (ctypes.c_int, [ctypes.POINTER(ctypes.POINTER(GemmF32)), ctypes.c_int32, _P, _I64,
                                                   ctypes.c_int32, ctypes.POINTER(ctypes.c_int32), _P]),
    "fs_splitk_sum": (ctypes.c_int, [_P, ctypes.c_int32, _I64, _I64, _P, _P]),
    "fs_adam_step": (ctypes.c_int, [_P, _P, _P, _P, _I64, _P, _P, _P] + [ctypes.c_double] * 5 + [_P]),
    "fs_target_energy": (ctypes.c_int, [_P, _I64, ctypes.c_int32, ctypes.c_double, ctypes.c_double, ctypes.c_int32]
                         + [ctypes.c_double] * 4 + [_P, _P, _P]),
    "fs_classify_wells": (ctypes.c_int, [_P, ctypes.c_int, _I64, ctypes.c_int32, ctypes.c_double, ctypes.c_double,
                                          _P, _P, _P, _P]),
    "fs_pair_hist": (ctypes.c_int, [_P, ctypes.c_int, _I64, ctypes.c_int32, ctypes.c_double, _P, ctypes.c_int32,
                                    _P, _P]),
    "fs_rdf_mean": (ctypes.c_int, [_P, _I64, ctypes.c_int32, _P, _P, _P]),
    "fs_hist2d": (ctypes.c_int, [_P, _I64, ctypes.c_int32, ctypes.c_double, _P, ctypes.c_int32, _P, _P]),
    "fs_well_stats": (ctypes.c_int, [_P, _P, _I64, ctypes.c_int32, ctypes.c_double, ctypes.c_double, _P, _P]),
}
EXPORTED = tuple(_SIGS)


def load(path=None):
    """Load (once) and return the library with argtypes set."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise FlowStateError(
            f"libflowstate.so not found at {p}: build the HIP extension first "
            "(python -c 'import __graft_entry__ as g; g.build()' or make -C flow-state_amd/csrc)")
    L = ctypes.CDLL(p)
    for name, (res, args) in _SIGS.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if path is None:
        _lib = L
    return L


def check(rc, what=""):
    if rc != 0:
        msg = load().fs_last_error().decode(errors="replace")
        raise FlowStateError(f"{what} failed (rc={rc}): {msg}")


def require_device(*tensors):
    """Every tensor is on the CURRENT HIP device.  The library launches on the stream
    passed in (stream_ptr(): the current device's current stream) and never switches
    devices itself, so a tensor on another device would be a cross-device access and
    unordered against torch's work on that device.  Public entry points enter the
    device of their tensors first (on_device), so this only fires on a mixed call."""
    if not torch.cuda.is_available():
        raise FlowStateError("flowstate needs a HIP device (MI355X); none is visible")
    cur = None
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise FlowStateError("flowstate kernels take device tensors; got a CPU tensor")
        if cur is None:
            cur = torch.cuda.current_device()
        if t.device.index != cur:
            raise FlowStateError(
                f"tensor on {t.device} but the current HIP device is cuda:{cur}: flowstate launches on the "
                "current device's stream; use `with torch.cuda.device(...)` or torch.cuda.set_device()")


def on_device(where):
    """Context entering the HIP device of a tensor / torch.device (no-op for CPU or None)."""
    dev = where.device if torch.is_tensor(where) else (torch.device(where) if where is not None else None)
    if dev is None or dev.type != "cuda" or dev.index is None:
        return contextlib.nullcontext()
    return torch.cuda.device(dev)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def stream_ptr():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
