"""CPU-only checks of the product's host side: the C-ABI library loads and
exports every symbol of include/flowstate.h, layouts agree with the module
tree, state_dict compatibility with the reference key set.  No GPU compute."""
import os
import re

import numpy as np
import pytest
import torch

from flowstate import _lib
from flowstate.models import build_flow, half_box
from oracle import flow as OF

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(REPO, "include", "flowstate.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(fs_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    L = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), f"{s} declared in include/flowstate.h but not exported"
    assert set(syms) == set(_lib.EXPORTED), "ctypes signature table out of sync with the header"
    assert L.fs_version() >= 10000


@pytest.mark.parametrize("N,L,H,nb,K", [(4, 2, 32, 1, 5), (16, 3, 64, 2, 8), (64, 2, 256, 3, 32), (64, 1, 128, 2, 15)])
def test_raw_layout_matches_module_tree(N, L, H, nb, K):
    m = build_flow(N, L, H, nb, K)
    n_mod = sum(t.numel() for f in m.flows for t in f.raw_param_tensors())
    assert _lib.load().fs_flow_raw_floats(m.dims()) == n_mod
    assert _lib.load().fs_flow_packed_bytes(m.dims()) > 0


def test_unsupported_dims_fail_loudly():
    m = build_flow(16, 1, 96, 1, 8)
    assert _lib.load().fs_flow_raw_floats(m.dims()) == -1
    assert b"unsupported" in _lib.load().fs_last_error()


def test_state_dict_keys_match_reference():
    dims = OF.FlowDims(N=16, L=3, H=64, nb=2, K=8, B=OF.half_box(16))
    sd_ref_format = OF.random_state_dict(dims, seed=0)  # reference key set, pinned by goldens
    m = build_flow(16, 3, 64, 2, 8)
    ours = m.state_dict()
    assert set(ours) == set(sd_ref_format)
    for k in ours:
        assert ours[k].shape == sd_ref_format[k].shape and ours[k].dtype == sd_ref_format[k].dtype, k
    m.load_state_dict(sd_ref_format, strict=True)


def test_init_matches_reference_rng_order(golden_dir):
    f = np.load(os.path.join(golden_dir, "init.npz"))
    torch.manual_seed(int(f["seed"]))
    m = build_flow(int(f["N"]), int(f["L"]), int(f["H"]), int(f["nb"]), int(f["K"]))
    sd = m.state_dict()
    for k in f.files:
        if k.startswith("sd/"):
            np.testing.assert_array_equal(sd[k[3:]].numpy(), f[k])


def test_product_has_no_oracle_dependency():
    pkg = os.path.join(REPO, "flow-state_amd")
    for root, _, files in os.walk(pkg):
        for fn in files:
            if fn.endswith((".py", ".hip", ".cpp", ".h")):
                src = open(os.path.join(root, fn)).read()
                assert "import oracle" not in src and "from oracle" not in src, fn


def test_half_box():
    assert half_box(64) == pytest.approx(np.sqrt(64 / 0.03) / 2)


def test_abi_rejects_invalid_arguments_before_touching_the_device():
    """Argument checks of the C ABI run on the host: bad shapes / nulls return FS_EINVAL
    (-1) or FS_EUNSUPPORTED (-2) with a message, and never launch."""
    import ctypes

    from flowstate import _lib

    L = _lib.load()
    ph = _lib.Phys()
    one = ctypes.c_void_p(1)  # never dereferenced: validation fails first
    rc = L.fs_local_moves(ph, 4, 65, one, None, one, None, one, one, one, one, one, None, 10, 0, 0, 0.5, 0, None,
                          None, None, None, None)
    assert rc == -1 and b"N=65" in L.fs_last_error()
    rc = L.fs_local_moves(ph, 4, 16, one, None, one, None, one, one, one, one, one, None, 10, 0, 50, 0.5, 0, None,
                          None, None, None, None)
    assert rc == -1 and b"adjust_every" in L.fs_last_error()
    rc = L.fs_local_moves_if(None, ph, 4, 16, one, None, one, None, one, one, one, one, one, None, 10, 0, 0, 0.5, 0,
                             None, None, None, None, None)
    assert rc == -1 and b"gate" in L.fs_last_error()
    full = _lib.LocalChains(*([1] * 10))
    part = _lib.LocalChains(*([1] * 9 + [None]))
    rc = L.fs_chains_copy_if(one, 4, 3, ctypes.byref(full), ctypes.byref(part), None)
    assert rc == -1 and b"same optional arrays" in L.fs_last_error()
    rc = L.fs_chains_copy_if(one, 4, 3, ctypes.byref(_lib.LocalChains()), ctypes.byref(full), None)
    assert rc == -1 and b"missing arrays" in L.fs_last_error()
    rc = L.fs_rqs_forward(8, 7, 0, one, one, one, one, 3.0, one, one, None, None)
    assert rc == -1 and b"K=7" in L.fs_last_error()
    rc = L.fs_pair_hist(one, 1, 4, 300, 5.0, one, 10, one, None)
    assert rc == -1
    d = _lib.FlowDims(N=16, L=2, H=96, nb=1, K=8, precision=0, tail_bound=5.0)
    assert L.fs_flow_packed_bytes(d) == -1 and b"H=96" in L.fs_last_error()
    rc = L.fs_nf_mh_step(_lib.FlowDims(N=16, L=2, H=64, nb=1, K=8, precision=0, tail_bound=5.0), one, ph, 4, 0, 0, 0,
                         None, None, None, None, None, None, None, None, None, None, None, 0, one, None)
    assert rc == -1
    d64 = _lib.FlowDims(N=16, L=2, H=64, nb=1, K=8, precision=0, tail_bound=5.0)
    rc = L.fs_nf_mh_steps(d64, one, ph, 4, 2, 0, 0, 0, one, one, one, one, one, None, one, None, None, None, None,
                          _lib.FS_MH_HYBRID, one, None)
    assert rc == -1 and b"FS_MH_HYBRID" in L.fs_last_error()
    assert L.fs_nf_mh_steps_ws_bytes(d64, 4, 0) == -1
    # proposal bank: S >= 1, step index inside the bank, aligned buffers, hybrid needs state
    rc = L.fs_nf_mh_bank(d64, one, ph, 4, 0, 0, 0, 0, None, one, None)
    assert rc == -1 and b"fs_nf_mh_bank" in L.fs_last_error()
    aligned = ctypes.c_void_p(256)
    rc = L.fs_nf_mh_step_banked(d64, one, ph, 4, 2, 2, aligned, one, one, one, one, one, None, one, None, None, None,
                                None, 0, aligned, None)
    assert rc == -1 and b"fs_nf_mh_step_banked" in L.fs_last_error()
    rc = L.fs_nf_mh_step_banked(d64, one, ph, 4, 2, 1, aligned, one, one, one, one, None, None, one, None, None, None,
                                None, _lib.FS_MH_HYBRID, aligned, None)
    assert rc == -1
    rc = L.fs_nf_mh_step_banked(d64, one, ph, 4, 2, 1, one, one, one, one, one, one, None, one, None, None, None,
                                None, 0, aligned, None)
    assert rc == -1 and b"aligned" in L.fs_last_error()
    assert L.fs_nf_mh_banked_ws_bytes(d64, 4) > 0 and L.fs_nf_mh_banked_ws_bytes(d64, -1) == -1
    # training kernels
    rc = L.fs_linear_f32(-1, 4, 4, one, 4, 1, one, 1, 4, None, None, 0, one, 4, None, None)
    assert rc == -1 and b"fs_linear_f32" in L.fs_last_error()
    rc = L.fs_linear_f32(4, 8, 4, one, 4, 1, one, 1, 4, None, None, 0, one, 4, None, None)  # ldc < N
    assert rc == -1
    rc = L.fs_bn_relu_train_fwd(1, 8, one, one, one, None, None, None, 0.1, 1e-3, one, one, one, None)
    assert rc == -1  # a batch of one has no batch statistics (torch raises)
    c = _lib.Coupling(rows=4, D=16, K=7, hidden=64, identity_features=1, transform_features=1, tail_bound=3.0)
    rc = L.fs_coupling_features_fwd(ctypes.byref(c), one, one, None)
    assert rc == -1 and b"K=7" in L.fs_last_error()
    c = _lib.Coupling(rows=4, D=15, K=8, hidden=64, identity_features=1, transform_features=1, tail_bound=3.0)
    rc = L.fs_coupling_density_fwd(ctypes.byref(c), one, one, one, one, one, None, one, one, None)
    assert rc == -1 and b"coupling description" in L.fs_last_error()
    c = _lib.Coupling(rows=4, D=16, K=8, hidden=64, identity_features=1, transform_features=1, tail_bound=3.0)
    rc = L.fs_coupling_sample_pre(ctypes.byref(c), one, one, one, one, one, one, one, None, None)  # out aliases z
    assert rc == -1 and b"alias" in L.fs_last_error()


class _FakeDeviceTensor:
    """Stands in for a tensor on cuda:1 (this container has no GPU)."""

    is_cuda = True
    device = torch.device("cuda", 1)


def test_require_device_rejects_tensor_on_non_current_device(monkeypatch):
    """The library launches on the current device's stream and never switches device,
    so a tensor on another device must raise, not launch (flowstate._lib.require_device)."""
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 0)
    with pytest.raises(_lib.FlowStateError, match="current HIP device is cuda:0"):
        _lib.require_device(_FakeDeviceTensor())
    with pytest.raises(_lib.FlowStateError, match="CPU tensor"):
        _lib.require_device(torch.zeros(1))
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 1)
    _lib.require_device(_FakeDeviceTensor(), None)  # on the current device: accepted


def test_on_device_context():
    import contextlib
    assert isinstance(_lib.on_device(torch.zeros(1)), contextlib.nullcontext)
    assert isinstance(_lib.on_device(None), contextlib.nullcontext)
    assert isinstance(_lib.on_device("cuda"), contextlib.nullcontext)  # no index: stay on the current device
    assert isinstance(_lib.on_device(torch.device("cuda", 1)), torch.cuda.device)


def test_default_proposal_seed_contract():
    """Ranks of one job share one global proposal stream (same base seed, disjoint
    chain_offset); jobs with different master seeds get different streams."""
    from flowstate.MCMC.batched import default_proposal_seed
    C = 256
    s0 = default_proposal_seed(np.arange(42, 42 + C, dtype=np.uint64), 0)
    s1 = default_proposal_seed(np.arange(42 + C, 42 + 2 * C, dtype=np.uint64), C)
    assert s0 == s1
    other = default_proposal_seed(np.arange(1042, 1042 + C, dtype=np.uint64), 0)
    assert other != s0
    assert 0 <= s0 < 2 ** 63 and 0 <= other < 2 ** 63


def test_pack_cache_tracks_versions_and_structure():
    """The packed image's key (normflows/core.py _PackCache): in-place updates bump a
    tensor's version, re-assigned parameters / buffers bump the module-structure
    generation, so a cached tensor list is never stale (no device work here)."""
    from flowstate.normflows import core as C

    m = build_flow(4, 2, 32, 1, 5).eval()
    layers = list(m.flows)
    cache = C._PackCache()
    t0 = cache._tensor_list(layers)
    k0 = C._tensor_key(t0)
    assert cache._tensor_list(layers) is t0  # no walk while nothing was re-registered
    with torch.no_grad():
        layers[0].prqct.transform_net.final_layer.weight.add_(1.0)
    assert C._tensor_key(cache._tensor_list(layers)) != k0
    fl = layers[1].prqct.transform_net.final_layer
    fl.weight = torch.nn.Parameter(fl.weight.detach().clone())
    t1 = cache._tensor_list(layers)
    assert t1 is not t0 and any(t is fl.weight for t in t1)
    bn = layers[0].prqct.transform_net.blocks[0].batch_norm_layers[0]
    bn.running_mean = torch.zeros_like(bn.running_mean)
    assert any(t is bn.running_mean for t in cache._tensor_list(layers))


def test_device_spline_with_uninstantiated_bins_raises():
    """circular_rqs on a device tensor with a bin count the HIP spline does not instantiate
    raises instead of falling back to torch ops on the device (no silent
    fallback); CPU tensors take the torch restatement."""
    from flowstate.normflows import autograd_flow as AF

    class FakeDevice:  # stands for a device tensor (no GPU here): only is_cuda is read
        is_cuda = True

    uw, ud = torch.zeros(4, 10), torch.zeros(4, 11)
    with pytest.raises(_lib.FlowStateError, match="K=10"):
        AF.circular_rqs(FakeDevice(), uw, uw, ud, 3.0, False)
    x = torch.linspace(-2.0, 2.0, 4)
    out, lad = AF.circular_rqs(x, uw, uw, ud, 3.0, False)
    assert out.shape == x.shape and torch.isfinite(lad).all()


def test_column_split_xcd_placement_is_a_bijection():
    """wide_trunk16g_kernel's block -> (tile, workgroup) map with a tile's workgroups at equal
    blockIdx.x % 8 (FS_GSPLIT_XCD, flow_kernels.hip): over its grid of ceil(T/8)*8*G blocks
    every (tile < T, g < G) appears exactly once, the tile's G blocks share b % 8, and every
    other block is a slot past the last tile (it exits before any barrier or hand-off)."""
    G = 4
    for T in range(1, 33):
        grid = (T + 7) // 8 * 8 * G
        seen = {}
        idle = 0
        for b in range(grid):
            xb, yb = b & 7, b >> 3
            g, t = yb % G, (yb // G) * 8 + xb
            if t >= T:
                idle += 1
                continue
            assert (t, g) not in seen
            seen[(t, g)] = b
        assert len(seen) == T * G and idle == grid - T * G
        for t in range(T):
            assert len({seen[(t, g)] % 8 for g in range(G)}) == 1


def test_pipeline_schedule():
    """algorithm1.pipeline_schedule: every stage after the first runs ahead; an accept in
    big move j sends stage j+1 back to the main stream (its next stage runs ahead again from
    the redone one), so the kept stages are those after a big move no chain accepted."""
    from flowstate.algorithm1 import pipeline_schedule

    acc = torch.zeros((10, 8), dtype=torch.uint8)
    spec, redo = pipeline_schedule(acc)
    assert spec == [False] + [True] * 7 and redo == [False] * 8
    acc[3, 2] = 1
    spec, redo = pipeline_schedule(acc)
    assert redo == [False, False, False, True, False, False, False, False]
    assert spec == [False] + [True] * 7
    acc[:, :] = 1  # every big move accepts: every stage after the first runs again
    spec, redo = pipeline_schedule(acc)
    assert redo == [False] + [True] * 7
    assert pipeline_schedule(torch.zeros((4, 1), dtype=torch.uint8)) == ([False], [False])
    assert pipeline_schedule(torch.zeros((4, 0), dtype=torch.uint8)) == ([], [])
