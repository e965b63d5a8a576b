"""Analysis reductions of the Algorithm-1 driver (hybrid_NF_MCMC/utils.py), drop-in
signatures, computed by the HIP kernels of csrc/analysis_kernels.hip:

  classify_particles(positions, halfbox, r0)                       utils.py:104-141
  calculate_well_statistics(configurations, start_idx, half_box, r0)  utils.py:61-101
  calculate_pair_correlation(final_samples, n_particles, bound, dr)   utils.py:530-574
  generate_samples(model, n_particles, n_dimension, ...)            utils.py:422-450

Inputs are numpy arrays or device tensors; float32 and float64 inputs keep
numpy's dtype semantics (the kernels reproduce numpy 2's weak-Python-float
promotion).  The host side only does the per-configuration bookkeeping of the
reference's Python loops (running counts, p = count / i) on the device results.
"""
import numpy as np
import torch

from . import _lib

_CLASS_NAMES = np.array(["A", "B", "Outside"])


def _device_array(a):
    """(M, N, 2) float32/float64 device tensor from numpy / torch input."""
    t = torch.as_tensor(a)
    if t.dtype not in (torch.float32, torch.float64):
        t = t.to(torch.float64)
    if t.dim() == 2:
        t = t[None]
    t = t.to("cuda").contiguous()
    _lib.require_device(t)
    return t


def classify_wells(positions, halfbox, r0):
    """Device results: cls (M, N) u8 (0 A, 1 B, 2 outside), state (M,) u8
    (1 all-in-A, 2 all-in-B), avg_x (M,) f64 (np.mean of the x column)."""
    pos = _device_array(positions)
    M, N, _ = pos.shape
    cls = torch.empty((M, N), dtype=torch.uint8, device=pos.device)
    state = torch.empty(M, dtype=torch.uint8, device=pos.device)
    avg_x = torch.empty(M, dtype=torch.float64, device=pos.device)
    _lib.check(_lib.load().fs_classify_wells(_lib.ptr(pos), int(pos.dtype == torch.float32), M, N, float(halfbox),
                                             float(r0), _lib.ptr(cls), _lib.ptr(state), _lib.ptr(avg_x),
                                             _lib.stream_ptr()), "fs_classify_wells")
    return cls, state, avg_x


def classify_particles(positions, halfbox, r0):
    """utils.py:104-141: array of 'A' / 'B' / 'Outside' per particle, shape (M, N)."""
    cls, _, _ = classify_wells(positions, halfbox, r0)
    return _CLASS_NAMES[cls.cpu().numpy()]


def calculate_well_statistics(configurations, start_idx, half_box, r0=1.2):
    """utils.py:61-101: (avg_x_values, p_a_values, p_b_values, deltaF_normalized_values, runs)."""
    _, state, avg_x = classify_wells(configurations, half_box, r0)
    state = state.cpu().numpy()
    avg_x = avg_x.cpu().numpy()
    f32 = torch.as_tensor(configurations).dtype == torch.float32
    count_left = count_right = 0
    avg_x_values, p_a_values, p_b_values, deltaF, runs = [], [], [], [], []
    for i, s in enumerate(state[start_idx:], start=1):
        avg_x_values.append(np.float32(avg_x[start_idx + i - 1]) if f32 else np.float64(avg_x[start_idx + i - 1]))
        if s == 1:
            count_left += 1
        elif s == 2:
            count_right += 1
        p_a = count_left / i
        p_b = count_right / i
        p_a_values.append(p_a)
        p_b_values.append(p_b)
        deltaF.append(np.log(p_b / p_a) if (p_a > 0 and p_b > 0) else 0)
        runs.append(i)
    return avg_x_values, p_a_values, p_b_values, deltaF, runs


def pair_histograms(final_samples, bound, edges):
    """Per-configuration pair-distance counts (M, nbins) int32 on the device."""
    pos = _device_array(final_samples)
    M, N, _ = pos.shape
    e = torch.as_tensor(np.asarray(edges, np.float64), device=pos.device)
    nb = e.numel() - 1
    counts = torch.empty((M, nb), dtype=torch.int32, device=pos.device)
    _lib.check(_lib.load().fs_pair_hist(_lib.ptr(pos), int(pos.dtype == torch.float32), M, N, float(bound),
                                        _lib.ptr(e), nb, _lib.ptr(counts), _lib.stream_ptr()), "fs_pair_hist")
    return counts


def calculate_pair_correlation(final_samples, n_particles, bound, dr=None):
    """utils.py:530-574: (r_vals, g_r) with g_r a pandas Series, as the reference returns."""
    import pandas as pd

    if dr is None:
        dr = bound / 50
    edges = np.arange(0, bound + dr, dr)
    counts = pair_histograms(final_samples, bound, edges)
    norm = n_particles * (n_particles - 1) / 2
    rou = n_particles / (4 * bound * bound)
    i_vals = np.arange(0, bound, dr)
    area = np.pi * ((i_vals + dr) ** 2 - i_vals ** 2)
    denom = norm * rou * area
    if denom.shape[0] != counts.shape[1]:
        raise ValueError(f"operands could not be broadcast together with shapes ({counts.shape[1]},) ({denom.shape[0]},)")
    d = torch.as_tensor(denom, device=counts.device)
    g = torch.empty(denom.shape[0], dtype=torch.float64, device=counts.device)
    _lib.check(_lib.load().fs_rdf_mean(_lib.ptr(counts), counts.shape[0], counts.shape[1], _lib.ptr(d), _lib.ptr(g),
                                       _lib.stream_ptr()), "fs_rdf_mean")
    return np.arange(0, bound, dr), pd.Series(g.cpu().numpy())


def generate_samples(model, n_particles, n_dimension, n_iterations=100, samples_per_iteration=5000,
                     device_output=False):
    """utils.py:422-450: n_iterations x model.sample(samples_per_iteration) reshaped to
    (n, n_particles, n_dimension).  device_output=True keeps the proposals on the GPU
    (one (n, N, d) float32 tensor) instead of the reference's numpy copy."""
    model.eval()
    out = []
    with torch.no_grad():
        for _ in range(n_iterations):
            z = model.sample(samples_per_iteration)
            out.append(z.reshape(-1, n_particles, n_dimension))
    if device_output:
        return torch.cat(out, 0)
    return np.concatenate([t.cpu().numpy() for t in out], axis=0)
