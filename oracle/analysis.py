"""ORACLE (test infrastructure only): numpy restatement of the analysis reductions
of hybrid_NF_MCMC/utils.py — classify_particles (:104-141), the per-configuration
part of calculate_well_statistics (:61-101) and calculate_pair_correlation
(:530-574) — vectorised over configurations, with numpy 2's weak-Python-float
promotion written out explicitly (float32 arrays round every Python float to
float32 first).  Pinned to the reference's outputs in tests/golden/analysis.npz
(tests/test_oracle_analysis.py)."""
import numpy as np


def classify(cfg, halfbox, r0):
    """-> cls (M, N) int (0 A, 1 B, 2 outside), state (M,) (1 all-A, 2 all-B, 0), avg_x (M,)."""
    cfg = np.asarray(cfg)
    T = cfg.dtype.type
    box = halfbox * 2
    radius = r0 * 1.1
    bx = T(box)

    def inside(cx, cy):
        dx = cfg[..., 0] - T(cx)
        dy = cfg[..., 1] - T(cy)
        dx = dx - bx * np.round(dx / bx)
        dy = dy - bx * np.round(dy / bx)
        return (dx * dx + dy * dy) <= T(radius ** 2)

    a = inside(box / 4, box / 2)
    b = ~a & inside(3 * box / 4, box / 2)
    cls = np.where(a, 0, np.where(b, 1, 2))
    state = np.where(a.all(1), 1, np.where(b.all(1), 2, 0))
    avg_x = np.array([np.mean(c[:, 0]) for c in cfg])
    return cls, state, avg_x


def pair_counts(samples, bound, edges):
    """(M, nbins) pair-distance counts per configuration (utils.py:546-556)."""
    s = np.asarray(samples)
    T = s.dtype.type
    out = np.zeros((s.shape[0], len(edges) - 1), np.int64)
    tb = T(2 * bound)
    for m, p in enumerate(s):
        d = p[:, None, :] - p[None, :, :]
        d = d - tb * np.round(d / tb)
        r = np.sqrt(d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]).ravel()
        r = r[r != 0]
        out[m], _ = np.histogram(r, edges)
    return out


def rdf(samples, n_particles, bound, dr=None):
    if dr is None:
        dr = bound / 50
    edges = np.arange(0, bound + dr, dr)
    counts = pair_counts(samples, bound, edges)
    norm = n_particles * (n_particles - 1) / 2
    rou = n_particles / (4 * bound * bound)
    i_vals = np.arange(0, bound, dr)
    area = np.pi * ((i_vals + dr) ** 2 - i_vals ** 2)
    res = counts / (norm * rou * area)
    # pandas DataFrame.apply(np.mean, axis=0): per column, numpy pairwise sum / count
    return i_vals, np.array([np.sum(res[:, k]) / res.shape[0] for k in range(res.shape[1])])
