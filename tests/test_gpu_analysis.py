"""GPU parity of the analysis reductions (fs_classify_wells, fs_pair_hist,
fs_rdf_mean) against the reference's own outputs (tests/golden/analysis.npz) and,
at larger sizes, against the pinned numpy oracle."""
import os

import numpy as np
import pytest

from flowstate import analysis as A
from oracle import analysis as OA

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_well_statistics_match_reference(dt):
    f = np.load(os.path.join(G, "analysis.npz"))
    cfg, hb = f[f"{dt}_cfg"], float(f["half_box"])
    np.testing.assert_array_equal(A.classify_particles(cfg, hb, 1.2), f[f"{dt}_cls"])
    ax, pa, pb, dF, runs = A.calculate_well_statistics(cfg, 3, hb, 1.2)
    np.testing.assert_array_equal(np.array(ax), f[f"{dt}_avg_x"])
    assert (np.asarray(ax).dtype == np.float32) == bool(f[f"{dt}_avg_x_dtype32"])
    np.testing.assert_array_equal(np.array(pa), f[f"{dt}_p_a"])
    np.testing.assert_array_equal(np.array(pb), f[f"{dt}_p_b"])
    np.testing.assert_array_equal(np.array(dF, np.float64), f[f"{dt}_dF"])
    np.testing.assert_array_equal(np.array(runs), f[f"{dt}_runs"])


def test_pair_correlation_matches_reference():
    f = np.load(os.path.join(G, "analysis.npz"))
    hb = float(f["half_box"])
    r, g = A.calculate_pair_correlation(f["rdf_samples"], 16, hb, dr=hb / 50)
    np.testing.assert_array_equal(r, f["rdf_r"])
    np.testing.assert_array_equal(g.to_numpy(), f["rdf_g"])
    r, g = A.calculate_pair_correlation(f["rdf_samples"].astype(np.float64)[:40], 16, hb, dr=hb / 30)
    np.testing.assert_array_equal(g.to_numpy(), f["rdf64_g"])


@pytest.mark.parametrize("N,M", [(64, 3000), (5, 1000)])
def test_analysis_matches_oracle_at_size(N, M):
    """Larger sets (M > 128 exercises the recursive pairwise mean) against the oracle."""
    hb = ((N / 0.03) ** 0.5) / 2
    rng = np.random.default_rng(N)
    cfg = (rng.random((M, N, 2)) * 2 * hb).astype(np.float32)
    cfg[::7, :, 0] = (hb / 2 + rng.normal(0, 0.3, (len(cfg[::7]), N))).astype(np.float32)
    cfg[::7, :, 1] = (hb + rng.normal(0, 0.3, (len(cfg[::7]), N))).astype(np.float32)
    cls, state, avg_x = A.classify_wells(cfg, hb, 1.2)
    c_o, s_o, a_o = OA.classify(cfg, hb, 1.2)
    np.testing.assert_array_equal(cls.cpu().numpy(), c_o)
    np.testing.assert_array_equal(state.cpu().numpy(), s_o)
    np.testing.assert_array_equal(avg_x.cpu().numpy().astype(np.float32), a_o)
    cen = cfg - np.float32(hb)
    r, g = A.calculate_pair_correlation(cen, N, hb)
    r_o, g_o = OA.rdf(cen, N, hb)
    np.testing.assert_array_equal(g.to_numpy(), g_o)
