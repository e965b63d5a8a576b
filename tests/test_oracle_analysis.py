"""The numpy analysis oracle against the reference's own outputs
(tests/golden/analysis.npz from hybrid_NF_MCMC/utils.py)."""
import os

import numpy as np
import pytest

from oracle import analysis as OA

G = os.path.join(os.path.dirname(__file__), "golden")
NAMES = np.array(["A", "B", "Outside"])


@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_classify_and_well_statistics(dt):
    f = np.load(os.path.join(G, "analysis.npz"))
    cls, state, avg_x = OA.classify(f[f"{dt}_cfg"], float(f["half_box"]), 1.2)
    np.testing.assert_array_equal(NAMES[cls], f[f"{dt}_cls"])
    np.testing.assert_array_equal(avg_x[3:], f[f"{dt}_avg_x"])
    assert avg_x.dtype == (np.float32 if dt == "f32" else np.float64)
    # cumulative probabilities from the per-configuration states, start_idx = 3
    a = np.cumsum(state[3:] == 1) / np.arange(1, len(state) - 2)
    b = np.cumsum(state[3:] == 2) / np.arange(1, len(state) - 2)
    np.testing.assert_array_equal(a, f[f"{dt}_p_a"])
    np.testing.assert_array_equal(b, f[f"{dt}_p_b"])


def test_pair_correlation():
    f = np.load(os.path.join(G, "analysis.npz"))
    hb = float(f["half_box"])
    r, g = OA.rdf(f["rdf_samples"], 16, hb, dr=hb / 50)
    np.testing.assert_array_equal(r, f["rdf_r"])
    np.testing.assert_array_equal(g, f["rdf_g"])
    r, g = OA.rdf(f["rdf_samples"].astype(np.float64)[:40], 16, hb, dr=hb / 30)
    np.testing.assert_array_equal(g, f["rdf64_g"])
