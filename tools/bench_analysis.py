"""Analysis-row kernels at the bench's scale: 65536 configurations of
N=64 (float32, flow-proposal-like): classify_wells (utils.py:104-141 / 61-101), the
pair-distance histogram of calculate_pair_correlation (utils.py:530-574, 50 bins), the
density histogram2d (utils.py:488-495, 99x99) and the per-chain well counters.  Reports
ms per launch, configurations/s and the algorithmic HBM rate (positions in + results out)
against the 8 TB/s HBM peak, plus pair terms/s for the O(N^2) pair histogram."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flow-state_amd"))
sys.path.insert(0, REPO)
from flowstate import analysis as A  # noqa: E402
from flowstate.MCMC import BatchedMonteCarlo, Physics  # noqa: E402
from bench import synthetic_states  # noqa: E402

N, M = 64, 65536
init, L = synthetic_states(N, M, 0)
B = L / 2
pos32 = torch.from_numpy(init.astype(np.float32)).cuda()
bmc = BatchedMonteCarlo(None, init, Physics(L, L), np.arange(42, 42 + M, dtype=np.uint64))


def timeit(f, reps=5):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return min(ts)


edges = np.arange(0, B + B / 50, B / 50)
cases = {
    "classify_wells": (lambda: A.classify_wells(pos32, B, 1.2), M * N * 8 + M * N + M * 9),
    "pair_hist_50bins": (lambda: A.pair_histograms(pos32, B, edges), M * N * 8 + M * 50 * 4),
    "hist2d_99x99": (lambda: bmc.histogram2d(100), M * N * 16 + 99 * 99 * 8),
    "well_counts": (lambda: bmc.well_counts(), M * N * 16 + M * 24),
}
out = {}
for name, (f, nbytes) in cases.items():
    ms = timeit(f)
    out[name] = {"ms": ms, "configs_per_s": M / (ms * 1e-3), "algorithmic_bytes": nbytes,
                 "achieved_GBs": nbytes / (ms * 1e-3) / 1e9, "frac_of_8TBs": nbytes / (ms * 1e-3) / 8e12}
out["pair_hist_50bins"]["pair_terms_per_s"] = M * N * (N - 1) / 2 / (out["pair_hist_50bins"]["ms"] * 1e-3)
print(json.dumps(out, indent=1))
