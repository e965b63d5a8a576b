"""GPU-side timeline of the Algorithm-1 pipeline without a profiler: timing events around each
stage's local moves (side stream), density pass (density streams) and big move (main
stream), read after the run.  Prints, for stages 100..(100+rows), the start / end of each
piece in microseconds from the first one, and the medians of the gaps that set the pace.
argv: attempts (default 300), rows (default 12)."""
import json
import os
import statistics as st
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "flow-state_amd"))
import bench  # noqa: E402
from flowstate import algorithm1 as A1  # noqa: E402

att = int(sys.argv[1]) if len(sys.argv) > 1 else 300
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 12
EV = {}


def ev(stream, key):
    e = torch.cuda.Event(enable_timing=True)
    e.record(stream)
    EV[key] = e


P = A1._Pipeline
orig_stage, orig_density, orig_attempt, orig_moves = P.stage, P._density, P.attempt, P._moves


def moves(self, m, k):
    st = torch.cuda.current_stream()
    ev(st, ("m0", k, st.cuda_stream))
    orig_moves(self, m, k)
    ev(st, ("m1", k, st.cuda_stream))


def stage(self, k, *args, **kw):
    ev(self.side, ("L0", k))  # queued on the side stream ahead of the stage's copy (after its waits: below)
    orig_stage(self, k, *args, **kw)
    ev(self.side, ("L1", k))


def density(self, k):
    ds = self.dens[k % len(self.dens)]
    orig_density(self, k)
    ev(ds, ("D1", k))


def attempt(self, k, configs, terms):
    r = orig_attempt(self, k, configs, terms)
    ev(self.main, ("M1", k))
    return r


P.stage, P._density, P.attempt, P._moves = stage, density, attempt, moves
r = bench.algorithm1_regime(attempts=att, speculate="pipeline")
torch.cuda.synchronize()
# the timed run is the second testing phase: its keys are the last `att` stages
ks = sorted({key[1] for key in EV if key[0] == "M1"})
base = EV[("M1", ks[0])]
t = lambda key: base.elapsed_time(EV[key]) * 1e3 if key in EV else float("nan")  # noqa: E731
lo = min(100, max(1, att // 3))
print(json.dumps({"value": r["value"], "seconds": r["seconds"], "speculated": r["speculated_attempts"]}))
print(f"{'k':>4} {'L0':>9} {'L1':>9} {'D1':>9} {'M1':>9}")
for k in range(lo, min(att, lo + rows)):
    print(f"{k:4d} " + " ".join(f"{t((n, k)):9.1f}" for n in ("L0", "L1", "D1", "M1")))
per = [t(("M1", k + 1)) - t(("M1", k)) for k in range(lo, att - 5)]
l_to_d = [t(("D1", k)) - t(("L1", k)) for k in range(lo, att - 5)]
d_to_m = [t(("M1", k)) - t(("D1", k)) for k in range(lo, att - 5)]
l_gap = [t(("L1", k + 1)) - t(("L1", k)) for k in range(lo, att - 5)]
m_to_l0 = [t(("L0", k + 3)) - t(("M1", k)) for k in range(lo, att - 5)]
side = {key[2] for key in EV if key[0] == "m0"}
lm = [base.elapsed_time(EV[("m1", k, sd)]) * 1e3 - base.elapsed_time(EV[("m0", k, sd)]) * 1e3
      for k in range(lo, att - 5) for sd in side if ("m0", k, sd) in EV and ("m1", k, sd) in EV]
print(json.dumps({"median_local_moves_launch_us": st.median(lm), "median_period_us": st.median(per), "median_L1_to_D1": st.median(l_to_d),
                  "median_D1_to_M1": st.median(d_to_m), "median_L1_step": st.median(l_gap),
                  "median_M1k_to_L0k+3": st.median(m_to_l0)}))
