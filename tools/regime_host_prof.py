"""Host-side time of the Algorithm-1 pipeline (flowstate.algorithm1._Pipeline): wraps its
methods with wall-clock timers and runs bench.algorithm1_regime, then prints the mean and
total host time per method (learn = the wait for the previous big move; attempt / stage /
_density = submission).  argv: attempts (default 300), mode (default pipeline)."""
import json
import os
import sys
import time
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "flow-state_amd"))
import bench  # noqa: E402
from flowstate import algorithm1 as A1  # noqa: E402

att = int(sys.argv[1]) if len(sys.argv) > 1 else 300
mode = sys.argv[2] if len(sys.argv) > 2 else "pipeline"
acc = defaultdict(lambda: [0, 0.0])


def timed(cls, name):
    f = getattr(cls, name)

    def w(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            acc[f"{cls.__name__}.{name}"][0] += 1
            acc[f"{cls.__name__}.{name}"][1] += time.perf_counter() - t

    setattr(cls, name, w)


for n in ("learn", "attempt", "stage", "_density", "_moves", "_copy"):
    timed(A1._Pipeline, n)
for n in ("begin", "finish"):
    timed(A1._Speculator, n)
timed(A1.BatchedMonteCarlo, "nf_big_move")
timed(A1.BatchedMonteCarlo, "state_nll")
r = bench.algorithm1_regime(attempts=att, speculate=mode)
print(json.dumps({"mode": mode, "value": r["value"], "seconds": r["seconds"], "speculated": r["speculated_attempts"]}))
for k, (c, t) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
    print(f"{k:36s} calls {c:6d}  total {t * 1e3:9.1f} ms  mean {t / max(c, 1) * 1e6:8.1f} us")
