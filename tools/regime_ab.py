"""Algorithm-1 regime (bench.algorithm1_regime) with and without the speculative local
moves (flowstate.algorithm1._Speculator), one JSON line each."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "flow-state_amd"))
import bench  # noqa: E402

att = int(sys.argv[1]) if len(sys.argv) > 1 else 300
modes = {"ab": (False, True, False, True), "on": (True,), "off": (False,)}[sys.argv[2] if len(sys.argv) > 2 else "ab"]
for spec in modes:
    r = bench.algorithm1_regime(attempts=att, speculate=spec)
    print(json.dumps({"speculate": spec, "value": r["value"], "seconds": r["seconds"],
                      "speculated": r["speculated_attempts"], "acc": r["big_move_acceptance"]}), flush=True)
