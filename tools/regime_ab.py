"""Algorithm-1 regime (bench.algorithm1_regime) by testing-phase overlap mode: the
pipeline (flowstate.algorithm1._Pipeline), the local-move speculation (_Speculator) and
none, one JSON line each.  argv: attempts, mode set (ab3 / ab / on / local / off)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "flow-state_amd"))
import bench  # noqa: E402

att = int(sys.argv[1]) if len(sys.argv) > 1 else 300
modes = {"ab3": ("local", "pipeline", False, "local", "pipeline"), "ab": ("local", "pipeline", "local", "pipeline"),
         "on": ("pipeline",), "local": ("local",), "off": (False,)}[sys.argv[2] if len(sys.argv) > 2 else "ab"]
for spec in modes:
    r = bench.algorithm1_regime(attempts=att, speculate=spec)
    print(json.dumps({"speculate": spec, "value": r["value"], "seconds": r["seconds"],
                      "speculated": r["speculated_attempts"], "acc": r["big_move_acceptance"]}), flush=True)
