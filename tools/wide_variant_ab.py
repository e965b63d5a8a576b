"""Wide-path A/B of a library variant (FLOWSTATE_LIB, tools/build_variant.sh): the
Algorithm-1 regime (speculative testing phase) and config 2 one step per launch.
One JSON line; run once per variant, each in its own process."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

att = int(sys.argv[1]) if len(sys.argv) > 1 else 300
r = [bench.algorithm1_regime(attempts=att)["value"] for _ in range(2)]
c = bench.config2(steps=16)
print(json.dumps({"lib": os.environ.get("FLOWSTATE_LIB") or "in-tree", "regime": r,
                  "config2_one_step": c["one_step_per_launch"]["value"], "config2": c["value"]}), flush=True)
