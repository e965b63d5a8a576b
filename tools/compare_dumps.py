"""Compare the per-chain final states of a sharded bench run (bench.py --dump A, world W)
with a 1-rank run over the same global chains (--dump B): every array concatenated in
chain-offset order must be identical.  Usage: compare_dumps.py A B  (prefixes)."""
import glob
import json
import sys

import numpy as np


def load(prefix):
    parts = [np.load(p) for p in sorted(glob.glob(prefix + ".rank*.npz"))]
    parts.sort(key=lambda z: int(z["chain_offset"]))
    keys = [k for k in parts[0].files if k != "chain_offset"]
    return len(parts), [int(z["chain_offset"]) for z in parts], {k: np.concatenate([z[k] for z in parts]) for k in keys}


wa, offs_a, a = load(sys.argv[1])
wb, offs_b, b = load(sys.argv[2])
res = {"ranks_a": wa, "offsets_a": offs_a, "ranks_b": wb, "chains": int(len(a["E_old"])),
       "identical": {k: bool(a[k].shape == b[k].shape
                             and np.array_equal(a[k], b[k], equal_nan=a[k].dtype.kind == "f"))
                     for k in a},
       "accepted_total": int(a["accepted"].sum()), "attempts_total": int(a["attempts"].sum())}
res["all_identical"] = all(res["identical"].values())
print(json.dumps(res))
sys.exit(0 if res["all_identical"] else 1)
