"""Average rocprofv3 --pmc counters per kernel (fs:: kernels only) into JSON, plus the
derived ratios DESIGN.md quotes for the flow kernel.  Usage:
  python tools/pmc_summary.py gpurun_out/pmc_flow1 [gpurun_out/pmc_flow2 ...] > profiles/r01/pmc/x.json
"""
import csv
import json
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        k = r["Kernel_Name"]
        if "fs::" not in k:
            continue
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}
for k, c in out.items():
    d = {}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
        # MFMA busy is summed over 256 CUs x 4 SIMDs; GRBM_GUI_ACTIVE over 8 XCDs
        d["mfma_busy"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 256 * 4)
    if "SQ_WAVE_CYCLES" in c:
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if n in c:
                d[n.lower().replace("sq_", "") + "_frac"] = c[n] / c["SQ_WAVE_CYCLES"]
    if d:
        c["derived"] = d
print(json.dumps(out, indent=1))
