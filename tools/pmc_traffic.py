"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes.

gfx950 calibration (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes
of wide coalesced 16-B-per-lane reads -> x2; WRITE_SIZE is exact for 16-B stores.
Both are in KiB.  Usage:
  python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write > profiles/traffic.json
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(d, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if r["Counter_Name"] == counter:
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
write = per_kernel(sys.argv[2], "WRITE_SIZE")
out = {"note": "bytes per launch = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE counts half of wide reads)",
       "kernels": {}}
flow = []
for k in fetch:
    if not k.startswith(("fs::", "void fs::")):
        continue
    b = 2 * fetch[k] * 1024 + write.get(k, 0.0) * 1024
    out["kernels"][k] = b
    if "flow_pass_kernel<256, 32" in k:
        flow.append(b)
out["flow_pass_bytes_per_launch"] = sum(flow) / len(flow) if flow else None
print(json.dumps(out, indent=1))
