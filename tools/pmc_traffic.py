"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes,
keyed by kernel AND grid size (a launch's row count: the flow kernels run 64 chains per
512-thread workgroup, so C rows = C/64*512 work-items; the hybrid step's 2C-row density
launch is a separate entry instead of being averaged in).

gfx950 calibration (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes
of wide coalesced 16-B-per-lane reads -> x2; WRITE_SIZE is exact for 16-B stores.
Both are in KiB.  Usage (in the build container, after the box's passes came back):
  python tools/pmc_traffic.py gpurun_out/<tag>_pmc_FETCH_SIZE gpurun_out/<tag>_pmc_WRITE_SIZE \
      > profiles/traffic.json
"""
import csv
import json
import os
import subprocess
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import flow_source_sha16  # noqa: E402


def per_kernel(d, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if r["Counter_Name"] == counter:
            vals[(r["Kernel_Name"], r["Grid_Size"])].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in vals.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    try:
        head = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True,
                              check=True).stdout.strip()
    except (OSError, subprocess.CalledProcessError):
        head = None
    out = {"note": "bytes per launch = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE counts half of "
                   "wide reads); kernels[name][grid_size] = [bytes, launches averaged]",
           "head": head, "flow_src_sha16": flow_source_sha16(), "source": [sys.argv[1], sys.argv[2]],
           "kernels": {}}
    for (k, grid), (f, n) in sorted(fetch.items()):
        if not k.startswith(("fs::", "void fs::")):
            continue
        w = write.get((k, grid), (0.0, 0))[0]
        out["kernels"].setdefault(k, {})[grid] = [2 * f * 1024 + w * 1024, n]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
