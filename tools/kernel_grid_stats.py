"""Per-(kernel, grid size) durations from a rocprofv3 --kernel-trace CSV (the --stats
summary averages every launch of a kernel together, e.g. the flow kernel's C-row and
2C-row launches):  python tools/kernel_grid_stats.py <dir with *kernel_trace.csv> > out.json"""
import csv
import glob
import json
import statistics
import sys


def main(d):
    files = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {d}")
    per = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"], int(r.get("Grid_Size") or r["Grid_Size_X"]))
            per.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    out = []
    for (name, grid), ms in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        out.append({"kernel": name[:160], "grid": grid, "calls": len(ms), "avg_ms": statistics.mean(ms),
                    "min_ms": min(ms), "max_ms": max(ms), "total_ms": sum(ms)})
    print(json.dumps(out[:40], indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
