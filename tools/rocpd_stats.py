"""Kernel statistics (rocprofv3 --stats layout) from a rocprofv3 rocpd SQLite database:
python tools/rocpd_stats.py <run_results.db> <out.csv>"""
import csv
import sqlite3
import statistics
import sys


def main(db, out):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else "kernel_name"
    rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
    per = {}
    for name, s, e in rows:
        per.setdefault(name, []).append(e - s)
    total = sum(sum(v) for v in per.values())
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for name, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, len(d), sum(d), sum(d) / len(d), 100.0 * sum(d) / total, min(d), max(d),
                        statistics.pstdev(d)])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
