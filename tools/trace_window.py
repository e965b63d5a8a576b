"""Summarise a rocprofv3 kernel trace after the last marker kernel (torch.cuda._sleep):
per-replay kernel count, busy time (sum of kernel durations), the span from the first
start to the last end, and the top kernels.  Usage:
  python tools/trace_window.py gpurun_out/prof_graph/run_kernel_trace.csv REPLAYS [seq] > summary.json
With "seq", the summary also lists the last replay's kernels in order (name, µs)."""
import csv
import json
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
reps = int(sys.argv[2])
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = max(i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"])
win = rows[last + 1:]
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win)
span = int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])
per = defaultdict(lambda: [0, 0])
for r in win:
    k = r["Kernel_Name"][:120]
    per[k][0] += 1
    per[k][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
top = sorted(per.items(), key=lambda kv: -kv[1][1])[:30]
print(json.dumps({"replays": reps, "kernels_per_replay": len(win) / reps, "busy_ms_per_replay": busy / reps / 1e6,
                  "span_ms_per_replay": span / reps / 1e6,
                  "top": [{"kernel": k, "calls_per_replay": c / reps, "ms_per_replay": t / reps / 1e6} for k, (c, t) in top],
                  **({"sequence": [[r["Kernel_Name"][:90], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3]
                                   for r in win[-(len(win) // reps):]]} if "seq" in sys.argv[3:] else {})},
                 indent=1))
