"""Print the kernel timeline of the last full training step (adam to adam) in a rocprofv3 kernel_trace.csv: start
offset, queue (compute stream / weight-gradient side stream), duration and grid; then per-queue busy time.

usage: python tools/step_timeline.py <kernel_trace.csv> [min_us]"""
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                     int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0), r.get("Queue_Id", "?")))
rows.sort()
idx = [i for i, r in enumerate(rows) if r[2].startswith("adam") and "tick" not in r[2]]
s, e = idx[-2] + 1, idx[-1] + 1
mn = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
t0 = rows[s][0]
busy = {}
for st, en, name, g, q in rows[s:e]:
    d = (en - st) / 1e3
    busy[q] = busy.get(q, 0.0) + d
    if d >= mn:
        print("%8.1f  q%-3s %-44s grid=%-9d %8.1f us" % ((st - t0) / 1e3, q, name[:44], g, d))
for q, b in sorted(busy.items()):
    print("queue %s busy %.3f ms" % (q, b / 1e3))
print("step wall %.3f ms (kernel trace; the profiler's per-launch cost stretches the host-bound stretches)"
      % ((rows[e - 1][1] - rows[s][0]) / 1e6))
