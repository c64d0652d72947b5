"""Print the kernel timeline of the last full training step in a rocprofv3 kernel_trace.csv."""
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                     int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)))
rows.sort()
idx = [i for i, r in enumerate(rows) if r[2].startswith("adam") and "tick" not in r[2]]
s, e = idx[-2] + 1, idx[-1] + 1
tot = 0
for st, en, name, g in rows[s:e]:
    d = (en - st) / 1e3
    tot += d
    if d >= float(sys.argv[2]) if len(sys.argv) > 2 else 20:
        print("%-44s grid=%-9d %9.1f us" % (name, g, d))
print("sum of kernel time in step: %.3f ms; wall %.3f ms" % (tot / 1e3, (rows[e - 1][1] - rows[s][0]) / 1e6))
